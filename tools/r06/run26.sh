#!/bin/bash
# r06 run 26: the config tests (they drive bench_configs.bench_coins) after the isolated-step addition
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run26
mkdir -p $O
step 900 python -u -m pytest -v -x --timeout 400 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_multi_rank.py > $O/pytest.log 2>&1
echo all-done >&2
