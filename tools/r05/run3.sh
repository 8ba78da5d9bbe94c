#!/bin/bash
# r05 session 3: hbtc_coin_decide (one coin round per call: checks + speculative combine + master
# check by the G1 identity) against the separate entry points; c1 / C2 lines.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run3
mkdir -p $O
step 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_coin_decide.py tests/test_gpu_comb_small.py tests/test_gpu_msm.py > $O/pytest.log 2>&1
step 300 python -u bench_configs.py --configs c1,c2 --no-cpu > $O/c12.json 2>> $O/c12.err
HBTC_COIN_SPEC=0 step 300 python -u bench_configs.py --configs c1 --no-cpu > $O/c1_nospec.json 2>> $O/c12.err
echo all-done >&2
