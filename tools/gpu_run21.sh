#!/bin/bash
# k_hash_cand register cap: hash tests, then C5 capped vs uncapped.
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/hw
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hash.py -m gpu > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python3 -u bench_configs.py --configs c5 > $O/cap_c5.json 2> $O/cap_c5.err || exit $?
HBTC_LIB_PATH=$PWD/hbbft_amd/libhbtc_hw1.so timeout -k 10 200 python3 -u bench_configs.py --configs c5 > $O/base_c5.json 2> $O/base_c5.err || exit $?
