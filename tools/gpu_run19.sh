#!/bin/bash
# k_msm_decode register cap: MSM / SyncKeyGen tests, then C5 with 2 (default), 1 and 4 waves.
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/dw
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_skg.py tests/test_gpu_skg_protocol.py -m gpu > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python3 -u bench_configs.py --configs c5 > $O/c5_w2.json 2> $O/c5_w2.err || exit $?
HBTC_LIB_PATH=$PWD/hbbft_amd/libhbtc_dw1.so timeout -k 10 200 python3 -u bench_configs.py --configs c5 > $O/c5_w1.json 2> $O/c5_w1.err || exit $?
HBTC_LIB_PATH=$PWD/hbbft_amd/libhbtc_dw4.so timeout -k 10 200 python3 -u bench_configs.py --configs c5 > $O/c5_w4.json 2> $O/c5_w4.err || exit $?
