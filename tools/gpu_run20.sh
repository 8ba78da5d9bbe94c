#!/bin/bash
# k_msm_buckets (G1) register cap: combine tests, then C3 (1000, 125) and C5, capped vs uncapped.
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/bw
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_parity.py -m gpu > $O/tests.log 2>&1 || exit $?
for v in cap base; do
  if [ $v = base ]; then export HBTC_LIB_PATH=$PWD/hbbft_amd/libhbtc_bw1.so; fi
  for c in 1000 125; do
    timeout -k 10 150 python -u bench.py --no-cpu --no-extra --steps 20 --cts $c > $O/${v}_$c.json 2> $O/${v}_$c.err || exit $?
  done
  timeout -k 10 200 python3 -u bench_configs.py --configs c5 > $O/${v}_c5.json 2> $O/${v}_c5.err || exit $?
done
