#!/bin/bash
# Lagrange scan: combine parity tests, then C2 and the 125 / 1000 ciphertext C3 lines.
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/lag
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_msm.py tests/test_protocol.py tests/test_gpu_configs.py tests/test_gpu_skg.py tests/test_gpu_skg_protocol.py -m gpu > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python3 -u bench_configs.py --configs c2 > $O/c2.json 2> $O/c2.err || exit $?
for c in 125 1000; do
  timeout -k 10 150 python -u bench.py --no-cpu --no-extra --steps 12 --cts $c > $O/c3_$c.json 2> $O/c3_$c.err || exit $?
done
