#!/bin/bash
# G1 GLV combine: parity tests, then C3 at 1000 / 250 / 125 ciphertexts (the rank slices of the
# strong-scaling bench) with and without the split.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/glv
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_msm.py tests/test_protocol.py tests/test_gpu_configs.py tests/test_gpu_skg.py -m gpu > gpurun_out/glv/tests.log 2>&1 || exit $?
for c in 1000 250 125; do
  timeout -k 10 150 python -u bench.py --no-cpu --no-extra --steps 12 --cts $c > gpurun_out/glv/glv_$c.json 2> gpurun_out/glv/glv_$c.err || exit $?
  HBTC_G1_GLV=0 timeout -k 10 150 python -u bench.py --no-cpu --no-extra --steps 12 --cts $c > gpurun_out/glv/base_$c.json 2> gpurun_out/glv/base_$c.err || exit $?
done
