#!/bin/bash
# r05 session 8: Lagrange coefficients from factorial tables (k_lagrange_fact) and the sized leaf
# chunks of SignatureShare calls: combine / parity tests, then C3, C4 and the 125 / 250 slices.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run8
mkdir -p $O
step 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_msm.py tests/test_gpu_configs.py > $O/pytest.log 2>&1
step 150 python -u bench.py --no-cpu --no-extra > $O/c3.json 2>> $O/c3.err
HBTC_LAGRANGE_FACT=0 step 150 python -u bench.py --no-cpu --no-extra > $O/c3_nofact.json 2>> $O/c3.err
step 300 python -u bench_configs.py --configs c4 --no-cpu > $O/c4.json 2>> $O/c4.err
for n in 125 250; do step 200 python -u bench.py --no-cpu --no-extra --cts $n > $O/slice$n.json 2>> $O/slice.err; done
echo all-done >&2
