#!/bin/bash
# r05 session 12: the DecryptionShare item pass split in two kernels (k_rlc_decode at 2 / 3 waves
# per SIMD, then the scalar half) against the single kernel (base): parity, then C3 and the slice.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run12
mkdir -p $O
HBTC_LIB_PATH=$(lib sp2) step 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_split.py > $O/pytest_sp2.log 2>&1
for v in base sp2 sp3 base sp2 sp3; do
  HBTC_LIB_PATH=$(lib $v) step 150 python -u bench.py --no-cpu --no-extra > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
done
for v in base sp2 sp3; do
  HBTC_LIB_PATH=$(lib $v) step 150 python -u bench.py --no-cpu --no-extra --cts 125 > $O/s125_$v.json 2>> $O/s.err
done
echo all-done >&2
