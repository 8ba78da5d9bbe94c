#!/bin/bash
# r05 session 1: k_rlc_items with the sign-aligned 8-entry table in registers at one wave per SIMD
# (default build, curve.h xadic_mul_sac8, 0 B/lane scratch) against the 15-entry scratch table
# (t16: -DHBTC_XADIC8=0, two waves) and the 8-entry table at two waves (s8w2).  Parity first.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run1
mkdir -p $O
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_coin_agreement.py > $O/pytest.log 2>&1
for v in base t16 s8w2 base t16; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench.py --no-cpu --no-extra > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
done
echo all-done >&2
