#!/bin/bash
# r05 session 18: k_rlc_items' table as a co-Z chain with entries 5..7 formed in LDS (572 -> 120
# B/lane of scratch) and k_rlc_decode's operands parked in memory (332 -> 192): the RLC parity
# tests, then C3 and the slices against the previous build (old).
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run18
mkdir -p $O
step 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_split.py > $O/parity.log 2>&1
for v in old base old base; do
  HBTC_LIB_PATH=$(lib $v) step 150 python -u bench.py --no-cpu --no-extra > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
done
for v in old base; do
  for n in 125 250; do HBTC_LIB_PATH=$(lib $v) step 150 python -u bench.py --no-cpu --no-extra --cts $n > $O/s${n}_$v.json 2>> $O/s.err; done
done
echo all-done >&2
