#!/bin/bash
# r05 session 21: k_sig_decode's psi subgroup test re-reading P from memory at its five additions
# (base: 772 -> 588 B/lane at two waves per SIMD) and the same at one wave (sd1: 0 B/lane),
# against the previous kernel (sgold): signature parity tests, then C4 and C2.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run21
mkdir -p $O
step 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_coin_decide.py tests/test_gpu_comb_small.py > $O/parity.log 2>&1
HBTC_LIB_PATH=$(lib sd1) step 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "sig or c1 or codec" > $O/parity_sd1.log 2>&1
for v in sgold base sd1 sgold base sd1; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_$v.$RANDOM.json 2>> $O/c4.err
done
for v in sgold base sd1; do
  HBTC_LIB_PATH=$(lib $v) step 200 python -u bench_configs.py --configs c2 --no-cpu > $O/c2_$v.json 2>> $O/c2.err
done
echo all-done >&2
