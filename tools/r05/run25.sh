#!/bin/bash
# r05 session 25: k_sig_decode in its own object with the Fq product inlined (base: 432 B/lane, no
# scratch in its loops) against the shared-subroutine build (sgsr: 588 B/lane, the G2 doubling
# loop re-reading spilled state): signature parity tests, then C4, C2 and c1.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run25
mkdir -p $O
step 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_coin_decide.py tests/test_gpu_comb_small.py tests/test_gpu_configs.py tests/test_gpu_coin_agreement.py > $O/parity.log 2>&1
for v in sgsr base sgsr base; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_$v.$RANDOM.json 2>> $O/c4.err
done
for v in sgsr base; do
  HBTC_LIB_PATH=$(lib $v) step 200 python -u bench_configs.py --configs c2,c1 --no-cpu > $O/c2c1_$v.json 2>> $O/c2.err
done
echo all-done >&2
