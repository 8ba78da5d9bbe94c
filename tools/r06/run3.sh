#!/bin/bash
# r06 run 3: k_sig_items and the G2 small combine in lane-pair form (pair.h) against the one-lane
# kernels (nopair): the signature / coin / pair-batch / config tests, then C4, C2 and c1 A/B/A/B.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run3
mkdir -p $O
step 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_coin_decide.py tests/test_gpu_comb_small.py tests/test_gpu_pair_batch.py tests/test_gpu_configs.py tests/test_gpu_coin_agreement.py > $O/pytest.log 2>&1
for v in nopair base nopair base; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_$v.$RANDOM.json 2>> $O/c4.err
done
for v in nopair base; do
  HBTC_LIB_PATH=$(lib $v) step 200 python -u bench_configs.py --configs c2,c1 --no-cpu > $O/c2c1_$v.json 2>> $O/c2.err
done
echo all-done >&2
