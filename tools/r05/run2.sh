#!/bin/bash
# r05 session 2: the small combines (hbtc_comb.hip) and three of the eight x-adic entries in LDS
# (default) against the 8-entry table at two waves without LDS (s8w2).  Parity first.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run2
mkdir -p $O
step 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_comb_small.py tests/test_gpu_parity.py tests/test_gpu_msm.py tests/test_gpu_split.py tests/test_gpu_coin_agreement.py > $O/pytest.log 2>&1
for v in base s8w2 base s8w2; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench.py --no-cpu --no-extra > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
done
step 300 python -u bench_configs.py --configs c1,c2 --no-cpu > $O/c12_small.json 2>> $O/c12.err
HBTC_COMB_SMALL=0 step 300 python -u bench_configs.py --configs c1,c2 --no-cpu > $O/c12_pip.json 2>> $O/c12.err
echo all-done >&2
