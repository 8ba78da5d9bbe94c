#!/bin/bash
# r05 session 23: square roots by a width-4 sliding window (8 odd powers: 25 products fewer per
# root) against width 3 (w3): codec / hash / parity tests, then C3 and C4.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run23
mkdir -p $O
step 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_hash.py tests/test_gpu_split.py > $O/parity.log 2>&1
for v in w3 base w3 base w3 base; do
  HBTC_LIB_PATH=$(lib $v) step 150 python -u bench.py --no-cpu --no-extra > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
done
for v in w3 base; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_$v.json 2>> $O/c4.err
done
echo all-done >&2
