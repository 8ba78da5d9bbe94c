#!/bin/bash
# r05 session 10: check levels on per-lane high-priority streams (OnCheckStream) against the lane
# stream (HBTC_CHECK_PRIO=0): parity subset, then C3, the slices, C2 / C4, A/B on one box.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run10
mkdir -p $O
step 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py tests/test_gpu_coin_decide.py > $O/pytest.log 2>&1
for p in 1 0 1 0; do
  HBTC_CHECK_PRIO=$p step 150 python -u bench.py --no-cpu --no-extra > $O/c3_p$p.$RANDOM.json 2>> $O/c3.err
done
for p in 1 0; do
  for n in 125 250; do HBTC_CHECK_PRIO=$p step 150 python -u bench.py --no-cpu --no-extra --cts $n > $O/s${n}_p$p.json 2>> $O/s.err; done
  HBTC_CHECK_PRIO=$p step 300 python -u bench_configs.py --configs c2,c4 --no-cpu > $O/c24_p$p.json 2>> $O/c24.err
done
echo all-done >&2
