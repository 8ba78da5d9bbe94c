#!/bin/bash
# r05 session 14 (rejected: the 125 slice 13.6 -> 26.6 ms, 250 unchanged; the variant was removed): the paired check levels (tiles -> leaves) in the latency form (HBTC_PAIR_REP=3,
# one group per wave) against the throughput form (five per wave): parity with the mode on, then
# the 125 / 250-ciphertext slices and C3 A/B on one box.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run14
mkdir -p $O
HBTC_PAIR_REP=3 step 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "rlc_single or batch_mode or 128bit or back_to_back" tests/test_gpu_split.py > $O/parity.log 2>&1
for p in 1 3 1 3; do
  for n in 125 250; do
    HBTC_PAIR_REP=$p step 150 python -u bench.py --no-cpu --no-extra --cts $n > $O/s${n}_p$p.$RANDOM.json 2>> $O/s.err
  done
done
echo all-done >&2
