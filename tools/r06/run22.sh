#!/bin/bash
# r06 run 22: small item passes staggered behind the previous lane's decode (HBTC_ITEMS_SERIAL=2)
# against the default (1): the 125 / 250-ciphertext slices and C3, interleaved
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run22
mkdir -p $O
for r in a b; do
  for v in 2 1; do
    for n in 125 250; do
      HBTC_ITEMS_SERIAL=$v step 300 python -u bench.py --cts $n --no-cpu --no-extra >> $O/s${n}_$v.json 2>> $O/err.log
    done
  done
done
for v in 2 1; do
  HBTC_ITEMS_SERIAL=$v step 300 python -u bench.py --no-cpu --no-extra >> $O/c3_$v.json 2>> $O/err.log
done
echo all-done >&2
