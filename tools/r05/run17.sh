#!/bin/bash
# r05 session 17 (no gain either way; serial kept): item passes of the lanes serialised (HBTC_ITEMS_SERIAL=1, default) or free to
# overlap (0): the 125 / 250-ciphertext slices and C3.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run17
mkdir -p $O
for p in 1 0 1 0; do
  for n in 125 250; do
    HBTC_ITEMS_SERIAL=$p step 150 python -u bench.py --no-cpu --no-extra --cts $n > $O/s${n}_ser$p.$RANDOM.json 2>> $O/s.err
  done
done
for p in 1 0; do HBTC_ITEMS_SERIAL=$p step 150 python -u bench.py --no-cpu --no-extra > $O/c3_ser$p.json 2>> $O/c3.err; done
echo all-done >&2
