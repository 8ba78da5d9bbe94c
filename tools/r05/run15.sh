#!/bin/bash
# r05 session 15 (kept 4: the gain needs more epochs in flight than hbbft has): verification lanes (epochs in flight) 4 (base) / 6 / 8: the 125 / 250-ciphertext
# slices and C3.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run15
mkdir -p $O
for v in base l6 l8 base l6 l8; do
  for n in 125 250; do
    HBTC_LIB_PATH=$(lib $v) step 150 python -u bench.py --no-cpu --no-extra --cts $n > $O/s${n}_$v.$RANDOM.json 2>> $O/s.err
  done
done
for v in base l6 l8; do
  HBTC_LIB_PATH=$(lib $v) step 150 python -u bench.py --no-cpu --no-extra > $O/c3_$v.json 2>> $O/c3.err
done
echo all-done >&2
