#!/bin/bash
# r05 session 24 (71.2 vs 71.4 ms, within noise; three waves kept for the smaller frame): k_rlc_decode at four waves per SIMD (dw4: 128 VGPRs, 524 B/lane, table entries
# of the square-root window re-read in the loop) against three (base): C3.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run24
mkdir -p $O
for v in dw4 base dw4 base dw4 base; do
  HBTC_LIB_PATH=$(lib $v) step 150 python -u bench.py --no-cpu --no-extra > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
done
echo all-done >&2
