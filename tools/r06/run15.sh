#!/bin/bash
# r06 run 15: k_rlc_decode at two waves (233 VGPRs, no scratch) against three (168, 192 B/lane),
# C3 twice each, interleaved
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run15
mkdir -p $O
for v in dec2 base dec2 base; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench.py --no-cpu --no-extra >> $O/c3_$v.json 2>> $O/c3.err
done
echo all-done >&2
