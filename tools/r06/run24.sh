#!/bin/bash
# r06 run 24: the rep-1 check kernels at two waves per SIMD (gtw2) against three (base) now that
# their operands are staged in LDS: C3 (+ adversarial) interleaved
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run24
mkdir -p $O
for v in gtw2 base gtw2 base; do
  HBTC_LIB_PATH=$(lib $v) step 400 python -u bench.py --no-cpu >> $O/c3_$v.json 2>> $O/err.log
done
echo all-done >&2
