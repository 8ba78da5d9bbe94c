#!/bin/bash
# r06 run 1: the re-validated VALU peak (tools/microbench/intmul.hip, in-kernel clock + issue cost)
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run1
mkdir -p $O
step 300 ./tools/microbench/intmul > $O/intmul.txt 2>&1
cat $O/intmul.txt
