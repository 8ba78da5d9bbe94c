#!/bin/bash
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run9
mkdir -p $O
step 200 python -u tools/r06/dbg_golden.py > $O/golden.txt 2>&1
cat $O/golden.txt
echo all-done >&2
