#!/bin/bash
# r06 run 25: C2 / C4 lines with the isolated item-pass roofline point
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run25
mkdir -p $O
step 600 python -u bench_configs.py --configs c2,c4 --no-cpu > $O/configs.json 2> $O/configs.err
echo all-done >&2
