#!/bin/bash
# r05 session 7: C4's exact-check count (leaf list length) and C2's, to see why C4 sends ~20 % of
# its shares to the leaf checks at 1 % wrong shares.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run7
mkdir -p $O
step 300 python -u bench_configs.py --configs c4,c2 --no-cpu --steps 3 > $O/c42.json 2>> $O/c42.err
HBTC_TRACK=0 step 300 python -u bench_configs.py --configs c4 --no-cpu --steps 3 > $O/c4_notrack.json 2>> $O/c42.err
echo all-done >&2
