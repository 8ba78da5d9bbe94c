#!/bin/bash
# r05 session 6: rocprofv3 evidence of this round's build: the C3 headline workload (kernel trace
# with per-launch durations + SQ / FETCH_SIZE / WRITE_SIZE passes) and kernel traces of c1, C2, C4.
source "$(dirname "$0")/lib.sh"
step 900 bash tools/profile.sh bench_1000ct_128b
for c in c4 c2 c1; do CONFIG=$c step 400 bash tools/profile.sh cfg_$c; done
echo all-done >&2
