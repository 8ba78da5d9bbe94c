#!/bin/bash
# r05 session 20: the headline profile (kernel trace + SQ / FETCH_SIZE / WRITE_SIZE passes) of the
# build with the co-Z chain table (tools/profile.sh -> profiles/r05/bench_1000ct_128b/).
source "$(dirname "$0")/lib.sh"
rm -rf gpurun_out/prof_bench_1000ct_128b
step 900 bash tools/profile.sh bench_1000ct_128b
echo all-done >&2
