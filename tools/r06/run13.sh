#!/bin/bash
# r06 run 13: the headline profile (kernel trace + full-size PMC passes) and bench line on the
# build with the lane-pair G2 kernels (k_g2_steps_pair in C3's table build)
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run13
mkdir -p $O
rm -rf gpurun_out/prof_bench_1000ct_128b
step 900 bash tools/profile.sh bench_1000ct_128b
rm -rf profiles/r06/bench_1000ct_128b && cp -r gpurun_out/prof_bench_1000ct_128b profiles/r06/bench_1000ct_128b
step 300 python -u bench.py > $O/bench.json 2> $O/bench.err
echo all-done >&2
