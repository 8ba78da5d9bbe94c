#!/bin/bash
# r06 run 18: kernel trace of the 125-ciphertext slice (one rank's share of C3 at 8 GPUs)
source "$(dirname "$0")/lib.sh"
rm -rf gpurun_out/prof_bench_125ct_128b
step 600 bash tools/profile.sh bench_125ct_128b --cts 125
echo all-done >&2
