#!/bin/bash
# r05 session 9: kernel traces of the 125- and 250-ciphertext slices (one rank's share of an epoch
# at 8 / 4 GPUs) for the slice work.
source "$(dirname "$0")/lib.sh"
step 400 bash tools/profile.sh bench_125ct_128b --cts 125
step 400 bash tools/profile.sh bench_250ct_128b --cts 250
echo all-done >&2
