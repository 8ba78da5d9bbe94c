#!/bin/bash
# r04 GPU session 12: rocprofv3 evidence at the round's build for the bench.py workloads
# (bench.py reads profiles/r04/bench_<cts>ct_<bits>b/ for its roofline).
cd "$(dirname "$0")/../.." || exit 1
bash tools/r04/profile.sh bench_1000ct_128b || exit $?
bash tools/r04/profile.sh bench_125ct_128b --cts 125 || exit $?
echo all-done >&2
