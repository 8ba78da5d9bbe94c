#!/bin/bash
# r04 GPU session 26: rocprofv3 evidence at the round's final build: the three bench.py
# workloads (bench.py reads profiles/r04/bench_<cts>ct_<bits>b/) and kernel traces of c1, c2, c4.
cd "$(dirname "$0")/../.." || exit 1
bash tools/r04/profile.sh bench_1000ct_128b || exit $?
bash tools/r04/profile.sh bench_125ct_128b --cts 125 || exit $?
bash tools/r04/profile.sh bench_250ct_128b --cts 250 || exit $?
bash tools/r04/profile_configs.sh c1 c2 c4 || exit $?
echo all-done >&2
