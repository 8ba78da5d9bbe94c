#!/bin/bash
# r04 GPU session 13: rocprofv3 evidence for the 250-ciphertext slice and kernel traces of the
# configuration lines c1, c2, c4.
cd "$(dirname "$0")/../.." || exit 1
bash tools/r04/profile.sh bench_250ct_128b --cts 250 || exit $?
bash tools/r04/profile_configs.sh c1 c2 c4 || exit $?
echo all-done >&2
