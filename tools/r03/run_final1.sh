#!/bin/bash
# r03 final pass 1: the whole GPU suite, then headline profiles (kernel trace + PMC passes).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03final
mkdir -p $O
export TMPDIR=/tmp
bash tools/r03/profile.sh final || exit $?
echo done >&2
