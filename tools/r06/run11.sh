#!/bin/bash
# r06 run 11: kernel traces of c1, c2, c4 on the round-6 build (tools/profile.sh CONFIG=...), and C4
# with the one-lane decode (nosdp) for the decode kernels' durations
source "$(dirname "$0")/lib.sh"
for c in c1 c2 c4; do
  rm -rf gpurun_out/prof_cfg_$c
  CONFIG=$c step 600 bash tools/profile.sh cfg_$c
done
rm -rf gpurun_out/prof_cfg_c4_nosdp
HBTC_LIB_PATH=$(lib nosdp) CONFIG=c4 step 600 bash tools/profile.sh cfg_c4_nosdp
echo all-done >&2
