#!/bin/bash
# r05 session 16: kernel traces of the configurations c1, c2, c4 with the final round-5 build
# (tools/profile.sh CONFIG mode -> gpurun_out/prof_cfg_<c>/, committed as profiles/r05/configs/<c>/).
source "$(dirname "$0")/lib.sh"
for c in c1 c2 c4; do
  CONFIG=$c step 400 bash tools/profile.sh cfg_$c
done
echo all-done >&2
