#!/bin/bash
# r06 run 5: debug of the 64-instance coin case (tools/r06/dbg_coin64.py) on base, unfused, nopair
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run5
mkdir -p $O
step 200 python -u tools/r06/dbg_coin64.py > $O/base.txt 2>&1
HBTC_SIG_FUSED=0 step 200 python -u tools/r06/dbg_coin64.py > $O/unfused.txt 2>&1
HBTC_LIB_PATH=$(lib nopair) step 200 python -u tools/r06/dbg_coin64.py > $O/nopair.txt 2>&1
cat $O/*.txt
echo all-done >&2
