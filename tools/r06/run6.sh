#!/bin/bash
# r06 run 6: which lane-pair kernel breaks the RLC leaves (dbg_coin64.py on variants)
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run6
mkdir -p $O
HBTC_LIB_PATH=$(lib noplp) step 200 python -u tools/r06/dbg_coin64.py > $O/noplp.txt 2>&1
HBTC_LIB_PATH=$(lib nostep) step 200 python -u tools/r06/dbg_coin64.py > $O/nostep.txt 2>&1
head -3 $O/noplp.txt $O/nostep.txt
echo all-done >&2
