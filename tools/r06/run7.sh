#!/bin/bash
# r06 run 7: k_plines_pair at one wave (plw1) and with nops before the DPP exchanges (xnop)
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run7
mkdir -p $O
HBTC_LIB_PATH=$(lib plw1) step 200 python -u tools/r06/dbg_coin64.py > $O/plw1.txt 2>&1
HBTC_LIB_PATH=$(lib xnop) step 200 python -u tools/r06/dbg_coin64.py > $O/xnop.txt 2>&1
head -3 $O/plw1.txt $O/xnop.txt
echo all-done >&2
