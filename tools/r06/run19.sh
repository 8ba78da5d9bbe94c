#!/bin/bash
# r06 run 19: SQ counters of C4 (bench_configs c4) for the SignatureShare item kernels
source "$(dirname "$0")/lib.sh"
OUT=gpurun_out/r06run19
mkdir -p $OUT
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
step 300 rocprofv3 --pmc $SQ --output-format csv -d $OUT/sq -o pmc -- python3 bench_configs.py --configs c4 --no-cpu > $OUT/sq.log 2>&1
python3 tools/pmc_summary.py $OUT/pmc_summary.json $OUT/sq > $OUT/pmc_summary.txt 2>&1
rm -rf $OUT/sq
echo all-done >&2
