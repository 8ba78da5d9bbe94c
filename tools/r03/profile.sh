#!/bin/bash
# Headline profiles of the current code (C3, RLC): kernel trace + stats, SQ / FETCH / WRITE PMC
# passes (each its own run), summarised by tools/pmc_summary.py; then an extra SQ pass of stall
# and memory-instruction counters.  Usage: tools/r03/profile.sh TAG
cd "$(dirname "$0")/../.." || exit 1
TAG=${1:-r03}
O=gpurun_out/prof_$TAG
mkdir -p $O
export TMPDIR=/tmp
# no cold-key-set probe pass: its small first call would join the per-dispatch means
export HBTC_PROBE=0
step() {
  local lim=$1; shift
  echo "== $*" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stopping: rc=$rc from: $*" >&2; exit $rc; fi
  return 0
}
B="bench.py --no-cpu --no-extra"
step 60 rocprofv3 -L > $O/pmc_list.txt 2>&1
step 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $B --steps 6 --warmup 2 > $O/kt.log 2>&1
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
step 240 rocprofv3 --pmc $SQ --output-format csv -d $O/sq -o pmc -- python3 $B --steps 1 --warmup 0 > $O/sq.log 2>&1
step 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o pmc -- python3 $B --steps 1 --warmup 0 > $O/fetch.log 2>&1
step 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o pmc -- python3 $B --steps 1 --warmup 0 > $O/write.log 2>&1
python3 tools/pmc_summary.py $O/pmc_summary.json $O/sq $O/fetch $O/write > $O/pmc_summary.txt 2>&1
SQ2="SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INST_CYCLES_VMEM_RD SQ_WAVES"
step 240 rocprofv3 --pmc $SQ2 --output-format csv -d $O/sq2 -o pmc -- python3 $B --steps 1 --warmup 0 > $O/sq2.log 2>&1
python3 tools/pmc_summary.py $O/pmc_summary2.json $O/sq2 > $O/pmc_summary2.txt 2>&1
echo done >&2
