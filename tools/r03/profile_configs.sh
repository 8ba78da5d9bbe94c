#!/bin/bash
# Secondary configuration lines (C2, C4, C5, bc) with their roofline / CPU baseline, then a
# rocprofv3 kernel trace and SQ / FETCH_SIZE / WRITE_SIZE PMC passes of each (every pass its own
# run).  Usage: tools/r03/profile_configs.sh TAG
cd "$(dirname "$0")/../.." || exit 1
TAG=${1:-r03}
O=gpurun_out/cfg_$TAG
mkdir -p $O
export TMPDIR=/tmp
step() {
  local lim=$1; shift
  echo "== $*" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stopping: rc=$rc from: $*" >&2; exit $rc; fi
  return 0
}
step 300 python3 -u bench_configs.py --configs c2,c4,bc > $O/bench_c2_c4_bc.json 2> $O/bench_c2_c4_bc.err
step 300 python3 -u bench_configs.py --configs c5 > $O/bench_c5.json 2> $O/bench_c5.err
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
for C in c2 c4 c5; do
  B="bench_configs.py --configs $C --no-cpu --steps 1 --warmup 0"
  step 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${C}_kt -o kt -- python3 $B > $O/${C}_kt.log 2>&1
  step 240 rocprofv3 --pmc $SQ GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/${C}_sq -o pmc -- python3 $B > $O/${C}_sq.log 2>&1
  step 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${C}_fetch -o pmc -- python3 $B > $O/${C}_fetch.log 2>&1
  step 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${C}_write -o pmc -- python3 $B > $O/${C}_write.log 2>&1
  python3 tools/pmc_summary.py $O/${C}_pmc_summary.json $O/${C}_sq $O/${C}_fetch $O/${C}_write > $O/${C}_pmc_summary.txt 2>&1
done
echo done >&2
