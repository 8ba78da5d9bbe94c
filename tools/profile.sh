#!/bin/bash
# rocprofv3 evidence for ONE bench.py workload, committed as profiles/<ROUND>/<TAG>/ (bench.py reads
# kt_launches.csv / kt_kernel_stats.csv + pmc_summary.json from profiles/r05/bench_<cts>ct_<bits>b):
#   1. --kernel-trace --stats of the bench command itself: per-kernel averages and, per launch,
#      kernel / grid / duration (tools/kt_launches.py)
#   2. three PMC passes, each its own run: SQ (VALU issue / instruction counts), FETCH_SIZE (HBM
#      reads, doubled on gfx950), WRITE_SIZE (HBM writes) -> tools/pmc_summary.py
# With CONFIG=<c1|c2|c4|c5|bc> the command is bench_configs.py --configs CONFIG instead (kernel
# trace only).  Every GPU step has its own time limit; a fault / abort / limit ends the script.
# Usage: tools/profile.sh TAG [bench args]   (outputs under gpurun_out/prof_TAG/)
cd "$(dirname "$0")/.." || exit 1
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local lim=$1; shift
  echo "== $*" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stopping: rc=$rc from: $*" >&2; exit $rc; fi
  return 0
}
if [ -n "$CONFIG" ]; then
  step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench_configs.py --configs $CONFIG --no-cpu "$@" > $OUT/kt_bench.json 2> $OUT/kt_bench.err
else
  B="bench.py --no-cpu --no-extra $*"
  step 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $B --steps 6 --warmup 1 > $OUT/kt_bench.json 2> $OUT/kt_bench.err
fi
cp "$(find $OUT/kt -name 'kt_kernel_stats.csv' | head -1)" $OUT/kt_kernel_stats.csv
python3 tools/kt_launches.py $OUT/kt $OUT/kt_launches.csv
rm -rf $OUT/kt
if [ -z "$CONFIG" ]; then
  SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
  step 240 rocprofv3 --pmc $SQ --output-format csv -d $OUT/sq -o pmc -- python3 $B --steps 2 --warmup 0 > $OUT/sq.log 2>&1
  step 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o pmc -- python3 $B --steps 2 --warmup 0 > $OUT/fetch.log 2>&1
  step 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o pmc -- python3 $B --steps 2 --warmup 0 > $OUT/write.log 2>&1
  python3 tools/pmc_summary.py $OUT/pmc_summary.json $OUT/sq $OUT/fetch $OUT/write > $OUT/pmc_summary.txt 2>&1
  rm -rf $OUT/sq $OUT/fetch $OUT/write
fi
echo done >&2
