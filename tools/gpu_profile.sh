#!/bin/bash
# One GPU session of profiles for the headline bench (C3, RLC, sender tracking on):
#   1. rocprofv3 --kernel-trace --stats (per-kernel durations; bench.py's live HIP-event timing
#      of the dominant kernel must agree with it)
#   2. three PMC passes, each its own run: SQ (occupancy / VALU issue / instruction counts),
#      FETCH_SIZE (HBM reads), WRITE_SIZE (HBM writes)  -> tools/pmc_summary.py
# Every GPU step has its own time limit; a fault / abort / time limit ends the script.
# Usage: tools/gpu_profile.sh TAG   (outputs under gpurun_out/prof_TAG*)
cd "$(dirname "$0")/.." || exit 1
TAG=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local lim=$1; shift
  echo "== $*" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stopping: rc=$rc from: $*" >&2; exit $rc; fi
  return 0
}
B="bench.py --no-cpu --no-extra"
step 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_kt -o kt -- python3 $B --steps 3 --warmup 1 > gpurun_out/prof_${TAG}_kt.log 2>&1
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
step 240 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/prof_${TAG}_sq -o pmc -- python3 $B --steps 1 --warmup 0 > gpurun_out/prof_${TAG}_sq.log 2>&1
step 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_${TAG}_fetch -o pmc -- python3 $B --steps 1 --warmup 0 > gpurun_out/prof_${TAG}_fetch.log 2>&1
step 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_${TAG}_write -o pmc -- python3 $B --steps 1 --warmup 0 > gpurun_out/prof_${TAG}_write.log 2>&1
python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_pmc_summary.json gpurun_out/prof_${TAG}_sq gpurun_out/prof_${TAG}_fetch gpurun_out/prof_${TAG}_write > gpurun_out/prof_${TAG}_pmc_summary.txt 2>&1
echo done >&2
