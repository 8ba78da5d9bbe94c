#!/bin/bash
# r03 session V: kernel trace of the 125-ciphertext C3 slice (one rank's share at 8 GPUs).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03v
mkdir -p $O
export TMPDIR=/tmp
export HBTC_PROBE=0
step() {
  local lim=$1; shift
  echo "== $*" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stopping: rc=$rc from: $*" >&2; exit $rc; fi
  return 0
}
step 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt125 -o kt -- python3 bench.py --cts 125 --no-cpu --no-extra --steps 10 --warmup 2 > $O/kt125.log 2>&1
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
step 200 rocprofv3 --pmc $SQ --output-format csv -d $O/sq125 -o pmc -- python3 bench.py --cts 125 --no-cpu --no-extra --steps 1 --warmup 0 > $O/sq125.log 2>&1
echo done >&2
