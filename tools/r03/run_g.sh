#!/bin/bash
# r03 session G: pair-batch probe (kernel trace + SQ PMC pass).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03g
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
step 200 python3 -u tools/pb_probe.py 65536 2 > $O/probe.txt 2>&1
step 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 tools/pb_probe.py 65536 1 > $O/kt.log 2>&1
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
step 240 rocprofv3 --pmc $SQ --output-format csv -d $O/sq -o pmc -- python3 tools/pb_probe.py 65536 1 > $O/sq.log 2>&1
echo done >&2
