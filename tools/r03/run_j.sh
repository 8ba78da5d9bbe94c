#!/bin/bash
# r03 session J: pair-batch item-pass occupancy variant (1 wave/SIMD, no spills) vs default.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03j
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
step 200 python3 -u tools/pb_probe.py 262144 2 > $O/probe_w2.txt 2>&1
step 200 env HBTC_LIB_PATH=hbbft_amd/libhbtc_pbw1.so python3 -u tools/pb_probe.py 262144 2 > $O/probe_w1.txt 2>&1
echo done >&2
