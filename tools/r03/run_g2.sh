#!/bin/bash
# r03: current-build refresh of the 128-bit-scalar C3 line and the 250-ciphertext slice.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03g2
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
step 200 python3 -u bench.py --rlc-bits 128 --no-extra --no-cpu > $O/c3_128.json 2> $O/c3_128.err
step 200 python3 -u bench.py --cts 250 --no-extra --no-cpu > $O/slice250.json 2> $O/slice250.err
step 200 python3 -u bench.py --cts 125 --no-extra --no-cpu > $O/slice125.json 2> $O/slice125.err
echo done >&2
