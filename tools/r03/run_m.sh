#!/bin/bash
# r03 session M: kernel traces of the 250-ciphertext slice, round start vs now (same box).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03m
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
step 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/old -o kt -- python3 oldtree/bench.py --cts 250 --no-extra --no-cpu --steps 12 --warmup 2 > $O/old.log 2>&1
step 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o kt -- python3 bench.py --cts 250 --no-extra --no-cpu --steps 12 --warmup 2 > $O/new.log 2>&1
echo done >&2
