#!/bin/bash
# r03 session L: A/B on one box: this round's start (oldtree/, commit 02a03cf) vs now, for the
# 125 / 250-ciphertext slices and full C3.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03l
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
for CT in 125 250 1000; do
  step 150 python3 -u oldtree/bench.py --cts $CT --no-extra --no-cpu > $O/old_${CT}.json 2> $O/old_${CT}.err
  step 150 python3 -u bench.py --cts $CT --no-extra --no-cpu > $O/new_${CT}.json 2> $O/new_${CT}.err
done
echo done >&2
