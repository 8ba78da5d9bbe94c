#!/bin/bash
# r04 GPU session 9: the C2-after-small-calls slowdown: host issue time per step by prelude, and
# a prelude followed by hbtc_trim_workspace.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run9
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
for p in none sig3 sig3trim lanes3; do
  step 120 python -u tools/r04/c2_after.py $p >> $O/c2_after.txt 2>> $O/c2_after.err
done
HBTC_ITEMS_SERIAL=0 step 120 python -u tools/r04/c2_after.py sig3 >> $O/c2_after.txt 2>> $O/c2_after.err
echo all-done >&2
