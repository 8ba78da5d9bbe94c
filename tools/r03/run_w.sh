#!/bin/bash
# r03 session W: check schedule at strong-scaling slice sizes (125 / 250 ciphertexts = one rank
# at 8 / 4 GPUs): auto (paired) vs plain-first, A/B/A/B.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03w
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
for r in 1 2; do
for n in 125 250; do
  step 150 python3 -u bench.py --cts $n --no-extra --no-cpu > $O/auto_${n}_$r.json 2> $O/auto_${n}_$r.err
  step 150 env HBTC_CHECK_MODE=plain python3 -u bench.py --cts $n --no-extra --no-cpu > $O/plain_${n}_$r.json 2> $O/plain_${n}_$r.err
  step 150 env HBTC_CHECK_MODE=pair2 python3 -u bench.py --cts $n --no-extra --no-cpu > $O/pair2_${n}_$r.json 2> $O/pair2_${n}_$r.err
done
done
echo done >&2
