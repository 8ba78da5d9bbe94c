#!/bin/bash
# r04 GPU session 8: the exact small-call path (RLC-mode share calls under 256 shares: decode +
# exact cooperative leaf checks), the suite, c1; and the C2-after-c1 slowdown by prelude.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run8
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
step 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
step 200 python -u bench_configs.py --configs c1 --no-cpu > $O/c1.json 2> $O/c1.err
for p in none sig1 sig3 keyset lanes3 c1; do
  step 120 python -u tools/r04/c2_after.py $p >> $O/c2_after.txt 2>> $O/c2_after.err
done
echo all-done >&2
