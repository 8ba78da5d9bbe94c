#!/bin/bash
# r03 session N: probe threshold fix: slices A/B vs round start, probe test, C3 with adversarial.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03n
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
step 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "probe or rlc_batch" > $O/tests.log 2>&1
for CT in 125 250; do
  step 150 python3 -u oldtree/bench.py --cts $CT --no-extra --no-cpu > $O/old_${CT}.json 2> $O/old_${CT}.err
  step 150 python3 -u bench.py --cts $CT --no-extra --no-cpu > $O/new_${CT}.json 2> $O/new_${CT}.err
done
step 400 python3 -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err
echo done >&2
