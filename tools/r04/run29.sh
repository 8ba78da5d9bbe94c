#!/bin/bash
# r04 GPU session 29 (evidence at the round's final build): the suite and smoke; the default
# bench line; the 125 / 250 slices (+ 125 at 64 bits); c1, c2, c4, c5 with CPU baselines; bc.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04final4
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
step 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
step 400 python -u bench.py > $O/bench.json 2> $O/bench.err
step 200 python -u bench.py --cts 125 --no-cpu --no-extra --steps 20 > $O/slice125.json 2> $O/slice125.err
step 200 python -u bench.py --cts 250 --no-cpu --no-extra --steps 20 > $O/slice250.json 2> $O/slice250.err
HBTC_RLC_BITS=64 step 200 python -u bench.py --cts 125 --no-cpu --no-extra --steps 20 > $O/slice125_64.json 2> $O/slice125_64.err
step 600 python -u bench_configs.py --configs c1,c2,c4,c5 > $O/configs.json 2> $O/configs.err
step 200 python -u bench_configs.py --configs bc --no-cpu > $O/bc.json 2> $O/bc.err
echo all-done >&2
