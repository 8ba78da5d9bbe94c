#!/bin/bash
# r04 GPU session 35 (final build, one call): rocprofv3 evidence first (the three bench.py
# workloads, kernel traces of c1 / c2 / c4), copied on the box into profiles/r04/bench_* so the
# bench lines below read THIS build's profiles; then the suite, smoke, the default bench line, the
# 125 / 250 slices (+ 125 at 64 bits), c1 / c2 / c4 / c5 with CPU baselines, and bc.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04final5
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
bash tools/r04/profile.sh bench_1000ct_128b || exit $?
bash tools/r04/profile.sh bench_125ct_128b --cts 125 || exit $?
bash tools/r04/profile.sh bench_250ct_128b --cts 250 || exit $?
bash tools/r04/profile_configs.sh c1 c2 c4 || exit $?
for t in bench_1000ct_128b bench_125ct_128b bench_250ct_128b; do
  mkdir -p profiles/r04/$t && cp gpurun_out/prof_$t/* profiles/r04/$t/ || exit 1
done
step 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
step 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
step 400 python -u bench.py > $O/bench.json 2> $O/bench.err
step 200 python -u bench.py --cts 125 --no-cpu --no-extra --steps 20 > $O/slice125.json 2> $O/slice125.err
step 200 python -u bench.py --cts 250 --no-cpu --no-extra --steps 20 > $O/slice250.json 2> $O/slice250.err
HBTC_RLC_BITS=64 step 200 python -u bench.py --cts 125 --no-cpu --no-extra --steps 20 > $O/slice125_64.json 2> $O/slice125_64.err
step 600 python -u bench_configs.py --configs c1,c2,c4,c5 > $O/configs.json 2> $O/configs.err
step 200 python -u bench_configs.py --configs bc --no-cpu > $O/bc.json 2> $O/bc.err
echo all-done >&2
