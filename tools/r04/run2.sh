#!/bin/bash
# r04 GPU session 2: the GPU suite, then the measurement lines (C3 headline with the rlc64 line,
# the 125- / 250-ciphertext slices with A/B variants of the check levels, the coin latency lines),
# then the per-workload rocprofv3 profiles.  Every GPU step has its own time limit; a failing
# step ends the script.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run2
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
step 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
step 300 python -u bench.py > $O/bench.json 2> $O/bench.err
step 200 python -u bench.py --cts 125 --no-cpu --no-extra > $O/slice125.json 2> $O/slice125.err
HBTC_SPLIT=0 step 200 python -u bench.py --cts 125 --no-cpu --no-extra > $O/slice125_nosplit.json 2> $O/slice125_nosplit.err
HBTC_GT_REP=1 step 200 python -u bench.py --cts 125 --no-cpu --no-extra > $O/slice125_rep1.json 2> $O/slice125_rep1.err
step 200 python -u bench.py --cts 250 --no-cpu --no-extra > $O/slice250.json 2> $O/slice250.err
step 300 python -u bench_configs.py --configs c1,c2 > $O/c1c2.json 2> $O/c1c2.err
step 900 bash tools/r04/profile.sh bench_1000ct_128b
step 600 bash tools/r04/profile.sh bench_125ct_128b --cts 125
echo all-done >&2
