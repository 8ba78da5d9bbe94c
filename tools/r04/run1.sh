#!/bin/bash
# r04 GPU session 1: the GPU suite, the headline bench (128-bit default + the rlc64 line), the
# coin latency lines (c1, c2), then the per-workload profiles of C3 and the 125-ciphertext slice.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run1
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
step 300 python -u bench.py > $O/bench.json 2> $O/bench.err
step 200 python -u bench.py --cts 125 --no-cpu > $O/slice125.json 2> $O/slice125.err
step 300 python -u bench_configs.py --configs c1,c2 > $O/c1c2.json 2> $O/c1c2.err
step 900 bash tools/r04/profile.sh bench_1000ct_128b
step 600 bash tools/r04/profile.sh bench_125ct_128b --cts 125
echo all-done >&2
