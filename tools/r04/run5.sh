#!/bin/bash
# r04 GPU session 5: the suite on the chosen defaults (lazy GT arithmetic, split levels on the
# plain-first schedule only, the latency form for the paired schedules' small levels), C3 and
# the 125-ciphertext slice, C2 at 64- and 128-bit scalars in separate processes (round 3
# measured C2 at 64 bits), c1, then the 16-queue suite and the context probe (churn + many
# contexts alive at once, with hbtc_ctx_create naming a failing HIP call).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run5
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
step 200 python -u bench.py --no-cpu --no-extra > $O/c3.json 2> $O/c3.err
step 200 python -u bench.py --cts 125 --no-cpu --no-extra --steps 20 > $O/slice125.json 2> $O/slice125.err
HBTC_RLC_BITS=64 step 200 python -u bench_configs.py --configs c2 --no-cpu > $O/c2_64.json 2> $O/c2_64.err
HBTC_RLC_BITS=128 step 200 python -u bench_configs.py --configs c2 --no-cpu > $O/c2_128.json 2> $O/c2_128.err
step 200 python -u bench_configs.py --configs c1 --no-cpu > $O/c1.json 2> $O/c1.err
step 600 bash tools/r04/hwq16.sh
echo all-done >&2
