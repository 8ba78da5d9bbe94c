#!/bin/bash
# r04 GPU session 28: C2 (100 coins x 100 shares: a latency-bound lane cycle) with every share on
# the exact cooperative leaf checks (HBTC_EXACT_BELOW=20000) against the RLC batch (default 256).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run28
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
for r in a b; do
  step 200 python -u bench_configs.py --configs c2 --no-cpu > $O/c2_rlc_$r.json 2>> $O/err
  HBTC_EXACT_BELOW=20000 step 200 python -u bench_configs.py --configs c2 --no-cpu > $O/c2_exact_$r.json 2>> $O/err
done
HBTC_EXACT_BELOW=200000 step 200 python -u bench.py --cts 100 --no-cpu --no-extra --steps 10 > $O/c3_100ct_exact.json 2>> $O/err
step 200 python -u bench.py --cts 100 --no-cpu --no-extra --steps 10 > $O/c3_100ct_rlc.json 2>> $O/err
echo all-done >&2
