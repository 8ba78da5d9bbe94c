#!/bin/bash
# r04 GPU session 3: A/B of the new check levels (HBTC_SPLIT) and the latency-form layout
# (HBTC_GT_REP) on the 125-ciphertext slice, C3 and the coin lines; then the GPU suite with 16
# HIP hardware queues for the whole process and a context create/destroy churn.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run3
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
S="--cts 125 --no-cpu --no-extra --steps 20"
for sp in 0 1; do for rep in 1 3; do
  HBTC_SPLIT=$sp HBTC_GT_REP=$rep step 200 python -u bench.py $S > $O/slice125_s${sp}_r${rep}.json 2> $O/slice125_s${sp}_r${rep}.err
done; done
HBTC_SPLIT=0 step 200 python -u bench.py --no-cpu --no-extra > $O/c3_s0.json 2> $O/c3_s0.err
HBTC_SPLIT=1 step 200 python -u bench.py --no-cpu --no-extra > $O/c3_s1.json 2> $O/c3_s1.err
HBTC_GT_REP=1 step 300 python -u bench_configs.py --configs c1,c2 --no-cpu > $O/c1c2_r1.json 2> $O/c1c2_r1.err
HBTC_GT_REP=3 step 300 python -u bench_configs.py --configs c1,c2 --no-cpu > $O/c1c2_r3.json 2> $O/c1c2_r3.err
step 600 bash tools/r04/hwq16.sh
echo all-done >&2
