#!/bin/bash
# r04 GPU session 4: the lazy-reduction GT arithmetic (gt6.h mul / sqr / line products with one
# Montgomery reduction per output half).  The GPU suite first, then A/B against the same build
# without it (hbbft_amd/libhbtc_nolazy.so: HBTC_GT_LAZY=0 in the check / sig / pb objects) on
# C3 and the 125-ciphertext slice, the split / latency-form A/B of run3 on the lazy build, the
# coin lines (small calls on the exact per-item checks, and batched as before), and the
# 16-queue suite + context churn.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run4
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
S="--cts 125 --no-cpu --no-extra --steps 20"
step 200 python -u bench.py --no-cpu --no-extra > $O/c3_lazy.json 2> $O/c3_lazy.err
HBTC_LIB_PATH=hbbft_amd/libhbtc_nolazy.so step 200 python -u bench.py --no-cpu --no-extra > $O/c3_nolazy.json 2> $O/c3_nolazy.err
HBTC_LIB_PATH=hbbft_amd/libhbtc_nolazy.so step 200 python -u bench.py $S > $O/slice125_nolazy.json 2> $O/slice125_nolazy.err
for sp in 0 1; do for rep in 1 3; do
  HBTC_SPLIT=$sp HBTC_GT_REP=$rep step 200 python -u bench.py $S > $O/slice125_s${sp}_r${rep}.json 2> $O/slice125_s${sp}_r${rep}.err
done; done
HBTC_SPLIT=0 step 200 python -u bench.py --no-cpu --no-extra > $O/c3_s0.json 2> $O/c3_s0.err
HBTC_GT_REP=1 step 300 python -u bench_configs.py --configs c1,c2 --no-cpu > $O/c1c2_r1.json 2> $O/c1c2_r1.err
HBTC_GT_REP=3 step 300 python -u bench_configs.py --configs c1,c2 --no-cpu > $O/c1c2_r3.json 2> $O/c1c2_r3.err
HBTC_EXACT_BELOW=0 step 200 python -u bench_configs.py --configs c1 --no-cpu > $O/c1_batch.json 2> $O/c1_batch.err
step 600 bash tools/r04/hwq16.sh
echo all-done >&2
