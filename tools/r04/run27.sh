#!/bin/bash
# r04 GPU session 27: runtime-knob A/B at the final build: the latency form on the 125 slice
# (HBTC_GT_REP 1 / 3), the split levels on C3 and on the 250 slice (HBTC_SPLIT 0 / 1).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run27
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
C3="--no-cpu --no-extra"
S1="--cts 125 --no-cpu --no-extra --steps 20"
S2="--cts 250 --no-cpu --no-extra --steps 20"
for r in a b; do
  HBTC_GT_REP=3 step 200 python -u bench.py $S1 > $O/s125_rep3_$r.json 2>> $O/err
  HBTC_GT_REP=1 step 200 python -u bench.py $S1 > $O/s125_rep1_$r.json 2>> $O/err
  HBTC_SPLIT=1 step 200 python -u bench.py $C3 > $O/c3_split1_$r.json 2>> $O/err
  HBTC_SPLIT=0 step 200 python -u bench.py $C3 > $O/c3_split0_$r.json 2>> $O/err
  HBTC_SPLIT=1 step 200 python -u bench.py $S2 > $O/s250_split1_$r.json 2>> $O/err
  HBTC_SPLIT=0 step 200 python -u bench.py $S2 > $O/s250_split0_$r.json 2>> $O/err
done
echo all-done >&2
