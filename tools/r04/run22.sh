#!/bin/bash
# r04 GPU session 22: runtime-knob A/B at the final build (no rebuild): item passes chained or
# not (HBTC_ITEMS_SERIAL), split levels on C3, the 250-ciphertext slice's schedule.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run22
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
  step 200 python -u bench.py $C3 > $O/c3_base_$r.json 2>> $O/err
  HBTC_ITEMS_SERIAL=0 step 200 python -u bench.py $C3 > $O/c3_noserial_$r.json 2>> $O/err
  step 200 python -u bench.py $S1 > $O/s125_base_$r.json 2>> $O/err
  HBTC_ITEMS_SERIAL=0 step 200 python -u bench.py $S1 > $O/s125_noserial_$r.json 2>> $O/err
  step 200 python -u bench.py $S2 > $O/s250_base_$r.json 2>> $O/err
  HBTC_CHECK_MODE=pair3 step 200 python -u bench.py $S2 > $O/s250_pair3_$r.json 2>> $O/err
done
echo all-done >&2
