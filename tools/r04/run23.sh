#!/bin/bash
# r04 GPU session 23: item passes chained or not on the 250-ciphertext slice; wave priority of the
# latency-bound levels (HBTC_LATENCY_PRIO_LEVEL 0 / 2 (default) / 3: libhbtc_prio0.so /
# libhbtc_prio3.so) on C3 and the 125 slice.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run23
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
  step 200 python -u bench.py $S2 > $O/s250_base_$r.json 2>> $O/err
  HBTC_ITEMS_SERIAL=0 step 200 python -u bench.py $S2 > $O/s250_noserial_$r.json 2>> $O/err
done
for v in p0 p3 p2; do
  case $v in p2) L="";; p0) L=hbbft_amd/libhbtc_prio0.so;; p3) L=hbbft_amd/libhbtc_prio3.so;; esac
  HBTC_LIB_PATH=$L step 200 python -u bench.py $C3 > $O/c3_$v.json 2>> $O/err
  HBTC_LIB_PATH=$L HBTC_ITEMS_SERIAL=0 step 200 python -u bench.py $S1 > $O/s125ns_$v.json 2>> $O/err
done
echo all-done >&2
