#!/bin/bash
# r04 GPU session 36: k_rlc_items with the 15-entry table -- default (next entry prefetched, two
# waves per SIMD) vs no prefetch (libhbtc_nopf.so), one wave (libhbtc_w1.so), three waves
# (libhbtc_w3.so): C3 interleaved, twice.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run36
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
for v in d nopf w1 w3 d nopf w1 w3; do
  case $v in d) L="";; *) L=hbbft_amd/libhbtc_$v.so;; esac
  HBTC_LIB_PATH=$L step 300 python -u bench.py --no-cpu > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
done
echo all-done >&2
