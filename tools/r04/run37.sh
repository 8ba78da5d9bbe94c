#!/bin/bash
# r04 GPU session 37: HBM bytes of k_rlc_items with the next table entry prefetched (default)
# vs loaded in its own iteration (libhbtc_nopf.so): one FETCH_SIZE and one WRITE_SIZE pass each
# over a short C3 run (tools/pmc_summary.py).
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
step() {
  local lim=$1; shift
  echo "== $*" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stopping: rc=$rc from: $*" >&2; exit $rc; fi
  return 0
}
B="bench.py --no-cpu --no-extra --steps 2 --warmup 0"
for v in d nopf; do
  case $v in d) L="";; *) L=hbbft_amd/libhbtc_$v.so;; esac
  OUT=gpurun_out/r04run37/$v
  mkdir -p $OUT
  HBTC_LIB_PATH=$L step 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o pmc -- python3 $B > $OUT/fetch.log 2>&1
  HBTC_LIB_PATH=$L step 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o pmc -- python3 $B > $OUT/write.log 2>&1
  python3 tools/pmc_summary.py $OUT/pmc_summary.json $OUT/fetch $OUT/write > $OUT/pmc_summary.txt 2>&1
  rm -rf $OUT/fetch $OUT/write
done
echo all-done >&2
