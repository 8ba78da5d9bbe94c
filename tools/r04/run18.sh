#!/bin/bash
# r04 GPU session 18: part-1 check kernels at 2 / 3 / 4 waves per SIMD (default build,
# libhbtc_gtw3.so, libhbtc_gtw4.so), interleaved: C3 with the adversarial line, then C4.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run18
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
for v in w4 w3 w2 w4 w3; do
  case $v in w2) L="";; w3) L=hbbft_amd/libhbtc_gtw3.so;; w4) L=hbbft_amd/libhbtc_gtw4.so;; esac
  HBTC_LIB_PATH=$L step 300 python -u bench.py --no-cpu > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
done
for v in w4 w3 w2; do
  case $v in w2) L="";; w3) L=hbbft_amd/libhbtc_gtw3.so;; w4) L=hbbft_amd/libhbtc_gtw4.so;; esac
  HBTC_LIB_PATH=$L step 200 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_$v.json 2>> $O/c4.err
done
echo all-done >&2
