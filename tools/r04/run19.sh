#!/bin/bash
# r04 GPU session 19: the round's build (part-1 check kernels at three waves) -- the suite; then
# part-2 check kernels (weighted / paired / split levels, latency-form leaves) at two waves per
# SIMD (libhbtc_gts2.so) against one: C3, the 125-ciphertext slice, C2.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run19
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
for v in s1 s2 s1 s2; do
  case $v in s1) L="";; s2) L=hbbft_amd/libhbtc_gts2.so;; esac
  HBTC_LIB_PATH=$L step 200 python -u bench.py --no-cpu --no-extra > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
  HBTC_LIB_PATH=$L step 200 python -u bench.py --cts 125 --no-cpu --no-extra --steps 20 > $O/slice125_$v.$RANDOM.json 2>> $O/slice.err
done
for v in s1 s2; do
  case $v in s1) L="";; s2) L=hbbft_amd/libhbtc_gts2.so;; esac
  HBTC_LIB_PATH=$L step 200 python -u bench_configs.py --configs c2 --no-cpu > $O/c2_$v.json 2>> $O/c2.err
done
echo all-done >&2
