#!/bin/bash
# r04 GPU session 32: r_i d_i in k_rlc_items with one mixed addition per bit from the 15-entry
# common-Z table (default build, curve.h xadic_mul_tab16) vs two per bit (libhbtc_x16off.so,
# -DHBTC_XADIC16=0): parity first, then C3 (exact-check counts must stay at 2344) and C4 / C2.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run32
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
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_pair_batch.py tests/test_gpu_coin_agreement.py > $O/pytest.log 2>&1
for v in k n k n; do
  case $v in k) L="";; n) L=hbbft_amd/libhbtc_x16off.so;; esac
  HBTC_LIB_PATH=$L step 300 python -u bench.py --no-cpu > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
done
for v in n k; do
  case $v in k) L="";; n) L=hbbft_amd/libhbtc_x16off.so;; esac
  HBTC_LIB_PATH=$L step 200 python -u bench_configs.py --configs c4,c2 --no-cpu > $O/c4_$v.json 2>> $O/c4.err
done
echo all-done >&2
