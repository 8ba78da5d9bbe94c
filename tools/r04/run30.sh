#!/bin/bash
# r04 GPU session 30: GT products with both Fq halves in one pass (two lazy accumulators,
# default build) vs two passes over one (libhbtc_lazy1.so, -DHBTC_GT_LAZY2=0): check-kernel
# parity first, then C3 (with the adversarial and slice lines) and C4, interleaved.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run30
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
for v in l2 l1 l2 l1; do
  case $v in l2) L="";; l1) L=hbbft_amd/libhbtc_lazy1.so;; esac
  HBTC_LIB_PATH=$L step 300 python -u bench.py --no-cpu > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
done
for v in l1 l2; do
  case $v in l2) L="";; l1) L=hbbft_amd/libhbtc_lazy1.so;; esac
  HBTC_LIB_PATH=$L step 200 python -u bench_configs.py --configs c4,c2 --no-cpu > $O/c4_$v.json 2>> $O/c4.err
done
echo all-done >&2
