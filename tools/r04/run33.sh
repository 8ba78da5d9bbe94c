#!/bin/bash
# r04 GPU session 33: the 15-entry common-Z x-adic table in the G2 item passes too (k_sig_items,
# k_pb_items; default build) vs the two-addition loop everywhere (libhbtc_x16off.so): parity
# first, then C4 / C2 / C5 alternating, one C3 each.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run33
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
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_pair_batch.py tests/test_gpu_coin_agreement.py tests/test_gpu_configs.py > $O/pytest.log 2>&1
for v in k n k n; do
  case $v in k) L="";; n) L=hbbft_amd/libhbtc_x16off.so;; esac
  HBTC_LIB_PATH=$L step 300 python -u bench_configs.py --configs c4,c2,c5 --no-cpu > $O/cfg_$v.$RANDOM.json 2>> $O/cfg.err
done
for v in n k; do
  case $v in k) L="";; n) L=hbbft_amd/libhbtc_x16off.so;; esac
  HBTC_LIB_PATH=$L step 300 python -u bench.py --no-cpu > $O/c3_$v.json 2>> $O/c3.err
done
echo all-done >&2
