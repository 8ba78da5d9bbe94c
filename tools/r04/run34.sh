#!/bin/bash
# r04 GPU session 34: the 15-entry x-adic table on the G1 item passes (k_rlc_items, k_pb_items'
# A) and on the throughput form of k_sig_items (on the exact stream; default build): the FULL
# GPU suite at 16 queues first (the per-queue scratch reservation), then C3, and
# C4 / C2 / C5 against libhbtc_x16off.so (the two-addition loop everywhere), alternating.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run34
mkdir -p $O
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
step() {
  local lim=$1; shift
  echo "== $*" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stopping: rc=$rc from: $*" >&2; exit $rc; fi
  return 0
}
step 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
step 300 python -u bench.py --no-cpu > $O/c3_k.json 2>> $O/c3.err
for v in k n k n; do
  case $v in k) L="";; n) L=hbbft_amd/libhbtc_x16off.so;; esac
  HBTC_LIB_PATH=$L step 300 python -u bench_configs.py --configs c4,c2,c5 --no-cpu > $O/cfg_$v.$RANDOM.json 2>> $O/cfg.err
done
echo all-done >&2
