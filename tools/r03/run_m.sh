#!/bin/bash
# r03 session M: where the strong-scaling merge's cost comes from at world size 1 (125-ciphertext
# slice): gloo vs RCCL, and RCCL with parts of the ordering skipped (diagnostic only).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03m
mkdir -p $O
export TMPDIR=/tmp
step() {
  local lim=$1; shift
  echo "== $*" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc=$rc from: $*" >&2; exit $rc; fi
  return 0
}
TR="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519"
B="bench.py --gpus 1 --cts 125 --no-extra --no-cpu --steps 20 --force-dist"
true
true
true
step 300 env HBTC_BENCH_SKIP=gather $TR $B > $O/nccl_nogather.json 2> $O/nccl_nogather.err
step 300 env HBTC_BENCH_SKIP=wait $TR $B > $O/nccl_nowait.json 2> $O/nccl_nowait.err
step 300 env HBTC_BENCH_SKIP=wait,order,gather $TR $B > $O/nccl_none.json 2> $O/nccl_none.err
step 300 env HBTC_BENCH_SKIP=order $TR $B > $O/nccl_noorder.json 2> $O/nccl_noorder.err
echo done >&2
