#!/bin/bash
# r03 session Q2: HIP hardware queues per process (GPU_MAX_HW_QUEUES, default 4) for the library's
# 4 lanes x 2 streams plus the strong-scaling merge's torch / RCCL streams: plain runs and the
# torchrun + RCCL merge at world size 1, C3 and the 125-ciphertext slice.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03q2
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
TR="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29520"
for q in 4 8 16; do
  step 200 env HBTC_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=$q HBTC_BENCH_HOSTT=1 python3 -u bench.py --cts 125 --no-extra --no-cpu --steps 20 > $O/plain125_q$q.json 2> $O/plain125_q$q.err
  step 300 env HBTC_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=$q HBTC_BENCH_HOSTT=1 $TR bench.py --gpus 1 --cts 125 --no-extra --no-cpu --steps 20 --force-dist > $O/nccl125_q$q.json 2> $O/nccl125_q$q.err
  step 200 env HBTC_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=$q HBTC_BENCH_HOSTT=1 python3 -u bench.py --no-extra --no-cpu --steps 20 > $O/plainc3_q$q.json 2> $O/plainc3_q$q.err
  step 300 env HBTC_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=$q HBTC_BENCH_HOSTT=1 $TR bench.py --gpus 1 --no-extra --no-cpu --steps 20 --force-dist > $O/ncclc3_q$q.json 2> $O/ncclc3_q$q.err
done
echo done >&2
