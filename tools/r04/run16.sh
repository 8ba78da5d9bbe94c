#!/bin/bash
# r04 GPU session 16: the multi-rank paths at the round's build: the strong-scaling bench through
# torchrun + RCCL at world size 1 (the merge's cost on the 125-ciphertext slice and on C3), and a
# 2-rank gloo rehearsal of the sharded path on the one GPU.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run16
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
step 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 2 --cts 125 --no-cpu --no-extra > $O/torchrun_125.json 2> $O/torchrun_125.err
step 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu --no-extra > $O/torchrun_c3.json 2> $O/torchrun_c3.err
step 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu --no-extra --backend gloo > $O/gloo_2rank.json 2> $O/gloo_2rank.err
echo all-done >&2
