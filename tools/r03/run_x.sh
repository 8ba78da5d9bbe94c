#!/bin/bash
# r03 session X: the torchrun / RCCL path of bench.py at world size 1 on the current build (the
# driver's N > 1 launch form), strong scaling, plus the gloo rehearsal backend.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03x
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
step 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 5 --warmup 1 --force-dist > $O/torchrun_nccl.json 2> $O/torchrun_nccl.err
echo done >&2
