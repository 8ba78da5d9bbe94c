#!/bin/bash
# r03 session Y: cost of the strong-scaling merge (torchrun + RCCL all-gather, world size 1) against
# the plain run, at C3 and at the 125-ciphertext slice.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03y
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
TR="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518"
for n in 125 1000; do
  step 200 python3 -u bench.py --cts $n --no-extra --no-cpu --steps 20 > $O/plain_$n.json 2> $O/plain_$n.err
  step 300 $TR bench.py --gpus 1 --cts $n --no-extra --no-cpu --steps 20 --force-dist > $O/nccl_$n.json 2> $O/nccl_$n.err
done
echo done >&2
