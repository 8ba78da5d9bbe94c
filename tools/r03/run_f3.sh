#!/bin/bash
# r03 final pass 3: the default bench line and the torchrun / RCCL strong-scaling path at world
# size 1 with bench.py's own 16 HIP hardware queues (C3 and the 125-ciphertext slice), C2 / C4.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03f3
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
TR="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29521"
step 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
step 300 $TR bench.py --gpus 1 --steps 20 --force-dist > $O/torchrun_c3.json 2> $O/torchrun_c3.err
step 300 $TR bench.py --gpus 1 --cts 125 --no-extra --no-cpu --steps 20 --force-dist > $O/torchrun_125.json 2> $O/torchrun_125.err
step 300 python3 -u bench_configs.py --configs c2,c4,bc > $O/configs.json 2> $O/configs.err
echo done >&2
