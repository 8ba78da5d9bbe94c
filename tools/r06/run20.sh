#!/bin/bash
# r06 run 20: the distributed bench path on the final build: torchrun at world size 1 over RCCL
# (as the driver launches N = 1), and a 2-rank gloo rehearsal of the strong-scaling merge on the
# one GPU; then the GPU suite at 16 hardware queues
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run20
mkdir -p $O
step 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu --no-extra --force-dist > $O/torchrun1.json 2> $O/torchrun1.err
step 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 6 --warmup 1 --no-cpu --no-extra --backend gloo --force-dist > $O/gloo2.json 2> $O/gloo2.err
GPU_MAX_HW_QUEUES=16 step 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_hwq16.log 2>&1
echo all-done >&2
