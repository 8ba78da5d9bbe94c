#!/bin/bash
# r03 session A: changed GPU tests (broadcast edge cases, SKG appended bytes, C4 / C2 node),
# the node bench path (two slots on one GPU) and the RCCL merge path at world size 1.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu \
  tests/test_broadcast.py tests/test_gpu_skg_protocol.py tests/test_gpu_configs.py::test_c2_node_slots_equal_single_context \
  tests/test_gpu_configs.py::test_c4_full_64_instances_single_context_and_node > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python3 -u bench.py --node --slots 0,0 --steps 6 --warmup 2 > $O/node_2slots.json 2> $O/node_2slots.err || exit $?
timeout -k 10 300 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --force-dist --no-extra --no-cpu --steps 6 --warmup 2 > $O/rccl_w1.json 2> $O/rccl_w1.err || exit $?
timeout -k 10 200 python3 -u bench_configs.py --configs c4 --slots 0,0 --steps 3 > $O/c4_node_2slots.json 2> $O/c4_node_2slots.err || exit $?
echo done
