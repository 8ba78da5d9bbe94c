#!/bin/bash
# r03 final pass 4 (bit-reversed trees, 16 HW queues in the benches): GPU suite, smoke, the
# default bench line, the torchrun / RCCL slice, C5, headline profiles.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03final4
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
TR="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29522"
step 600 python3 -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu_log.txt 2>&1
step 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
step 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
step 300 $TR bench.py --gpus 1 --cts 125 --no-extra --no-cpu --steps 20 --force-dist > $O/torchrun_125.json 2> $O/torchrun_125.err
step 400 python3 -u bench_configs.py --configs c5 > $O/c5.json 2> $O/c5.err
bash tools/r03/profile.sh final4 || exit $?
echo done >&2
