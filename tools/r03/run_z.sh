#!/bin/bash
# r03 session Z: bit-reversed location weights (one doubling per tree level) vs the previous build
# (base): GPU suite on the new default, then C3 / 125-ciphertext slice / C2-C4 A/B/A/B; the merge
# cost of the strong-scaling path at world size 1 (torchrun + RCCL) vs the plain run.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03z2
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
step 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_default.txt 2>&1
for r in 1 2; do
for v in base default; do
  if [ $v = default ]; then L=""; else L="HBTC_LIB_PATH=hbbft_amd/libhbtc_$v.so"; fi
  step 200 env $L python3 -u bench.py --no-cpu --no-extra --steps 20 > $O/${v}_c3_$r.json 2> $O/${v}_c3_$r.err
  step 150 env $L python3 -u bench.py --cts 125 --no-extra --no-cpu > $O/${v}_125_$r.json 2> $O/${v}_125_$r.err
  step 200 env $L python3 -u bench_configs.py --configs c2,c4 --no-cpu > $O/${v}_c2c4_$r.json 2> $O/${v}_c2c4_$r.err
done
done
TR="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518"
step 300 $TR bench.py --gpus 1 --no-extra --no-cpu --steps 20 --force-dist > $O/nccl_c3.json 2> $O/nccl_c3.err
step 300 $TR bench.py --gpus 1 --cts 125 --no-extra --no-cpu --steps 20 --force-dist > $O/nccl_125.json 2> $O/nccl_125.err
echo done >&2
