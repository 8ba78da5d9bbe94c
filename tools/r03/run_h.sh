#!/bin/bash
# r03 session H: split pair-batch checks (partials per sub-tile): parity, probe, C5 era.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03h
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
step 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pair_batch.py tests/test_gpu_skg_protocol.py -k "pair or decrypt or ciphertext or sigs" > $O/tests_pb.log 2>&1
step 200 python3 -u tools/pb_probe.py 131072 2 > $O/probe.txt 2>&1
step 300 python3 -u bench_configs.py --configs c5 --no-cpu > $O/bench_c5.json 2> $O/bench_c5.err
echo done >&2
