#!/bin/bash
# r03 session F: pair-batch RLC path (Ciphertext::verify / PublicKey::verify / decrypt) parity,
# cold-key-set probe tests, C5 era, C3 bench + adversarial, item-pass priority variant.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03f
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
step 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pair_batch.py > $O/tests_pb.log 2>&1
step 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_skg_protocol.py tests/test_gpu_parity.py -k "probe or decrypt or ciphertext or sigs or golden or c1" > $O/tests.log 2>&1
step 300 python3 -u bench_configs.py --configs c5 --no-cpu > $O/bench_c5.json 2> $O/bench_c5.err
step 400 python3 -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err
step 300 env HBTC_LIB_PATH=hbbft_amd/libhbtc_prio3.so python3 -u bench.py --no-cpu --no-extra > $O/bench_prio3.json 2> $O/bench_prio3.err
echo done >&2
