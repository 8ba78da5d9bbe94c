#!/bin/bash
# r03 session I: psi-based G2 cofactor clearing (hash tests), pair batch, C5 era, C2/C4.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03i
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
step 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hash.py tests/test_gpu_pair_batch.py tests/test_gpu_skg_protocol.py tests/test_gpu_coin_agreement.py > $O/tests.log 2>&1
step 300 python3 -u bench_configs.py --configs c5 --no-cpu > $O/bench_c5.json 2> $O/bench_c5.err
step 300 python3 -u bench_configs.py --configs c2,c4 --no-cpu > $O/bench_c2_c4.json 2> $O/bench_c2_c4.err
echo done >&2
step 200 python3 -u bench.py --cts 125 --no-extra --no-cpu > $O/bench_125.json 2> $O/bench_125.err
step 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt125 -o kt -- python3 bench.py --cts 125 --no-extra --no-cpu --steps 20 --warmup 2 > $O/kt125.log 2>&1
echo done2 >&2
step 200 python3 -u tools/pb_probe.py 262144 2 > $O/probe_w2.txt 2>&1
step 200 env HBTC_LIB_PATH=hbbft_amd/libhbtc_pbw1.so python3 -u tools/pb_probe.py 262144 2 > $O/probe_w1.txt 2>&1
echo done >&2
