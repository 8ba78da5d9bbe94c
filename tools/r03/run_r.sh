#!/bin/bash
# r03 session R: GT operand loops of the line product / easy part / Miller step unrolled with the
# shared-subroutine product (unr) vs the committed default; C3, 125-ciphertext slice, C2 / C4.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03r
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
step 300 env HBTC_LIB_PATH=hbbft_amd/libhbtc_unr.so python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_pair_batch.py > $O/pytest_unr.txt 2>&1
for r in 1 2; do
for v in base unr; do
  if [ $v = base ]; then L=""; else L="HBTC_LIB_PATH=hbbft_amd/libhbtc_$v.so"; fi
  step 200 env $L python3 -u bench.py --no-cpu --no-extra --steps 10 > $O/${v}_c3_$r.json 2> $O/${v}_c3_$r.err
  step 150 env $L python3 -u bench.py --cts 125 --no-extra --no-cpu > $O/${v}_125_$r.json 2> $O/${v}_125_$r.err
done
done
step 200 python3 -u bench_configs.py --configs c2,c4 --no-cpu > $O/base_c2c4.json 2> $O/base_c2c4.err
step 200 env HBTC_LIB_PATH=hbbft_amd/libhbtc_unr.so python3 -u bench_configs.py --configs c2,c4 --no-cpu > $O/unr_c2c4.json 2> $O/unr_c2c4.err
echo done >&2
