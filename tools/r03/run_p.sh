#!/bin/bash
# r03 session P: Fq product / squaring as shared s_swappc subroutines (fq_fips_sr.h) in the RLC
# item pass: microbench cross-check + throughput, RLC parity with the variant, C3 A/B/A/B.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03p
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
step 120 ./tools/kbench/fqbench_sr > $O/fqbench_sr.txt 2>&1
grep -q "products ok.*squarings ok" $O/fqbench_sr.txt || { echo "fqbench cross-check failed" >&2; exit 1; }
step 400 env HBTC_LIB_PATH=hbbft_amd/libhbtc_sr.so python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/parity_sr.txt 2>&1
step 200 python3 -u bench.py --no-cpu --no-extra --steps 10 > $O/base1.json 2> $O/base1.err
step 200 env HBTC_LIB_PATH=hbbft_amd/libhbtc_sr.so python3 -u bench.py --no-cpu --no-extra --steps 10 > $O/sr1.json 2> $O/sr1.err
step 200 python3 -u bench.py --no-cpu --no-extra --steps 10 > $O/base2.json 2> $O/base2.err
step 200 env HBTC_LIB_PATH=hbbft_amd/libhbtc_sr.so python3 -u bench.py --no-cpu --no-extra --steps 10 > $O/sr2.json 2> $O/sr2.err
echo done >&2
