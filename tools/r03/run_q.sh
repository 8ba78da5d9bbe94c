#!/bin/bash
# r03 session Q: SQ counters of the Fq product microbenchmark (per-wave VALU issue share at 1-8
# waves/SIMD); the shared-subroutine product in the check kernels (srchk) and everywhere but the
# MSMs (srall): GPU suite with srall, C3 / 125-ciphertext slice / C2-C4 A/B.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03q
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
step 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/fq_sq -o pmc -- ./tools/kbench/fqbench_sr > $O/fq_sq.log 2>&1
step 600 env HBTC_LIB_PATH=hbbft_amd/libhbtc_srall.so python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_srall.txt 2>&1
for v in base srchk srall; do
  if [ $v = base ]; then L=""; else L="HBTC_LIB_PATH=hbbft_amd/libhbtc_$v.so"; fi
  step 200 env $L python3 -u bench.py --no-cpu --no-extra --steps 10 > $O/${v}_c3.json 2> $O/${v}_c3.err
  step 150 env $L python3 -u bench.py --cts 125 --no-extra --no-cpu > $O/${v}_125.json 2> $O/${v}_125.err
done
step 200 python3 -u bench_configs.py --configs c2,c4 --no-cpu > $O/base_c2c4.json 2> $O/base_c2c4.err
step 200 env HBTC_LIB_PATH=hbbft_amd/libhbtc_srall.so python3 -u bench_configs.py --configs c2,c4 --no-cpu > $O/srall_c2c4.json 2> $O/srall_c2c4.err
step 200 python3 -u bench.py --no-cpu --no-extra --steps 10 > $O/base_c3b.json 2> $O/base_c3b.err
step 200 env HBTC_LIB_PATH=hbbft_amd/libhbtc_srall.so python3 -u bench.py --no-cpu --no-extra --steps 10 > $O/srall_c3b.json 2> $O/srall_c3b.err
echo done >&2
