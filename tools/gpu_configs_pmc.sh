#!/bin/bash
# One GPU session: the secondary config bench lines (bench_configs.py), then three rocprofv3 PMC
# passes over the headline bench (SQ occupancy/VALU, HBM reads, HBM writes), each pass its own
# run.  Every GPU step has its own time limit; a fault / abort / time limit ends the script
# (exit 1 = an ordinary Python error, reported and the next step still runs).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local lim=$1; shift
  echo "== $*" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc=$rc from: $*" >&2; exit $rc; fi
  return 0
}
step 400 python3 -u bench_configs.py --configs c2,c4 > gpurun_out/bench_c2_c4.json 2> gpurun_out/bench_c2_c4.err
step 500 python3 -u bench_configs.py --configs c5 --steps 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
step 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
step 180 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/pmc_sq -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 > gpurun_out/pmc_sq.log 2>&1
step 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 > gpurun_out/pmc_fetch.log 2>&1
step 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 > gpurun_out/pmc_write.log 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc_summary.json gpurun_out/pmc_sq gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_summary.txt 2>&1
echo done >&2
