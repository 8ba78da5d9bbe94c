#!/bin/bash
# C2 (100 x 100 SignatureShares, latency-bound) under each verification mode / check schedule.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/c2modes
export TMPDIR=/tmp
timeout -k 10 150 python3 -u bench_configs.py --configs c2 --mode per_share > gpurun_out/c2modes/per_share.json 2> gpurun_out/c2modes/per_share.err || exit $?
for m in auto plain pair3 pair2; do
  if [ $m = auto ]; then unset HBTC_CHECK_MODE; else export HBTC_CHECK_MODE=$m; fi
  timeout -k 10 150 python3 -u bench_configs.py --configs c2 > gpurun_out/c2modes/rlc_$m.json 2> gpurun_out/c2modes/rlc_$m.err || exit $?
done
