#!/bin/bash
# rocprofv3 kernel traces of bench_configs.py lines (one run per config), committed under
# profiles/r04/configs/<config>/: per-kernel call counts and average / total durations
# (kt_kernel_stats.csv) beside the line the same run printed (kt_bench.json).
# Usage: tools/r04/profile_configs.sh c1 c2 ...   (outputs under gpurun_out/prof_cfg_<config>/)
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
step() {
  local lim=$1; shift
  echo "== $*" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stopping: rc=$rc from: $*" >&2; exit $rc; fi
  return 0
}
for cfg in "$@"; do
  OUT=gpurun_out/prof_cfg_$cfg
  mkdir -p $OUT
  step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench_configs.py --configs $cfg --no-cpu > $OUT/kt_bench.json 2> $OUT/kt_bench.err
  cp "$(find $OUT/kt -name 'kt_kernel_stats.csv' | head -1)" $OUT/kt_kernel_stats.csv
  rm -rf $OUT/kt
done
echo done >&2
