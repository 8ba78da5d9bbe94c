#!/bin/bash
# r06 run 21: the G1 item pass (k_rlc_decode + k_rlc_items) with the shared-subroutine product
# (p6sr) against the inlined one (base), C3 interleaved, and a kernel trace of p6sr
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run21
mkdir -p $O
for v in p6sr base p6sr base; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench.py --no-cpu --no-extra >> $O/c3_$v.json 2>> $O/c3.err
done
HBTC_LIB_PATH=$(lib p6sr) step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --no-cpu --no-extra --steps 6 --warmup 1 > $O/kt_bench.json 2> $O/kt_bench.err
cp "$(find $O/kt -name 'kt_kernel_stats.csv' | head -1)" $O/kt_kernel_stats_p6sr.csv
python3 tools/kt_launches.py $O/kt $O/kt_launches_p6sr.csv
rm -rf $O/kt
echo all-done >&2
