#!/bin/bash
# r05 session 13: the throughput-form check kernels at two waves per SIMD (256 VGPRs, ~290 B/lane)
# against three (168 VGPRs, ~576 B/lane): C3, adversarial C3, C4.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run13
mkdir -p $O
for v in base gt2 base gt2; do
  HBTC_LIB_PATH=$(lib $v) step 150 python -u bench.py --no-cpu --no-extra > $O/c3_$v.$RANDOM.json 2>> $O/c3.err
done
for v in base gt2; do
  HBTC_LIB_PATH=$(lib $v) step 200 python -u bench.py --no-cpu --no-extra --corrupt-mode senders --steps 6 > $O/adv_$v.json 2>> $O/c3.err
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_$v.json 2>> $O/c4.err
done
echo all-done >&2
