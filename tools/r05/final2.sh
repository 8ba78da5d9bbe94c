#!/bin/bash
# r05 final 2: bench.py as the driver runs it (defaults: C3, CPU baseline, adversarial / 64-bit /
# host-buffer lines) and the configurations c1 / c2 / c4 / c5 / bc with their CPU baselines.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05final
mkdir -p $O
step 400 python -u bench.py > $O/bench.json 2> $O/bench.err
step 700 python -u bench_configs.py --configs c1,c2,c4,c5,bc > $O/configs.json 2> $O/configs.err
echo all-done >&2
