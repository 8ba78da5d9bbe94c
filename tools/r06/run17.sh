#!/bin/bash
# r06 run 17: pair-form G2 halves of the pair batches (k_pb_wsum_pair) and of the hash
# (k_g2_clear_cofactor), one-wave G2 bucket pass, unused one-lane G2 kernels out of the build:
# the whole GPU suite, smoke, C5 / c1 / C2 / C4
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run17
mkdir -p $O
step 1200 python -u -m pytest -v -x --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
step 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step 600 python -u bench_configs.py --configs c1,c2,c4,c5 --no-cpu > $O/configs.json 2> $O/configs.err
echo all-done >&2
