#!/bin/bash
# r05 final 4 (after the width-4 square roots): the headline profile (kernel trace + PMC passes,
# tools/profile.sh -> profiles/r05/bench_1000ct_128b/), then the whole GPU suite, smoke() and
# bench.py as the driver runs them.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05final4
mkdir -p $O
rm -rf gpurun_out/prof_bench_1000ct_128b
step 900 bash tools/profile.sh bench_1000ct_128b
step 1000 python -u -m pytest -v -x --timeout 240 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
step 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo all-done >&2
