#!/bin/bash
# r06 run 23: the GPU suite, smoke and the default bench line on the last build
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run23
mkdir -p $O
step 1200 python -u -m pytest -v -x --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
step 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step 400 python -u bench.py > $O/bench.json 2> $O/bench.err
echo all-done >&2
