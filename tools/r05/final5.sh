#!/bin/bash
# r05 final 5 (after k_sig_decode moved to its own object): the whole GPU suite and smoke().
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05final5
mkdir -p $O
step 1000 python -u -m pytest -v -x --timeout 240 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
step 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step 200 python -u bench.py --no-cpu --no-extra > $O/c3.json 2> $O/c3.err
echo all-done >&2
