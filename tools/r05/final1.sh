#!/bin/bash
# r05 final 1: the whole GPU suite (as the driver runs it) and smoke() on the round's final build.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05final
mkdir -p $O
step 1000 python -u -m pytest -v -x --timeout 240 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
step 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo all-done >&2
