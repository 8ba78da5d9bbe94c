#!/bin/bash
# r05 final 3 (after the G2 item-pass changes): the whole GPU suite, smoke(), and the signature
# configurations c1 / c2 / c4 with their CPU baselines.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05final3
mkdir -p $O
step 1000 python -u -m pytest -v -x --timeout 240 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
step 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step 600 python -u bench_configs.py --configs c1,c2,c4 > $O/configs.json 2> $O/configs.err
echo all-done >&2
