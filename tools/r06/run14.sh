#!/bin/bash
# r06 run 14: LDS-staged GT operands (gt6.h) in the check kernels: the whole GPU suite, then C3
# and the adversarial line against the unstaged build (nogtlds)
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run14
mkdir -p $O
step 1200 python -u -m pytest -v -x --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
for v in nogtlds base; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench.py --no-cpu > $O/c3_$v.json 2>> $O/c3.err
done
echo all-done >&2
