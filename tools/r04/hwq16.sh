#!/bin/bash
# The GPU suite in ONE process with GPU_MAX_HW_QUEUES=16 (round-3 VERDICT item 4: with 16 queues
# the suite's contexts once failed hipStreamCreate after ~80 tests).  Then a context create /
# destroy loop at 16 queues (tools/r04/ctx_churn.py) reports whether streams or queues leak.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04hwq
mkdir -p $O
export GPU_MAX_HW_QUEUES=16
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_hwq16.log 2>&1
rc=$?
echo "pytest rc=$rc" >&2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/r04/ctx_churn.py > $O/ctx_churn.log 2>&1
echo "churn rc=$?" >&2
