#!/bin/bash
# r04 GPU session 38: the full-size C3 and C4 tests with the new exact-check bounds (the group
# sums of the table forms are right, not only the decisions).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/r04run38
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py -k "c3_full_epoch or c4_full" > gpurun_out/r04run38/pytest.log 2>&1
