#!/bin/bash
# r03 session B: pipelined host-buffer epochs (tests), then the default bench line.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pipeline.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo done
