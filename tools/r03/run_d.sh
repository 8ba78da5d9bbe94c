#!/bin/bash
# r03 session D: 128-bit RLC scalars (parity tests + C3 cost), default bench line unchanged.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench64.json 2> $O/bench64.err || exit $?
timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu --rlc-bits 128 > $O/bench128.json 2> $O/bench128.err || exit $?
echo done
