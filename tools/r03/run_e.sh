#!/bin/bash
# r03 session E: cold-key-set probe (tests + adversarial first epoch), item-pass priority variant.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "probe or rlc_batch or location" > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || exit $?
HBTC_LIB_PATH=hbbft_amd/libhbtc_prio3.so timeout -k 10 300 python3 -u bench.py --no-cpu --no-extra > $O/bench_prio3.json 2> $O/bench_prio3.err || exit $?
echo done
