#!/bin/bash
# r03 session C: the one-block asm Fq product / squaring.  Full GPU test suite, then the
# headline bench and the secondary configs, A/B against the C++-glued product build.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench_oneblock.json 2> $O/bench_oneblock.err || exit $?
HBTC_LIB_PATH=$PWD/hbbft_amd/libhbtc_glued.so timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench_glued.json 2> $O/bench_glued.err || exit $?
timeout -k 10 300 python3 -u bench_configs.py --configs c2,c4 > $O/c2c4_oneblock.json 2> $O/c2c4_oneblock.err || exit $?
HBTC_LIB_PATH=$PWD/hbbft_amd/libhbtc_glued.so timeout -k 10 300 python3 -u bench_configs.py --configs c2,c4 > $O/c2c4_glued.json 2> $O/c2c4_glued.err || exit $?
timeout -k 10 300 python3 -u bench_configs.py --configs c5 > $O/c5_oneblock.json 2> $O/c5_oneblock.err || exit $?
echo done
