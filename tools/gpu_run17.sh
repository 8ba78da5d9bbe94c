#!/bin/bash
# Final check of the round: the whole -m gpu suite, smoke(), the default bench line and the
# secondary configs (c2, c4, bc, c5), each under its own time limit; the first failure ends it.
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${OUT_DIR:-final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python3 -u bench_configs.py --configs c2,c4,bc > $O/bench_c2_c4_bc.json 2> $O/bench_c2_c4_bc.err || exit $?
timeout -k 10 300 python3 -u bench_configs.py --configs c5 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
