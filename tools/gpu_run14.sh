#!/bin/bash
# Round-end check: the whole -m gpu suite, smoke(), and the default bench line (N = 1), each
# under its own time limit; the first failure ends the script.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r02g
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02g/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02g/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r02g/bench.json 2> gpurun_out/r02g/bench.err || exit $?
timeout -k 10 150 python3 -u bench_configs.py --configs bc --steps 20 --warmup 2 > gpurun_out/r02g/bench_bc.json 2> gpurun_out/r02g/bench_bc.err || exit $?
