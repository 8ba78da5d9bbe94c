#!/bin/bash
# r06 run 2: coin_decide golden test + smoke, then the headline profile (kernel trace + full-size
# PMC passes, tools/profile.sh) and the bench line that reads it.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run2
mkdir -p $O
step 300 python -u -m pytest -v -x --timeout 240 --timeout-method thread -m gpu tests/test_gpu_coin_decide.py tests/test_gpu_parity.py > $O/pytest.log 2>&1
step 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rm -rf gpurun_out/prof_bench_1000ct_128b
step 900 bash tools/profile.sh bench_1000ct_128b
mkdir -p profiles/r06 && rm -rf profiles/r06/bench_1000ct_128b && cp -r gpurun_out/prof_bench_1000ct_128b profiles/r06/bench_1000ct_128b
step 300 python -u bench.py > $O/bench.json 2> $O/bench.err
echo all-done >&2
