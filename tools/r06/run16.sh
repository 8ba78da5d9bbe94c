#!/bin/bash
# r06 run 16 (final build): the whole GPU suite, smoke, the headline profile (kernel trace + PMC
# passes) and bench line, the configs (c1 c2 c4 c5 bc), and the 125 / 250-ciphertext slices
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06final
mkdir -p $O
step 1200 python -u -m pytest -v -x --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
step 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rm -rf gpurun_out/prof_bench_1000ct_128b
step 900 bash tools/profile.sh bench_1000ct_128b
step 400 python -u bench.py > $O/bench.json 2> $O/bench.err
step 600 python -u bench_configs.py --configs c1,c2,c4,c5,bc > $O/configs.json 2> $O/configs.err
for n in 125 250; do
  step 300 python -u bench.py --cts $n --no-cpu --no-extra > $O/slice_$n.json 2>> $O/slice.err
done
echo all-done >&2
