#!/bin/bash
# r06 run 4: the whole GPU suite and smoke after the lane-pair line tables (k_g2_steps, k_plines),
# the fused exact path (k_sig_exact), prepared G2 tables and the faster coin speculation; then c1
# / C2 / C4 against the one-lane build (nopair).
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run4
mkdir -p $O
step 1200 python -u -m pytest -v -x --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
step 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for v in nopair base; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench_configs.py --configs c2,c1 --no-cpu > $O/c2c1_$v.json 2>> $O/c2.err
done
for v in nopair base; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_$v.json 2>> $O/c4.err
done
echo all-done >&2
