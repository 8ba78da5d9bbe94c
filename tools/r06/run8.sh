#!/bin/bash
# r06 run 8: the whole GPU suite and smoke with the pair_all fix; then c1 / C2 against the one-lane
# build (nopair), and C4 with the pair decode chain (base) against without (nosdp) and nopair.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run8
mkdir -p $O
step 1200 python -u -m pytest -v -x --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
step 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for v in nopair base; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench_configs.py --configs c2,c1 --no-cpu > $O/c2c1_$v.json 2>> $O/c2.err
done
for v in nopair nosdp base; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_$v.json 2>> $O/c4.err
done
echo all-done >&2
