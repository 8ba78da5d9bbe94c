#!/bin/bash
# r06 run 12: the G2 MSM passes on lane pairs (k_msm_*_g2p): the MSM / combine GPU tests, then C4
# and C2 against the one-lane MSM (nomsmp) and the one-wave bucket pass (msmpw1)
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r06run12
mkdir -p $O
step 600 python -u -m pytest -v -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_coin_decide.py tests/test_gpu_comb_small.py > $O/pytest.log 2>&1
for v in nomsmp msmpw1 base; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench_configs.py --configs c4,c2 --no-cpu > $O/c4_$v.json 2>> $O/c4.err
done
echo all-done >&2
