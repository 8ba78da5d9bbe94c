#!/bin/bash
# r05 session 5: after the scratch removal (one-wave k_sig_items, pb_items at one wave with the
# 8-entry table, inlined decode / line / G2 MSM parts): the GPU tests that touch those kernels,
# then C3, c1 / C2 / C4 / C5 / bc lines.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run5
mkdir -p $O
step 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_pair_batch.py tests/test_gpu_hash.py tests/test_gpu_skg.py > $O/pytest.log 2>&1
step 150 python -u bench.py --no-cpu --no-extra > $O/c3.json 2>> $O/c3.err
step 600 python -u bench_configs.py --configs c1,c2,c4,c5,bc --no-cpu > $O/configs.json 2>> $O/configs.err
echo all-done >&2
