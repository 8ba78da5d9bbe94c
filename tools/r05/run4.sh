#!/bin/bash
# r05 session 4: the whole GPU suite once with 16 HIP hardware queues per process, after the
# per-item exact kernels, the two-wave / 15-entry-table k_sig_items and the exact-kernel stream
# were removed (no kernel above 1 KB/lane of scratch); then C3.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run4
mkdir -p $O
export GPU_MAX_HW_QUEUES=16 HBTC_KEEP_HW_QUEUES=1
step 1000 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests > $O/pytest_hwq16.log 2>&1
step 150 python -u bench.py --no-cpu --no-extra > $O/c3.json 2>> $O/c3.err
echo all-done >&2
