#!/bin/bash
# r05 session 11: the SignatureShare item pass split in two kernels (k_sig_decode at two waves per
# SIMD, k_sig_items at one) against the single one-wave kernel (nosplit): parity, then C4 / C2.
source "$(dirname "$0")/lib.sh"
O=gpurun_out/r05run11
mkdir -p $O
step 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_coin_agreement.py tests/test_gpu_coin_decide.py tests/test_gpu_pair_batch.py tests/test_gpu_configs.py -k "sig or coin or c2 or c4 or pair or small or parity" > $O/pytest.log 2>&1
for v in base nosplit base nosplit; do
  HBTC_LIB_PATH=$(lib $v) step 300 python -u bench_configs.py --configs c4,c2 --no-cpu > $O/c42_$v.$RANDOM.json 2>> $O/c42.err
done
step 120 python -u bench_configs.py --configs c1 --no-cpu > $O/c1.json 2>> $O/c42.err
echo all-done >&2
