#!/bin/bash
# r04 GPU session 17: the check kernels of part 1 (plain tiles, rep-1 leaves, SignatureShare
# tiles / sub-tiles / leaves, pair-batch Miller partials / final exponentiations) at three waves
# per SIMD (libhbtc_gtw3.so: 168 VGPRs, ~500 B/lane of scratch) against two (256, ~200 B): C3
# with the adversarial line, C4.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run17
mkdir -p $O
export TMPDIR=/tmp
step() {
  local lim=$1; shift
  echo "== $*" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stopping: rc=$rc from: $*" >&2; exit $rc; fi
  return 0
}
step 300 python -u bench.py --no-cpu > $O/c3_w2.json 2> $O/c3_w2.err
HBTC_LIB_PATH=hbbft_amd/libhbtc_gtw3.so step 300 python -u bench.py --no-cpu > $O/c3_w3.json 2> $O/c3_w3.err
step 200 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_w2.json 2> $O/c4_w2.err
HBTC_LIB_PATH=hbbft_amd/libhbtc_gtw3.so step 200 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_w3.json 2> $O/c4_w3.err
echo all-done >&2
