#!/bin/bash
# r03 session U: the G2 item pass always in its one-wave form (sigw1) vs the default (two-wave
# form above 1024 tiles, i.e. C4): signature-share parity with sigw1, then C4 / C2 A/B/A/B.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03u
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
step 300 env HBTC_LIB_PATH=hbbft_amd/libhbtc_sigw1.so python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k "sig or coin or c4 or c2" tests > $O/pytest_sigw1.txt 2>&1
for r in 1 2; do
for v in base sigw1; do
  if [ $v = base ]; then L=""; else L="HBTC_LIB_PATH=hbbft_amd/libhbtc_$v.so"; fi
  step 200 env $L python3 -u bench_configs.py --configs c2,c4 --no-cpu > $O/${v}_c2c4_$r.json 2> $O/${v}_c2c4_$r.err
done
done
echo done >&2
