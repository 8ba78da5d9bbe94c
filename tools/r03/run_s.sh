#!/bin/bash
# r03 session S: Karatsuba cooperative Fq12 mul / sqr (kara) vs the committed default.
# C3, 125-ciphertext slice, C2 / C4; GPU suite with kara.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03s
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
step 300 env HBTC_LIB_PATH=hbbft_amd/libhbtc_kara.so python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_kara.txt 2>&1
for r in 1 2; do
for v in base kara; do
  if [ $v = base ]; then L=""; else L="HBTC_LIB_PATH=hbbft_amd/libhbtc_$v.so"; fi
  step 200 env $L python3 -u bench.py --no-cpu --no-extra --steps 10 > $O/${v}_c3_$r.json 2> $O/${v}_c3_$r.err
  step 150 env $L python3 -u bench.py --cts 125 --no-extra --no-cpu > $O/${v}_125_$r.json 2> $O/${v}_125_$r.err
done
done
step 200 python3 -u bench_configs.py --configs c2,c4 --no-cpu > $O/base_c2c4.json 2> $O/base_c2c4.err
step 200 env HBTC_LIB_PATH=hbbft_amd/libhbtc_kara.so python3 -u bench_configs.py --configs c2,c4 --no-cpu > $O/kara_c2c4.json 2> $O/kara_c2c4.err
echo done >&2
