#!/bin/bash
# r03 session T: one v_mov per product column (rotating accumulator pairs) and the Karatsuba
# cooperative Fq12 mul / sqr.  base = round-3 default before both; kara = Karatsuba only;
# rotonly = rotation only; default (libhbtc.so) = both.  Product microbench cross-check, GPU
# suite on the default, then C3 / 125-ciphertext slice / C2-C4.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03t
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
step 120 ./tools/kbench/fqbench_sr > $O/fqbench_sr.txt 2>&1
grep -q "products ok.*squarings ok" $O/fqbench_sr.txt || { echo "fqbench cross-check failed" >&2; exit 1; }
step 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_default.txt 2>&1
for r in 1 2; do
for v in base kara rotonly default; do
  if [ $v = default ]; then L=""; else L="HBTC_LIB_PATH=hbbft_amd/libhbtc_$v.so"; fi
  step 200 env $L python3 -u bench.py --no-cpu --no-extra --steps 10 > $O/${v}_c3_$r.json 2> $O/${v}_c3_$r.err
  step 150 env $L python3 -u bench.py --cts 125 --no-extra --no-cpu > $O/${v}_125_$r.json 2> $O/${v}_125_$r.err
done
done
for v in base default; do
  if [ $v = default ]; then L=""; else L="HBTC_LIB_PATH=hbbft_amd/libhbtc_$v.so"; fi
  step 200 env $L python3 -u bench_configs.py --configs c2,c4 --no-cpu > $O/${v}_c2c4.json 2> $O/${v}_c2c4.err
done
echo done >&2
