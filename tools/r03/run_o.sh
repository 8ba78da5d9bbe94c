#!/bin/bash
# r03 session O: check kernels with the GT helpers inlined (scratch 960 -> ~330 B/lane) vs default.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03o
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
step 300 python3 -u bench.py --no-cpu > $O/base.json 2> $O/base.err
step 300 env HBTC_LIB_PATH=hbbft_amd/libhbtc_gtinl.so python3 -u bench.py --no-cpu > $O/gtinl.json 2> $O/gtinl.err
step 150 python3 -u bench.py --cts 125 --no-extra --no-cpu > $O/base_125.json 2> $O/base_125.err
step 150 env HBTC_LIB_PATH=hbbft_amd/libhbtc_gtinl.so python3 -u bench.py --cts 125 --no-extra --no-cpu > $O/gtinl_125.json 2> $O/gtinl_125.err
step 200 python3 -u bench_configs.py --configs c2,c4 --no-cpu > $O/base_c2c4.json 2> $O/base_c2c4.err
step 200 env HBTC_LIB_PATH=hbbft_amd/libhbtc_gtinl.so python3 -u bench_configs.py --configs c2,c4 --no-cpu > $O/gtinl_c2c4.json 2> $O/gtinl_c2c4.err
echo done >&2
