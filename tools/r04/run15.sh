#!/bin/bash
# r04 GPU session 15: C4 with the one-wave SignatureShare item pass (libhbtc_sigw1.so) against the
# two-wave default; smoke().
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run15
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
step 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
step 200 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_w2.json 2> $O/c4_w2.err
HBTC_LIB_PATH=hbbft_amd/libhbtc_sigw1.so step 200 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_w1.json 2> $O/c4_w1.err
step 200 python -u bench_configs.py --configs c4 --no-cpu > $O/c4_w2b.json 2> $O/c4_w2b.err
echo all-done >&2
