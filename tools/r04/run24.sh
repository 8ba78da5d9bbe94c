#!/bin/bash
# r04 GPU session 24: item passes chained only above one chip round (8 n_cu tiles): the suite,
# C3, the 125 / 250 slices, C2, C4.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run24
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
step 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for r in a b; do
  step 200 python -u bench.py --no-cpu --no-extra > $O/c3_$r.json 2>> $O/err
  step 200 python -u bench.py --cts 125 --no-cpu --no-extra --steps 20 > $O/s125_$r.json 2>> $O/err
  step 200 python -u bench.py --cts 250 --no-cpu --no-extra --steps 20 > $O/s250_$r.json 2>> $O/err
done
step 300 python -u bench_configs.py --configs c2,c4 --no-cpu > $O/c2c4.json 2>> $O/err
echo all-done >&2
