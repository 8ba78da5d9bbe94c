#!/bin/bash
# r04 GPU session 10: workspace buffers and pinned stage slots grow on every lane at once (old
# ones retired until the next sync): the suite, c1 then c2 in one process, C2 after small calls,
# C3 and the 125-ciphertext slice.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run10
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
step 200 python -u bench_configs.py --configs c1,c2 --no-cpu > $O/c1c2.json 2> $O/c1c2.err
for p in none sig3 c1; do
  step 120 python -u tools/r04/c2_after.py $p >> $O/c2_after.txt 2>> $O/c2_after.err
done
step 200 python -u bench.py --no-cpu --no-extra > $O/c3.json 2> $O/c3.err
step 200 python -u bench.py --cts 125 --no-cpu --no-extra --steps 20 > $O/slice125.json 2> $O/slice125.err
echo all-done >&2
