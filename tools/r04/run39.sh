#!/bin/bash
# r04 GPU session 39: the round-end tree as built by __graft_entry__.build(): the GPU suite,
# smoke and the default bench line.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run39
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
step 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
step 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
step 400 python -u bench.py > $O/bench.json 2> $O/bench.err
echo all-done >&2
