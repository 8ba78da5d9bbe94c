#!/bin/bash
# r03 final pass 2 (after the shared-subroutine product and the accumulator rotation): GPU suite,
# smoke, headline profiles (kernel trace + PMC passes), the default bench line, C2 / C4 / C5 / bc.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03final2
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
step 600 python3 -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu_log.txt 2>&1
step 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
bash tools/r03/profile.sh final2 || exit $?
step 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
step 400 python3 -u bench_configs.py --configs c2,c4,bc > $O/configs.json 2> $O/configs.err
step 400 python3 -u bench_configs.py --configs c5 > $O/c5.json 2> $O/c5.err
echo done >&2
