#!/bin/bash
# r04 GPU session 6: the per-item exact kernels on one process-wide stream (their ~6 KB/lane
# scratch reserved on ONE hardware queue): the suite at HIP's default queues and at 16 queues
# for the whole process + the context probe; then why C2 runs slower after c1 in one process:
# c2 alone, after c1, after c1 without its master verification, after c1 without its combine.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run6
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
step 600 bash tools/r04/hwq16.sh
step 200 python -u bench_configs.py --configs c2 --no-cpu > $O/c2.json 2> $O/c2.err
step 200 python -u bench_configs.py --configs c1,c2 --no-cpu > $O/c1c2.json 2> $O/c1c2.err
HBTC_C1_SKIP=master step 200 python -u bench_configs.py --configs c1,c2 --no-cpu > $O/c1nomaster_c2.json 2> $O/c1nomaster_c2.err
HBTC_C1_SKIP=combine,master step 200 python -u bench_configs.py --configs c1,c2 --no-cpu > $O/c1verifyonly_c2.json 2> $O/c1verifyonly_c2.err
echo all-done >&2
