#!/bin/bash
# r04 GPU session 7: workspace buffers that grow are retired until the next sync instead of
# freed (hipFree waited for the whole device mid-pipeline): c2 alone and after c1 in one
# process; the suite (16 hardware queues for the whole process now: test_gpu_configs imports
# bench.py); the default bench line (C3 + 64-bit + host buffers + adversarial + CPU baseline);
# the 125- and 250-ciphertext slices.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run7
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
step 200 python -u bench_configs.py --configs c1,c2 --no-cpu > $O/c1c2.json 2> $O/c1c2.err
step 200 python -u bench_configs.py --configs c2 --no-cpu > $O/c2.json 2> $O/c2.err
step 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
step 400 python -u bench.py > $O/bench.json 2> $O/bench.err
step 200 python -u bench.py --cts 125 --no-cpu --no-extra --steps 20 > $O/slice125.json 2> $O/slice125.err
step 200 python -u bench.py --cts 250 --no-cpu --no-extra --steps 20 > $O/slice250.json 2> $O/slice250.err
echo all-done >&2
