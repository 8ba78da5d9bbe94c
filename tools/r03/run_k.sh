#!/bin/bash
# r03 session K: 125- and 250-ciphertext slices (one rank's share at 8 / 4 GPUs): item-pass
# chaining and priority variants.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r03k
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
for CT in 125 250; do
  step 120 python3 -u bench.py --cts $CT --no-extra --no-cpu > $O/s${CT}_default.json 2> $O/s${CT}_default.err
  step 120 env HBTC_ITEMS_SERIAL=0 python3 -u bench.py --cts $CT --no-extra --no-cpu > $O/s${CT}_noserial.json 2> $O/s${CT}_noserial.err
  step 120 env HBTC_LIB_PATH=hbbft_amd/libhbtc_prio3.so python3 -u bench.py --cts $CT --no-extra --no-cpu > $O/s${CT}_prio3.json 2> $O/s${CT}_prio3.err
  step 120 env HBTC_LIB_PATH=hbbft_amd/libhbtc_prio3.so HBTC_ITEMS_SERIAL=0 python3 -u bench.py --cts $CT --no-extra --no-cpu > $O/s${CT}_prio3_noserial.json 2> $O/s${CT}_prio3_noserial.err
done
echo done >&2
