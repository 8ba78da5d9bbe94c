#!/bin/bash
# r04 GPU session 14: small pair-check calls (PublicKey::verify / Ciphertext::verify / decrypt of
# fewer than 256 items) through the SignatureShare exact path: the suite, c1 and its kernel
# trace, C5 (its pair batches are large: unchanged path).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r04run14
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
step 200 python -u bench_configs.py --configs c1 > $O/c1.json 2> $O/c1.err
bash tools/r04/profile_configs.sh c1 || exit $?
echo all-done >&2
