# Shared helpers of the round-6 GPU sessions (sourced by tools/r06/*.sh): every GPU step runs under
# its own time limit and the session stops at the first failing step.
cd "$(dirname "${BASH_SOURCE[0]}")/../.." || exit 1
export TMPDIR=/tmp
step() {
  local lim=$1; shift
  echo "== $*" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stopping: rc=$rc from: $*" >&2; exit $rc; fi
  return 0
}
# lib NAME -> the HBTC_LIB_PATH of a variant build (tools/build_variant.sh), "" = the default build
lib() { if [ "$1" = base ]; then echo ""; else echo "hbbft_amd/libhbtc_$1.so"; fi; }
