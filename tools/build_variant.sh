#!/bin/bash
# Build a variant of libhbtc.so with extra compile flags on chosen objects, for occupancy /
# register-allocation / inlining experiments:
#   tools/build_variant.sh NAME OBJ "FLAGS" [OBJ "FLAGS" ...]
#   OBJ is a build/ object stem: hbtc_check.c1, hbtc_sig.s2, hbtc_rlc.p6, hbtc_msm.p8, ...
#   -> hbbft_amd/libhbtc_NAME.so   (select it with HBTC_LIB_PATH=... python bench.py)
# Every other object comes from the regular build (make lib must have run).  FQMUL / CHKFQ / G2FQ
# override the product mode of rlc.p6 + msm.p8 / the check objects / sig + pb (Makefile defaults).
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Ihbbft_amd/csrc"
out=build/var_$name
mkdir -p "$out"
declare -A extra
while [ $# -ge 2 ]; do extra[$1]=$2; shift 2; done
objs=()
for o in build/*.o; do
  stem=$(basename "$o" .o)
  if [ -n "${extra[$stem]+x}" ]; then
    src=${stem%%.*}
    part=""
    if [[ $stem == *.p* ]]; then part="-DHBTC_PART=${stem##*.p}"; fi
    if [[ $stem == hbtc_sig.s* ]]; then part="-DHBTC_SIG_PART=${stem##*.s}"; fi
    if [[ $stem == hbtc_check.c* ]]; then src=hbtc_check; part="-DHBTC_CHECK_PART=${stem##*.c} -DHBTC_GT_INLINE ${CHKFQ:--DHBTC_FQMUL_SR}"; fi
    base=""
    case $stem in hbtc_rlc.p6|hbtc_msm.p8) base="-DHBTC_INLINE_ALL ${FQMUL:--DHBTC_FQMUL_INLINE}";; hbtc_sig.s1) base="-DHBTC_INLINE_ALL -DHBTC_FQMUL_INLINE";; hbtc_sig.s2|hbtc_pb|hbtc_comb) base="-DHBTC_INLINE_ALL ${G2FQ:--DHBTC_FQMUL_SR}";; hbtc_kernels.p*|hbtc_hash|hbtc_msm.p9) base="-DHBTC_INLINE_ALL -DHBTC_FQMUL_SR";; esac
    $HIPCC $FLAGS $part $base ${extra[$stem]} -c "hbbft_amd/csrc/$src.hip" -o "$out/$stem.o" &
    objs+=("$out/$stem.o")
  else
    objs+=("$o")
  fi
done
wait
$HIPCC --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "hbbft_amd/libhbtc_$name.so"
echo "built hbbft_amd/libhbtc_$name.so"
