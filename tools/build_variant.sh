#!/bin/bash
# Build a variant of libhbtc.so whose RLC kernels (hbtc_rlc.hip parts 6 and 7) use extra
# compile flags, for occupancy / register-allocation experiments:
#   tools/build_variant.sh NAME "P6 FLAGS" "P7 FLAGS"
#   -> hbbft_amd/libhbtc_NAME.so   (select it with HBTC_LIB_PATH=... python bench.py)
# The other objects come from the regular build (make lib must have run).
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1
p6flags=${2:-}
p7flags=${3:-}
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Ihbbft_amd/csrc"
out=build/var_$name
mkdir -p "$out"
$HIPCC $FLAGS -DHBTC_PART=6 -DHBTC_INLINE_ALL $p6flags -c hbbft_amd/csrc/hbtc_rlc.hip -o "$out/p6.o" &
$HIPCC $FLAGS -DHBTC_PART=7 $p7flags -c hbbft_amd/csrc/hbtc_rlc.hip -o "$out/p7.o" &
wait
$HIPCC --offload-arch=gfx950 -shared -fPIC build/hbtc_kernels.p{1,2,3,4,5}.o "$out/p6.o" "$out/p7.o" \
  build/hbtc_api.o -o "hbbft_amd/libhbtc_$name.so"
echo "built hbbft_amd/libhbtc_$name.so"
