#!/bin/bash
# Per-kernel VGPR / AGPR / scratch / occupancy of every object of libhbtc.so, with the Makefile's
# flags (a kernel resource report: tools/resources.sh [min_scratch_bytes]).
cd "$(dirname "$0")/.." || exit 1
MIN=${1:-0}
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Ihbbft_amd/csrc"
run() {
  $H "$@" -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 |
    awk -v min="$MIN" '/Function Name:/ {n=$(NF-1)} /VGPRs:/ && !/Spill/ {v=$(NF-1)} /AGPRs:/ {a=$(NF-1)}
      /ScratchSize/ {s=$(NF-1)} /Occupancy/ {o=$(NF-1); if (s+0 >= min+0) printf "%6s B  v%-4s a%-4s w%-2s %s\n", s, v, a, o, n}'
}
run -DHBTC_PART=1 -DHBTC_INLINE_ALL -DHBTC_FQMUL_SR -c hbbft_amd/csrc/hbtc_kernels.hip &
run -DHBTC_PART=6 -DHBTC_INLINE_ALL -DHBTC_FQMUL_INLINE -c hbbft_amd/csrc/hbtc_rlc.hip &
run -DHBTC_PART=8 -DHBTC_INLINE_ALL -DHBTC_FQMUL_INLINE -c hbbft_amd/csrc/hbtc_msm.hip &
run -DHBTC_PART=9 -DHBTC_INLINE_ALL -DHBTC_FQMUL_SR -c hbbft_amd/csrc/hbtc_msm.hip &
run -DHBTC_PART=10 -c hbbft_amd/csrc/hbtc_skg.hip &
wait
for p in 1 2; do run -DHBTC_CHECK_PART=$p -DHBTC_GT_INLINE -DHBTC_FQMUL_SR -c hbbft_amd/csrc/hbtc_check.hip & done
run -DHBTC_SIG_PART=1 -DHBTC_INLINE_ALL -DHBTC_FQMUL_INLINE -c hbbft_amd/csrc/hbtc_sig.hip &
run -DHBTC_SIG_PART=2 -DHBTC_INLINE_ALL -DHBTC_FQMUL_SR -c hbbft_amd/csrc/hbtc_sig.hip &
run -DHBTC_INLINE_ALL -DHBTC_FQMUL_SR -c hbbft_amd/csrc/hbtc_pb.hip &
run -DHBTC_INLINE_ALL -DHBTC_FQMUL_SR -c hbbft_amd/csrc/hbtc_comb.hip &
run -DHBTC_INLINE_ALL -DHBTC_FQMUL_SR -c hbbft_amd/csrc/hbtc_hash.hip &
run -c hbbft_amd/csrc/hbtc_bcast.hip &
wait
