# Build recipes.  The product is hbbft_amd/libhbtc.so (gfx950 HIP kernels + host C++ behind the
# C ABI of include/hbtc.h).  The kernel file is compiled once per kernel group (HBTC_PART=1..5)
# so the groups build in parallel (`make -j8 lib`); hbtc_rlc.hip (parts 6-7) and hbtc_msm.hip
# (parts 8-9) likewise.
#   hosttest : the kernel arithmetic headers compiled for the HOST (tests/native, test-only)
#   oracle   : the C restatement of threshold_crypto (oracle/c, test + CPU-baseline only)
HIPCC ?= /opt/rocm/bin/hipcc
CLANGXX ?= /opt/rocm/lib/llvm/bin/clang++
CC ?= gcc
ARCH ?= gfx950
CSRC := hbbft_amd/csrc
HDRS := $(wildcard $(CSRC)/*.h) include/hbtc.h
BUILD := build
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -I$(CSRC)
PARTS := 1
RLC_PARTS := 6
MSM_PARTS := 8 9
SKG_PARTS := 10
KOBJS := $(foreach p,$(PARTS),$(BUILD)/hbtc_kernels.p$(p).o) $(foreach p,$(RLC_PARTS),$(BUILD)/hbtc_rlc.p$(p).o) \
         $(foreach p,$(MSM_PARTS),$(BUILD)/hbtc_msm.p$(p).o) $(foreach p,$(SKG_PARTS),$(BUILD)/hbtc_skg.p$(p).o) \
         $(BUILD)/hbtc_check.c1.o $(BUILD)/hbtc_check.c2.o $(BUILD)/hbtc_sig.s1.o $(BUILD)/hbtc_sig.s2.o $(BUILD)/hbtc_pb.o \
         $(BUILD)/hbtc_bcast.o $(BUILD)/hbtc_comb.o
LIB := hbbft_amd/libhbtc.so

.PHONY: all lib hosttest oracle clean resources roofline-constants
all: lib hosttest oracle

lib: $(LIB)

# the one-block asm Fq product / squaring (generated; `make gen-fips` after editing the generator)
.PHONY: gen-fips
gen-fips:
	python3 tools/gen_fips_asm.py --selftest
	python3 tools/gen_fips_asm.py --selftest-lazy
	python3 tools/gen_fips_asm.py > $(CSRC)/fq_fips_asm.h
	python3 tools/gen_fips_asm.py --sr > $(CSRC)/fq_fips_sr.h

$(BUILD):
	mkdir -p $(BUILD)

# decode, line tables, key-set tables, scalar multiplication: helpers inlined, the product as the
# shared subroutine (no stack frames: k_point_mul 1.5 KB -> 0, k_g2_steps 1.1 KB -> 264 B/lane)
$(BUILD)/hbtc_kernels.p%.o: $(CSRC)/hbtc_kernels.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_PART=$* -DHBTC_INLINE_ALL -DHBTC_FQMUL_SR -c $< -o $@

# part 6 (per-item G1 work) is built with every helper and the Fq product inlined: no calls
# (each call saves / restores live registers through scratch; 72.6 -> 67.9 ms per C3 launch).
# The shared-subroutine product (HBTC_FQMUL_SR) is 1.2 MB -> 150 KB of code here but no faster
# (isolated 48.5 vs 49.9 ms): the pass is VALU-issue-bound, not instruction-fetch-bound.
$(BUILD)/hbtc_rlc.p6.o: $(CSRC)/hbtc_rlc.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_PART=6 -DHBTC_INLINE_ALL -DHBTC_FQMUL_INLINE -c $< -o $@

$(BUILD)/hbtc_rlc.p%.o: $(CSRC)/hbtc_rlc.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_PART=$* -c $< -o $@

# part 8 (G1 MSMs: the decryption combines) with every helper and the Fq product inlined: the
# bucket loop's mixed addition fits the instruction cache (k_msm_buckets 17.4 -> 15.1 ms per C3
# launch, k_msm_final 5.2 -> 4.3)
$(BUILD)/hbtc_msm.p8.o: $(CSRC)/hbtc_msm.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_PART=8 -DHBTC_FQMUL_INLINE -DHBTC_INLINE_ALL -c $< -o $@

# part 9 (G2 MSMs: the signature combines past 64 shares) with helpers inlined and the product as
# the shared subroutine: no stack frames (k_msm_decode<Fq2> 1,008 -> 0 B/lane of scratch)
$(BUILD)/hbtc_msm.p9.o: $(CSRC)/hbtc_msm.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_PART=9 -DHBTC_INLINE_ALL -DHBTC_FQMUL_SR -c $< -o $@

$(BUILD)/hbtc_msm.p%.o: $(CSRC)/hbtc_msm.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_PART=$* -c $< -o $@

$(BUILD)/hbtc_skg.p%.o: $(CSRC)/hbtc_skg.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_PART=$* -c $< -o $@

# the group checks in two translation units: the one-wave weighted passes (part 2) must not share
# the out-of-line GT helpers with the two-wave kernels (part 1)
# with the GT helpers (gt6.h mul / frob / exp_by_x) inlined: 960 -> ~330 B/lane of scratch (the
# by-reference operands of the calls went through the stack), C3 unchanged, the 125-ciphertext
# slice 18.3 -> 17.8 ms per epoch (profiles/r03/gt_inline/)
# with the Fq product / squaring as ONE shared subroutine each (HBTC_FQMUL_SR, fq_fips_sr.h):
# straight-line Fq2 products instead of the rolled select loop, ~100 B/lane less scratch; C3
# 11.35 -> 11.62 M shares/s (profiles/r03/fq_sr/)
$(BUILD)/hbtc_check.c%.o: $(CSRC)/hbtc_check.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_CHECK_PART=$* -DHBTC_GT_INLINE -DHBTC_FQMUL_SR -c $< -o $@

# the G2 item pass, all helpers inlined, the product as the shared subroutine (no ABI calls:
# C2 658k -> 696k, C4 3.67M -> 3.93M shares/s with the check kernels, profiles/r03/fq_sr/)
$(BUILD)/hbtc_sig.s2.o: $(CSRC)/hbtc_sig.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_SIG_PART=2 -DHBTC_INLINE_ALL -DHBTC_FQMUL_SR -c $< -o $@

# the G2 decode half (k_sig_decode) with the product inlined: no scratch in its loops
# (588 -> 432 B/lane, the doubling loop's ~150 spilled dwords per bit gone)
$(BUILD)/hbtc_sig.s1.o: $(CSRC)/hbtc_sig.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_SIG_PART=1 -DHBTC_INLINE_ALL -DHBTC_FQMUL_INLINE -c $< -o $@

# the pair-batch item pass (Ciphertext::verify / PublicKey::verify by RLC), helpers inlined,
# the product as the shared subroutine
$(BUILD)/hbtc_pb.o: $(CSRC)/hbtc_pb.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_INLINE_ALL -DHBTC_FQMUL_SR -c $< -o $@

# the small combines (t <= 64: one workgroup per instance), helpers inlined, the product as the
# shared subroutine
$(BUILD)/hbtc_comb.o: $(CSRC)/hbtc_comb.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_INLINE_ALL -DHBTC_FQMUL_SR -c $< -o $@

# Reliable Broadcast: Reed-Solomon over GF(2^8), SHA3 Merkle trees and proofs
$(BUILD)/hbtc_bcast.o: $(CSRC)/hbtc_bcast.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/hbtc_api.o: $(CSRC)/hbtc_api.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/hbtc_hash.o: $(CSRC)/hbtc_hash.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DHBTC_INLINE_ALL -DHBTC_FQMUL_SR -c $< -o $@

# host-only C++ over the public ABI (no device code)
$(BUILD)/hbtc_node.o: $(CSRC)/hbtc_node.cpp include/hbtc.h | $(BUILD)
	g++ -O2 -std=c++17 -fPIC -pthread -Wall -Iinclude -c $< -o $@

$(LIB): $(KOBJS) $(BUILD)/hbtc_api.o $(BUILD)/hbtc_hash.o $(BUILD)/hbtc_node.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@

# per-kernel VGPR / scratch / occupancy report (one part at a time: make resources PART=2)
PART ?= 2
resources:
	$(HIPCC) $(HIPFLAGS) -DHBTC_PART=$(PART) -c $(CSRC)/hbtc_kernels.hip -o /dev/null \
	  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs|AGPRs|Scratch|Occupancy|Spill"

hosttest: tests/native/libhbtc_hosttest.so
tests/native/libhbtc_hosttest.so: tests/native/hbtc_hosttest.cpp tests/native/gt_sim.cpp $(HDRS)
	$(CLANGXX) -O2 -std=c++17 -shared -fPIC -pthread -I$(CSRC) tests/native/hbtc_hosttest.cpp tests/native/gt_sim.cpp -o $@

oracle: oracle/c/libtcoracle.so
oracle/c/libtcoracle.so: oracle/c/tc_oracle.c
	$(CC) -O3 -std=gnu11 -shared -fPIC -pthread $< -o $@

clean:
	rm -rf $(BUILD) tests/native/*.so hbbft_amd/*.so oracle/c/*.so

# Fqm per unit of work, measured on the kernels' own headers (host build, counting on)
roofline-constants: bench/roofline_constants.json
bench/roofline_constants.json: tools/fqm_count.cpp $(HDRS)
	mkdir -p bench build
	$(CLANGXX) -O1 -std=c++17 -DHBTC_COUNT_FQM -I$(CSRC) $< -o build/fqm_count
	build/fqm_count > $@
