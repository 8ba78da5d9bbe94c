# Build recipes.  The product is hbbft_amd/libhbtc.so (gfx950 HIP + host C++, C ABI in
# include/hbtc.h).  hosttest = the kernel arithmetic headers compiled for the host (tests).
HIPCC ?= /opt/rocm/bin/hipcc
CLANGXX ?= /opt/rocm/lib/llvm/bin/clang++
ARCH ?= gfx950
CSRC := hbbft_amd/csrc
HDRS := $(wildcard $(CSRC)/*.h) include/hbtc.h

.PHONY: all hosttest lib oracle clean
all: lib hosttest oracle

hosttest: tests/native/libhbtc_hosttest.so
tests/native/libhbtc_hosttest.so: tests/native/hbtc_hosttest.cpp $(HDRS)
	$(CLANGXX) -O2 -std=c++17 -shared -fPIC -I$(CSRC) $< -o $@

clean:
	rm -f tests/native/*.so hbbft_amd/*.so oracle/c/*.so
