// Fq Montgomery multiplication for gfx950 by product scanning (FIPS: "finely integrated
// product scanning"), the fast form of field.h's fq_mul on the device.
//
// Replaces the 12-limb CIOS loop of round 1: that form needs the 64-bit addend of every
// v_mad_u64_u32 zero-extended from a 32-bit limb and, rolled, rotates the multiplier through
// registers — ~1,680 VALU instructions per multiplication, of which ~1,050 are moves
// (tools/kbench/fqbench.hip).  Here each output column k of  a*b + q*p  is summed in a 96-bit
// accumulator: a 64-bit VGPR pair fed by v_mad_u64_u32 (whose carry-out goes to an SGPR
// lane mask) and a 32-bit overflow counter fed by v_addc_co_u32 from that mask:
//     per product: 1 v_mad_u64_u32 + 1 v_addc_co_u32, no moves
// 288 products + 12 v_mul_lo_u32 (the Montgomery quotient digits) + 3 moves per column
// ≈ 660 VALU instructions.  The MACs are issued in groups of up to four per inline-asm
// statement (hipcc pads every asm statement with one s_nop).  Only VALU instructions on
// registers: no memory access, no scalar stores.
//
// Bounds: inputs a, b < 2p (field.h's lazy range), so a*b + q*p < 4p^2 + 2^384 p < 2^384 * 2p:
// the result is < 2p, and every column sum (<= 24 products < 2^64 plus the carried-in word)
// fits the 96-bit accumulator with room to spare.
#pragma once
#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define HBTC_FIPS_FN __host__ __device__ __forceinline__
#else
#define HBTC_FIPS_FN static inline
#endif

namespace hbtc {

#if defined(__HIP_DEVICE_COMPILE__)
namespace fips {

#define HBTC_MAC_ASM(A, B) \
  "v_mad_u64_u32 %0, %2, %" #A ", %" #B ", %0\n\tv_addc_co_u32_e64 %1, %2, %1, 0, %2\n\t"

__device__ __forceinline__ void mac1(uint64_t& acc, uint32_t& c2, uint32_t a0, uint32_t b0) {
  uint64_t cc;
  asm(HBTC_MAC_ASM(3, 4) : "+v"(acc), "+v"(c2), "=&s"(cc) : "v"(a0), "v"(b0));
}
__device__ __forceinline__ void mac2(uint64_t& acc, uint32_t& c2, uint32_t a0, uint32_t b0,
                                     uint32_t a1, uint32_t b1) {
  uint64_t cc;
  asm(HBTC_MAC_ASM(3, 4) HBTC_MAC_ASM(5, 6)
      : "+v"(acc), "+v"(c2), "=&s"(cc)
      : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
}
__device__ __forceinline__ void mac4(uint64_t& acc, uint32_t& c2, uint32_t a0, uint32_t b0,
                                     uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2,
                                     uint32_t a3, uint32_t b3) {
  uint64_t cc;
  asm(HBTC_MAC_ASM(3, 4) HBTC_MAC_ASM(5, 6) HBTC_MAC_ASM(7, 8) HBTC_MAC_ASM(9, 10)
      : "+v"(acc), "+v"(c2), "=&s"(cc)
      : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3));
}
#undef HBTC_MAC_ASM

// acc += sum_{i = LO..HI} x[i] * y[K - i]
template <int K, int LO, int HI>
__device__ __forceinline__ void column(uint64_t& acc, uint32_t& c2, const uint32_t* x,
                                       const uint32_t* y) {
  constexpr int n = HI - LO + 1;
  if constexpr (n >= 4) {
    mac4(acc, c2, x[LO], y[K - LO], x[LO + 1], y[K - LO - 1], x[LO + 2], y[K - LO - 2],
         x[LO + 3], y[K - LO - 3]);
    if constexpr (n > 4) column<K, LO + 4, HI>(acc, c2, x, y);
  } else if constexpr (n >= 2) {
    mac2(acc, c2, x[LO], y[K - LO], x[LO + 1], y[K - LO - 1]);
    if constexpr (n > 2) column<K, LO + 2, HI>(acc, c2, x, y);
  } else if constexpr (n == 1) {
    mac1(acc, c2, x[LO], y[K - LO]);
  }
}

// Column K of the integrated product a*b + q*p: K < 12 produces the quotient digit q[K]
// (which zeroes the column's low word), K >= 12 produces result limb K - 12.
template <int K>
__device__ __forceinline__ void step(uint64_t& acc, uint32_t& c2, const uint32_t* a,
                                     const uint32_t* b, uint32_t* q, const uint32_t* m,
                                     uint32_t np, uint32_t* r) {
  constexpr int lo = K < 12 ? 0 : K - 11, hi = K < 12 ? K : 11;
  column<K, lo, hi>(acc, c2, a, b);
  constexpr int qhi = K < 12 ? K - 1 : 11;
  if constexpr (qhi >= lo) column<K, lo, qhi>(acc, c2, q, m);
  if constexpr (K < 12) {
    q[K] = (uint32_t)acc * np;
    mac1(acc, c2, q[K], m[0]);
  } else {
    r[K - 12] = (uint32_t)acc;
  }
  acc = (acc >> 32) | ((uint64_t)c2 << 32);
  c2 = 0;
  if constexpr (K < 22) step<K + 1>(acc, c2, a, b, q, m, np, r);
}

}  // namespace fips

// r = a * b * 2^-384 mod p for 12-limb a, b < 2p (lazy range) -> r < 2p.
HBTC_FIPS_FN void mont_mul_fips(uint32_t* r, const uint32_t* a, const uint32_t* b,
                                              const uint32_t* p, uint32_t np) {
  uint32_t q[12], m[12], out[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) m[i] = p[i];
  uint64_t acc = 0;
  uint32_t c2 = 0;
  fips::step<0>(acc, c2, a, b, q, m, np, out);
  out[11] = (uint32_t)acc;
#pragma unroll
  for (int i = 0; i < 12; ++i) r[i] = out[i];
}
#else
// Host build (tests/native, host hashing): the same product-scanning algorithm in portable C.
HBTC_FIPS_FN void mont_mul_fips(uint32_t* r, const uint32_t* a, const uint32_t* b,
                                const uint32_t* p, uint32_t np) {
  uint32_t q[12], out[12];
  uint64_t acc = 0;
  uint32_t c2 = 0;
  auto mac = [&](uint32_t x, uint32_t y) {
    const uint64_t t = (uint64_t)x * y + acc;
    c2 += t < acc;
    acc = t;
  };
  for (int k = 0; k < 23; ++k) {
    const int lo = k < 12 ? 0 : k - 11, hi = k < 12 ? k : 11;
    for (int i = lo; i <= hi; ++i) mac(a[i], b[k - i]);
    for (int i = lo; i <= hi && i < k; ++i) mac(q[i], p[k - i]);
    if (k < 12) {
      q[k] = (uint32_t)acc * np;
      mac(q[k], p[0]);
    } else {
      out[k - 12] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
    c2 = 0;
  }
  out[11] = (uint32_t)acc;
  for (int i = 0; i < 12; ++i) r[i] = out[i];
}
#endif

}  // namespace hbtc
