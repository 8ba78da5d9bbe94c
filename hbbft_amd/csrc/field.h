// BLS12-381 field arithmetic for gfx950 (and, for tests/host hashing, the host).
//
// Replaces the field layer of pairing 0.14.2 (src/bls12_381/{fq,fq2,fq6,fq12,fr}.rs,
// an external crate used by hbbft at /root/reference/Cargo.toml:27) — see SURVEY.md §8a A15.
//
// Representation (MI355X-first):
//   * Fq: 12 x 32-bit limbs, Montgomery form with R = 2^384.  Because 4p < R the product
//     of two values in [0, 2p) is again in [0, 2p) without a final subtraction, so every
//     Fq value lives in the "lazy" range [0, 2p) and is canonicalised only for
//     comparisons and encoding.
//   * The Montgomery product is CIOS written so that hipcc emits one v_mad_u64_u32 per
//     32x32->64 partial product followed by one v_addc_co_u32 carry step (the measured
//     fastest multiply on gfx950: tools/microbench/intmul.hip, profiles/r01_intmul_microbench.txt).
//   * The outer CIOS loop is a real (non-unrolled by default) loop over the multiplier
//     limbs with the multiplier rotated through registers, which keeps each Fq
//     multiplication ~70 instructions of code: the pairing is ~10^4 multiplications
//     per share and a fully unrolled body would not fit the instruction cache.
//   * Fr: 8 x 32-bit limbs, Montgomery with R = 2^256 (Lagrange coefficients, scalars).
#pragma once
#include <cstdint>

// HD  = always inlined (the small field/curve steps that make up the hot loop bodies).
// HDN = kept out of line: operations executed a handful of times per item that wrap a long
//       loop or a large body (exponentiations, decode, final-exponentiation pieces, the Miller
//       loops themselves).  Inlining those into one kernel body produces ~10^5-instruction
//       functions whose register allocation takes the compiler tens of minutes and whose code
//       does not fit the instruction cache; a call boundary costs a few hundred bytes of
//       scratch traffic per call, negligible next to the work inside.
// A translation unit that only runs light group arithmetic (G1 decode / scalar mult) defines
// HBTC_INLINE_ALL: with no calls the compiler can size registers for the real working set and
// run several waves per SIMD.
#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define HD __host__ __device__ __forceinline__
#if defined(HBTC_INLINE_ALL)
#define HDN __host__ __device__ __forceinline__
#else
#define HDN __host__ __device__ inline __attribute__((noinline))
#endif
#define HBTC_CONST static constexpr
// Latency-bound kernels (the group-check levels and the per-instance G2 preparation: a few
// waves per SIMD, each a long dependent chain) raise their wave priority, so when the next
// epoch's item pass shares the SIMDs with them the arbiter issues their instructions first and
// the item waves fill the remaining slots.  HBTC_LATENCY_PRIO_LEVEL=0 turns it off.
#ifndef HBTC_LATENCY_PRIO_LEVEL
#define HBTC_LATENCY_PRIO_LEVEL 2
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define HBTC_LATENCY_PRIO() __builtin_amdgcn_s_setprio(HBTC_LATENCY_PRIO_LEVEL)
#else
#define HBTC_LATENCY_PRIO() ((void)0)
#endif
#else
#define HD static inline
#define HDN static inline __attribute__((noinline))
#define HBTC_CONST static constexpr
#endif

#include "bls_constants.h"
#include "fq_fips.h"
// One inline-asm block per product / squaring (tools/gen_fips_asm.py): no per-statement s_nop
// padding, and a squaring with 222 instead of 288 MACs.  HBTC_FIPS_ONEBLOCK=0 keeps the
// C++-glued product of fq_fips.h for both.
#ifndef HBTC_FIPS_ONEBLOCK
#define HBTC_FIPS_ONEBLOCK 1
#endif
#if HBTC_FIPS_ONEBLOCK
#include "fq_fips_asm.h"
#endif
#if defined(HBTC_FQMUL_SR)
#include "fq_fips_sr.h"
#endif

#ifndef HBTC_FQ_UNROLL
#define HBTC_FQ_UNROLL 1
#endif

#define HBTC_PRAGMA(x) _Pragma(#x)
#define HBTC_UNROLL_N(n) HBTC_PRAGMA(unroll n)

namespace hbtc {

// ============================================================================ limbs
template <int N>
struct Limbs {
  uint32_t v[N];
};

typedef Limbs<12> Fq;
typedef Limbs<8> Fr;

HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  return __builtin_addc(a, b, cin, cout);
}
HD uint32_t subb32(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  return __builtin_subc(a, b, bin, bout);
}

// r = a + b (N limbs), returns carry
template <int N>
HD uint32_t limbs_add(Limbs<N>& r, const Limbs<N>& a, const Limbs<N>& b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r.v[i] = addc32(a.v[i], b.v[i], c, &c);
  return c;
}

// r = a - b, returns borrow
template <int N>
HD uint32_t limbs_sub(Limbs<N>& r, const Limbs<N>& a, const Limbs<N>& b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r.v[i] = subb32(a.v[i], b.v[i], c, &c);
  return c;
}

template <int N>
HD uint32_t limbs_sub_const(Limbs<N>& r, const Limbs<N>& a, const uint32_t* m) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r.v[i] = subb32(a.v[i], m[i], c, &c);
  return c;
}

template <int N>
HD uint32_t limbs_add_const(Limbs<N>& r, const Limbs<N>& a, const uint32_t* m) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r.v[i] = addc32(a.v[i], m[i], c, &c);
  return c;
}

template <int N>
HD void limbs_select(Limbs<N>& r, bool take_b, const Limbs<N>& a, const Limbs<N>& b) {
#pragma unroll
  for (int i = 0; i < N; ++i) r.v[i] = take_b ? b.v[i] : a.v[i];
}

template <int N>
HD bool limbs_is_zero(const Limbs<N>& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) acc |= a.v[i];
  return acc == 0;
}

template <int N>
HD bool limbs_eq(const Limbs<N>& a, const Limbs<N>& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) acc |= a.v[i] ^ b.v[i];
  return acc == 0;
}

// a < m (constant), unsigned
template <int N>
HD bool limbs_lt_const(const Limbs<N>& a, const uint32_t* m) {
  Limbs<N> t;
  return limbs_sub_const<N>(t, a, m) != 0;
}

template <int N>
HD void limbs_set_const(Limbs<N>& r, const uint32_t* m) {
#pragma unroll
  for (int i = 0; i < N; ++i) r.v[i] = m[i];
}

template <int N>
HD void limbs_zero(Limbs<N>& r) {
#pragma unroll
  for (int i = 0; i < N; ++i) r.v[i] = 0;
}

// ============================================================================ Montgomery core
// CIOS: r = a * b * 2^(-32N) mod m.  Inputs < 2m (lazy) give output < 2m provided 4m < 2^(32N).
// Two-pass inner steps: N independent v_mad_u64_u32 (a_j * b_i + t_j), then one carry chain.
template <int N, int UNROLL>
HD void mont_mul(Limbs<N>& r, const Limbs<N>& a, const Limbs<N>& bin, const uint32_t* m,
                 uint32_t np) {
  uint32_t t[N + 2];
#pragma unroll
  for (int j = 0; j < N + 2; ++j) t[j] = 0;
  Limbs<N> b = bin;
  HBTC_UNROLL_N(UNROLL)
  for (int i = 0; i < N; ++i) {
    const uint32_t bi = b.v[0];
#pragma unroll
    for (int j = 0; j < N - 1; ++j) b.v[j] = b.v[j + 1];  // rotate multiplier (static indexing)
    uint64_t s[N];
#pragma unroll
    for (int j = 0; j < N; ++j) s[j] = (uint64_t)a.v[j] * bi + t[j];
    uint32_t c = 0;
    t[0] = (uint32_t)s[0];
#pragma unroll
    for (int j = 1; j < N; ++j) t[j] = addc32((uint32_t)s[j], (uint32_t)(s[j - 1] >> 32), c, &c);
    t[N] = addc32(t[N], (uint32_t)(s[N - 1] >> 32), c, &c);
    t[N + 1] = c;
    const uint32_t q = t[0] * np;
#pragma unroll
    for (int j = 0; j < N; ++j) s[j] = (uint64_t)q * m[j] + t[j];
    c = 0;
#pragma unroll
    for (int j = 1; j < N; ++j)
      t[j - 1] = addc32((uint32_t)s[j], (uint32_t)(s[j - 1] >> 32), c, &c);
    t[N - 1] = addc32(t[N], (uint32_t)(s[N - 1] >> 32), c, &c);
    t[N] = t[N + 1] + c;
  }
#pragma unroll
  for (int j = 0; j < N; ++j) r.v[j] = t[j];
}

// ============================================================================ Fq
HD void fq_zero(Fq& r) { limbs_zero<12>(r); }
HD void fq_one(Fq& r) { limbs_set_const<12>(r, FQ_ONE); }
HD void fq_set(Fq& r, const uint32_t* c) { limbs_set_const<12>(r, c); }

// reduce [0, 4p) -> [0, 2p)
HD void fq_reduce_2p(Fq& r) {
  Fq t;
  uint32_t borrow = limbs_sub_const<12>(t, r, FQ_2P);
  limbs_select<12>(r, borrow == 0, r, t);
}

HD void fq_add(Fq& r, const Fq& a, const Fq& b) {
  limbs_add<12>(r, a, b);  // < 4p < 2^384: no carry out
  fq_reduce_2p(r);
}

HD void fq_dbl(Fq& r, const Fq& a) { fq_add(r, a, a); }

HD void fq_sub(Fq& r, const Fq& a, const Fq& b) {
  uint32_t borrow = limbs_sub<12>(r, a, b);
  Fq t;
  limbs_add_const<12>(t, r, FQ_2P);
  limbs_select<12>(r, borrow != 0, r, t);
}

HD void fq_neg(Fq& r, const Fq& a) {
  Fq z;
  fq_zero(z);
  fq_sub(r, z, a);
}

// Host-only instrumentation (tools/fqm_count.cpp): counts Fq Montgomery multiplications so the
// roofline's algorithmic work per item is measured on the very code the kernels run.
#if defined(HBTC_COUNT_FQM) && !defined(__HIP_DEVICE_COMPILE__)
extern unsigned long long hbtc_fqm_count;
#define HBTC_COUNT_FQ_MUL() (++hbtc_fqm_count)
#else
#define HBTC_COUNT_FQ_MUL() ((void)0)
#endif

// Device multiplication: product scanning with carry-out MACs (fq_fips.h; 0.58-0.62 of the
// v_mad_u64_u32 roofline at 4-8 waves/SIMD vs 0.43-0.48 for the rolled CIOS loop, and 1.8x
// lower single-wave latency: profiles/r02_fqbench.txt).  The product is ~660 instructions, so
// by default every call site calls ONE out-of-line copy (operands and result in VGPRs): the
// tower and curve code inlines dozens of products per loop body, and inlined copies put a G2
// scalar-multiplication loop at ~55k instructions, far past the instruction cache.  A
// translation unit whose hot loops hold few product sites (the cooperative GT kernels,
// hbtc_check.hip) defines HBTC_FQMUL_INLINE; HBTC_FQMUL_CIOS selects round 1's CIOS loop.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void fq_mul_dev(uint32_t* r, const uint32_t* a, const uint32_t* b) {
#if HBTC_FIPS_ONEBLOCK
  fips::mont_mul_asm(r, a, b);
#else
  mont_mul_fips(r, a, b, FQ_P, FQ_NP);
#endif
}
__device__ __forceinline__ void fq_sqr_dev(uint32_t* r, const uint32_t* a) {
#if HBTC_FIPS_ONEBLOCK
  fips::mont_sqr_asm(r, a);
#else
  mont_mul_fips(r, a, a, FQ_P, FQ_NP);
#endif
}
__device__ __attribute__((noinline)) Fq fq_mul_call(Fq a, Fq b) {
  Fq r;
  fq_mul_dev(r.v, a.v, b.v);
  return r;
}
__device__ __attribute__((noinline)) Fq fq_sqr_call(Fq a) {
  Fq r;
  fq_sqr_dev(r.v, a.v);
  return r;
}
#endif
#if defined(__HIP_DEVICE_COMPILE__) && defined(HBTC_FQMUL_SR)
// One shared copy of each as a subroutine on fixed registers (fq_fips_sr.h): the hot loops of a
// fully inlined translation unit shrink ~15x and fit the instruction cache.
HD void fq_mul(Fq& r, const Fq& a, const Fq& b) { fips::mont_mul_sr(r.v, a.v, b.v); }
HD void fq_sqr(Fq& r, const Fq& a) { fips::mont_sqr_sr(r.v, a.v); }
#elif defined(__HIP_DEVICE_COMPILE__) && defined(HBTC_FQMUL_INLINE)
HD void fq_mul(Fq& r, const Fq& a, const Fq& b) { fq_mul_dev(r.v, a.v, b.v); }
HD void fq_sqr(Fq& r, const Fq& a) { fq_sqr_dev(r.v, a.v); }
#elif defined(__HIP_DEVICE_COMPILE__) && !defined(HBTC_FQMUL_CIOS)
HD void fq_mul(Fq& r, const Fq& a, const Fq& b) { r = fq_mul_call(a, b); }
HD void fq_sqr(Fq& r, const Fq& a) { r = fq_sqr_call(a); }
#else
HD void fq_mul(Fq& r, const Fq& a, const Fq& b) {
  HBTC_COUNT_FQ_MUL();
  mont_mul<12, HBTC_FQ_UNROLL>(r, a, b, FQ_P, FQ_NP);
}
HD void fq_sqr(Fq& r, const Fq& a) { fq_mul(r, a, a); }  // counted as one Fqm
#endif
// Product through the single out-of-line copy on the device (code-size-bound callers).
HD void fq_mul_ol(Fq& r, const Fq& a, const Fq& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  r = fq_mul_call(a, b);
#else
  fq_mul(r, a, b);
#endif
}

// ---------------------------------------------------------------- lazy (double-width) reduction
// A sum of products of reduced operands (< 2p each) kept unreduced in 25 words and reduced ONCE:
// fq_acc_mac is the product half of a Montgomery multiplication (144 v_mad_u64_u32), fq_acc_redc
// the reduction half plus conditional subtractions of 4p and 2p (result < 2p).  At most 12
// products per accumulator (< 48 p^2, so the Montgomery quotient is < 5.6p).  Device
// builds with the shared-subroutine product run both as subroutines on fixed registers (the
// accumulator pinned to v60..v84 across calls: tools/gen_fips_asm.py); elsewhere plain C++ with
// the same arithmetic (same Montgomery quotient, same subtractions: the same representative).
struct FqAcc {
  uint32_t v[25];
};
HD void fq_acc_zero(FqAcc& a) {
#pragma unroll
  for (int i = 0; i < 25; ++i) a.v[i] = 0;
}
// Karatsuba accumulation of an Fq2 sum (fq_acc_kara below): X starts at 24 p^2 (a multiple of p,
// so the residue is unchanged) and ends at 24 p^2 + sum (a0 b0 - a1 b1) < 48 p^2 for up to 6 terms
// of operands < 2p; Y ends at sum (a0 b1 + a1 b0) < 48 p^2.  In between both wrap modulo 2^800.
HBTC_CONST uint32_t FQ_ACC_K24[25] = {
    0xaaa55558u, 0x9ff00002u, 0x1544600bu, 0xb6420ac3u, 0x319db7c3u, 0x1424d451u, 0xdaa92e4au, 0xa1f5ae3du, 0x8da706e1u, 0xdc5c87cau, 0x9248ab8bu, 0xc1c926acu, 0xe356681au, 0xfc9edcc8u, 0x24cafa66u, 0x8f9437bau, 0xeedd1b87u, 0xa586d6dcu, 0x5a86a0e9u, 0x44ad9579u, 0x346b8dedu, 0x1bbb55ffu, 0x5250faafu, 0x3f653771u, 0x00000000u};
HD void fq_acc_k24(FqAcc& a) {
#pragma unroll
  for (int i = 0; i < 25; ++i) a.v[i] = FQ_ACC_K24[i];
}
// a + b without the reduction: < 4p < 2^384 for operands < 2p (a Karatsuba sum operand)
HD void fq_add_nr(Fq& r, const Fq& a, const Fq& b) { limbs_add<12>(r, a, b); }
#if defined(__HIP_DEVICE_COMPILE__) && defined(HBTC_FQMUL_SR)
HD void fq_acc_mac(FqAcc& acc, const Fq& a, const Fq& b) { fips::fq_mac_sr(acc.v, a.v, b.v); }
HD void fq_acc_redc(Fq& r, const FqAcc& acc) { fips::fq_redc_sr(r.v, acc.v); }
// the second accumulator's pair (pinned to v85..v109): a sum of two accumulators in one pass
HD void fq_acc_mac2(FqAcc& acc, const Fq& a, const Fq& b) { fips::fq_mac2_sr(acc.v, a.v, b.v); }
HD void fq_acc_redc2(Fq& r, const FqAcc& acc) { fips::fq_redc2_sr(r.v, acc.v); }
// x += a b, y -= a b  /  x -= a b, y -= a b  (both accumulators in one product)
HD void fq_acc_macsub(FqAcc& x, FqAcc& y, const Fq& a, const Fq& b) { fips::fq_macsub_sr(x.v, y.v, a.v, b.v); }
HD void fq_acc_subsub(FqAcc& x, FqAcc& y, const Fq& a, const Fq& b) { fips::fq_subsub_sr(x.v, y.v, a.v, b.v); }
#else
HD void fq_acc_mac(FqAcc& acc, const Fq& a, const Fq& b) {
  uint32_t p[24];
#pragma unroll
  for (int i = 0; i < 24; ++i) p[i] = 0;
  for (int i = 0; i < 12; ++i) {
    uint32_t c = 0;
    for (int j = 0; j < 12; ++j) {
      const uint64_t t = (uint64_t)a.v[i] * b.v[j] + p[i + j] + c;
      p[i + j] = (uint32_t)t;
      c = (uint32_t)(t >> 32);
    }
    p[i + 12] = c;
  }
  uint32_t c = 0;
  for (int i = 0; i < 24; ++i) acc.v[i] = addc32(acc.v[i], p[i], c, &c);
  acc.v[24] += c;
}
HD void fq_acc_redc(Fq& r, const FqAcc& acc) {
  uint32_t t[26];
  for (int i = 0; i < 25; ++i) t[i] = acc.v[i];
  t[25] = 0;
  for (int i = 0; i < 12; ++i) {
    const uint32_t q = t[i] * FQ_NP;
    uint32_t c = 0;
    for (int j = 0; j < 12; ++j) {
      const uint64_t s = (uint64_t)q * FQ_P[j] + t[i + j] + c;
      t[i + j] = (uint32_t)s;
      c = (uint32_t)(s >> 32);
    }
    for (int j = i + 12; j < 26; ++j) t[j] = addc32(t[j], 0, c, &c);
  }
  uint32_t x[12];
  for (int i = 0; i < 12; ++i) x[i] = t[12 + i];  // < 5.6p: words 24, 25 are 0
  for (int sh = 2; sh >= 1; --sh) {  // subtract 4p, then 2p, where they fit
    uint32_t m[12], d[12], b = 0;
    for (int i = 0; i < 12; ++i) m[i] = (FQ_P[i] << sh) | (i > 0 ? FQ_P[i - 1] >> (32 - sh) : 0u);
    for (int i = 0; i < 12; ++i) d[i] = subb32(x[i], m[i], b, &b);
    if (!b)
      for (int i = 0; i < 12; ++i) x[i] = d[i];
  }
  for (int i = 0; i < 12; ++i) r.v[i] = x[i];
}
HD void fq_acc_mac2(FqAcc& acc, const Fq& a, const Fq& b) { fq_acc_mac(acc, a, b); }
HD void fq_acc_redc2(Fq& r, const FqAcc& acc) { fq_acc_redc(r, acc); }
// acc -= a b modulo 2^800
HD void fq_acc_msb(FqAcc& acc, const Fq& a, const Fq& b) {
  FqAcc p;
  fq_acc_zero(p);
  fq_acc_mac(p, a, b);
  uint32_t c = 0;
  for (int i = 0; i < 25; ++i) acc.v[i] = subb32(acc.v[i], p.v[i], c, &c);
}
HD void fq_acc_macsub(FqAcc& x, FqAcc& y, const Fq& a, const Fq& b) {
  fq_acc_mac(x, a, b);
  fq_acc_msb(y, a, b);
}
HD void fq_acc_subsub(FqAcc& x, FqAcc& y, const Fq& a, const Fq& b) {
  fq_acc_msb(x, a, b);
  fq_acc_msb(y, a, b);
}
#endif
// x += a0 b0 - a1 b1, y += a0 b1 + a1 b0 (three half products: Karatsuba)
HD void fq_acc_kara(FqAcc& x, FqAcc& y, const Fq& a0, const Fq& a1, const Fq& b0, const Fq& b1) {
  Fq sa, sb;
  fq_add_nr(sa, a0, a1);
  fq_add_nr(sb, b0, b1);
  fq_acc_macsub(x, y, a0, b0);
  fq_acc_subsub(x, y, a1, b1);
  fq_acc_mac2(y, sa, sb);
}

// canonical value in [0, p)
HD void fq_canon(Fq& r, const Fq& a) {
  Fq t;
  uint32_t borrow = limbs_sub_const<12>(t, a, FQ_P);
  limbs_select<12>(r, borrow == 0, a, t);
}

HD bool fq_is_zero(const Fq& a) {
  Fq c;
  fq_canon(c, a);
  return limbs_is_zero<12>(c);
}

HD bool fq_eq(const Fq& a, const Fq& b) {
  Fq d;
  fq_sub(d, a, b);
  return fq_is_zero(d);
}

HD void fq_to_mont(Fq& r, const Fq& a) {
  Fq r2;
  fq_set(r2, FQ_R2);
  fq_mul(r, a, r2);
}

// Montgomery -> canonical integer
HD void fq_from_mont(Fq& r, const Fq& a) {
  Fq one;
  limbs_zero<12>(one);
  one.v[0] = 1;
  Fq t;
  fq_mul(t, a, one);
  fq_canon(r, t);
}

HD void fq_sel(Fq& r, bool c, const Fq& a, const Fq& b) {  // r = c ? a : b (no branch)
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = c ? a.v[i] : b.v[i];
}

// a^e for a constant 12-limb exponent e (square-and-multiply, MSB first)
HDN void fq_pow_const(Fq& r, const Fq& a, const uint32_t* e) {
  Fq acc;
  fq_one(acc);
  for (int w = 11; w >= 0; --w) {
    const uint32_t word = e[w];
    for (int b = 31; b >= 0; --b) {
      fq_sqr(acc, acc);
      if ((word >> b) & 1u) fq_mul(acc, acc, a);
    }
  }
  r = acc;
}

HD void fq_inv(Fq& r, const Fq& a) { fq_pow_const(r, a, EXP_P_MINUS_2); }

// a^e for a constant exponent by a left-to-right sliding window of width POW_W over the odd
// powers a, a^3, ..., a^(2^POW_W - 1) (2^(POW_W-1) Fq of table).  For the 379-bit (p-3)/4 of the
// square roots: width 3 (4 entries) 377 squarings + 105 multiplications + 4 for the table, width
// 4 (8 entries) 375 + 78 + 8 -- 25 products fewer per square root (G1 decode 1,528 -> 1,503 Fqm,
// G2 decode two square roots).  The schedule is computed at compile time: each step squares `nsq`
// times, then multiplies by table entry `idx` (POW_NONE: no multiplication).
#ifndef HBTC_POW_W
#define HBTC_POW_W 4
#endif
constexpr int POW_W = HBTC_POW_W;
constexpr int POW_TAB = 1 << (POW_W - 1);
constexpr uint8_t POW_NONE = 0xff;
struct PowStep {
  uint16_t nsq;
  uint8_t idx;
};
struct PowPlan {
  PowStep s[400];
  int n = 0;
  uint8_t first = 0;
};
constexpr int pow_bit(const uint32_t* e, int i) { return (int)((e[i >> 5] >> (i & 31)) & 1u); }
constexpr PowPlan pow_plan(const uint32_t* e) {
  PowPlan pl{};
  int i = 383;
  while (i >= 0 && !pow_bit(e, i)) --i;
  auto window = [&](int top, int& low) {  // odd window [top .. low], at most POW_W bits
    low = top - (POW_W - 1) < 0 ? 0 : top - (POW_W - 1);
    while (!pow_bit(e, low)) ++low;
    int v = 0;
    for (int b = top; b >= low; --b) v = 2 * v + pow_bit(e, b);
    return v;
  };
  int low = 0;
  pl.first = (uint8_t)((window(i, low) - 1) / 2);
  i = low - 1;
  int nsq = 0;
  while (i >= 0) {
    if (!pow_bit(e, i)) {
      ++nsq;
      --i;
      continue;
    }
    const int v = window(i, low);
    nsq += i - low + 1;
    pl.s[pl.n++] = PowStep{(uint16_t)nsq, (uint8_t)((v - 1) / 2)};
    nsq = 0;
    i = low - 1;
  }
  if (nsq) pl.s[pl.n++] = PowStep{(uint16_t)nsq, POW_NONE};
  return pl;
}
HBTC_CONST PowPlan POW_SQRT_PLAN = pow_plan(EXP_P_MINUS_3_DIV_4);

HDN void fq_pow_window(Fq& r, const Fq& a, const PowPlan& pl) {
  Fq t[POW_TAB], a2;
  t[0] = a;
  fq_sqr(a2, a);
#pragma unroll
  for (int k = 1; k < POW_TAB; ++k) fq_mul(t[k], t[k - 1], a2);
  Fq acc = t[0];
#pragma unroll
  for (int k = 1; k < POW_TAB; ++k) fq_sel(acc, pl.first == k, t[k], acc);
#pragma unroll 1
  for (int k = 0; k < pl.n; ++k) {
    const PowStep st = pl.s[k];
#pragma unroll 1
    for (int q = 0; q < st.nsq; ++q) fq_sqr(acc, acc);
    // the entry by a wave-uniform branch over constant indices (the table stays in registers)
#pragma unroll
    for (int j = 0; j < POW_TAB; ++j)
      if (st.idx == j) fq_mul(acc, acc, t[j]);
  }
  r = acc;
}


// Wave-wide OR of a predicate (the device loops below stay wave-uniform); the host build has
// one "lane".
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ bool fq_wave_any(bool p) { return __ballot(p) != 0ull; }
#else
inline bool fq_wave_any(bool p) { return p; }
#endif

// Inversion in Fq by the binary extended Euclidean algorithm (variable time: every input is
// public), about a quarter of the instruction count of the Fermat power a^(p-2).
// Invariants x1 A = u, x2 A = v (mod p) with A the canonical input, u, v odd after the first
// step; each iteration subtracts the smaller of u, v from the larger and strips the difference's
// factors of two (up to 31 per iteration: x <- x / 2^k mod p as (x + m p) / 2^k with
// m = -x p^-1 mod 2^k, the Montgomery digit).  The loop is wave-uniform: lanes that finished
// keep their state until every lane has.  Montgomery in, Montgomery out: for the input aR the
// loop finds x = (aR)^-1 and the result is x R^3 R^-1 = a^-1 R.
HD void half_k(Fq& x, uint32_t k) {  // x / 2^k mod p for x < p, 0 <= k <= 31  (result < p)
  const uint32_t mask = k ? (0xffffffffu >> (32 - k)) : 0u;
  const uint32_t m = (x.v[0] * FQ_NP) & mask;
  uint32_t t[13];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    c += (uint64_t)m * FQ_P[i] + x.v[i];
    t[i] = (uint32_t)c;
    c >>= 32;
  }
  t[12] = (uint32_t)c;
#pragma unroll
  for (int i = 0; i < 12; ++i)
    x.v[i] = k ? ((t[i] >> k) | (t[i + 1] << (32 - k))) : t[i];
  fq_canon(x, x);  // (x + m p) / 2^k < 2p
}
HD uint32_t ctz31(const Fq& a) {
  const uint32_t w = a.v[0];
  return w ? (uint32_t)__builtin_ctz(w) : 31u;
}
HD void shr_k(Fq& a, uint32_t k) {
#pragma unroll
  for (int i = 0; i < 11; ++i) a.v[i] = k ? ((a.v[i] >> k) | (a.v[i + 1] << (32 - k))) : a.v[i];
  a.v[11] = a.v[11] >> k;
}
HD void fq_inv_binary(Fq& r, const Fq& a_mont) {
  Fq u, v, x1, x2, one;
  fq_canon(u, a_mont);
  limbs_set_const<12>(v, FQ_P);
  limbs_zero<12>(x1);
  x1.v[0] = 1;
  limbs_zero<12>(x2);
  limbs_zero<12>(one);
  one.v[0] = 1;
  bool zero = limbs_is_zero<12>(u);
  {  // make u odd
    uint32_t k = ctz31(u);
#pragma unroll 1
    for (int rep = 0; rep < 13 && k && !zero; ++rep) {
      shr_k(u, k);
      half_k(x1, k);
      k = ctz31(u);
    }
  }
  bool done = zero || limbs_eq<12>(u, one);
#pragma unroll 1
  for (int it = 0; it < 2 * 384; ++it) {
    if (!fq_wave_any(!done)) break;
    Fq duv, dvu, d, xd, t;
    const bool ge = limbs_sub<12>(duv, u, v) == 0;  // u >= v
    limbs_sub<12>(dvu, v, u);
    fq_sel(d, ge, duv, dvu);
    // xd = ge ? x1 - x2 : x2 - x1 (mod p, canonical)
    Fq xa, xb;
    fq_sel(xa, ge, x1, x2);
    fq_sel(xb, ge, x2, x1);
    const uint32_t bw = limbs_sub<12>(xd, xa, xb);
    limbs_add_const<12>(t, xd, FQ_P);
    fq_sel(xd, bw != 0, t, xd);
    uint32_t k = ctz31(d);
    shr_k(d, k);
    half_k(xd, k);
    if (!done) {
      fq_sel(u, ge, d, u);
      fq_sel(x1, ge, xd, x1);
      fq_sel(v, ge, v, d);
      fq_sel(x2, ge, x2, xd);
    }
    done = done || limbs_eq<12>(u, one) || limbs_eq<12>(v, one);
  }
  Fq x, r3;
  fq_sel(x, limbs_eq<12>(u, one), x1, x2);
  limbs_set_const<12>(r3, FQ_R3);
  fq_mul(r, x, r3);
}

// Returns true and r = sqrt(a) if a is a square (p = 3 mod 4: a^((p+1)/4)).
HD bool fq_sqrt(Fq& r, const Fq& a) {
  Fq t, y;
  fq_pow_window(t, a, POW_SQRT_PLAN);  // a^((p-3)/4)
  fq_mul(y, t, a);                          // a^((p+1)/4)
  Fq y2;
  fq_sqr(y2, y);
  r = y;
  return fq_eq(y2, a);
}

// canonical(a) > (p-1)/2   <=>  a > -a  (pairing 0.14 ordering on canonical values, a != 0)
HD bool fq_is_lex_largest(const Fq& a) {
  Fq c;
  fq_from_mont(c, a);
  Fq t;
  uint32_t borrow = limbs_sub_const<12>(t, c, P_MINUS_1_DIV_2);  // c - (p-1)/2
  return borrow == 0 && !limbs_is_zero<12>(t);
}

// ============================================================================ Fr (scalars)
HD void fr_canon(Fr& r, const Fr& a) {
  Fr t;
  uint32_t borrow = limbs_sub_const<8>(t, a, FR_R);
  limbs_select<8>(r, borrow == 0, a, t);
}

// 4r > 2^256, so Fr cannot use Fq's lazy [0, 2m) range: inputs must be canonical (< r), the
// CIOS output is < 2r and one conditional subtraction makes it canonical again.
HD void fr_mul(Fr& r, const Fr& a, const Fr& b) {
  Fr t;
  mont_mul<8, 8>(t, a, b, FR_R, FR_NP);
  fr_canon(r, t);
}

HD void fr_add(Fr& r, const Fr& a, const Fr& b) {
  // inputs canonical (< r < 2^255): sum < 2^256
  limbs_add<8>(r, a, b);
  fr_canon(r, r);
}

HD void fr_sub(Fr& r, const Fr& a, const Fr& b) {
  uint32_t borrow = limbs_sub<8>(r, a, b);
  Fr t;
  limbs_add_const<8>(t, r, FR_R);
  limbs_select<8>(r, borrow != 0, r, t);
}

HD void fr_to_mont(Fr& r, const Fr& a) {
  Fr r2;
  limbs_set_const<8>(r2, FR_R2);
  fr_mul(r, a, r2);
  fr_canon(r, r);
}

HD void fr_from_mont(Fr& r, const Fr& a) {
  Fr one;
  limbs_zero<8>(one);
  one.v[0] = 1;
  fr_mul(r, a, one);
  fr_canon(r, r);
}

HDN void fr_pow_const(Fr& r, const Fr& a, const uint32_t* e) {
  Fr acc;
  limbs_set_const<8>(acc, FR_ONE);
  for (int w = 7; w >= 0; --w) {
    const uint32_t word = e[w];
    for (int b = 31; b >= 0; --b) {
      fr_mul(acc, acc, acc);
      if ((word >> b) & 1u) fr_mul(acc, acc, a);
    }
  }
  fr_canon(r, acc);
}

HD void fr_inv(Fr& r, const Fr& a) { fr_pow_const(r, a, EXP_R_MINUS_2); }

// small canonical integer -> Montgomery Fr
HD void fr_from_u64(Fr& r, uint64_t x) {
  Fr a;
  limbs_zero<8>(a);
  a.v[0] = (uint32_t)x;
  a.v[1] = (uint32_t)(x >> 32);
  fr_to_mont(r, a);
}

// ============================================================================ Fq2 = Fq[u]/(u^2+1)
struct Fq2 {
  Fq c0, c1;
};

HD void fq2_zero(Fq2& r) {
  fq_zero(r.c0);
  fq_zero(r.c1);
}
HD void fq2_one(Fq2& r) {
  fq_one(r.c0);
  fq_zero(r.c1);
}
HD void fq2_set(Fq2& r, const uint32_t* c) {
  fq_set(r.c0, c);
  fq_set(r.c1, c + 12);
}
HD void fq2_add(Fq2& r, const Fq2& a, const Fq2& b) {
  fq_add(r.c0, a.c0, b.c0);
  fq_add(r.c1, a.c1, b.c1);
}
HD void fq2_sub(Fq2& r, const Fq2& a, const Fq2& b) {
  fq_sub(r.c0, a.c0, b.c0);
  fq_sub(r.c1, a.c1, b.c1);
}
HD void fq2_dbl(Fq2& r, const Fq2& a) { fq2_add(r, a, a); }
HD void fq2_neg(Fq2& r, const Fq2& a) {
  fq_neg(r.c0, a.c0);
  fq_neg(r.c1, a.c1);
}
HD void fq2_conj(Fq2& r, const Fq2& a) {
  r.c0 = a.c0;
  fq_neg(r.c1, a.c1);
}
// Karatsuba: 3 Fq multiplications
HD void fq2_mul(Fq2& r, const Fq2& a, const Fq2& b) {
  Fq t0, t1, s0, s1;
  fq_mul(t0, a.c0, b.c0);
  fq_mul(t1, a.c1, b.c1);
  fq_add(s0, a.c0, a.c1);
  fq_add(s1, b.c0, b.c1);
  fq_mul(s0, s0, s1);
  fq_sub(r.c0, t0, t1);
  fq_sub(s0, s0, t0);
  fq_sub(r.c1, s0, t1);
}
// (a0 + a1 u)^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u
HD void fq2_sqr(Fq2& r, const Fq2& a) {
  Fq s, d, m;
  fq_add(s, a.c0, a.c1);
  fq_sub(d, a.c0, a.c1);
  fq_mul(m, a.c0, a.c1);
  fq_mul(r.c0, s, d);
  fq_dbl(r.c1, m);
}
HD void fq2_mul_fq(Fq2& r, const Fq2& a, const Fq& b) {
  fq_mul(r.c0, a.c0, b);
  fq_mul(r.c1, a.c1, b);
}
// multiply by xi = 1 + u
HD void fq2_mul_xi(Fq2& r, const Fq2& a) {
  Fq t0, t1;
  fq_sub(t0, a.c0, a.c1);
  fq_add(t1, a.c0, a.c1);
  r.c0 = t0;
  r.c1 = t1;
}
HD bool fq2_is_zero(const Fq2& a) { return fq_is_zero(a.c0) && fq_is_zero(a.c1); }
HD bool fq2_eq(const Fq2& a, const Fq2& b) { return fq_eq(a.c0, b.c0) && fq_eq(a.c1, b.c1); }
HD void fq2_inv(Fq2& r, const Fq2& a) {
  Fq t0, t1;
  fq_sqr(t0, a.c0);
  fq_sqr(t1, a.c1);
  fq_add(t0, t0, t1);
  fq_inv(t0, t0);
  fq_mul(r.c0, a.c0, t0);
  fq_mul(t1, a.c1, t0);
  fq_neg(r.c1, t1);
}

// Square root in Fq2 via the norm: two Fq exponentiations.  Returns false if a is a
// non-square.  Any root is fine: callers choose between y and -y by pairing 0.14's order.
HDN bool fq2_sqrt(Fq2& r, const Fq2& a) {
  Fq n, t;
  fq_sqr(n, a.c0);
  fq_sqr(t, a.c1);
  fq_add(n, n, t);  // norm a0^2 + a1^2
  Fq s;
  fq_sqrt(s, n);    // validity checked at the end (r^2 == a)
  Fq half;
  fq_set(half, FQ_INV2);
  Fq d;
  fq_add(d, a.c0, s);
  fq_mul(d, d, half);  // delta = (a0 + s)/2
  if (fq_is_zero(d)) {
    fq_sub(d, a.c0, s);
    fq_mul(d, d, half);
  }
  Fq tt, x0;
  fq_pow_window(tt, d, POW_SQRT_PLAN);  // t = delta^((p-3)/4)
  fq_mul(x0, tt, d);                         // x0 = delta^((p+1)/4)
  Fq chk;
  fq_mul(chk, tt, x0);  // delta^((p-1)/2) = +-1
  Fq one;
  fq_one(one);
  Fq2 cand;
  if (fq_eq(chk, one)) {
    // x = (x0, a1 * t / 2)
    cand.c0 = x0;
    fq_mul(cand.c1, a.c1, tt);
    fq_mul(cand.c1, cand.c1, half);
  } else {
    // delta non-square: x = (-a1 * t / 2, x0)
    Fq u;
    fq_mul(u, a.c1, tt);
    fq_mul(u, u, half);
    fq_neg(cand.c0, u);
    cand.c1 = x0;
  }
  Fq2 sq;
  fq2_sqr(sq, cand);
  r = cand;
  return fq2_eq(sq, a);
}

// pairing 0.14 Ord for Fq2 (c1, then c0): is a > -a ?
HD bool fq2_is_lex_largest(const Fq2& a) {
  if (!fq_is_zero(a.c1)) return fq_is_lex_largest(a.c1);
  return fq_is_lex_largest(a.c0);
}

// a^(p^k): conjugation for odd k
HD void fq2_frob(Fq2& r, const Fq2& a, int k) {
  if (k & 1)
    fq2_conj(r, a);
  else
    r = a;
}

// ============================================================================ Fq6 = Fq2[v]/(v^3 - xi)
struct Fq6 {
  Fq2 c0, c1, c2;
};

HD void fq6_zero(Fq6& r) {
  fq2_zero(r.c0);
  fq2_zero(r.c1);
  fq2_zero(r.c2);
}
HD void fq6_one(Fq6& r) {
  fq2_one(r.c0);
  fq2_zero(r.c1);
  fq2_zero(r.c2);
}
HD void fq6_add(Fq6& r, const Fq6& a, const Fq6& b) {
  fq2_add(r.c0, a.c0, b.c0);
  fq2_add(r.c1, a.c1, b.c1);
  fq2_add(r.c2, a.c2, b.c2);
}
HD void fq6_sub(Fq6& r, const Fq6& a, const Fq6& b) {
  fq2_sub(r.c0, a.c0, b.c0);
  fq2_sub(r.c1, a.c1, b.c1);
  fq2_sub(r.c2, a.c2, b.c2);
}
HD void fq6_neg(Fq6& r, const Fq6& a) {
  fq2_neg(r.c0, a.c0);
  fq2_neg(r.c1, a.c1);
  fq2_neg(r.c2, a.c2);
}
// multiply by v: (c0, c1, c2) -> (xi c2, c0, c1)
HD void fq6_mul_v(Fq6& r, const Fq6& a) {
  Fq2 t;
  fq2_mul_xi(t, a.c2);
  r.c2 = a.c1;
  r.c1 = a.c0;
  r.c0 = t;
}
// Karatsuba: 6 Fq2 multiplications
HD void fq6_mul(Fq6& r, const Fq6& a, const Fq6& b) {
  Fq2 v0, v1, v2, s, t, c0, c1, c2;
  fq2_mul(v0, a.c0, b.c0);
  fq2_mul(v1, a.c1, b.c1);
  fq2_mul(v2, a.c2, b.c2);
  // c0 = v0 + xi((a1 + a2)(b1 + b2) - v1 - v2)
  fq2_add(s, a.c1, a.c2);
  fq2_add(t, b.c1, b.c2);
  fq2_mul(s, s, t);
  fq2_sub(s, s, v1);
  fq2_sub(s, s, v2);
  fq2_mul_xi(s, s);
  fq2_add(c0, v0, s);
  // c1 = (a0 + a1)(b0 + b1) - v0 - v1 + xi v2
  fq2_add(s, a.c0, a.c1);
  fq2_add(t, b.c0, b.c1);
  fq2_mul(s, s, t);
  fq2_sub(s, s, v0);
  fq2_sub(s, s, v1);
  fq2_mul_xi(t, v2);
  fq2_add(c1, s, t);
  // c2 = (a0 + a2)(b0 + b2) - v0 - v2 + v1
  fq2_add(s, a.c0, a.c2);
  fq2_add(t, b.c0, b.c2);
  fq2_mul(s, s, t);
  fq2_sub(s, s, v0);
  fq2_sub(s, s, v2);
  fq2_add(c2, s, v1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
// CH-SQR2
HD void fq6_sqr(Fq6& r, const Fq6& a) {
  Fq2 s0, s1, s2, s3, s4, t;
  fq2_sqr(s0, a.c0);
  fq2_mul(s1, a.c0, a.c1);
  fq2_dbl(s1, s1);
  fq2_sub(t, a.c0, a.c1);
  fq2_add(t, t, a.c2);
  fq2_sqr(s2, t);
  fq2_mul(s3, a.c1, a.c2);
  fq2_dbl(s3, s3);
  fq2_sqr(s4, a.c2);
  Fq6 o;
  fq2_mul_xi(t, s3);
  fq2_add(o.c0, s0, t);
  fq2_mul_xi(t, s4);
  fq2_add(o.c1, s1, t);
  fq2_add(t, s1, s2);
  fq2_add(t, t, s3);
  fq2_sub(t, t, s0);
  fq2_sub(o.c2, t, s4);
  r = o;
}
// a * (b0 + b1 v)   (5 Fq2 multiplications)
HD void fq6_mul_by_01(Fq6& r, const Fq6& a, const Fq2& b0, const Fq2& b1) {
  Fq2 t0, t1, s, t, c0, c1, c2;
  fq2_mul(t0, a.c0, b0);
  fq2_mul(t1, a.c1, b1);
  // c0 = t0 + xi * a2 * b1
  fq2_mul(s, a.c2, b1);
  fq2_mul_xi(s, s);
  fq2_add(c0, t0, s);
  // c1 = (a0 + a1)(b0 + b1) - t0 - t1
  fq2_add(s, a.c0, a.c1);
  fq2_add(t, b0, b1);
  fq2_mul(s, s, t);
  fq2_sub(s, s, t0);
  fq2_sub(c1, s, t1);
  // c2 = t1 + a2 * b0
  fq2_mul(s, a.c2, b0);
  fq2_add(c2, t1, s);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
// a * (b1 v)   (3 Fq2 multiplications)
HD void fq6_mul_by_1(Fq6& r, const Fq6& a, const Fq2& b1) {
  Fq2 t0, t1, t2;
  fq2_mul(t2, a.c2, b1);
  fq2_mul_xi(t2, t2);
  fq2_mul(t0, a.c0, b1);
  fq2_mul(t1, a.c1, b1);
  r.c0 = t2;
  r.c1 = t0;
  r.c2 = t1;
}
HDN void fq6_inv(Fq6& r, const Fq6& a) {
  Fq2 t0, t1, t2, s, d;
  // t0 = c0^2 - xi c1 c2
  fq2_sqr(t0, a.c0);
  fq2_mul(s, a.c1, a.c2);
  fq2_mul_xi(s, s);
  fq2_sub(t0, t0, s);
  // t1 = xi c2^2 - c0 c1
  fq2_sqr(t1, a.c2);
  fq2_mul_xi(t1, t1);
  fq2_mul(s, a.c0, a.c1);
  fq2_sub(t1, t1, s);
  // t2 = c1^2 - c0 c2
  fq2_sqr(t2, a.c1);
  fq2_mul(s, a.c0, a.c2);
  fq2_sub(t2, t2, s);
  // d = c0 t0 + xi (c2 t1 + c1 t2)
  fq2_mul(d, a.c2, t1);
  fq2_mul(s, a.c1, t2);
  fq2_add(d, d, s);
  fq2_mul_xi(d, d);
  fq2_mul(s, a.c0, t0);
  fq2_add(d, d, s);
  fq2_inv(d, d);
  fq2_mul(r.c0, t0, d);
  fq2_mul(r.c1, t1, d);
  fq2_mul(r.c2, t2, d);
}
HD void fq6_frob(Fq6& r, const Fq6& a, int k) {
  Fq2 c1, c2;
  fq2_frob(r.c0, a.c0, k);
  fq2_frob(c1, a.c1, k);
  fq2_frob(c2, a.c2, k);
  Fq2 g1, g2;
  if (k == 1) {
    fq2_set(g1, FROB6_C1_1);
    fq2_set(g2, FROB6_C2_1);
  } else if (k == 2) {
    fq2_set(g1, FROB6_C1_2);
    fq2_set(g2, FROB6_C2_2);
  } else {
    fq2_set(g1, FROB6_C1_3);
    fq2_set(g2, FROB6_C2_3);
  }
  fq2_mul(r.c1, c1, g1);
  fq2_mul(r.c2, c2, g2);
}

// ============================================================================ Fq12 = Fq6[w]/(w^2 - v)
struct Fq12 {
  Fq6 c0, c1;
};

HD void fq12_one(Fq12& r) {
  fq6_one(r.c0);
  fq6_zero(r.c1);
}
HD void fq12_conj(Fq12& r, const Fq12& a) {
  r.c0 = a.c0;
  fq6_neg(r.c1, a.c1);
}
HDN void fq12_mul(Fq12& r, const Fq12& a, const Fq12& b) {
  Fq6 aa, bb, s, t;
  fq6_mul(aa, a.c0, b.c0);
  fq6_mul(bb, a.c1, b.c1);
  fq6_add(s, a.c0, a.c1);
  fq6_add(t, b.c0, b.c1);
  fq6_mul(s, s, t);
  fq6_sub(s, s, aa);
  fq6_sub(r.c1, s, bb);
  fq6_mul_v(t, bb);
  fq6_add(r.c0, aa, t);
}
// complex squaring: 2 Fq6 multiplications
HD void fq12_sqr(Fq12& r, const Fq12& a) {
  Fq6 ab, s, t;
  fq6_mul(ab, a.c0, a.c1);
  fq6_add(s, a.c0, a.c1);
  fq6_mul_v(t, a.c1);
  fq6_add(t, a.c0, t);
  fq6_mul(s, s, t);
  fq6_sub(s, s, ab);
  fq6_mul_v(t, ab);
  fq6_sub(r.c0, s, t);
  fq6_add(r.c1, ab, ab);
}
// f * line where line = (l00 + l01 v) + (l11 v) w
HD void fq12_mul_by_line(Fq12& f, const Fq2& l00, const Fq2& l01, const Fq2& l11) {
  Fq6 t0, t1, s;
  fq6_mul_by_01(t0, f.c0, l00, l01);
  fq6_mul_by_1(t1, f.c1, l11);
  fq6_add(s, f.c0, f.c1);
  Fq2 m;
  fq2_add(m, l01, l11);
  fq6_mul_by_01(s, s, l00, m);
  fq6_sub(s, s, t0);
  fq6_sub(f.c1, s, t1);
  fq6_mul_v(s, t1);
  fq6_add(f.c0, t0, s);
}
HDN void fq12_inv(Fq12& r, const Fq12& a) {
  Fq6 t0, t1;
  fq6_sqr(t0, a.c0);
  fq6_sqr(t1, a.c1);
  fq6_mul_v(t1, t1);
  fq6_sub(t0, t0, t1);
  fq6_inv(t0, t0);
  fq6_mul(r.c0, a.c0, t0);
  fq6_mul(t1, a.c1, t0);
  fq6_neg(r.c1, t1);
}
HDN void fq12_frob(Fq12& r, const Fq12& a, int k) {
  Fq6 c1;
  fq6_frob(r.c0, a.c0, k);
  fq6_frob(c1, a.c1, k);
  Fq2 g;
  if (k == 1)
    fq2_set(g, FROB12_C1_1);
  else if (k == 2)
    fq2_set(g, FROB12_C1_2);
  else
    fq2_set(g, FROB12_C1_3);
  fq2_mul(r.c1.c0, c1.c0, g);
  fq2_mul(r.c1.c1, c1.c1, g);
  fq2_mul(r.c1.c2, c1.c2, g);
}
HD bool fq12_is_one(const Fq12& a) {
  Fq2 one;
  fq2_one(one);
  return fq2_eq(a.c0.c0, one) && fq2_is_zero(a.c0.c1) && fq2_is_zero(a.c0.c2) &&
         fq2_is_zero(a.c1.c0) && fq2_is_zero(a.c1.c1) && fq2_is_zero(a.c1.c2);
}
HD bool fq12_eq(const Fq12& a, const Fq12& b) {
  return fq2_eq(a.c0.c0, b.c0.c0) && fq2_eq(a.c0.c1, b.c0.c1) && fq2_eq(a.c0.c2, b.c0.c2) &&
         fq2_eq(a.c1.c0, b.c1.c0) && fq2_eq(a.c1.c1, b.c1.c1) && fq2_eq(a.c1.c2, b.c1.c2);
}

// Granger-Scott squaring in the cyclotomic subgroup (6 Fq2 multiplications).
// Fq12 viewed as Fq4^3: (c0.c0, c1.c1), (c1.c0, c0.c2), (c0.c1, c1.c2).
HD void fq4_sqr(Fq2& t0, Fq2& t1, const Fq2& a, const Fq2& b) {
  Fq2 tmp, s, u;
  fq2_mul(tmp, a, b);
  fq2_add(s, a, b);
  fq2_mul_xi(u, b);
  fq2_add(u, u, a);
  fq2_mul(s, s, u);
  fq2_sub(s, s, tmp);
  fq2_mul_xi(u, tmp);
  fq2_sub(t0, s, u);  // a^2 + xi b^2
  fq2_dbl(t1, tmp);   // 2ab
}
HD void fq12_cyclotomic_sqr(Fq12& r, const Fq12& a) {
  Fq2 t0, t1, t2, t3, t4, t5, tmp;
  fq4_sqr(t0, t1, a.c0.c0, a.c1.c1);
  fq4_sqr(t2, t3, a.c1.c0, a.c0.c2);
  fq4_sqr(t4, t5, a.c0.c1, a.c1.c2);
  Fq12 o;
  // z0 = 3 t0 - 2 z0
  fq2_sub(tmp, t0, a.c0.c0);
  fq2_dbl(tmp, tmp);
  fq2_add(o.c0.c0, tmp, t0);
  // z1 = 3 t1 + 2 z1
  fq2_add(tmp, t1, a.c1.c1);
  fq2_dbl(tmp, tmp);
  fq2_add(o.c1.c1, tmp, t1);
  // z2 = 3 xi t5 + 2 z2
  Fq2 x5;
  fq2_mul_xi(x5, t5);
  fq2_add(tmp, x5, a.c1.c0);
  fq2_dbl(tmp, tmp);
  fq2_add(o.c1.c0, tmp, x5);
  // z3 = 3 t4 - 2 z3
  fq2_sub(tmp, t4, a.c0.c2);
  fq2_dbl(tmp, tmp);
  fq2_add(o.c0.c2, tmp, t4);
  // z4 = 3 t2 - 2 z4
  fq2_sub(tmp, t2, a.c0.c1);
  fq2_dbl(tmp, tmp);
  fq2_add(o.c0.c1, tmp, t2);
  // z5 = 3 t3 + 2 z5
  fq2_add(tmp, t3, a.c1.c2);
  fq2_dbl(tmp, tmp);
  fq2_add(o.c1.c2, tmp, t3);
  r = o;
}

}  // namespace hbtc
