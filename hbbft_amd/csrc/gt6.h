// Wavefront-cooperative pairing arithmetic for gfx950: one GT / Fq12 value spread over a
// group of 6 lanes, one Fq2 coefficient per lane.
//
// Replaces the single-lane Miller loop + final exponentiation (pairing.h) for the pairing
// checks of PublicKeyShare::verify_decryption_share (/root/reference/src/
// threshold_decryption.rs:159) and PublicKeyShare::verify (src/coin.rs:151) as batched by
// hbtc_rlc.hip.  A single lane holding a whole Fq12 (144 VGPRs) plus temporaries spills to
// scratch and runs the ~17k Fq multiplications of a check serially; here a check's state
// is 24 VGPRs per lane and each Fq12 operation's Fq2 products run on 6 lanes at once.
//
// Basis.  Fq12 = Fq2[w] / (w^6 - xi), xi = 1 + u: f = sum_{k<6} f_k w^k.  It is the tower
// Fq6[w]/(w^2 - v), Fq6 = Fq2[v]/(v^3 - xi) of field.h flattened (v = w^2):
//     f_0 = c0.c0, f_1 = c1.c0, f_2 = c0.c1, f_3 = c1.c1, f_4 = c0.c2, f_5 = c1.c2.
// Lane l of a wave holds coefficient k = l mod 6 of group g = l / 6; lanes 60..63 form a
// partial group whose results are never used (they take part in every exchange so the
// exchanges stay in converged control flow).
//
// Operations (Fq2 products on the critical path of one lane, vs the serial tower):
//     mul        f_k = sum_i a_i b_{k-i} (xi on wrap)            6 Fq2 mul   (18 Fq2 on 1 lane)
//     sqr        symmetric terms, doubled                         4 Fq2 mul   (12)
//     line mul   f*(A + B w^2 + Y w^3)                            2 Fq2 + 1 Fq2xFq
//     cyclotomic Granger-Scott over the pairs (k, k+3)             2 Fq2 mul   (6)
//     frobenius  conj^j(f_k) * xi^(k (p^j - 1)/6)                 1 Fq2 mul
// Values are exchanged with ds_bpermute (no LDS storage, no barriers: a group never spans
// two waves).  Every lane of a group executes the same instruction stream; data-dependent
// choices are selects.
#pragma once
#include "pairing.h"

namespace hbtc {
namespace gt {

// ------------------------------------------------------------------------------ lane plumbing
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t shfl(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0ull; }
__device__ __forceinline__ void fetch(Fq& r, const Fq& x, uint32_t src) {
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = shfl(x.v[i], src);
}
#else
// Host build (tests/native): the cooperative code runs on host threads, one per lane, that
// meet at every exchange (tests/native/gt_sim.cpp provides the simulator).
uint32_t lane_id();
uint32_t shfl(uint32_t v, uint32_t src);
bool wave_any(bool p);
void fetch_words(uint32_t* r, const uint32_t* x, int n, uint32_t src);
inline void fetch(Fq& r, const Fq& x, uint32_t src) { fetch_words(r.v, x.v, 12, src); }
#endif
HD void fetch2(Fq2& r, const Fq2& x, uint32_t src) {
  fetch(r.c0, x.c0, src);
  fetch(r.c1, x.c1, src);
}

// Position of the calling lane inside its group.  rep = 1: 6 lanes per group, lane k holds
// coefficient k.  rep = 3 (the latency form): 18 lanes per group, coefficient k replicated on
// the three lanes 3k + j (sub-lane j), and every Fq2 product split over them (mul2 below: one
// Fq product per lane instead of three): a check's chain of dependent instructions shrinks by
// ~1.7x for ~1.7x the lane-instructions, the trade for check levels too small to fill the chip.
struct Pos {
  uint32_t k;     // coefficient index 0..5
  uint32_t base;  // lane holding coefficient 0 (sub-lane 0)
  uint32_t sub;   // 0..rep-1
  uint32_t rep;   // lanes per coefficient: 1 or 3
};
HD Pos pos(uint32_t rep = 1) {
  const uint32_t l = lane_id();
  const uint32_t gs = 6u * rep;
  const uint32_t g = l / gs, w = l - gs * g;
  return Pos{w / rep, gs * g, w % rep, rep};
}
// the lane holding coefficient k of the caller's group, on the caller's sub-lane
HD uint32_t src(const Pos& ps, uint32_t k) { return ps.base + ps.rep * k + ps.sub; }

HD void fq2_sel(Fq2& r, bool c, const Fq2& a, const Fq2& b) {
  fq_sel(r.c0, c, a.c0, b.c0);
  fq_sel(r.c1, c, a.c1, b.c1);
}
// r = t ? xi * a : a
HD void fq2_xi_if(Fq2& r, bool t, const Fq2& a) {
  Fq2 x;
  fq2_mul_xi(x, a);
  fq2_sel(r, t, x, a);
}

// Fq2 product (Karatsuba) with ONE Fq multiplication site in a rolled 3-step loop: with the
// ~660-instruction product-scanning multiply inlined, three sites per Fq2 product put the
// cooperative kernels far past the instruction cache; the operand selects cost ~10%.
// With the product as a shared subroutine (HBTC_FQMUL_SR) a site is a few dozen instructions:
// straight-line Karatsuba, no operand selects.
#if defined(__HIP_DEVICE_COMPILE__) && defined(HBTC_FQMUL_SR)
HD void mul2_one(Fq2& r, const Fq2& a, const Fq2& b) {
  Fq sa, sb, t0, t1, t2;
  fq_add(sa, a.c0, a.c1);
  fq_add(sb, b.c0, b.c1);
  fq_mul(t0, a.c0, b.c0);
  fq_mul(t1, a.c1, b.c1);
  fq_mul(t2, sa, sb);
  fq_sub(r.c0, t0, t1);
  fq_sub(t2, t2, t0);
  fq_sub(r.c1, t2, t1);
}
HD void mul2_fq_one(Fq2& r, const Fq2& a, const Fq& y) {
  fq_mul(r.c0, a.c0, y);
  fq_mul(r.c1, a.c1, y);
}
#else
HD void mul2_one(Fq2& r, const Fq2& a, const Fq2& b) {
  Fq sa, sb;
  fq_add(sa, a.c0, a.c1);
  fq_add(sb, b.c0, b.c1);
  Fq t0, t1, t2;
#pragma unroll 1
  for (uint32_t t = 0; t < 3; ++t) {
    Fq x, y, q;
    fq_sel(x, t == 1, a.c1, sa);
    fq_sel(x, t == 0, a.c0, x);
    fq_sel(y, t == 1, b.c1, sb);
    fq_sel(y, t == 0, b.c0, y);
    fq_mul(q, x, y);
    fq_sel(t0, t == 0, q, t0);
    fq_sel(t1, t == 1, q, t1);
    t2 = q;
  }
  fq_sub(r.c0, t0, t1);
  fq_sub(t2, t2, t0);
  fq_sub(r.c1, t2, t1);
}
// a * (y + 0u): two Fq products through the same single site
HD void mul2_fq_one(Fq2& r, const Fq2& a, const Fq& y) {
  Fq t0;
#pragma unroll 1
  for (uint32_t t = 0; t < 2; ++t) {
    Fq q;
    Fq x;
    fq_sel(x, t == 0, a.c0, a.c1);
    fq_mul(q, x, y);
    fq_sel(t0, t == 0, q, t0);
    r.c1 = q;
  }
  r.c0 = t0;
}
#endif

// Fq2 products of the group's lanes.  rep = 1: the whole product on each lane.  rep = 3: the
// three sub-lanes of a coefficient each form one Karatsuba term (a0 b0, a1 b1, (a0 + a1)(b0 +
// b1)) and exchange them, so every sub-lane ends with the same product (the operands are
// replicated, hence so is the result).  ps.rep is uniform over the wave: a uniform branch.
HD void mul2(Fq2& r, const Fq2& a, const Fq2& b, const Pos& ps) {
  if (ps.rep == 1) {
    mul2_one(r, a, b);
    return;
  }
  Fq x, y, t, t0, t1, t2;
  {
    Fq sa, sb;
    fq_add(sa, a.c0, a.c1);
    fq_add(sb, b.c0, b.c1);
    fq_sel(x, ps.sub == 1, a.c1, sa);
    fq_sel(x, ps.sub == 0, a.c0, x);
    fq_sel(y, ps.sub == 1, b.c1, sb);
    fq_sel(y, ps.sub == 0, b.c0, y);
  }
  fq_mul(t, x, y);
  const uint32_t l0 = ps.base + ps.rep * ps.k;  // sub-lane 0 of this coefficient
  fetch(t0, t, l0);
  fetch(t1, t, l0 + 1);
  fetch(t2, t, l0 + 2);
  fq_sub(r.c0, t0, t1);
  fq_sub(t2, t2, t0);
  fq_sub(r.c1, t2, t1);
}
// a * (y + 0u): sub-lanes 0 and 1 form the two products (sub-lane 2 repeats sub-lane 1's)
HD void mul2_fq(Fq2& r, const Fq2& a, const Fq& y, const Pos& ps) {
  if (ps.rep == 1) {
    mul2_fq_one(r, a, y);
    return;
  }
  Fq x, t;
  fq_sel(x, ps.sub == 0, a.c0, a.c1);
  fq_mul(t, x, y);
  const uint32_t l0 = ps.base + ps.rep * ps.k;
  fetch(r.c0, t, l0);
  fetch(r.c1, t, l0 + 1);
}

// The short operand-choice loops of the line product, the easy part and the Miller step stay
// rolled where the product is inlined (code size: instruction cache); with the shared-subroutine
// product they are unrolled, so the operand choices are compile-time.  (Unrolling mul's and
// sqr's term loops too hoists their operand fetches: 220 -> 960 B/lane of scratch.)
#if defined(__HIP_DEVICE_COMPILE__) && defined(HBTC_FQMUL_SR) && !defined(HBTC_GT_ROLLED)
#define HBTC_GT_SMALL_LOOP HBTC_PRAGMA(unroll)
#else
#define HBTC_GT_SMALL_LOOP HBTC_PRAGMA(unroll 1)
#endif

// ------------------------------------------------------------------------------ GT operations
// Out-of-line on the device unless HBTC_GT_INLINE: the glue of the final exponentiation and the
// location search call these a few dozen times per check; their by-reference operands cost
// ~100 dwords of stack traffic per call.  The check kernels are built with HBTC_GT_INLINE
// (Makefile): scratch 960 -> ~330 B/lane at the same C3 throughput, the latency-bound small
// calls slightly faster.
#if defined(__HIP_DEVICE_COMPILE__) && defined(HBTC_GT_INLINE)
#define GTN __device__ __forceinline__
#elif defined(__HIP_DEVICE_COMPILE__)
#define GTN __device__ __attribute__((noinline))
#else
#define GTN static inline
#endif

// ------------------------------------------------------------ lazy reduction (rep = 1 layout)
// Every output coefficient of mul / sqr / the line product is a sum of 3-6 Fq2 products.  With
// the double-width accumulator (field.h FqAcc) the products stay unreduced and each Fq half of
// the coefficient is reduced ONCE: Fq2 schoolbook with xi and the sign folded into the operands,
//     half 0: sum x0 y0 + x1 (-y1),   half 1: sum x0 y1 + x1 y0,
// -y1 as the reduced negation (< 2p), so every term is a product of two values < 2p and a half
// sums at most 12 of them (< 48 p^2).  Per lane of a mul: 24 half products (144 MADs each) + 2
// reductions, instead of 18 full Montgomery products (288 each).  HBTC_GT_LAZY2 / HBTC_GT_KARA
// below: one pass over two accumulators, Karatsuba terms (18 half products).
#ifndef HBTC_GT_LAZY
#if !defined(__HIP_DEVICE_COMPILE__) || defined(HBTC_FQMUL_SR)
#define HBTC_GT_LAZY 1
#else
#define HBTC_GT_LAZY 0
#endif
#endif

// With HBTC_GT_LAZY2 (default) both halves accumulate in ONE pass over the terms, half 1 in the
// second accumulator (v85..v109 in the subroutine builds): each term's operands are fetched and
// xi / the negation applied once instead of once per half.
#ifndef HBTC_GT_LAZY2
#define HBTC_GT_LAZY2 1
#endif
// With HBTC_GT_KARA (default, one-pass only) a term is Karatsuba on the two accumulators,
// three half products instead of four (field.h fq_acc_kara): X = c0 + 24 p^2, Y = c1.
#ifndef HBTC_GT_KARA
#define HBTC_GT_KARA HBTC_GT_LAZY2
#endif
#if HBTC_GT_LAZY
#if HBTC_GT_LAZY2
constexpr uint32_t GT_LAZY_PASSES = 1;
#else
constexpr uint32_t GT_LAZY_PASSES = 2;
#endif
// pass h: one-pass mode adds half 0 of x * y to a0 and half 1 to a1; two-pass mode adds half h
// to a0
HD void acc_init(FqAcc& a0, FqAcc& a1) {
  if (HBTC_GT_KARA)
    fq_acc_k24(a0);
  else
    fq_acc_zero(a0);
  fq_acc_zero(a1);
}
HD void mac2_pass(FqAcc& a0, FqAcc& a1, const Fq2& x, const Fq2& y, uint32_t h) {
  if (HBTC_GT_KARA) {
    fq_acc_kara(a0, a1, x.c0, x.c1, y.c0, y.c1);
  } else if (GT_LAZY_PASSES == 1) {
    Fq ny1;
    fq_neg(ny1, y.c1);
    fq_acc_mac(a0, x.c0, y.c0);
    fq_acc_mac2(a1, x.c0, y.c1);
    fq_acc_mac(a0, x.c1, ny1);
    fq_acc_mac2(a1, x.c1, y.c0);
  } else if (h == 0) {
    Fq ny1;
    fq_neg(ny1, y.c1);
    fq_acc_mac(a0, x.c0, y.c0);
    fq_acc_mac(a0, x.c1, ny1);
  } else {
    fq_acc_mac(a0, x.c0, y.c1);
    fq_acc_mac(a0, x.c1, y.c0);
  }
}
// x * (y + 0u), y in Fq
HD void mac1_pass(FqAcc& a0, FqAcc& a1, const Fq2& x, const Fq& y, uint32_t h) {
  if (GT_LAZY_PASSES == 1) {
    fq_acc_mac(a0, x.c0, y);
    fq_acc_mac2(a1, x.c1, y);
  } else {
    fq_acc_mac(a0, h ? x.c1 : x.c0, y);
  }
}
HD void redc_pass(Fq2& r, const FqAcc& a0, const FqAcc& a1, uint32_t h) {
  if (GT_LAZY_PASSES == 1) {
    fq_acc_redc(r.c0, a0);
    fq_acc_redc2(r.c1, a1);
  } else {
    fq_acc_redc(h ? r.c1 : r.c0, a0);
  }
}

// LDS staging of the operands of mul / sqr (device, rep = 1): each lane stores its coefficient
// once and every term reads the one it needs from the group's lanes, so the operands are not
// live in VGPRs across the term loop.  With them live (48 VGPRs) beside the accumulators and the
// shared subroutines' fixed registers, the three-wave check kernels reloaded a and b from
// scratch in every iteration (k_chk_plain: 576 B/lane, 618 spill instructions).  The stage is one
// [word][lane] array per wave (12 KB; every kernel using these runs one wave per block), read
// in program order by the same wave (LDS operations of a wave complete in order).
#ifndef HBTC_GT_LDS
#define HBTC_GT_LDS 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && HBTC_GT_LDS
constexpr uint32_t GT_STAGE_WORDS = 24u * 64u;
__device__ __forceinline__ uint32_t* gt_stage() {
  __shared__ uint32_t s_gt_stage[2 * GT_STAGE_WORDS];
  return s_gt_stage;
}
__device__ __forceinline__ void stage_put(uint32_t* s, const Fq2& x) {
  const uint32_t l = lane_id();
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&x);
#pragma unroll
  for (int i = 0; i < 24; ++i) s[i * 64 + l] = w[i];
}
__device__ __forceinline__ void stage_get(Fq2& x, const uint32_t* s, uint32_t from) {
  uint32_t* w = reinterpret_cast<uint32_t*>(&x);
#pragma unroll
  for (int i = 0; i < 24; ++i) w[i] = s[i * 64 + from];
}
#define HBTC_GT_STAGED 1
#else
#define HBTC_GT_STAGED 0
#endif

#if HBTC_GT_STAGED
// f = a * b with both operands staged (sa, sb)
GTN void mul_staged(Fq2& f, const uint32_t* sa, const uint32_t* sb, const Pos& ps) {
  Fq2 r;
#pragma unroll
  for (uint32_t h = 0; h < GT_LAZY_PASSES; ++h) {
    FqAcc a0, a1;
    acc_init(a0, a1);
#pragma unroll 1
    for (uint32_t i = 0; i < 6; ++i) {
      const bool wrap = i > ps.k;
      const uint32_t j = wrap ? ps.k + 6 - i : ps.k - i;
      Fq2 ai, bj;
      stage_get(ai, sa, src(ps, i));
      stage_get(bj, sb, src(ps, j));
      fq2_xi_if(bj, wrap, bj);
      mac2_pass(a0, a1, ai, bj, h);
    }
    redc_pass(r, a0, a1, h);
  }
  f = r;
}
GTN void mul_lazy(Fq2& f, const Fq2& a, const Fq2& b, const Pos& ps) {
  uint32_t* sa = gt_stage();
  uint32_t* sb = sa + GT_STAGE_WORDS;
  stage_put(sa, a);
  stage_put(sb, b);
  mul_staged(f, sa, sb, ps);
}
#else
GTN void mul_lazy(Fq2& f, const Fq2& a, const Fq2& b, const Pos& ps) {
  Fq2 r;
#pragma unroll
  for (uint32_t h = 0; h < GT_LAZY_PASSES; ++h) {
    FqAcc a0, a1;
    acc_init(a0, a1);
#pragma unroll 1
    for (uint32_t i = 0; i < 6; ++i) {
      const bool wrap = i > ps.k;
      const uint32_t j = wrap ? ps.k + 6 - i : ps.k - i;
      Fq2 ai, bj;
      fetch2(ai, a, src(ps, i));
      fetch2(bj, b, src(ps, j));
      fq2_xi_if(bj, wrap, bj);
      mac2_pass(a0, a1, ai, bj, h);
    }
    redc_pass(r, a0, a1, h);
  }
  f = r;
}
#endif
#endif

// f = a * b
GTN void mul(Fq2& f, const Fq2& a, const Fq2& b, const Pos& ps) {
#if HBTC_GT_LAZY
  if (ps.rep == 1) {
    mul_lazy(f, a, b, ps);
    return;
  }
#endif
  Fq2 acc;
  fq2_zero(acc);
#pragma unroll 1
  for (uint32_t i = 0; i < 6; ++i) {
    const bool wrap = i > ps.k;
    const uint32_t j = wrap ? ps.k + 6 - i : ps.k - i;
    Fq2 ai, bj, z;
    fetch2(ai, a, src(ps, i));
    fetch2(bj, b, src(ps, j));
    mul2(z, ai, bj, ps);
    fq2_xi_if(z, wrap, z);
    fq2_add(acc, acc, z);
  }
  f = acc;
}

// f = a^2: the unordered pairs {i, j} with i + j = k (mod 6), cross terms doubled.  Per lane
// 4 (even k) or 3 (odd k) terms, packed one byte each: i | j << 3 | xi << 6 | double << 7,
// 0xff = no term.
constexpr uint32_t sqr_word(uint32_t k) {
  uint32_t w = 0xffffffffu;
  int t = 0;
  for (uint32_t i = 0; i < 6; ++i)
    for (uint32_t j = i; j < 6; ++j)
      if ((i + j) % 6 == k) {
        const uint32_t e = i | (j << 3) | (i + j >= 6 ? 64u : 0u) | (i != j ? 128u : 0u);
        w = (w & ~(0xffu << (8 * t))) | (e << (8 * t));
        ++t;
      }
  return w;
}
static_assert(sqr_word(0) == 0x5be2e900u && sqr_word(1) == 0xffe3ea88u &&
                  sqr_word(5) == 0xff9aa1a8u,
              "squaring term table: (0,0) (1,5)x2 (2,4)x2 (3,3)x | (0,1)2 (2,5)x2 (3,4)x2");
HD uint32_t sqr_terms(uint32_t k) {
  uint32_t w = sqr_word(0);
  w = k == 1 ? sqr_word(1) : w;
  w = k == 2 ? sqr_word(2) : w;
  w = k == 3 ? sqr_word(3) : w;
  w = k == 4 ? sqr_word(4) : w;
  w = k == 5 ? sqr_word(5) : w;
  return w;
}

HD void sqr(Fq2& f, const Fq2& a, const Pos& ps) {
  const uint32_t terms = sqr_terms(ps.k);
#if HBTC_GT_LAZY
  if (ps.rep == 1) {
    // the doubling and xi go on the second operand (reduced: < 2p), a missing term multiplies 0
    Fq2 r;
#if HBTC_GT_STAGED
    uint32_t* sa = gt_stage();
    stage_put(sa, a);
#endif
#pragma unroll
    for (uint32_t h = 0; h < GT_LAZY_PASSES; ++h) {
      FqAcc lacc, lacc1;
      acc_init(lacc, lacc1);
#pragma unroll 1
      for (uint32_t t = 0; t < 4; ++t) {
        const uint32_t e = (terms >> (8 * t)) & 0xffu;
        const bool none = e == 0xffu;
        Fq2 ai, aj, d, z;
#if HBTC_GT_STAGED
        stage_get(ai, sa, src(ps, e & 7u));
        stage_get(aj, sa, src(ps, (e >> 3) & 7u));
#else
        fetch2(ai, a, src(ps, e & 7u));
        fetch2(aj, a, src(ps, (e >> 3) & 7u));
#endif
        fq2_xi_if(aj, ((e >> 6) & 1u) && !none, aj);
        fq2_dbl(d, aj);
        fq2_sel(aj, ((e >> 7) & 1u) && !none, d, aj);
        fq2_zero(z);
        fq2_sel(aj, none, z, aj);
        mac2_pass(lacc, lacc1, ai, aj, h);
      }
      redc_pass(r, lacc, lacc1, h);
    }
    f = r;
    return;
  }
#endif
  Fq2 acc;
  fq2_zero(acc);
#pragma unroll 1
  for (uint32_t t = 0; t < 4; ++t) {
    const uint32_t e = (terms >> (8 * t)) & 0xffu;
    const bool none = e == 0xffu;
    Fq2 ai, aj, z;
    fetch2(ai, a, src(ps, e & 7u));
    fetch2(aj, a, src(ps, (e >> 3) & 7u));
    mul2(z, ai, aj, ps);
    fq2_xi_if(z, ((e >> 6) & 1u) && !none, z);
    Fq2 z2;
    fq2_dbl(z2, z);
    fq2_sel(z, ((e >> 7) & 1u) && !none, z2, z);
    fq2_add(z2, acc, z);
    fq2_sel(acc, none, acc, z2);
  }
  f = acc;
}

// f = f * (A + B w^2 + Y w^3) for a Miller-loop line evaluated at a G1 point (scaled by a
// subfield factor).  The coefficients are not materialised: they sit on the lanes that computed
// them — B = (pb on lane b, pb on lane b+1), Y = py on lane y (Fq) or (py on y, py on y+1)
// (Fq2 when Y2) — and A is either (pa on lane a, pa on lane a+1) or, with A_DIRECT, the Fq2
// value Ad every lane already holds.  Each term fetches its operand, which keeps a Miller
// step's live set small.  use = false makes the line 1 (A = 1, B = Y = 0: the caller zeroes
// pa / Ad, pb, py).
template <bool A_DIRECT, bool Y2>
HD void mul_line_t(Fq2& f, const Fq& pa, uint32_t a, const Fq2& Ad, const Fq& pb, uint32_t b,
                   const Fq& py, uint32_t y, bool use, const Pos& ps) {
  const uint32_t k = ps.k;
#if HBTC_GT_LAZY
  if (ps.rep == 1) {
    // xi on the f coefficient (the operand every term has), so an Fq Y stays one product a half
    Fq2 r;
#if HBTC_GT_STAGED
    uint32_t* sa = gt_stage();  // f staged: not live across the terms
    stage_put(sa, f);
#endif
#pragma unroll
    for (uint32_t h = 0; h < GT_LAZY_PASSES; ++h) {
      FqAcc lacc, lacc1;
      acc_init(lacc, lacc1);
HBTC_GT_SMALL_LOOP
      for (uint32_t t = 0; t < 3; ++t) {
        const uint32_t fk = t == 0 ? k : (t == 1 ? (k >= 2 ? k - 2 : k + 4) : (k >= 3 ? k - 3 : k + 3));
        Fq2 x, q;
#if HBTC_GT_STAGED
        stage_get(x, sa, src(ps, fk));
#else
        fetch2(x, f, src(ps, fk));
#endif
        Fq o0, o1;  // element-wise selects (no conditional between two referenced objects)
        fq_sel(o0, t == 1, pb, py);
        fq_sel(o0, t == 0, pa, o0);
        o1 = o0;
        const uint32_t l0 = t == 0 ? a : (t == 1 ? b : y);
        fetch(q.c0, o0, src(ps, l0));
        fetch(q.c1, o1, src(ps, l0 + 1));  // unused for an Fq Y
        if (A_DIRECT && t == 0) q = Ad;
        if (t == 0 && !use) {
          fq_one(q.c0);
          fq_zero(q.c1);
        }
        fq2_xi_if(x, (t == 1 && k < 2) || (t == 2 && k < 3), x);
        if (!Y2 && t == 2)  // uniform branch
          mac1_pass(lacc, lacc1, x, q.c0, h);
        else
          mac2_pass(lacc, lacc1, x, q, h);
      }
      redc_pass(r, lacc, lacc1, h);
    }
    f = r;
    return;
  }
#endif
  Fq2 acc;
  fq2_zero(acc);
HBTC_GT_SMALL_LOOP
  for (uint32_t t = 0; t < 3; ++t) {
    // term t: f_k A, f_{k-2} B (xi if k < 2), f_{k-3} Y (xi if k < 3)
    const uint32_t fk = t == 0 ? k : (t == 1 ? (k >= 2 ? k - 2 : k + 4) : (k >= 3 ? k - 3 : k + 3));
    Fq2 x, q, z;
    fetch2(x, f, src(ps, fk));
    Fq o0, o1;
    fq_sel(o0, t == 1, pb, py);
    fq_sel(o0, t == 0, pa, o0);
    o1 = o0;
    const uint32_t l0 = t == 0 ? a : (t == 1 ? b : y);
    fetch(q.c0, o0, src(ps, l0));
    fetch(q.c1, o1, src(ps, l0 + 1));  // unused for an Fq Y
    if (A_DIRECT && t == 0) q = Ad;
    if (t == 0 && !use) {
      fq_one(q.c0);
      fq_zero(q.c1);
    }
    if (!Y2 && t == 2)  // Y in Fq: two products (t is the same on every lane: a uniform branch)
      mul2_fq(z, x, q.c0, ps);
    else
      mul2(z, x, q, ps);
    fq2_xi_if(z, (t == 1 && k < 2) || (t == 2 && k < 3), z);
    fq2_add(acc, acc, z);
  }
  f = acc;
}
HD void mul_line(Fq2& f, const Fq& pa, uint32_t a, const Fq& pb, uint32_t b, const Fq& py,
                 uint32_t y, bool use, const Pos& ps) {
  Fq2 unused;
  mul_line_t<false, false>(f, pa, a, unused, pb, b, py, y, use, ps);
}

HD void conj(Fq2& f, const Pos& ps) {
  Fq2 n;
  fq2_neg(n, f);
  fq2_sel(f, (ps.k & 1u) != 0, n, f);
}

// f = phi^j(f), j = 1, 2, 3
GTN void frob(Fq2& f, int j, const Pos& ps) {
  const uint32_t* tab = j == 1 ? GT_FROB_1 : (j == 2 ? GT_FROB_2 : GT_FROB_3);
  Fq2 g, x;
  // the table row of this lane's coefficient (selects: no per-lane memory indexing)
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint32_t a = tab[i], b = tab[12 + i];
#pragma unroll
    for (uint32_t c = 1; c < 6; ++c) {
      a = ps.k == c ? tab[24 * c + i] : a;
      b = ps.k == c ? tab[24 * c + 12 + i] : b;
    }
    g.c0.v[i] = a;
    g.c1.v[i] = b;
  }
  if (j & 1)
    fq2_conj(x, f);
  else
    x = f;
  mul2(f, x, g, ps);
}

// Granger-Scott squaring of a cyclotomic element, Fq12 seen as Fq4^3 over the coefficient
// pairs (k, k+3), a = f_k, b = f_{k+3}: (a + b s)^2 = (a^2 + xi b^2) + 2ab s with s = w^3.
// Karatsuba across the pair: lane k + 3 forms m = ab, lane k forms q = (a + b)(a + xi b), so
// a^2 + xi b^2 = q - m - xi m — ONE Fq2 product per lane.  Then each output needs one value:
//     z_0 = 3 T_0 - 2 f_0   z_1 = 3 xi T_5 + 2 f_1   z_2 = 3 T_1 - 2 f_2
//     z_3 = 3 T_3 + 2 f_3   z_4 = 3 T_2 - 2 f_4      z_5 = 3 T_4 + 2 f_5
// with T_k = a^2 + xi b^2 on lanes k < 3 and 2ab on lanes k >= 3.
HD void cyc_sqr(Fq2& f, const Pos& ps) {
  const bool lo = ps.k < 3;
  const uint32_t pk = lo ? ps.k + 3 : ps.k - 3;
  Fq2 partner;
  fetch2(partner, f, src(ps, pk));
  Fq2 x, y, r;
  {
    Fq2 b, a, xb, apb, apxb;
    fq2_sel(b, lo, partner, f);
    fq2_sel(a, lo, f, partner);
    fq2_mul_xi(xb, b);
    fq2_add(apb, a, b);
    fq2_add(apxb, a, xb);
    fq2_sel(x, lo, apb, a);
    fq2_sel(y, lo, apxb, b);
  }
  mul2(r, x, y, ps);  // lo: (a + b)(a + xi b); hi: ab
  Fq2 m;
  fetch2(m, r, src(ps, pk));  // lo lanes take ab from their partner
  Fq2 T, t1, xm;
  fq2_mul_xi(xm, m);
  fq2_sub(t1, r, m);
  fq2_sub(t1, t1, xm);    // a^2 + xi b^2
  Fq2 t2;
  fq2_dbl(t2, r);         // 2ab
  fq2_sel(T, lo, t1, t2);
  // route T: lane k reads T from lane s(k) = {0, 5, 1, 3, 2, 4}[k]
  const uint32_t sk = ps.k == 0 ? 0u : ps.k == 1 ? 5u : ps.k == 2 ? 1u : ps.k == 3 ? 3u : ps.k == 4 ? 2u : 4u;
  Fq2 Ts;
  fetch2(Ts, T, src(ps, sk));
  fq2_xi_if(Ts, ps.k == 1, Ts);
  Fq2 three, two;
  fq2_dbl(three, Ts);
  fq2_add(three, three, Ts);
  fq2_dbl(two, f);
  Fq2 plus, minus;
  fq2_add(plus, three, two);
  fq2_sub(minus, three, two);
  fq2_sel(f, (ps.k & 1u) != 0, plus, minus);
}

// Group-wide AND of a per-lane predicate.
HD bool group_all(bool ok, const Pos& ps) {
  uint32_t acc = 1;
#pragma unroll
  for (uint32_t c = 0; c < 6; ++c) acc &= shfl(ok ? 1u : 0u, src(ps, c));
  return acc != 0;
}

HD bool is_one(const Fq2& f, const Pos& ps) {
  Fq2 one;
  fq2_one(one);
  const bool ok = ps.k == 0 ? fq2_eq(f, one) : fq2_is_zero(f);
  return group_all(ok, ps);
}

HD bool equal(const Fq2& a, const Fq2& b, const Pos& ps) { return group_all(fq2_eq(a, b), ps); }

HD void set_one(Fq2& f, const Pos& ps) {
  Fq2 one, zero;
  fq2_one(one);
  fq2_zero(zero);
  fq2_sel(f, ps.k == 0, one, zero);
}

// y^x for cyclotomic y (x < 0: y^|x| then conjugate)
GTN void exp_by_x(Fq2& r, const Fq2& y, const Pos& ps) {
  Fq2 acc = y;
#if HBTC_GT_STAGED
  // y stays in the second stage for the whole chain (cyc_sqr does not use the stages): not live
  // in VGPRs across the 63 squarings, and not re-staged by each of the five products
  uint32_t* sa = gt_stage();
  uint32_t* sb = sa + GT_STAGE_WORDS;
  const bool staged = ps.rep == 1;
  if (staged) stage_put(sb, y);
#endif
#pragma unroll 1
  for (int bit = 62; bit >= 0; --bit) {
    cyc_sqr(acc, ps);
    if ((BLS_X_ABS >> bit) & 1ull) {
#if HBTC_GT_STAGED
      if (staged) {
        stage_put(sa, acc);
        mul_staged(acc, sa, sb, ps);
        continue;
      }
#endif
      mul(acc, acc, y, ps);
    }
  }
  conj(acc, ps);
  r = acc;
}

// fq_inv_binary: field.h (binary extended Euclid, also used by the item passes).

// f^(p^6 - 1) = conj(f)^2 / N with N = f conj(f) in Fq6 (coefficients 0, 2, 4 = its
// v-basis digits n0, n1, n2); N^-1 = (t0 + t1 v + t2 v^2) / d with
//   t0 = n0^2 - xi n1 n2,  t1 = xi n2^2 - n0 n1,  t2 = n1^2 - n0 n2,  d = n0 t0 + xi (n2 t1 + n1 t2)
// computed on lanes 0, 2, 4 (one t each), d^-1 in Fq2 through one Fq inversion.
HD void easy_part(Fq2& r, const Fq2& f, const Pos& ps) {
  Fq2 cf = f;
  conj(cf, ps);
  Fq2 N;
  mul(N, f, cf, ps);
  Fq2 n0, n1, n2;
  fetch2(n0, N, src(ps, 0));
  fetch2(n1, N, src(ps, 2));
  fetch2(n2, N, src(ps, 4));
  const uint32_t k = ps.k;
  // t_m = tx * x * x' - ty * y * y'
  Fq2 z0, z1;
HBTC_GT_SMALL_LOOP
  for (uint32_t t = 0; t < 2; ++t) {
    Fq2 x, y, q, sx, px, py;
    // the square term, then the product term: (n1 n2), (n0 n1), (n0 n2)
    fq2_sel(sx, k == 2, n2, n0);
    fq2_sel(sx, k == 4, n1, sx);
    fq2_sel(px, k == 0, n1, n0);
    fq2_sel(py, k == 2, n1, n2);
    fq2_sel(x, t == 0, sx, px);
    fq2_sel(y, t == 0, sx, py);
    mul2(q, x, y, ps);
    fq2_sel(z0, t == 0, q, z0);
    z1 = q;
  }
  fq2_xi_if(z0, k == 2, z0);
  fq2_xi_if(z1, k == 0, z1);
  Fq2 tm;
  fq2_sub(tm, z0, z1);
  // d: lane 0 n0 t0, lane 2 xi n2 t1, lane 4 xi n1 t2
  Fq2 m, u;
  fq2_sel(m, k == 2, n2, n0);
  fq2_sel(m, k == 4, n1, m);
  mul2(u, m, tm, ps);
  fq2_xi_if(u, k != 0, u);
  Fq2 d, d2, d4;
  fetch2(d, u, src(ps, 0));
  fetch2(d2, u, src(ps, 2));
  fetch2(d4, u, src(ps, 4));
  fq2_add(d, d, d2);
  fq2_add(d, d, d4);
  // d^-1 = conj(d) / (d0^2 + d1^2)
  Fq nrm, t1;
  fq_sqr(nrm, d.c0);
  fq_sqr(t1, d.c1);
  fq_add(nrm, nrm, t1);
  Fq inv;
  fq_inv_binary(inv, nrm);
  Fq2 dinv;
  fq_mul(dinv.c0, d.c0, inv);
  fq_mul(t1, d.c1, inv);
  fq_neg(dinv.c1, t1);
  Fq2 ninv, zero;
  mul2(ninv, tm, dinv, ps);
  fq2_zero(zero);
  fq2_sel(ninv, (k & 1u) == 0, ninv, zero);
  Fq2 c2;
  sqr(c2, cf, ps);
  mul(r, c2, ninv, ps);
}

// Final exponentiation (easy part, then the hard part by the Hayashida-Hayasaka-Teruya
// x-chain, which yields the cube of the standard pairing: equality decisions are unchanged
// since gcd(3, r) = 1) — the chain of pairing.h's final_exponentiation.
HD void final_exp(Fq2& out, const Fq2& f, const Pos& ps) {
  Fq2 r, t0;
  easy_part(r, f, ps);
  t0 = r;
  frob(t0, 2, ps);
  mul(r, t0, r, ps);
  Fq2 y0, y1, y2;
  y0 = r;
  cyc_sqr(y0, ps);
  exp_by_x(y1, r, ps);
  y2 = r;
  conj(y2, ps);
  mul(y1, y1, y2, ps);
  exp_by_x(y2, y1, ps);
  conj(y1, ps);
  mul(y1, y1, y2, ps);
  exp_by_x(y2, y1, ps);
  frob(y1, 1, ps);
  mul(y1, y1, y2, ps);
  mul(r, r, y0, ps);
  exp_by_x(y0, y1, ps);
  exp_by_x(y2, y0, ps);
  y0 = y1;
  frob(y0, 2, ps);
  conj(y1, ps);
  mul(y1, y1, y2, ps);
  mul(y1, y1, y0, ps);
  mul(out, r, y1, ps);
}

// ------------------------------------------------------------------------------ Miller loop
// One argument of a pairing product.  Either (PROJ = false) a precomputed affine-normalised line
// table of the G2 argument (pairing.h Line: a + b xP v + yP v w at step j) with the G1 point P
// Jacobian — the line times Z^3 (an Fq factor, removed by the final exponentiation) is
//     Z^3 a + (X Z) b w^2 + Y w^3
// so the loop needs no inversion — or (PROJ = true, second argument only) a projective table of
// (A, B, C) per step (g2_dbl_step / g2_add_step of a G2 point that varies per check) with the
// G1 point affine (Z = 1): the line is A + B xP w^2 + C yP w^3.  An unused pair (an argument at
// infinity) contributes 1.
struct MillerArg {
  const Line* lines;   // affine-normalised table (PROJ = false)
  const Fq2* plines;   // projective (A, B, C) table, 3 * MILLER_STEPS Fq2 (PROJ = true)
  G1J P;               // the G1 argument (sign already applied)
  bool use;
};

// f = prod_{pairs} f_{|x|,Q}(P), conjugated (x < 0).  Per step the 8 Fq products that scale the
// two lines run on separate lanes (lane k: product k; lanes 0, 1: products 6, 7).
template <bool PROJ2>
HD void miller2_t(Fq2& f, const MillerArg& m1, const MillerArg& m2, const Pos& ps) {
  const uint32_t k = ps.k;
  // Round-1 product of lane k: k = 0,1 a1.c{k} Z1^3; 2,3 b1.c{k-2} X1Z1; 4,5 a2.c{k-4} Z2^3
  // (PROJ2: B2.c{k-4} x2).  Lanes 0, 1, round 2: b2.c{k} X2Z2 (PROJ2: C2.c{k} y2).  Lane 0
  // keeps Y1, the others Y2 (unused with PROJ2).  Unused pairs get zero scalars.
  Fq s1, s2, ymine, zero;
  fq_zero(zero);
  {
    const bool second = k >= 4;
    // element-wise selects, not a reference chosen between m1.P and m2.P: a select of two
    // objects' addresses keeps both in private memory (scratch) for the whole kernel
    G1J P;
    fq_sel(P.x, second, m2.P.x, m1.P.x);
    fq_sel(P.y, second, m2.P.y, m1.P.y);
    fq_sel(P.z, second, m2.P.z, m1.P.z);
    Fq z2, z3, xz;
    fq_sqr(z2, P.z);
    fq_mul(z3, z2, P.z);
    fq_mul(xz, P.x, P.z);
    fq_sel(s1, k < 2 || second, z3, xz);
    if (PROJ2 && second) s1 = m2.P.x;
    fq_sel(s1, second ? m2.use : m1.use, s1, zero);
    if (PROJ2)
      s2 = m2.P.y;
    else
      fq_mul(s2, m2.P.x, m2.P.z);
    fq_sel(s2, m2.use, s2, zero);
    fq_sel(ymine, k == 0, m1.P.y, m2.P.y);
    fq_sel(ymine, k == 0 ? m1.use : m2.use, ymine, zero);
  }
  const uint32_t c1 = k < 4 ? k : (PROJ2 ? k - 2 : k - 4);  // Fq component: a.c0 a.c1 b.c0 b.c1 / A B C
  const uint32_t c2 = (PROJ2 ? 4 : 2) + (k & 1u);            // round-2 component (b2 / C2)
  set_one(f, ps);
#if HBTC_GT_STAGED
  // s1 | s2 in the second stage for the whole loop (sqr and the line products use only the
  // first): two Fq off the loop's live set
  uint32_t* ss = gt_stage() + GT_STAGE_WORDS;
  const bool s_staged = ps.rep == 1;
  if (s_staged) {
    Fq2 s12;
    s12.c0 = s1;
    s12.c1 = s2;
    stage_put(ss, s12);
  }
#endif
  int j = 0;
  bool first = true;
#pragma unroll 1
  for (int bit = 62; bit >= 0; --bit) {
    const bool add = ((BLS_X_ABS >> bit) & 1ull) != 0;
#pragma unroll 1
    for (int rep = 0; rep < (add ? 2 : 1); ++rep) {
      if (rep == 0 && !first) sqr(f, f, ps);
      first = false;
      const Fq* L1 = reinterpret_cast<const Fq*>(m1.lines + j);
      const Fq* L2 = PROJ2 ? reinterpret_cast<const Fq*>(m2.plines + 3 * j)
                           : reinterpret_cast<const Fq*>(m2.lines + j);
      const Fq* Lr1 = k < 4 ? L1 : L2;
      Fq p1, p2;
HBTC_GT_SMALL_LOOP
      for (uint32_t t = 0; t < 2; ++t) {
        Fq q;
        Fq sv;
#if HBTC_GT_STAGED
        if (s_staged) {
          const uint32_t l = lane_id();
#pragma unroll
          for (int i = 0; i < 12; ++i) sv.v[i] = ss[(12 * t + i) * 64 + l];
        } else {
          fq_sel(sv, t == 0, s1, s2);
        }
#else
        fq_sel(sv, t == 0, s1, s2);
#endif
        fq_mul(q, t == 0 ? Lr1[c1] : L2[c2], sv);
        fq_sel(p1, t == 0, q, p1);
        p2 = q;
      }
      // line 1: A1 = p1@{0,1}, B1 = p1@{2,3}, Y1 = ymine@0
      mul_line(f, p1, 0, p1, 2, ymine, 0, m1.use, ps);
      if (PROJ2) {
        // line 2: A2 from the table, B2 = p1@{4,5} (B x2), Y2 = p2@{0,1} (C y2)
        Fq2 A2;
        A2.c0 = L2[0];
        A2.c1 = L2[1];
        mul_line_t<true, true>(f, p1, 0, A2, p1, 4, p2, 0, m2.use, ps);
      } else {
        // line 2: A2 = p1@{4,5}, B2 = p2@{0,1}, Y2 = ymine@1
        mul_line(f, p1, 4, p2, 0, ymine, 1, m2.use, ps);
      }
      ++j;
    }
  }
  conj(f, ps);
}
HD void miller2(Fq2& f, const MillerArg& m1, const MillerArg& m2, const Pos& ps) {
  miller2_t<false>(f, m1, m2, ps);
}

}  // namespace gt
}  // namespace hbtc
