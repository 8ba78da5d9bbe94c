// Pairing-product checks of the RLC batch verification (hbtc_rlc.hip) on the cooperative GT
// arithmetic of gt6.h: one check per 6-lane group, two checks (a "unit") per 12 lanes, five
// units per wave.
//
// Replaces, for batches, the per-share PublicKeyShare::verify_decryption_share
// (/root/reference/src/threshold_decryption.rs:159): for a group G of shares of one
// ciphertext, T = e(sum r_i d_i, H) e(-sum r_i pk_i, w) == 1 iff (except with probability
// 2^-64) every share of G is valid; T_w, the same with position-weighted r_i, locates a single
// wrong share as the weight w with T_w == T^w (hbtc_rlc.hip explains both; share i of a group of
// 2^k has the weight bitrev_k(i), rlc_common.h).
//
// Levels:
//   k_chk_tiles   every 64-share tile: (plain, weighted) unit; a failing tile's single wrong
//                 share is located, a tile with more goes to the sub-tile list
//   k_chk_subs    the 8 sub-tiles of each listed tile, likewise; an unlocated sub-tile sends
//                 its pending shares to the leaf list
//   k_chk_leaves  two exact per-share checks per unit (decoded shares from k_rlc_items)
// A unit's two groups run the same instruction stream; the location search is split between
// them (the plain group tries positions [0, half), the weighted group [half, count) starting
// from T^half), with a wave-wide early exit once every failing unit has its answer.
// few product sites per hot loop (gt6.h's rolled Fq2 product): inline the multiplication
#ifndef HBTC_FQMUL_SR
#define HBTC_FQMUL_INLINE
#endif
#include <algorithm>

#include "gt6.h"
#include "hbtc_kernels.h"

namespace hbtc {

using gt::Pos;

// Minimum waves per SIMD the check kernels' register budget must allow.  Three since round 4
// (168 VGPRs, ~500 B/lane of scratch against 256 / ~200 at two): C3 11.74 -> 11.94-12.03 M
// shares/s, adversarial 4.39 -> 4.55 M, C4 4.83 -> 4.96 M on one box; four (128 VGPRs, ~700 B)
// falls back (profiles/r04/run18/).
#ifndef HBTC_GT_WAVES
#define HBTC_GT_WAVES 3
#endif
// The weighted passes run few groups (the failing ones: fewer waves than SIMDs): one wave per
// SIMD, the full register file, no spills (C3: 13.9 -> 11.5 ms; the plain passes, whose grids
// fill the chip, lose 17.4 -> 21.7 ms at one wave, so they keep two).
#ifndef HBTC_GT_WAVES_SMALL
#define HBTC_GT_WAVES_SMALL 1
#endif
// The file is compiled twice (Makefile): part 1 = every kernel but the weighted passes, part 2 =
// the weighted passes.  The out-of-line GT helpers take the register budget of their most
// generous caller, so one-wave and two-wave kernels must not share a translation unit.
#ifndef HBTC_CHECK_PART
#define HBTC_CHECK_PART 0
#endif
#define HBTC_CHECK_IN(n) (HBTC_CHECK_PART == 0 || HBTC_CHECK_PART == (n))

namespace {

constexpr uint32_t UNITS_PER_WAVE = 5;
// units per wave of a layout: 5 of 12 lanes (rep 1), 1 of 36 lanes (rep 3, the latency form:
// gt6.h Pos.rep; lanes 36..63 idle)
template <uint32_t REP>
struct Units {
  static constexpr uint32_t PER_WAVE = REP == 1 ? UNITS_PER_WAVE : 1u;
};

struct UnitLane {
  uint32_t unit;     // 0..4 (5: the idle lanes 60..63); rep 3: 0 (1: idle)
  uint32_t side;     // 0: first group of the unit, 1: second
  uint32_t partner;  // the same coefficient's lane in the other group
  Pos ps;
};

__device__ __forceinline__ UnitLane unit_lane(uint32_t rep = 1) {
  const uint32_t l = gt::lane_id();
  const uint32_t gs = 6u * rep;
  UnitLane u;
  u.unit = l / (2u * gs);
  u.side = (l / gs) & 1u;
  u.partner = u.side ? l - gs : l + gs;
  u.ps = gt::pos(rep);
  return u;
}

__device__ __forceinline__ G1J g1j_of(const G1A& a) {
  G1J r;
  jac_from_aff(r, a);
  return r;
}

// e = FE( f_{|x|,H}(S) * f_{|x|,w}(-P) ): the pairing-product value of one group.
__device__ __forceinline__ void pair_value(Fq2& e, const G1J& S, bool use1, const Line* hl, const G1J& P,
                           bool use2, const Line* wl, const Pos& ps) {
  gt::MillerArg m1{hl, nullptr, S, use1};
  gt::MillerArg m2{wl, nullptr, P, use2};
  fq_neg(m2.P.y, P.y);
  Fq2 f;
  gt::miller2(f, m1, m2, ps);
  gt::final_exp(e, f, ps);
}

// The trees of the item passes give share i of a group of 2^k the weight bitrev_k(i)
// (rlc_common.h): the position of weight w, or -1 past the group's count.
__device__ __forceinline__ int32_t weight_pos(int32_t w, int k, uint32_t count) {
  if (w < 0) return -1;
  const uint32_t i = __builtin_bitreverse32((uint32_t)w) >> (32 - k);
  return i < count ? (int32_t)i : -1;
}

// Single-error location for a failing unit of a group of 2^(lg+1) shares: the weight w with
// Tw == T^w (unique: T has prime order), mapped to its position, or -1.  The group on side 0
// tries [0, half), side 1 tries [half, 2 half) from T^half (half = 2^lg).  Every lane of the wave
// runs the loop; `need` is false on units that passed or are idle.
__device__ __forceinline__ int32_t locate(const Fq2& T, const Fq2& Tw, uint32_t count, int lg, bool need,
                          const UnitLane& ul) {
  const uint32_t half = 1u << lg;
  Fq2 acc;
  gt::set_one(acc, ul.ps);
  if (ul.side) {
    acc = T;
#pragma unroll 1
    for (int i = 0; i < lg; ++i) gt::cyc_sqr(acc, ul.ps);
  }
  const uint32_t p0 = ul.side ? half : 0u;
  int32_t found = -1;
#pragma unroll 1
  for (uint32_t q = 0; q < half; ++q) {
    const bool live = need && found < 0;
    if (!gt::wave_any(live)) break;
    if (gt::equal(acc, Tw, ul.ps) && live) found = (int32_t)(p0 + q);
    gt::mul(acc, acc, T, ul.ps);
  }
  // combine the two halves
  const int32_t other = (int32_t)gt::shfl((uint32_t)found, ul.partner);
  const int32_t f0 = ul.side ? other : found, f1 = ul.side ? found : other;
  return weight_pos(f0 >= 0 ? f0 : f1, lg + 1, count);
}

// T (plain, side 0) and Tw (weighted, side 1) on both groups of a unit, the plain verdict.
__device__ __forceinline__ bool unit_values(Fq2& T, Fq2& Tw, const Fq2& e, const UnitLane& ul) {
  Fq2 other;
  gt::fetch2(other, e, ul.partner);
  gt::fq2_sel(T, ul.side == 0, e, other);
  gt::fq2_sel(Tw, ul.side == 0, other, e);
  return gt::is_one(T, ul.ps);
}

}  // namespace

// ------------------------------------------------------------------------------ group levels
// Plain first: a group's weighted check (needed only to locate a wrong share) runs only when
// its plain check failed.  Every group of a level is one 6-lane check; a unit carries two
// groups.  Level 0 = the 64-share tiles (group g = tile g); level 1 = the 8-share sub-tiles of
// the listed tiles (group g = sub-tile g & 7 of tile sub_list[g >> 3], the paired schedules);
// level 2 = the 32-share halves of the listed tiles (group g = half g & 1 of tile
// sub_list[g >> 1]); level 3 = the 4 sub-tiles of the listed halves (half code list2[g >> 2],
// sub-tile 4 (code & 1) + (g & 3) of tile sub_list[code >> 1]).  Halves between the tiles and
// the sub-tiles cut a tile with two wrong shares from 8 sub-tile checks to 1 half check (the
// other half's value is the tile's divided by it) plus the halves' own location.
namespace {

struct GroupRef {
  uint32_t inst, t, sub, lo, hi;
  bool active, inst_ok;
};

template <int LEVEL>
__device__ __forceinline__ GroupRef group_ref(uint32_t g, uint32_t n, const Tile* tiles,
                                              const uint32_t* sub_list, const uint32_t* list2,
                                              const int32_t* h_status, const int32_t* w_status) {
  GroupRef r{0, 0, 8, 0, 0, false, false};
  if (g >= n) return r;
  uint32_t t, sub = 8;
  if (LEVEL == 0) {
    t = g;
  } else if (LEVEL == 1) {
    t = sub_list[g >> 3];
    sub = g & 7u;
  } else if (LEVEL == 2) {
    t = sub_list[g >> 1];
    sub = g & 1u;  // the half
  } else {
    const uint32_t code = list2[g >> 2];
    t = sub_list[code >> 1];
    sub = 4u * (code & 1u) + (g & 3u);
  }
  const Tile tile = tiles[t];
  r.t = t;
  r.inst = tile.inst;
  r.sub = sub;
  if (LEVEL == 0) {
    r.lo = tile.first;
    r.hi = tile.first + tile.count;
    r.inst_ok = h_status[tile.inst] == HBTC_ACCEPT && w_status[tile.inst] == HBTC_ACCEPT;
  } else {
    const uint32_t span = LEVEL == 2 ? 32u : 8u;
    r.lo = tile.first + sub * span;
    r.hi = min(tile.first + tile.count, r.lo + span);
    r.inst_ok = true;  // listed tiles belong to instances whose H and w decoded
  }
  r.active = r.lo < r.hi;
  return r;
}

// the (plain or weighted) G1 sums of a group
template <int LEVEL>
__device__ __forceinline__ void group_sums(G1J& S, G1J& P, const TileSums& ts, uint32_t sub,
                                           bool weighted) {
  if (LEVEL == 2) {
    S = weighted ? ts.SHW[sub] : ts.SH[sub];
    P = weighted ? ts.PHW[sub] : ts.PH[sub];
  } else {
    S = weighted ? ts.SW[sub] : ts.S[sub];
    P = weighted ? ts.PW[sub] : ts.P[sub];
  }
}

// 64-bit fingerprint of a GT value (canonical low words of coefficients 0 and 3), group-wide.
__device__ __forceinline__ void gt_fingerprint(uint32_t& a, uint32_t& b, const Fq2& x, const Pos& ps) {
  Fq c;
  fq_canon(c, x.c0);
  a = gt::shfl(c.v[0], gt::src(ps, 0));
  b = gt::shfl(c.v[0], gt::src(ps, 3));
}

// Single-error location inside one group of 2^lg shares: the weight w < 2^lg with Tw == T^w
// mapped to its position (weight_pos), or -1.  Baby-step giant-step over w = 8 a + b:
// fingerprints of T^b (b < 8), then Tw T^(-8 a) (T^-8 = conj(T^8): T is cyclotomic) for
// 8 a < 2^lg — at most 16 products instead of 64 — and the match is confirmed exactly (T^w
// recomputed by square-and-multiply and compared in full).
__device__ __forceinline__ int32_t locate_group(const Fq2& T, const Fq2& Tw, uint32_t count, int lg,
                                                bool need, const Pos& ps) {
  const uint32_t size = 1u << lg;
  uint32_t fa[8], fb[8];
  Fq2 acc;
  gt::set_one(acc, ps);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    gt_fingerprint(fa[b], fb[b], acc, ps);
    gt::mul(acc, acc, T, ps);  // ends as T^8
  }
  Fq2 step = acc;
  gt::conj(step, ps);  // T^-8
  Fq2 g = Tw;
  int32_t found = -1;
#pragma unroll 1
  for (uint32_t a = 0; a < 8u; ++a) {
    const bool live = need && found < 0 && 8u * a < size;
    if (!gt::wave_any(live)) break;
    uint32_t ga, gb;
    gt_fingerprint(ga, gb, g, ps);
#pragma unroll
    for (int b = 0; b < 8; ++b)
      if (live && found < 0 && ga == fa[b] && gb == fb[b] && 8u * a + (uint32_t)b < size)
        found = (int32_t)(8u * a + (uint32_t)b);
    gt::mul(g, g, step, ps);
  }
  // confirm: T^found == Tw (a fingerprint match is only a candidate)
  const uint32_t pe = found >= 0 ? (uint32_t)found : 0u;
  Fq2 tp;
  gt::set_one(tp, ps);
#pragma unroll 1
  for (int bit = 5; bit >= 0; --bit) {
    gt::cyc_sqr(tp, ps);
    Fq2 m;
    gt::mul(m, tp, T, ps);
    gt::fq2_sel(tp, ((pe >> bit) & 1u) != 0, m, tp);
  }
  const bool ok = gt::equal(tp, Tw, ps);
  return weight_pos(found >= 0 && ok ? found : -1, lg, count);
}

// Append a group's node to a split level's list with its GT values (T, U) and weight form
// (ab = log2 alpha | beta << 8: U = prod E_i^(r_i (alpha w_i + beta)), w_i the node-local
// bit-reversed weights).  Called by every lane of the group (converged: the slot is broadcast).
__device__ __forceinline__ void split_list(const SplitOut& o, bool list, uint32_t code, const Fq2& T,
                                           const Fq2& U, uint32_t ab, const Pos& ps) {
  uint32_t pos = 0;
  if (list && ps.k == 0 && ps.sub == 0) pos = atomicAdd(o.count, 1u);
  pos = gt::shfl(pos, ps.base);
  if (!list || ps.sub != 0) return;
  o.T[(size_t)pos * 6u + ps.k] = T;
  o.U[(size_t)pos * 6u + ps.k] = U;
  if (ps.k == 0) {
    o.list[pos] = code;
    o.ab[pos] = ab;
  }
}

// y^e for a small non-negative e < 2^NB (square-and-multiply, uniform over the wave)
template <int NB>
__device__ __forceinline__ void gt_pow_small(Fq2& r, const Fq2& y, uint32_t e, const Pos& ps) {
  Fq2 acc;
  gt::set_one(acc, ps);
#pragma unroll 1
  for (int bit = NB - 1; bit >= 0; --bit) {
    gt::cyc_sqr(acc, ps);
    Fq2 m;
    gt::mul(m, acc, y, ps);
    gt::fq2_sel(acc, ((e >> bit) & 1u) != 0, m, acc);
  }
  r = acc;
}

// y^(2^k) for k <= KMAX (uniform: KMAX squarings, the extra ones discarded)
template <int KMAX>
__device__ __forceinline__ void gt_pow2k(Fq2& r, const Fq2& y, uint32_t k, const Pos& ps) {
  Fq2 acc = y;
#pragma unroll 1
  for (int i = 0; i < KMAX; ++i) {
    Fq2 sq = acc;
    gt::cyc_sqr(sq, ps);
    gt::fq2_sel(acc, (uint32_t)i < k, sq, acc);
  }
  r = acc;
}

}  // namespace

#if HBTC_CHECK_IN(1)
// Plain check of every group of the level; a failing group stores its value T (6 lanes, one
// Fq2 each) and joins the list of the weighted pass.
template <int LEVEL>
__global__ void __launch_bounds__(64, HBTC_GT_WAVES) k_chk_plain(
    uint32_t n_direct, const uint32_t* __restrict__ n_listed, const uint32_t* __restrict__ sub_list,
    const uint32_t* __restrict__ list2, const Tile* __restrict__ tiles,
    const TileSums* __restrict__ sums,
    const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    const G2A* __restrict__ w_aff, const Line* __restrict__ w_lines,
    const int32_t* __restrict__ h_status, const int32_t* __restrict__ w_status,
    Fq2* __restrict__ Tbuf, uint32_t* __restrict__ fail_count, uint32_t* __restrict__ fail_list) {
  HBTC_LATENCY_PRIO();
  const uint32_t n = LEVEL == 0 ? n_direct : *n_listed * (LEVEL == 1 ? 8u : 4u);
  if (blockIdx.x * 2u * UNITS_PER_WAVE >= n) return;  // wave-uniform: grids are sized for the worst case
  const UnitLane ul = unit_lane();
  const uint32_t g = (blockIdx.x * UNITS_PER_WAVE + ul.unit) * 2u + ul.side;
  const GroupRef r = group_ref<LEVEL>(ul.unit < UNITS_PER_WAVE ? g : n, n, tiles, sub_list, list2,
                                      h_status, w_status);
  G1J S, P;
  jac_set_inf(S);
  jac_set_inf(P);
  if (r.active) group_sums<LEVEL>(S, P, sums[r.t], r.sub, false);
  const bool use1 = r.active && r.inst_ok && !jac_is_inf(S) && !h_aff[r.inst].inf;
  const bool use2 = r.active && r.inst_ok && !jac_is_inf(P) && !w_aff[r.inst].inf;
  Fq2 e;
  pair_value(e, S, use1, h_lines + (size_t)r.inst * MILLER_STEPS, P, use2,
             w_lines + (size_t)r.inst * MILLER_STEPS, ul.ps);
  const bool pass = gt::is_one(e, ul.ps);
  // undecodable H / w: k_rlc_finalize decides the group's items
  if (!r.active || !r.inst_ok || pass) return;
  Tbuf[(size_t)g * 6u + ul.ps.k] = e;
  if (ul.ps.k == 0) fail_list[atomicAdd(fail_count, 1u)] = g;
}

// Level 2: the halves of every listed tile i (tile sub_list[i]).  One pairing check per listed
// tile: half 0's value T_0; half 1's is T_tile / T_0 (T_tile stored by k_chk_plain<0> at the
// tile's index; GT values are cyclotomic, so the inverse is the conjugate).  A failing half
// stores its value and joins the list of the weighted pass as code 2 i + h.
__global__ void __launch_bounds__(64, HBTC_GT_WAVES) k_chk_halves(
    const uint32_t* __restrict__ n_listed, const uint32_t* __restrict__ tile_list,
    const Tile* __restrict__ tiles, const TileSums* __restrict__ sums,
    const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    const G2A* __restrict__ w_aff, const Line* __restrict__ w_lines,
    const Fq2* __restrict__ Ttile, Fq2* __restrict__ Thalf, uint32_t* __restrict__ fail_count,
    uint32_t* __restrict__ fail_list) {
  HBTC_LATENCY_PRIO();
  const uint32_t n = *n_listed;
  if (blockIdx.x * 2u * UNITS_PER_WAVE >= n) return;
  const UnitLane ul = unit_lane();
  const uint32_t i = (blockIdx.x * UNITS_PER_WAVE + ul.unit) * 2u + ul.side;
  const bool active = ul.unit < UNITS_PER_WAVE && i < n;
  uint32_t t = 0, inst = 0, count = 0;
  G1J S, P;
  jac_set_inf(S);
  jac_set_inf(P);
  Fq2 T;
  gt::set_one(T, ul.ps);
  if (active) {
    t = tile_list[i];
    const Tile tile = tiles[t];
    inst = tile.inst;
    count = tile.count;
    S = sums[t].SH[0];
    P = sums[t].PH[0];
    T = Ttile[(size_t)t * 6u + ul.ps.k];
  }
  const bool use1 = active && !jac_is_inf(S) && !h_aff[inst].inf;
  const bool use2 = active && !jac_is_inf(P) && !w_aff[inst].inf;
  Fq2 e0, e1;
  pair_value(e0, S, use1, h_lines + (size_t)inst * MILLER_STEPS, P, use2,
             w_lines + (size_t)inst * MILLER_STEPS, ul.ps);
  {
    Fq2 c0 = e0;
    gt::conj(c0, ul.ps);
    gt::mul(e1, T, c0, ul.ps);
  }
  const bool pass0 = gt::is_one(e0, ul.ps), pass1 = gt::is_one(e1, ul.ps);
  if (!active) return;
  if (!pass0) {
    Thalf[(size_t)(2u * i) * 6u + ul.ps.k] = e0;
    if (ul.ps.k == 0) fail_list[atomicAdd(fail_count, 1u)] = 2u * i;
  }
  if (count > 32u && !pass1) {
    Thalf[(size_t)(2u * i + 1u) * 6u + ul.ps.k] = e1;
    if (ul.ps.k == 0) fail_list[atomicAdd(fail_count, 1u)] = 2u * i + 1u;
  }
}

#endif  // part 1

#if HBTC_CHECK_IN(2)
// Weighted check of every listed group: locate its single wrong share (REJECT it), else pass
// the group down (level 0: its tile to the sub-tile list; level 1: its pending shares to the
// exact leaf checks).
template <int LEVEL>
__global__ void __launch_bounds__(64, HBTC_GT_WAVES_SMALL) k_chk_weighted(
    const uint32_t* __restrict__ fail_count, const uint32_t* __restrict__ fail_list,
    const uint32_t* __restrict__ sub_list_in, const uint32_t* __restrict__ list2,
    const Tile* __restrict__ tiles, const TileSums* __restrict__ sums,
    const G2A* __restrict__ h_aff,
    const Line* __restrict__ h_lines, const G2A* __restrict__ w_aff,
    const Line* __restrict__ w_lines, const int32_t* __restrict__ h_status,
    const int32_t* __restrict__ w_status, const Fq2* __restrict__ Tbuf,
    int32_t* __restrict__ status, uint32_t* __restrict__ out_count, uint32_t* __restrict__ out_list,
    SplitOut split) {
  HBTC_LATENCY_PRIO();
  const uint32_t n = *fail_count;
  if (blockIdx.x * 2u * UNITS_PER_WAVE >= n) return;
  const UnitLane ul = unit_lane();
  const uint32_t j = (blockIdx.x * UNITS_PER_WAVE + ul.unit) * 2u + ul.side;
  const bool listed = ul.unit < UNITS_PER_WAVE && j < n;
  const uint32_t g = listed ? fail_list[j] : 0u;
  const GroupRef r = group_ref<LEVEL>(listed ? g : ~0u, ~0u, tiles, sub_list_in, list2, h_status,
                                      w_status);
  G1J S, P;
  jac_set_inf(S);
  jac_set_inf(P);
  Fq2 T;
  gt::set_one(T, ul.ps);
  if (r.active) {
    group_sums<LEVEL>(S, P, sums[r.t], r.sub, true);
    T = Tbuf[(size_t)g * 6u + ul.ps.k];
  }
  const bool use1 = r.active && !jac_is_inf(S) && !h_aff[r.inst].inf;
  const bool use2 = r.active && !jac_is_inf(P) && !w_aff[r.inst].inf;
  Fq2 Tw;
  pair_value(Tw, S, use1, h_lines + (size_t)r.inst * MILLER_STEPS, P, use2,
             w_lines + (size_t)r.inst * MILLER_STEPS, ul.ps);
  const int32_t loc = locate_group(T, Tw, r.hi - r.lo, LEVEL == 0 ? 6 : (LEVEL == 2 ? 5 : 3),
                                   r.active, ul.ps);
  if (LEVEL == 0 && split.list) {
    // the split levels: an unlocated tile is listed with its values (T, T_w; alpha = 1, beta = 0)
    const bool located = loc >= 0 && status[r.lo + loc] == HBTC_RLC_PENDING;
    split_list(split, r.active && !located, r.t << 3, T, Tw, 0u, ul.ps);
    if (r.active && located && ul.ps.k == 0) status[r.lo + loc] = HBTC_REJECT;
    return;
  }
  if (!r.active || ul.ps.k != 0) return;
  if (loc >= 0 && status[r.lo + loc] == HBTC_RLC_PENDING) {
    status[r.lo + loc] = HBTC_REJECT;
    return;
  }
  if (LEVEL == 0) {
    out_list[atomicAdd(out_count, 1u)] = r.t;
  } else if (LEVEL == 2) {
    out_list[atomicAdd(out_count, 1u)] = g;  // the half code 2 i + h
  } else {
    for (uint32_t i = r.lo; i < r.hi; ++i)
      if (status[i] == HBTC_RLC_PENDING) {
        const uint32_t pos = atomicAdd(out_count, 1u);
        out_list[2 * pos] = i;
        out_list[2 * pos + 1] = r.inst;
      }
  }
}

// Paired check (the latency form, for calls too small to fill the chip): a unit carries ONE
// group, its plain value T on side 0 and its weighted value T_w on side 1, so a failing group's
// single wrong share is located in the same launch.  An unlocated group either joins the
// sub-tile list (LEVEL 0, !TO_LEAVES) or sends its pending shares to the exact leaf checks.
// Levels per call: tiles -> leaves (2 check latencies) or tiles -> sub-tiles -> leaves (3),
// instead of the plain-first form's 5 (hbtc_api.hip picks by the call's tile count).
template <int LEVEL, bool TO_LEAVES>
__global__ void __launch_bounds__(64, HBTC_GT_WAVES_SMALL) k_chk_pair(
    uint32_t n_direct, const uint32_t* __restrict__ n_listed, const uint32_t* __restrict__ sub_list,
    const Tile* __restrict__ tiles, const TileSums* __restrict__ sums,
    const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    const G2A* __restrict__ w_aff, const Line* __restrict__ w_lines,
    const int32_t* __restrict__ h_status, const int32_t* __restrict__ w_status,
    int32_t* __restrict__ status, uint32_t* __restrict__ out_count, uint32_t* __restrict__ out_list,
    SplitOut split) {
  HBTC_LATENCY_PRIO();
  const uint32_t n = LEVEL == 0 ? n_direct : *n_listed * 8u;
  if (blockIdx.x * UNITS_PER_WAVE >= n) return;  // wave-uniform: grids are sized for the worst case
  const UnitLane ul = unit_lane();
  const uint32_t g = blockIdx.x * UNITS_PER_WAVE + ul.unit;
  const GroupRef r = group_ref<LEVEL>(ul.unit < UNITS_PER_WAVE ? g : n, n, tiles, sub_list, nullptr,
                                      h_status, w_status);
  G1J S, P;
  jac_set_inf(S);
  jac_set_inf(P);
  if (r.active) group_sums<LEVEL>(S, P, sums[r.t], r.sub, ul.side != 0);
  const bool use1 = r.active && r.inst_ok && !jac_is_inf(S) && !h_aff[r.inst].inf;
  const bool use2 = r.active && r.inst_ok && !jac_is_inf(P) && !w_aff[r.inst].inf;
  Fq2 e, T, Tw;
  pair_value(e, S, use1, h_lines + (size_t)r.inst * MILLER_STEPS, P, use2,
             w_lines + (size_t)r.inst * MILLER_STEPS, ul.ps);
  const bool pass = unit_values(T, Tw, e, ul);
  // undecodable H / w: k_rlc_finalize decides the group's items
  const bool fail = r.active && r.inst_ok && !pass;
  const int32_t loc = locate(T, Tw, r.hi - r.lo, LEVEL == 0 ? 5 : 2, fail, ul);
  // (the split levels follow the plain-first tile level only: `split` is unused here)
  if (!fail || ul.side != 0 || ul.ps.k != 0) return;
  if (loc >= 0 && status[r.lo + loc] == HBTC_RLC_PENDING) {
    status[r.lo + loc] = HBTC_REJECT;
    return;
  }
  if (LEVEL == 0 && !TO_LEAVES) {
    out_list[atomicAdd(out_count, 1u)] = r.t;
  } else {
    uint32_t m = 0;
    for (uint32_t i = r.lo; i < r.hi; ++i) m += status[i] == HBTC_RLC_PENDING;
    uint32_t pos = atomicAdd(out_count, m);
    for (uint32_t i = r.lo; i < r.hi; ++i)
      if (status[i] == HBTC_RLC_PENDING) {
        out_list[2 * pos] = i;
        out_list[2 * pos + 1] = r.inst;
        ++pos;
      }
  }
}

// Split level LVL (1: listed tiles, 2: listed halves, 3: listed quarters).  A listed node X
// (>= 2 wrong shares, or one its location could not confirm) carries its values T_X and
// U_X = prod_X E_i^(r_i (alpha w_i + beta)).  A unit checks X's LEFT child L (plain T_L on side
// 0, weighted W_L on side 1: one paired check) and derives the right child R without pairings:
//     T_R = T_X / T_L,   U_R = U_X / (W_L^(2 alpha) T_L^beta)   (alpha_R = 2 alpha, beta_R = alpha + beta)
// since the parent's local weight of a share is 2 w_L in L and 2 w_R + 1 in R (bit-reversed
// weights).  GT values are cyclotomic: division is multiplication by the conjugate.  Then side 0
// locates a single wrong share in L (W_L = T_L^w) and side 1 in R (U_R = T_R^(alpha_R w + beta_R):
// G = T_R^alpha_R, Y = U_R / T_R^beta_R, G^w = Y), both by the baby-step giant-step search.  A
// child whose value is 1 passes; an unlocated child is listed for level LVL + 1 (LVL 3: its
// pending shares go to the exact leaf checks).  Two checks per listed node instead of 16 for its
// eight sub-tiles; soundness as every group check (hbtc_rlc.hip): a derived value is the plain /
// weighted RLC value of the child itself.
template <int LVL, uint32_t REP>
__global__ void __launch_bounds__(64, HBTC_GT_WAVES_SMALL) k_chk_split(
    const uint32_t* __restrict__ n_in, const uint32_t* __restrict__ in_list,
    const Fq2* __restrict__ in_T, const Fq2* __restrict__ in_U, const uint32_t* __restrict__ in_ab,
    const Tile* __restrict__ tiles, const TileSums* __restrict__ sums,
    const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    const G2A* __restrict__ w_aff, const Line* __restrict__ w_lines,
    int32_t* __restrict__ status, uint32_t* __restrict__ leaf_count, uint32_t* __restrict__ leaves,
    SplitOut split) {
  HBTC_LATENCY_PRIO();
  constexpr uint32_t SIZE = 64u >> (LVL - 1), HALF = SIZE / 2;
  constexpr int LG = 6 - LVL;  // log2(HALF)
  constexpr uint32_t UPW = Units<REP>::PER_WAVE;
  const uint32_t n = *n_in;
  if (blockIdx.x * UPW >= n) return;  // wave-uniform: grids are sized for the worst case
  const UnitLane ul = unit_lane(REP);
  const uint32_t u = blockIdx.x * UPW + ul.unit;
  const bool active = ul.unit < UPW && u < n;
  const uint32_t code = active ? in_list[u] : 0u;
  const uint32_t t = code >> 3, j = code & 7u;
  Tile tile{0, 0, 0, 0};
  if (active) tile = tiles[t];
  const uint32_t end = tile.first + tile.count;
  const uint32_t x_lo = min(end, tile.first + j * SIZE);
  const uint32_t x_hi = min(end, x_lo + SIZE);
  const uint32_t l_hi = min(x_hi, x_lo + HALF);  // L = [x_lo, l_hi), R = [l_hi, x_hi)
  G1J S, P;
  jac_set_inf(S);
  jac_set_inf(P);
  if (active) {
    const TileSums& ts = sums[t];
    const bool wt = ul.side != 0;
    if (LVL == 1) {
      S = wt ? ts.SHW[0] : ts.SH[0];
      P = wt ? ts.PHW[0] : ts.PH[0];
    } else if (LVL == 2) {  // the left quarter of half j
      S = wt ? ts.SQW[j] : ts.SQ[j];
      P = wt ? ts.PQW[j] : ts.PQ[j];
    } else {  // the left eighth of quarter j
      S = wt ? ts.SW[2 * j] : ts.S[2 * j];
      P = wt ? ts.PW[2 * j] : ts.P[2 * j];
    }
  }
  const uint32_t inst = tile.inst;
  const bool use1 = active && !jac_is_inf(S) && !h_aff[inst].inf;
  const bool use2 = active && !jac_is_inf(P) && !w_aff[inst].inf;
  Fq2 e, TL, WL;
  pair_value(e, S, use1, h_lines + (size_t)inst * MILLER_STEPS, P, use2,
             w_lines + (size_t)inst * MILLER_STEPS, ul.ps);
  unit_values(TL, WL, e, ul);
  Fq2 TX, UX;
  gt::set_one(TX, ul.ps);
  gt::set_one(UX, ul.ps);
  uint32_t ab = 0;
  if (active) {
    TX = in_T[(size_t)u * 6u + ul.ps.k];
    UX = in_U[(size_t)u * 6u + ul.ps.k];
    ab = in_ab[u];
  }
  const uint32_t ka = ab & 0xffu, beta = ab >> 8;  // alpha = 2^ka: ka <= LVL - 1, beta < 2^(LVL-1)
  Fq2 TR, UR;
  {
    Fq2 c = TL;
    gt::conj(c, ul.ps);
    gt::mul(TR, TX, c, ul.ps);
    Fq2 m, tb;
    gt_pow2k<LVL>(m, WL, ka + 1u, ul.ps);              // W_L^(2 alpha)
    gt_pow_small<(LVL > 1 ? LVL - 1 : 1)>(tb, TL, beta, ul.ps);  // T_L^beta
    gt::mul(m, m, tb, ul.ps);
    gt::conj(m, ul.ps);
    gt::mul(UR, UX, m, ul.ps);
  }
  const uint32_t kaR = ka + 1u, betaR = (1u << ka) + beta;
  const bool passL = gt::is_one(TL, ul.ps), passR = gt::is_one(TR, ul.ps);
  // location inputs of this side
  Fq2 G = TL, Y = WL;
  {
    Fq2 g, tb;
    gt_pow2k<LVL>(g, TR, kaR, ul.ps);
    gt_pow_small<LVL>(tb, TR, betaR, ul.ps);
    gt::conj(tb, ul.ps);
    Fq2 y;
    gt::mul(y, UR, tb, ul.ps);
    gt::fq2_sel(G, ul.side != 0, g, TL);
    gt::fq2_sel(Y, ul.side != 0, y, WL);
  }
  const uint32_t lo = ul.side ? l_hi : x_lo, hi = ul.side ? x_hi : l_hi;
  const bool pass = ul.side ? passR : passL;
  const bool need = active && !pass && lo < hi;
  const int32_t loc = locate_group(G, Y, hi - lo, LG, need, ul.ps);
  // decide on every lane of the group before any write (the status reads must not race)
  const bool located = need && loc >= 0 && status[lo + loc] == HBTC_RLC_PENDING;
  const bool unresolved = need && !located;
  if (LVL < 3) {
    const uint32_t ab_child = ul.side ? (kaR | (betaR << 8)) : 0u;
    // values selected element-wise: `side ? TR : TL` as a reference argument would select
    // between two addresses and keep all four values in scratch (388 B/lane)
    Fq2 To, Uo;
    gt::fq2_sel(To, ul.side != 0, TR, TL);
    gt::fq2_sel(Uo, ul.side != 0, UR, WL);
    split_list(split, unresolved, (t << 3) | (2u * j + ul.side), To, Uo, ab_child, ul.ps);
  }
  if (ul.ps.k != 0 || ul.ps.sub != 0) return;
  if (located) status[lo + loc] = HBTC_REJECT;
  if (LVL == 3 && unresolved) {
    uint32_t m = 0;
    for (uint32_t i = lo; i < hi; ++i) m += status[i] == HBTC_RLC_PENDING;
    uint32_t pos = atomicAdd(leaf_count, m);
    for (uint32_t i = lo; i < hi; ++i)
      if (status[i] == HBTC_RLC_PENDING) {
        leaves[2 * pos] = i;
        leaves[2 * pos + 1] = inst;
        ++pos;
      }
  }
}

#endif  // part 2

// ------------------------------------------------------------------------------ level 3: leaves
// (a template in both parts: <1> is instantiated by part 1's launcher, <3> by part 2's)
// e(d_i, H_k) e(-pk_i, w_k) == 1 for two listed shares per unit.
template <uint32_t REP>
__global__ void __launch_bounds__(64, REP == 1 ? HBTC_GT_WAVES : HBTC_GT_WAVES_SMALL) k_chk_leaves(
    const uint32_t* __restrict__ leaf_count, const uint32_t* __restrict__ leaves,
    const uint32_t* __restrict__ idx, const G1A* __restrict__ dec, const G1A* __restrict__ pk,
    const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    const G2A* __restrict__ w_aff, const Line* __restrict__ w_lines,
    int32_t* __restrict__ status, uint32_t rep3_limit) {
  HBTC_LATENCY_PRIO();
  constexpr uint32_t UPW = Units<REP>::PER_WAVE;
  const uint32_t n = *leaf_count;
  // a list of at most rep3_limit leaves is the latency form's (REP 3), a longer one the
  // throughput form's: both are launched, one of them exits at once
  if ((REP == 3) == (n > rep3_limit)) return;
  if (blockIdx.x * 2 * UPW >= n) return;
  const UnitLane ul = unit_lane(REP);
  const uint32_t li = (blockIdx.x * UPW + ul.unit) * 2u + ul.side;
  const bool active = ul.unit < UPW && li < n;
  uint32_t item = 0, k = 0;
  G1J S, P;
  jac_set_inf(S);
  jac_set_inf(P);
  if (active) {
    item = leaves[2 * li];
    k = leaves[2 * li + 1];
    S = g1j_of(dec[item]);
    P = g1j_of(pk[idx[item]]);
  }
  const bool use1 = active && !jac_is_inf(S) && !h_aff[k].inf;
  const bool use2 = active && !jac_is_inf(P) && !w_aff[k].inf;
  Fq2 e;
  pair_value(e, S, use1, h_lines + (size_t)k * MILLER_STEPS, P, use2,
             w_lines + (size_t)k * MILLER_STEPS, ul.ps);
  const bool ok = gt::is_one(e, ul.ps);
  if (active && ul.ps.k == 0 && ul.ps.sub == 0) status[item] = ok ? HBTC_ACCEPT : HBTC_REJECT;
}

// ------------------------------------------------------------------------------ SignatureShares
// (templates on the layout: rep 1 instantiated by part 1, the latency form rep 3 by part 2)
// e(sum r_i pk_i, H) e(-G1, sum r_i sigma_i) == 1: the first pair over H's precomputed lines,
// the second over the group's projective line table (hbtc_sig.hip k_plines) at the fixed -G1.
namespace {
__device__ __forceinline__ void sig_pair_value(Fq2& e, const G1J& P, bool use1, const Line* hl,
                                               const Fq2* table, bool use2, const Pos& ps) {
  G1J ng;
  fq_set(ng.x, G1_GEN_X);
  fq_set(ng.y, G1_GEN_Y);
  fq_neg(ng.y, ng.y);
  fq_one(ng.z);
  gt::MillerArg m1{hl, nullptr, P, use1};
  gt::MillerArg m2{nullptr, table, ng, use2};
  Fq2 f;
  gt::miller2_t<true>(f, m1, m2, ps);
  gt::final_exp(e, f, ps);
}
}  // namespace

template <uint32_t REP>
__global__ void __launch_bounds__(64, REP == 1 ? HBTC_GT_WAVES : HBTC_GT_WAVES_SMALL) k_sigchk_tiles(
    uint32_t n_tiles, const Tile* __restrict__ tiles, const SigTileSums* __restrict__ sums,
    const Fq2* __restrict__ tables, const uint32_t* __restrict__ inf,
    const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    const int32_t* __restrict__ h_status, int32_t* __restrict__ status,
    uint32_t* __restrict__ sub_count, uint32_t* __restrict__ sub_list, bool to_leaves) {
  HBTC_LATENCY_PRIO();
  constexpr uint32_t UPW = Units<REP>::PER_WAVE;
  const UnitLane ul = unit_lane(REP);
  const uint32_t t = blockIdx.x * UPW + ul.unit;
  const bool active = ul.unit < UPW && t < n_tiles;
  uint32_t k = 0, first = 0, count = 0, g = 0;
  bool inst_ok = false, inf2 = true;
  G1J P;
  jac_set_inf(P);
  if (active) {
    const Tile tile = tiles[t];
    k = tile.inst;
    first = tile.first;
    count = tile.count;
    inst_ok = h_status[k] == HBTC_ACCEPT;
    P = ul.side ? sums[t].PW[8] : sums[t].P[8];
    g = 2 * t + ul.side;
    inf2 = inf[g] != 0;
  }
  const bool use1 = inst_ok && !jac_is_inf(P) && !h_aff[k].inf;
  const bool use2 = inst_ok && !inf2;
  Fq2 e, T, Tw;
  sig_pair_value(e, P, use1, h_lines + (size_t)k * MILLER_STEPS, tables + (size_t)g * PLINES_FQ2,
                 use2, ul.ps);
  const bool pass = unit_values(T, Tw, e, ul);
  const bool fail = active && inst_ok && !pass;
  const int32_t loc = locate(T, Tw, count, 5, fail, ul);
  if (!fail || ul.side != 0 || ul.ps.k != 0 || ul.ps.sub != 0) return;
  if (loc >= 0 && status[first + loc] == HBTC_RLC_PENDING) {
    status[first + loc] = HBTC_REJECT;
    return;
  }
  if (!to_leaves) {
    sub_list[atomicAdd(sub_count, 1u)] = t;
    return;
  }
  // the paired tiles -> leaves schedule: every pending share of the tile to the exact checks
  // (sub_count / sub_list are then the leaf counter and list)
  uint32_t m = 0;
  for (uint32_t i = first; i < first + count; ++i) m += status[i] == HBTC_RLC_PENDING;
  uint32_t pos = atomicAdd(sub_count, m);
  for (uint32_t i = first; i < first + count; ++i)
    if (status[i] == HBTC_RLC_PENDING) {
      sub_list[2 * pos] = i;
      sub_list[2 * pos + 1] = k;
      ++pos;
    }
}

#if HBTC_CHECK_IN(1)
__global__ void __launch_bounds__(64, HBTC_GT_WAVES) k_sigchk_subs(
    const uint32_t* __restrict__ sub_count, const uint32_t* __restrict__ sub_list,
    const Tile* __restrict__ tiles, const SigTileSums* __restrict__ sums,
    const Fq2* __restrict__ tables, const uint32_t* __restrict__ inf,
    const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    int32_t* __restrict__ status, uint32_t* __restrict__ leaf_count,
    uint32_t* __restrict__ leaves) {
  HBTC_LATENCY_PRIO();
  const uint32_t n_units = *sub_count * 8u;
  if (blockIdx.x * UNITS_PER_WAVE >= n_units) return;
  const UnitLane ul = unit_lane();
  const uint32_t u = blockIdx.x * UNITS_PER_WAVE + ul.unit;
  bool active = ul.unit < UNITS_PER_WAVE && u < n_units;
  uint32_t k = 0, lo = 0, hi = 0, g = 0;
  bool inf2 = true;
  G1J P;
  jac_set_inf(P);
  if (active) {
    const uint32_t t = sub_list[u >> 3], sub = u & 7u;
    const Tile tile = tiles[t];
    k = tile.inst;
    lo = tile.first + sub * 8u;
    hi = min(tile.first + tile.count, lo + 8u);
    active = lo < hi;
    if (active) {
      P = ul.side ? sums[t].PW[sub] : sums[t].P[sub];
      g = 16u * (u >> 3) + 2u * sub + ul.side;  // k_plines mode 1 numbering
      inf2 = inf[g] != 0;
    }
  }
  const bool use1 = active && !jac_is_inf(P) && !h_aff[k].inf;
  const bool use2 = active && !inf2;
  Fq2 e, T, Tw;
  sig_pair_value(e, P, use1, h_lines + (size_t)k * MILLER_STEPS, tables + (size_t)g * PLINES_FQ2,
                 use2, ul.ps);
  const bool pass = unit_values(T, Tw, e, ul);
  const bool fail = active && !pass;
  const int32_t loc = locate(T, Tw, hi - lo, 2, fail, ul);
  if (!fail || ul.side != 0 || ul.ps.k != 0) return;
  if (loc >= 0 && status[lo + loc] == HBTC_RLC_PENDING) {
    status[lo + loc] = HBTC_REJECT;
    return;
  }
  for (uint32_t i = lo; i < hi; ++i)
    if (status[i] == HBTC_RLC_PENDING) {
      const uint32_t pos = atomicAdd(leaf_count, 1u);
      leaves[2 * pos] = i;
      leaves[2 * pos + 1] = k;
    }
}

#endif  // part 1

// rep3_limit: a list of at most rep3_limit leaves is the latency form's (REP 3, first chunk
// only), a longer one the throughput form's; both are launched, one exits at once
template <uint32_t REP>
__global__ void __launch_bounds__(64, REP == 1 ? HBTC_GT_WAVES : HBTC_GT_WAVES_SMALL) k_sigchk_leaves(
    uint32_t base, uint32_t chunk, const uint32_t* __restrict__ leaf_count,
    const uint32_t* __restrict__ leaves,
    const uint32_t* __restrict__ idx, const G1A* __restrict__ pk,
    const Fq2* __restrict__ tables, const uint32_t* __restrict__ inf,
    const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    int32_t* __restrict__ status, uint32_t rep3_limit) {
  HBTC_LATENCY_PRIO();
  constexpr uint32_t UPW = Units<REP>::PER_WAVE;
  // leaves [base, base + chunk) of the list; tables are numbered from the chunk start
  const uint32_t c = *leaf_count;
  if ((REP == 3) == (c > rep3_limit)) return;
  const uint32_t n = c > base ? min(c - base, chunk) : 0u;
  if (blockIdx.x * 2 * UPW >= n) return;
  const UnitLane ul = unit_lane(REP);
  const uint32_t g = (blockIdx.x * UPW + ul.unit) * 2u + ul.side;
  const bool active = ul.unit < UPW && g < n;
  uint32_t item = 0, k = 0;
  bool inf2 = true;
  G1J P;
  jac_set_inf(P);
  if (active) {
    item = leaves[2 * (base + g)];
    k = leaves[2 * (base + g) + 1];
    P = g1j_of(pk[idx[item]]);
    inf2 = inf[g] != 0;
  }
  const bool use1 = active && !jac_is_inf(P) && !h_aff[k].inf;
  const bool use2 = active && !inf2;
  Fq2 e;
  sig_pair_value(e, P, use1, h_lines + (size_t)k * MILLER_STEPS,
                 tables + (size_t)(active ? g : 0) * PLINES_FQ2, use2, ul.ps);
  const bool ok = gt::is_one(e, ul.ps);
  // a share the fused exact pass (k_sig_exact) listed before its psi test failed keeps DECODE_ERR
  if (active && ul.ps.k == 0 && ul.ps.sub == 0 && status[item] != HBTC_DECODE_ERR)
    status[item] = ok ? HBTC_ACCEPT : HBTC_REJECT;
}

// ------------------------------------------------------------------------------ launchers
static inline uint32_t unit_blocks(uint64_t units) {
  return (uint32_t)((units + UNITS_PER_WAVE - 1) / UNITS_PER_WAVE);
}

#if HBTC_CHECK_IN(1)
hipError_t launch_chk_plain(hipStream_t s, int level, uint32_t max_groups, uint32_t n_direct,
                            const uint32_t* n_listed, const uint32_t* sub_list,
                            const uint32_t* list2, const Tile* tiles,
                            const TileSums* sums, const G2A* h_aff, const Line* h_lines,
                            const G2A* w_aff, const Line* w_lines, const int32_t* h_status,
                            const int32_t* w_status, Fq2* Tbuf, uint32_t* fail_count,
                            uint32_t* fail_list) {
  if (max_groups == 0) return hipSuccess;
  const dim3 grid(unit_blocks(((uint64_t)max_groups + 1) / 2));
#define HBTC_PLAIN_ARGS                                                                         \
  grid, dim3(64), 0, s, n_direct, n_listed, sub_list, list2, tiles, sums, h_aff, h_lines, w_aff, \
      w_lines, h_status, w_status, Tbuf, fail_count, fail_list
  if (level == 0)
    hipLaunchKernelGGL(k_chk_plain<0>, HBTC_PLAIN_ARGS);
  else if (level == 1)
    hipLaunchKernelGGL(k_chk_plain<1>, HBTC_PLAIN_ARGS);
  else
    hipLaunchKernelGGL(k_chk_plain<3>, HBTC_PLAIN_ARGS);
#undef HBTC_PLAIN_ARGS
  return hipGetLastError();
}

hipError_t launch_chk_halves(hipStream_t s, uint32_t max_tiles, const uint32_t* n_listed,
                             const uint32_t* tile_list, const Tile* tiles, const TileSums* sums,
                             const G2A* h_aff, const Line* h_lines, const G2A* w_aff,
                             const Line* w_lines, const Fq2* Ttile, Fq2* Thalf,
                             uint32_t* fail_count, uint32_t* fail_list) {
  if (max_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_chk_halves, dim3(unit_blocks(((uint64_t)max_tiles + 1) / 2)), dim3(64), 0, s,
                     n_listed, tile_list, tiles, sums, h_aff, h_lines, w_aff, w_lines, Ttile, Thalf,
                     fail_count, fail_list);
  return hipGetLastError();
}

#endif

#if HBTC_CHECK_IN(2)
hipError_t launch_chk_weighted(hipStream_t s, int level, uint32_t max_groups,
                               const uint32_t* fail_count, const uint32_t* fail_list,
                               const uint32_t* sub_list, const uint32_t* list2, const Tile* tiles,
                               const TileSums* sums,
                               const G2A* h_aff, const Line* h_lines, const G2A* w_aff,
                               const Line* w_lines, const int32_t* h_status,
                               const int32_t* w_status, const Fq2* Tbuf, int32_t* status,
                               uint32_t* out_count, uint32_t* out_list, SplitOut split) {
  if (max_groups == 0) return hipSuccess;
  const dim3 grid(unit_blocks(((uint64_t)max_groups + 1) / 2));
#define HBTC_WEIGHTED_ARGS                                                                     \
  grid, dim3(64), 0, s, fail_count, fail_list, sub_list, list2, tiles, sums, h_aff, h_lines, w_aff, \
      w_lines, h_status, w_status, Tbuf, status, out_count, out_list, split
  if (level == 0)
    hipLaunchKernelGGL(k_chk_weighted<0>, HBTC_WEIGHTED_ARGS);
  else if (level == 1)
    hipLaunchKernelGGL(k_chk_weighted<1>, HBTC_WEIGHTED_ARGS);
  else if (level == 2)
    hipLaunchKernelGGL(k_chk_weighted<2>, HBTC_WEIGHTED_ARGS);
  else
    hipLaunchKernelGGL(k_chk_weighted<3>, HBTC_WEIGHTED_ARGS);
#undef HBTC_WEIGHTED_ARGS
  return hipGetLastError();
}

hipError_t launch_chk_pair(hipStream_t s, int level, bool to_leaves, uint32_t max_groups,
                           uint32_t n_direct, const uint32_t* n_listed, const uint32_t* sub_list,
                           const Tile* tiles, const TileSums* sums, const G2A* h_aff,
                           const Line* h_lines, const G2A* w_aff, const Line* w_lines,
                           const int32_t* h_status, const int32_t* w_status, int32_t* status,
                           uint32_t* out_count, uint32_t* out_list, SplitOut split) {
  if (max_groups == 0) return hipSuccess;
  const dim3 grid(unit_blocks(max_groups));
#define HBTC_PAIR_ARGS                                                                       \
  grid, dim3(64), 0, s, n_direct, n_listed, sub_list, tiles, sums, h_aff, h_lines, w_aff, w_lines, \
      h_status, w_status, status, out_count, out_list, split
  if (level == 0 && to_leaves)
    hipLaunchKernelGGL((k_chk_pair<0, true>), HBTC_PAIR_ARGS);
  else if (level == 0)
    hipLaunchKernelGGL((k_chk_pair<0, false>), HBTC_PAIR_ARGS);
  else
    hipLaunchKernelGGL((k_chk_pair<1, true>), HBTC_PAIR_ARGS);
#undef HBTC_PAIR_ARGS
  return hipGetLastError();
}

hipError_t launch_chk_split(hipStream_t s, int level, int rep, uint32_t max_nodes,
                            const uint32_t* n_in, const uint32_t* in_list, const Fq2* in_T,
                            const Fq2* in_U, const uint32_t* in_ab, const Tile* tiles,
                            const TileSums* sums, const G2A* h_aff, const Line* h_lines,
                            const G2A* w_aff, const Line* w_lines, int32_t* status,
                            uint32_t* leaf_count, uint32_t* leaves, SplitOut split) {
  if (max_nodes == 0) return hipSuccess;
  // the split levels run on the plain-first schedule only, which keeps the throughput layout
  // (rep 1): the latency-form instantiations were never launched and are gone (round 5)
  if (rep != 1) return hipErrorInvalidValue;
  const dim3 grid(unit_blocks(max_nodes));
#define HBTC_SPLIT_ARGS                                                                       \
  grid, dim3(64), 0, s, n_in, in_list, in_T, in_U, in_ab, tiles, sums, h_aff, h_lines, w_aff, \
      w_lines, status, leaf_count, leaves, split
  if (level == 1)
    hipLaunchKernelGGL((k_chk_split<1, 1>), HBTC_SPLIT_ARGS);
  else if (level == 2)
    hipLaunchKernelGGL((k_chk_split<2, 1>), HBTC_SPLIT_ARGS);
  else
    hipLaunchKernelGGL((k_chk_split<3, 1>), HBTC_SPLIT_ARGS);
#undef HBTC_SPLIT_ARGS
  return hipGetLastError();
}

// the latency-form leaf checks (one check per 18-lane group, two per wave), compiled with the
// one-wave kernels of this part
hipError_t launch_chk_leaves_rep3(hipStream_t s, uint32_t max_leaves, uint32_t rep3_limit,
                                  const uint32_t* leaf_count, const uint32_t* leaves,
                                  const uint32_t* idx, const G1A* dec, const G1A* pk,
                                  const G2A* h_aff, const Line* h_lines, const G2A* w_aff,
                                  const Line* w_lines, int32_t* status) {
  if (max_leaves == 0 || rep3_limit == 0) return hipSuccess;
  const uint32_t m = std::min(max_leaves, rep3_limit);
  hipLaunchKernelGGL(k_chk_leaves<3>, dim3((m + 1) / 2), dim3(64), 0, s, leaf_count, leaves, idx, dec,
                     pk, h_aff, h_lines, w_aff, w_lines, status, rep3_limit);
  return hipGetLastError();
}

// SignatureShare tiles and leaves in the latency form (one unit per wave)
hipError_t launch_sigchk_tiles_rep3(hipStream_t s, uint32_t n_tiles, const Tile* tiles,
                                    const SigTileSums* sums, const Fq2* tables, const uint32_t* inf,
                                    const G2A* h_aff, const Line* h_lines, const int32_t* h_status,
                                    int32_t* status, uint32_t* sub_count, uint32_t* sub_list,
                                    bool to_leaves) {
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sigchk_tiles<3>, dim3(n_tiles), dim3(64), 0, s, n_tiles, tiles, sums, tables, inf,
                     h_aff, h_lines, h_status, status, sub_count, sub_list, to_leaves);
  return hipGetLastError();
}
hipError_t launch_sigchk_leaves_rep3(hipStream_t s, uint32_t chunk, uint32_t rep3_limit,
                                     const uint32_t* leaf_count, const uint32_t* leaves,
                                     const uint32_t* idx, const G1A* pk, const Fq2* tables,
                                     const uint32_t* inf, const G2A* h_aff, const Line* h_lines,
                                     int32_t* status) {
  if (chunk == 0 || rep3_limit == 0) return hipSuccess;
  const uint32_t m = std::min(chunk, rep3_limit);
  hipLaunchKernelGGL(k_sigchk_leaves<3>, dim3((m + 1) / 2), dim3(64), 0, s, 0u, chunk, leaf_count, leaves,
                     idx, pk, tables, inf, h_aff, h_lines, status, rep3_limit);
  return hipGetLastError();
}

#endif

#if HBTC_CHECK_IN(1)
hipError_t launch_chk_leaves(hipStream_t s, uint32_t max_leaves, const uint32_t* leaf_count,
                             const uint32_t* leaves, const uint32_t* idx, const G1A* dec,
                             const G1A* pk, const G2A* h_aff, const Line* h_lines,
                             const G2A* w_aff, const Line* w_lines, int32_t* status,
                             uint32_t rep3_limit) {
  if (max_leaves == 0) return hipSuccess;
  hipLaunchKernelGGL(k_chk_leaves<1>, dim3(unit_blocks(((uint64_t)max_leaves + 1) / 2)), dim3(64), 0,
                     s, leaf_count, leaves, idx, dec, pk, h_aff, h_lines, w_aff, w_lines, status,
                     rep3_limit);
  return hipGetLastError();
}

hipError_t launch_sigchk_tiles(hipStream_t s, uint32_t n_tiles, const Tile* tiles,
                               const SigTileSums* sums, const Fq2* tables, const uint32_t* inf,
                               const G2A* h_aff, const Line* h_lines, const int32_t* h_status,
                               int32_t* status, uint32_t* sub_count, uint32_t* sub_list,
                               bool to_leaves) {
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sigchk_tiles<1>, dim3(unit_blocks(n_tiles)), dim3(64), 0, s, n_tiles, tiles, sums,
                     tables, inf, h_aff, h_lines, h_status, status, sub_count, sub_list, to_leaves);
  return hipGetLastError();
}

hipError_t launch_sigchk_subs(hipStream_t s, uint32_t max_tiles, const uint32_t* sub_count,
                              const uint32_t* sub_list, const Tile* tiles,
                              const SigTileSums* sums, const Fq2* tables, const uint32_t* inf,
                              const G2A* h_aff, const Line* h_lines, int32_t* status,
                              uint32_t* leaf_count, uint32_t* leaves) {
  if (max_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sigchk_subs, dim3(unit_blocks((uint64_t)max_tiles * 8)), dim3(64), 0, s,
                     sub_count, sub_list, tiles, sums, tables, inf, h_aff, h_lines, status,
                     leaf_count, leaves);
  return hipGetLastError();
}

hipError_t launch_sigchk_leaves(hipStream_t s, uint32_t base, uint32_t chunk,
                                const uint32_t* leaf_count, const uint32_t* leaves,
                                const uint32_t* idx, const G1A* pk, const Fq2* tables,
                                const uint32_t* inf, const G2A* h_aff, const Line* h_lines,
                                int32_t* status, uint32_t rep3_limit) {
  if (chunk == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sigchk_leaves<1>, dim3(unit_blocks(((uint64_t)chunk + 1) / 2)), dim3(64), 0, s,
                     base, chunk, leaf_count, leaves, idx, pk, tables, inf, h_aff, h_lines, status,
                     rep3_limit);
  return hipGetLastError();
}

#endif

#if HBTC_CHECK_IN(1)
// ------------------------------------------------------------------------------ pair batches
// e(A_i, Q_i) == e(G1, W_i) batches (hbtc_pb.hip).  A group's value is
//     FE( conj( prod_i f_{|x|,Q_i}(r_i A_i) * f_{|x|,W}(-G1) ) ),  W = the group's sum of r_i W_i:
// every pair is an affine G1 point with a projective line table.  The Miller loops are cut by
// 8-item sub-tile so a batch yields enough independent chains to fill the chip: k_pb_ml runs one
// 6-lane group per sub-tile (its items' pairs share the 63 squarings) and stores the partial
// product; k_pb_fe runs one group per checked group: the product of its partials (a tile: 8),
// the Miller loop of its W sum at -G1, the final exponentiation.  Level 0: the 64-item tiles;
// level 1: the 8 sub-tiles of failing tiles (their partials are reused).  A passing group
// ACCEPTs its pending items; a failing tile is listed for level 1, a failing sub-tile's pending
// items for the exact per-item checks.
constexpr uint32_t PB_GROUPS_PER_WAVE = 10;

namespace {
// f *= prod_{p < bound} line_p: the pair loader sets, per lane, the line's A (Fq2, every lane),
// `prod` (lanes 0, 1: C.c{k} y; lanes 2, 3: B.c{k-2} x; zero elsewhere) and whether pair p is
// used; `bound` is wave-uniform (groups with fewer pairs mark the rest unused).  The 63
// squarings are shared by all pairs.  Unconjugated (x < 0: the caller conjugates the product).
template <class Loader>
__device__ __forceinline__ void pb_miller(Fq2& f, uint32_t bound, const Loader& load, const Pos& ps) {
  gt::set_one(f, ps);
  int j = 0;
  bool first = true;
#pragma unroll 1
  for (int bit = 62; bit >= 0; --bit) {
    const bool add = ((BLS_X_ABS >> bit) & 1ull) != 0;
#pragma unroll 1
    for (int rep = 0; rep < (add ? 2 : 1); ++rep) {
      if (rep == 0 && !first) gt::sqr(f, f, ps);
      first = false;
#pragma unroll 1
      for (uint32_t p = 0; p < bound; ++p) {
        Fq2 A;
        Fq prod;
        bool u;
        load(p, j, A, prod, u);
        gt::mul_line_t<true, true>(f, prod, 0, A, prod, 2, prod, 0, u, ps);
      }
      ++j;
    }
  }
}

// The per-lane line values of one pair at step j: table L (3 Fq2 per step), affine point (x, y).
__device__ __forceinline__ void pb_line_values(const Fq2* L, const Fq& x, const Fq& y, bool u,
                                               uint32_t k, Fq2& A, Fq& prod) {
  fq2_zero(A);
  fq_zero(prod);
  if (u) {
    A = L[0];
    const Fq2& BC = k < 2 ? L[2] : L[1];
    const Fq& m = (k & 1u) ? BC.c1 : BC.c0;
    Fq s;  // element-wise: a reference select would keep x and y in scratch
    fq_sel(s, k < 2, y, x);
    fq_mul(prod, m, s);
    if (k >= 4) fq_zero(prod);
  }
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}
}  // namespace

// Partial Miller products of the 8-item sub-tiles: group g = items [8g, 8g + 8) of the chunk.
__global__ void __launch_bounds__(64, HBTC_GT_WAVES) k_pb_ml(uint32_t n_items, const G1A* __restrict__ rA,
                                                           const Fq2* __restrict__ qtab,
                                                           const int32_t* __restrict__ status,
                                                           Fq2* __restrict__ fbuf) {
  HBTC_LATENCY_PRIO();
  const uint32_t n_groups = (n_items + 7u) / 8u;
  if (blockIdx.x * PB_GROUPS_PER_WAVE >= n_groups) return;  // wave-uniform
  const Pos ps = gt::pos();
  const uint32_t slot = gt::lane_id() / 6u;
  const uint32_t g = blockIdx.x * PB_GROUPS_PER_WAVE + slot;
  const bool active = slot < PB_GROUPS_PER_WAVE && g < n_groups;
  const uint32_t lo = active ? 8u * g : 0u;
  const uint32_t cnt = active ? min(8u, n_items - lo) : 0u;
  uint32_t use = 0;  // pending items whose r A is finite (A = O or Q = O: the pair is 1)
  for (uint32_t q = 0; q < cnt; ++q)
    if (status[lo + q] == HBTC_RLC_PENDING && !rA[lo + q].inf) use |= 1u << q;
  const uint32_t k = ps.k;
  Fq2 f;
  pb_miller(f, wave_max(cnt), [&](uint32_t p, int j, Fq2& A, Fq& prod, bool& u) {
    u = ((use >> p) & 1u) != 0;
    const uint32_t i = lo + (u ? p : 0u);
    pb_line_values(qtab + ((size_t)i * MILLER_STEPS + j) * 3, rA[i].x, rA[i].y, u, k, A, prod);
  }, ps);
  if (active) fbuf[(size_t)g * 6 + k] = f;
}

// Group checks from the partials: level 0 group g = tile g (partials 8g .. 8g + 7); level 1
// group g = sub-tile g & 7 of tile list[g >> 3] (one partial).
template <int LEVEL>
__global__ void __launch_bounds__(64, HBTC_GT_WAVES) k_pb_fe(
    uint32_t n_items, uint32_t n_direct, const uint32_t* __restrict__ n_listed,
    const uint32_t* __restrict__ list, const Fq2* __restrict__ fbuf, const Fq2* __restrict__ wtab,
    const uint32_t* __restrict__ winf, int32_t* __restrict__ status, uint32_t* __restrict__ out_count,
    uint32_t* __restrict__ out_list) {
  HBTC_LATENCY_PRIO();
  const uint32_t n_groups = LEVEL == 0 ? n_direct : *n_listed * 8u;
  if (blockIdx.x * PB_GROUPS_PER_WAVE >= n_groups) return;  // wave-uniform
  const Pos ps = gt::pos();
  const uint32_t slot = gt::lane_id() / 6u;
  const uint32_t g = blockIdx.x * PB_GROUPS_PER_WAVE + slot;
  const bool active = slot < PB_GROUPS_PER_WAVE && g < n_groups;
  const uint32_t k = ps.k;
  uint32_t t = 0, s0 = 0, ns = 0;  // partials [s0, s0 + ns)
  if (active) {
    t = LEVEL == 0 ? g : list[g >> 3];
    s0 = LEVEL == 0 ? 8u * t : 8u * t + (g & 7u);
    const uint32_t n_subs = (n_items + 7u) / 8u;
    ns = s0 < n_subs ? min(LEVEL == 0 ? 8u : 1u, n_subs - s0) : 0u;
  }
  const bool w_use = active && winf[g] == 0;
  Fq gx, ngy;  // -G1
  fq_set(gx, G1_GEN_X);
  fq_set(ngy, G1_GEN_Y);
  fq_neg(ngy, ngy);
  const Fq2* wt = wtab + (size_t)g * PLINES_FQ2;
  Fq2 f;
  pb_miller(f, 1u, [&](uint32_t, int j, Fq2& A, Fq& prod, bool& u) {
    u = w_use;
    pb_line_values(wt + 3 * j, gx, ngy, u, k, A, prod);
  }, ps);
#pragma unroll 1
  for (uint32_t s = 0; s < wave_max(ns); ++s) {
    Fq2 x;
    gt::set_one(x, ps);
    if (s < ns) x = fbuf[(size_t)(s0 + s) * 6 + k];
    gt::mul(f, f, x, ps);
  }
  gt::conj(f, ps);
  Fq2 e;
  gt::final_exp(e, f, ps);
  const bool ok = gt::is_one(e, ps);
  if (!active) return;
  const uint32_t lo = 8u * s0, hi = min(n_items, 8u * (s0 + ns));
  if (ok) {
    for (uint32_t q = lo + k; q < hi; q += 6u)
      if (status[q] == HBTC_RLC_PENDING) status[q] = HBTC_ACCEPT;
  } else if (LEVEL == 0) {
    if (k == 0) out_list[atomicAdd(out_count, 1u)] = t;
  } else if (k == 0) {
    for (uint32_t q = lo; q < hi; ++q)
      if (status[q] == HBTC_RLC_PENDING) out_list[atomicAdd(out_count, 1u)] = q;
  }
}

hipError_t launch_pb_ml(hipStream_t s, uint32_t n_items, const G1A* rA, const Fq2* qtab,
                        const int32_t* status, Fq2* fbuf) {
  if (n_items == 0) return hipSuccess;
  const uint32_t groups = (n_items + 7u) / 8u;
  hipLaunchKernelGGL(k_pb_ml, dim3((groups + PB_GROUPS_PER_WAVE - 1) / PB_GROUPS_PER_WAVE), dim3(64), 0, s,
                     n_items, rA, qtab, status, fbuf);
  return hipGetLastError();
}

hipError_t launch_pb_fe(hipStream_t s, int level, uint32_t max_groups, uint32_t n_items,
                        uint32_t n_direct, const uint32_t* n_listed, const uint32_t* list,
                        const Fq2* fbuf, const Fq2* wtab, const uint32_t* winf, int32_t* status,
                        uint32_t* out_count, uint32_t* out_list) {
  if (max_groups == 0) return hipSuccess;
  const dim3 grid((max_groups + PB_GROUPS_PER_WAVE - 1) / PB_GROUPS_PER_WAVE);
  if (level == 0)
    hipLaunchKernelGGL(k_pb_fe<0>, grid, dim3(64), 0, s, n_items, n_direct, n_listed, list, fbuf, wtab,
                       winf, status, out_count, out_list);
  else
    hipLaunchKernelGGL(k_pb_fe<1>, grid, dim3(64), 0, s, n_items, n_direct, n_listed, list, fbuf, wtab,
                       winf, status, out_count, out_list);
  return hipGetLastError();
}
#endif

}  // namespace hbtc
