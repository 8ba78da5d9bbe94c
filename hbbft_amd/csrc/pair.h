// G2 arithmetic on LANE PAIRS (round 6).  Every Fq2 of one item is held by two lanes of a wave:
// lane 2j + e holds component c_e (an Fq, 12 words), so a G2 Jacobian point is 36 registers per
// lane instead of 72 and a G2 kernel's state fits a register budget that allows two or more waves
// per SIMD (a lone wave issues v_mad_u64_u32 at half rate: 8.2 against 4.2 cycles per
// instruction, profiles/r06/intmul_peak.txt).  The templates of curve.h (Jacobian doubling, mixed
// addition, the x-adic double-and-add, ...) run unchanged on the type Fq2p below; only the field
// operations know about the pair.
//
// Products (the partner's operand comes over one DPP exchange per word, quad_perm [1,0,3,2]):
//   a b:  lane 0: a0 b0 + (-a1) b1,  lane 1: a0 b1 + a1 b0  -- ONE Montgomery reduction of a sum
//         of two products per lane (fq_mul2: both products and the reduction in one product
//         scanning, 432 MACs), against Karatsuba's three full products (864 MACs) on one lane:
//         the same multiplications in total, half the latency;
//   a^2:  lane 0: (a0 + a1)(a0 - a1),  lane 1: a0 (2 a1)  -- one product per lane (two on one lane).
// Control flow: every data-dependent condition is made pair-uniform (fis_zero / feq AND the two
// lanes' answers), so the two lanes of a pair always execute the same instructions and the DPP
// partner is always active.  Callers keep items pair-aligned (item = lane / 2).
#pragma once
#include "pairing.h"

namespace hbtc {

struct Fq2p {
  Fq v;  // component (lane & 1) of the Fq2
};
typedef Aff<Fq2p> G2Ap;
typedef Jac<Fq2p> G2Jp;

// lane parity and the partner lane's value (lanes 2j <-> 2j + 1, DPP quad_perm [1,0,3,2]); host
// builds (tests/native) never run pair code, the host bodies only keep the templates compilable
HD bool pair_odd() {
#if defined(__HIP_DEVICE_COMPILE__)
  return (__lane_id() & 1u) != 0;
#else
  return false;
#endif
}
HD uint32_t pair_xchg(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
#else
  return x;
#endif
}

HD void fq_xchg(Fq& r, const Fq& a) {
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = pair_xchg(a.v[i]);
}
// both lanes' b.  The exchange runs on both lanes unconditionally: a short-circuit `b && xchg(b)`
// would leave the lane with b = false out of the DPP, and its partner would read a disabled lane
// (this broke every pair test of a point with one zero component, e.g. Z = (1, 0) after
// jac_from_aff).
HD bool pair_all(bool b) {
  const uint32_t mine = b ? 1u : 0u;
  const uint32_t other = pair_xchg(mine);
  return (mine & other) != 0u;
}

// MONT(a b + c d) for operands < 2p: < 8p^2 before the reduction, < 2p after (one product
// scanning of both products: fq_fips_sr.h hbtc_fqmul2_sr, 432 MACs)
HD void fq_mul2(Fq& r, const Fq& a, const Fq& b, const Fq& c, const Fq& d) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(HBTC_FQMUL_SR)
  fips::mont_mul2_sr(r.v, a.v, b.v, c.v, d.v);
#else
  Fq t, u;
  fq_mul(t, a, b);
  fq_mul(u, c, d);
  fq_add(r, t, u);
#endif
}

HD void fadd(Fq2p& r, const Fq2p& a, const Fq2p& b) { fq_add(r.v, a.v, b.v); }
HD void fsub(Fq2p& r, const Fq2p& a, const Fq2p& b) { fq_sub(r.v, a.v, b.v); }
HD void fdbl(Fq2p& r, const Fq2p& a) { fq_dbl(r.v, a.v); }
HD void fneg(Fq2p& r, const Fq2p& a) { fq_neg(r.v, a.v); }
HD void fzero(Fq2p& r) { fq_zero(r.v); }
HD void fone(Fq2p& r) {
  Fq o, z;
  fq_one(o);
  fq_zero(z);
  fq_sel(r.v, pair_odd(), z, o);
}
HD bool fis_zero(const Fq2p& a) { return pair_all(fq_is_zero(a.v)); }
HD bool feq(const Fq2p& a, const Fq2p& b) { return pair_all(fq_eq(a.v, b.v)); }
template <>
HD void fsel<Fq2p>(Fq2p& r, bool c, const Fq2p& a, const Fq2p& b) { fq_sel(r.v, c, a.v, b.v); }

HD void fmul(Fq2p& r, const Fq2p& a, const Fq2p& b) {
  Fq pa, pb, npa, u1, u2;
  fq_xchg(pa, a.v);
  fq_xchg(pb, b.v);
  fq_neg(npa, pa);
  const bool odd = pair_odd();
  fq_sel(u1, odd, pa, a.v);   // a0
  fq_sel(u2, odd, a.v, npa);  // lane 0: -a1, lane 1: a1
  fq_mul2(r.v, u1, b.v, u2, pb);
}
HD void fsqr(Fq2p& r, const Fq2p& a) {
  Fq pa, s, d, t, u, w;
  fq_xchg(pa, a.v);
  fq_add(s, a.v, pa);
  fq_sub(d, a.v, pa);
  fq_dbl(t, a.v);
  const bool odd = pair_odd();
  fq_sel(u, odd, pa, s);  // lane 0: a0 + a1, lane 1: a0
  fq_sel(w, odd, t, d);   // lane 0: a0 - a1, lane 1: 2 a1
  fq_mul(r.v, u, w);
}
HD void fmul_by_fq(Fq2p& r, const Fq2p& a, const Fq& c) { fq_mul(r.v, a.v, c); }
// 1/a = conj(a) / (a0^2 + a1^2): the norm by one square per lane, one binary-GCD inversion
HD void finv_fast(Fq2p& r, const Fq2p& a) {
  Fq s, ps, n, ni, t, nt;
  fq_sqr(s, a.v);
  fq_xchg(ps, s);
  fq_add(n, s, ps);
  fq_inv_binary(ni, n);
  fq_mul(t, a.v, ni);
  fq_neg(nt, t);
  fq_sel(r.v, pair_odd(), nt, t);
}
HD void finv(Fq2p& r, const Fq2p& a) { finv_fast(r, a); }
HD void fconj(Fq2p& r, const Fq2p& a) {
  Fq n;
  fq_neg(n, a.v);
  fq_sel(r.v, pair_odd(), n, a.v);
}
// an Fq2 constant (24 words: c0 then c1) in pair form
HD void fq2p_set(Fq2p& r, const uint32_t* c) {
  Fq a, b;
  fq_set(a, c);
  fq_set(b, c + 12);
  fq_sel(r.v, pair_odd(), b, a);
}

// psi(x, y) = (conj(x) cx, conj(y) cy) with cx = (0, cx1) purely imaginary:
// conj(x) (cx1 u) = x1 cx1 + x0 cx1 u -> the partner's component times cx1 (one product per lane)
HD void g2p_psi(Fq2p& rx, Fq2p& ry, const G2Ap& p) {
  Fq px, c;
  fq_xchg(px, p.x.v);
  fq_set(c, G2_PSI_CX + 12);
  fq_mul(rx.v, px, c);
  Fq2p cy, yc;
  fq2p_set(cy, G2_PSI_CY);
  fconj(yc, p.y);
  fmul(ry, yc, cy);
}

// Loads and stores between the single-lane layouts (G2A, G2J in memory) and pair form.
HD void g2p_load_aff(G2Ap& r, const G2A* p) {
  const bool odd = pair_odd();
  r.x.v = odd ? p->x.c1 : p->x.c0;
  r.y.v = odd ? p->y.c1 : p->y.c0;
  r.inf = p->inf;
}
HD void g2p_store_jac(G2J* p, const G2Jp& a) {
  Fq* base = reinterpret_cast<Fq*>(p) + (pair_odd() ? 1 : 0);  // x.c0 x.c1 y.c0 y.c1 z.c0 z.c1
  base[0] = a.x.v;
  base[2] = a.y.v;
  base[4] = a.z.v;
}
HD void g2p_load_jac(G2Jp& r, const G2J* p) {
  const Fq* base = reinterpret_cast<const Fq*>(p) + (pair_odd() ? 1 : 0);
  r.x.v = base[0];
  r.y.v = base[2];
  r.z.v = base[4];
}

HD void fq2p_store(Fq2* p, const Fq2p& a) { (reinterpret_cast<Fq*>(p) + (pair_odd() ? 1 : 0))[0] = a.v; }
HD void fq2p_load(Fq2p& a, const Fq2* p) { a.v = (reinterpret_cast<const Fq*>(p) + (pair_odd() ? 1 : 0))[0]; }

// The 68 projective Miller lines (A, B, C) of a G2 point Q (not infinity) in pair form, written
// as Fq2 triples (pairing.h g2_proj_lines' layout); T ends as [|x|] Q, the first half of the psi
// subgroup test (curve.h g2_in_subgroup): psi(Q) == -T.
HD void g2p_walk_lines(Fq2* out, G2Jp& T, const G2Ap& Q) {
  jac_from_aff(T, Q);
  int j = 0;
#pragma unroll 1
  for (int bit = 62; bit >= 0; --bit) {
    Fq2p A, B, C;
    g2_dbl_line(T, A, B, C);
    fq2p_store(out + 3 * j, A);
    fq2p_store(out + 3 * j + 1, B);
    fq2p_store(out + 3 * j + 2, C);
    ++j;
    if ((BLS_X_ABS >> bit) & 1ull) {
      g2_add_step(T, Q, A, B, C);
      fq2p_store(out + 3 * j, A);
      fq2p_store(out + 3 * j + 1, B);
      fq2p_store(out + 3 * j + 2, C);
      ++j;
    }
  }
}
// psi(Q) == -T for T = [|x|] Q (pair form): Q in the prime-order subgroup (Q not infinity)
HD bool g2p_psi_test(const G2Jp& T, const G2Ap& Q) {
  if (jac_is_inf(T)) return false;
  Fq2p px, py;
  g2p_psi(px, py, Q);
  fneg(py, py);
  return jac_eq_aff(T, px, py);
}
// psi on Jacobian coordinates (curve.h g2j_psi) in pair form: X and Y as in g2p_psi, Z conjugated
HD void g2p_psi_jac(G2Jp& r, const G2Jp& p) {
  Fq px, c;
  fq_xchg(px, p.x.v);
  fq_set(c, G2_PSI_CX + 12);
  Fq2p cy, yc;
  fq2p_set(cy, G2_PSI_CY);
  fconj(yc, p.y);
  fq_mul(r.x.v, px, c);
  fmul(r.y, yc, cy);
  fconj(r.z, p.z);
}

// [h2] P (curve.h g2_clear_cofactor: Budroni-Pintore g(P), then [s] g(P) by the m-split) in pair
// form; the same chain of group operations, so the same point
HD void g2p_clear_cofactor(G2Jp& out, const G2Ap& p) {
  if (p.inf) {  // pair-uniform
    jac_set_inf(out);
    return;
  }
  G2Jp pj, t1, t2, t3;
  jac_from_aff(pj, p);
  jac_mul_u64(t1, p, BLS_X_ABS);
  jac_neg(t1, t1);  // [x] P
  G2Ap ps;
  g2p_psi(ps.x, ps.y, p);
  ps.inf = 0;
  jac_dbl(t3, pj);
  g2p_psi_jac(t3, t3);
  g2p_psi_jac(t3, t3);  // psi^2(2P)
  {
    G2Ap nps;
    aff_neg(nps, ps);
    jac_add_aff(t3, t3, nps);
  }
  jac_add_aff(t2, t1, ps);
  jac_mul_u64_jac(t2, t2, BLS_X_ABS);
  jac_neg(t2, t2);
  jac_add(t3, t3, t2);
  {
    G2Jp nt1;
    jac_neg(nt1, t1);
    jac_add(t3, t3, nt1);
  }
  {
    G2Ap np;
    aff_neg(np, p);
    jac_add_aff(t3, t3, np);  // Q = g(P)
  }
  if (jac_is_inf(t3)) {
    out = t3;
    return;
  }
  G2Jp mq = t3;  // m(Q) = (zeta X, Y, Z)
  {
    Fq zeta;
    fq_set(zeta, G2_ZETA);
    fmul_by_fq(mq.x, t3.x, zeta);
  }
  G2Jp bj;
  jac_add(bj, t3, mq);
  G2Ap b;
  {
    Fq2p zi, zi2, zi3;
    finv_fast(zi, bj.z);
    fsqr(zi2, zi);
    fmul(zi3, zi2, zi);
    fmul(b.x, bj.x, zi2);
    fmul(b.y, bj.y, zi3);
    b.inf = 0;
  }
  G2Jp acc;
  jac_from_aff(acc, b);
#pragma unroll 1
  for (int bit = 125; bit >= 0; --bit) {
    jac_dbl(acc, acc);
    if ((cofactor_c0_word(bit >> 5) >> (bit & 31)) & 1u) jac_add_aff(acc, acc, b);
  }
  jac_add(out, acc, mq);
}

// An Fq2 point decoded on both lanes of the pair (one-lane code) -> pair form
HD void g2p_from_full(G2Ap& r, const G2A& f) {
  const bool odd = pair_odd();
  r.x.v = odd ? f.x.c1 : f.x.c0;
  r.y.v = odd ? f.y.c1 : f.y.c0;
  r.inf = f.inf;
}

}  // namespace hbtc
