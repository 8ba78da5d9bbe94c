// BLS12-381 groups G1 (over Fq) and G2 (over Fq2): Jacobian arithmetic, the zcash point
// codec with pairing 0.14's decode checks, and fast subgroup membership tests.
//
// Replaces pairing 0.14.2 src/bls12_381/ec.rs (external crate, /root/reference/Cargo.toml:27)
// as used through threshold_crypto's serde and combine paths (A3/A6).
//
// Decode semantics (bit-exact with G{1,2}Compressed::into_affine):
//   bit7 must be set (compressed); bit6 = infinity -> all remaining bits must be zero;
//   bit5 = "y is lexicographically largest"; coordinates must be < p; x^3 + b must be a
//   square; the point must lie in the r-order subgroup.  Any failure = HBTC_DECODE_ERR.
// The subgroup test uses the curve endomorphisms instead of pairing 0.14's [r]P == O:
//   G1: phi(P) == [-x^2] P   (phi(x, y) = (beta x, y));   G2: psi(P) == [x] P.
// Both are exact membership tests for BLS12-381 (Scott, "A note on group membership tests
// for G1, G2 and GT on BLS pairing-friendly curves", 2021); tests/ cross-check them against
// [r]P on points with every small cofactor component.
#pragma once
#include "field.h"

namespace hbtc {

// ---------------------------------------------------------------- generic field wrappers
HD void fadd(Fq& r, const Fq& a, const Fq& b) { fq_add(r, a, b); }
HD void fadd(Fq2& r, const Fq2& a, const Fq2& b) { fq2_add(r, a, b); }
HD void fsub(Fq& r, const Fq& a, const Fq& b) { fq_sub(r, a, b); }
HD void fsub(Fq2& r, const Fq2& a, const Fq2& b) { fq2_sub(r, a, b); }
HD void fmul(Fq& r, const Fq& a, const Fq& b) { fq_mul(r, a, b); }
HD void fmul(Fq2& r, const Fq2& a, const Fq2& b) { fq2_mul(r, a, b); }
HD void fsqr(Fq& r, const Fq& a) { fq_sqr(r, a); }
HD void fsqr(Fq2& r, const Fq2& a) { fq2_sqr(r, a); }
HD void fdbl(Fq& r, const Fq& a) { fq_dbl(r, a); }
HD void fdbl(Fq2& r, const Fq2& a) { fq2_dbl(r, a); }
HD void fneg(Fq& r, const Fq& a) { fq_neg(r, a); }
HD void fneg(Fq2& r, const Fq2& a) { fq2_neg(r, a); }
HD bool fis_zero(const Fq& a) { return fq_is_zero(a); }
HD bool fis_zero(const Fq2& a) { return fq2_is_zero(a); }
HD bool feq(const Fq& a, const Fq& b) { return fq_eq(a, b); }
HD bool feq(const Fq2& a, const Fq2& b) { return fq2_eq(a, b); }
HD void fone(Fq& r) { fq_one(r); }
HD void fone(Fq2& r) { fq2_one(r); }
HD void fzero(Fq& r) { fq_zero(r); }
HD void fzero(Fq2& r) { fq2_zero(r); }
HD void finv(Fq& r, const Fq& a) { fq_inv(r, a); }
HD void finv(Fq2& r, const Fq2& a) { fq2_inv(r, a); }

template <class F>
struct Aff {
  F x, y;
  uint32_t inf;  // 1 = point at infinity
};

template <class F>
struct Jac {
  F x, y, z;  // (X/Z^2, Y/Z^3); Z == 0 is infinity
};

typedef Aff<Fq> G1A;
typedef Aff<Fq2> G2A;
typedef Jac<Fq> G1J;
typedef Jac<Fq2> G2J;

template <class F>
HD void jac_set_inf(Jac<F>& r) {
  fone(r.x);
  fone(r.y);
  fzero(r.z);
}
template <class F>
HD bool jac_is_inf(const Jac<F>& p) {
  return fis_zero(p.z);
}
template <class F>
HD void jac_from_aff(Jac<F>& r, const Aff<F>& a) {
  if (a.inf) {
    jac_set_inf(r);
  } else {
    r.x = a.x;
    r.y = a.y;
    fone(r.z);
  }
}

// dbl-2009-l (a = 0): 2M + 5S
template <class F>
HD void jac_dbl(Jac<F>& r, const Jac<F>& p) {
  F A, B, C, D, E, Fv, t;
  fsqr(A, p.x);
  fsqr(B, p.y);
  fsqr(C, B);
  fadd(t, p.x, B);
  fsqr(t, t);
  fsub(t, t, A);
  fsub(t, t, C);
  fdbl(D, t);
  fdbl(E, A);
  fadd(E, E, A);
  fsqr(Fv, E);
  F z3;
  fmul(z3, p.y, p.z);
  fdbl(z3, z3);
  F x3;
  fdbl(t, D);
  fsub(x3, Fv, t);
  F y3;
  fsub(t, D, x3);
  fmul(y3, E, t);
  fdbl(C, C);
  fdbl(C, C);
  fdbl(C, C);
  fsub(y3, y3, C);
  r.x = x3;
  r.y = y3;
  r.z = z3;  // Y == 0 never happens for points of odd order; Z stays 0 for infinity
}

// madd-2007-bl: r = p + q (q affine), handles all special cases
template <class F>
HD void jac_add_aff(Jac<F>& r, const Jac<F>& p, const Aff<F>& q) {
  if (q.inf) {
    r = p;
    return;
  }
  if (jac_is_inf(p)) {
    jac_from_aff(r, q);
    return;
  }
  F z1z1, u2, s2, H, HH, I, J, rr, V, t;
  fsqr(z1z1, p.z);
  fmul(u2, q.x, z1z1);
  fmul(s2, q.y, p.z);
  fmul(s2, s2, z1z1);
  fsub(H, u2, p.x);
  fsub(rr, s2, p.y);
  if (fis_zero(H)) {
    if (fis_zero(rr)) {
      jac_dbl(r, p);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  fsqr(HH, H);
  fdbl(I, HH);
  fdbl(I, I);
  fmul(J, H, I);
  fdbl(rr, rr);
  fmul(V, p.x, I);
  F x3, y3, z3;
  fsqr(x3, rr);
  fsub(x3, x3, J);
  fdbl(t, V);
  fsub(x3, x3, t);
  fsub(t, V, x3);
  fmul(y3, rr, t);
  fmul(t, p.y, J);
  fdbl(t, t);
  fsub(y3, y3, t);
  fadd(z3, p.z, H);
  fsqr(z3, z3);
  fsub(z3, z3, z1z1);
  fsub(z3, z3, HH);
  r.x = x3;
  r.y = y3;
  r.z = z3;
}

// add-2007-bl: r = p + q (both Jacobian)
template <class F>
HD void jac_add(Jac<F>& r, const Jac<F>& p, const Jac<F>& q) {
  if (jac_is_inf(p)) {
    r = q;
    return;
  }
  if (jac_is_inf(q)) {
    r = p;
    return;
  }
  F z1z1, z2z2, u1, u2, s1, s2, H, I, J, rr, V, t;
  fsqr(z1z1, p.z);
  fsqr(z2z2, q.z);
  fmul(u1, p.x, z2z2);
  fmul(u2, q.x, z1z1);
  fmul(s1, p.y, q.z);
  fmul(s1, s1, z2z2);
  fmul(s2, q.y, p.z);
  fmul(s2, s2, z1z1);
  fsub(H, u2, u1);
  fsub(rr, s2, s1);
  if (fis_zero(H)) {
    if (fis_zero(rr)) {
      jac_dbl(r, p);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  fdbl(I, H);
  fsqr(I, I);
  fmul(J, H, I);
  fdbl(rr, rr);
  fmul(V, u1, I);
  F x3, y3, z3;
  fsqr(x3, rr);
  fsub(x3, x3, J);
  fdbl(t, V);
  fsub(x3, x3, t);
  fsub(t, V, x3);
  fmul(y3, rr, t);
  fmul(t, s1, J);
  fdbl(t, t);
  fsub(y3, y3, t);
  fadd(z3, p.z, q.z);
  fsqr(z3, z3);
  fsub(z3, z3, z1z1);
  fsub(z3, z3, z2z2);
  fmul(z3, z3, H);
  r.x = x3;
  r.y = y3;
  r.z = z3;
}

// add-2007-bl in place, a += q, ordered so that at most four temporaries are live beside a and q
// (the same formulas and special cases as jac_add; for register-tight kernels: the lane-pair G2
// trees, pair.h)
template <class F>
HD void jac_add_lean(Jac<F>& a, const Jac<F>& q) {
  if (jac_is_inf(q)) return;
  if (jac_is_inf(a)) {
    a = q;
    return;
  }
  F z1z1, z2z2, h, rr;
  fsqr(z1z1, a.z);
  fsqr(z2z2, q.z);
  fmul(a.x, a.x, z2z2);  // U1
  fmul(h, q.x, z1z1);
  fsub(h, h, a.x);       // H = U2 - U1
  fmul(a.y, a.y, q.z);
  fmul(a.y, a.y, z2z2);  // S1
  fmul(rr, q.y, a.z);
  fmul(rr, rr, z1z1);
  fsub(rr, rr, a.y);     // S2 - S1
  if (fis_zero(h)) {
    if (fis_zero(rr)) {
      jac_dbl(a, q);
    } else {
      jac_set_inf(a);
    }
    return;
  }
  fadd(a.z, a.z, q.z);
  fsqr(a.z, a.z);
  fsub(a.z, a.z, z1z1);
  fsub(a.z, a.z, z2z2);
  fmul(a.z, a.z, h);     // Z3
  F i, j;
  fdbl(i, h);
  fsqr(i, i);            // I = (2H)^2
  fmul(j, h, i);         // J = H I
  fmul(i, a.x, i);       // V = U1 I
  fdbl(rr, rr);          // r
  F x3;
  fsqr(x3, rr);
  fsub(x3, x3, j);
  fsub(x3, x3, i);
  fsub(x3, x3, i);       // X3 = r^2 - J - 2 V
  fsub(i, i, x3);
  fmul(i, rr, i);        // r (V - X3)
  fmul(j, a.y, j);
  fdbl(j, j);            // 2 S1 J
  fsub(a.y, i, j);
  a.x = x3;
}

template <class F>
HD void jac_neg(Jac<F>& r, const Jac<F>& p) {
  r.x = p.x;
  fneg(r.y, p.y);
  r.z = p.z;
}

template <class F>
HD void aff_neg(Aff<F>& r, const Aff<F>& p) {
  r.x = p.x;
  fneg(r.y, p.y);
  r.inf = p.inf;
}

template <class F>
HDN void jac_to_aff(Aff<F>& r, const Jac<F>& p) {
  if (jac_is_inf(p)) {
    fzero(r.x);
    fzero(r.y);
    r.inf = 1;
    return;
  }
  F zi, zi2;
  finv(zi, p.z);
  fsqr(zi2, zi);
  fmul(r.x, p.x, zi2);
  fmul(zi2, zi2, zi);
  fmul(r.y, p.y, zi2);
  r.inf = 0;
}

// [k] q for a 64-bit k (MSB-first double-and-add, q affine)
template <class F>
HDN void jac_mul_u64(Jac<F>& r, const Aff<F>& q, uint64_t k) {
  Jac<F> acc;
  jac_set_inf(acc);
  for (int b = 63; b >= 0; --b) {
    jac_dbl(acc, acc);
    if ((k >> b) & 1ull) jac_add_aff(acc, acc, q);
  }
  r = acc;
}

// [a] p + [b] q for 32-bit a, b (joint MSB-first double-and-add, p and q affine)
template <class F>
HDN void jac_mul2_u32(Jac<F>& r, const Aff<F>& p, uint32_t a, const Aff<F>& q, uint32_t b) {
  Jac<F> acc;
  jac_set_inf(acc);
  const uint32_t m = a | b;
  const int top = m ? 31 - __builtin_clz(m) : -1;
  for (int bit = top; bit >= 0; --bit) {
    jac_dbl(acc, acc);
    if ((a >> bit) & 1u) jac_add_aff(acc, acc, p);
    if ((b >> bit) & 1u) jac_add_aff(acc, acc, q);
  }
  r = acc;
}

// 1/a by one binary-GCD inversion in Fq (Fq2: through the norm, conj(a) / (a0^2 + a1^2))
HD void finv_fast(Fq& r, const Fq& a) { fq_inv_binary(r, a); }
HD void finv_fast(Fq2& r, const Fq2& a) {
  Fq n, t, ni;
  fq_sqr(n, a.c0);
  fq_sqr(t, a.c1);
  fq_add(n, n, t);
  fq_inv_binary(ni, n);
  fq_mul(r.c0, a.c0, ni);
  fq_mul(t, a.c1, ni);
  fq_neg(r.c1, t);
}
template <class F>
HD void fsel(F& r, bool c, const F& a, const F& b);
template <>
HD void fsel<Fq>(Fq& r, bool c, const Fq& a, const Fq& b) { fq_sel(r, c, a, b); }
template <>
HD void fsel<Fq2>(Fq2& r, bool c, const Fq2& a, const Fq2& b) {
  fq_sel(r.c0, c, a.c0, b.c0);
  fq_sel(r.c1, c, a.c1, b.c1);
}

// [a] p + [b] q (32-bit a, b) with ONE mixed addition per bit from the table {p, q, p + q}
// (p + q made affine by one binary-GCD inversion): every lane of a wave runs the same 32
// doublings and 32 additions.  The two-branch form (jac_mul2_u32) diverges on random scalars,
// so a wave pays both additions on nearly every bit (32 doublings + 64 additions).
template <class F>
HD void jac_mul2_u32_uniform(Jac<F>& r, const Aff<F>& p, uint32_t a, const Aff<F>& q, uint32_t b) {
  Jac<F> s;
  jac_from_aff(s, p);
  jac_add_aff(s, s, q);
  Aff<F> pq;
  pq.inf = jac_is_inf(s) ? 1u : 0u;
  {
    F zi, zi2, zi3;
    finv_fast(zi, s.z);  // s.z = 0 (infinity): garbage, unused (pq.inf)
    fsqr(zi2, zi);
    fmul(zi3, zi2, zi);
    fmul(pq.x, s.x, zi2);
    fmul(pq.y, s.y, zi3);
  }
  Jac<F> acc;
  jac_set_inf(acc);
  for (int bit = 31; bit >= 0; --bit) {
    jac_dbl(acc, acc);
    const bool ba = ((a >> bit) & 1u) != 0, bb = ((b >> bit) & 1u) != 0;
    Aff<F> t;
    fsel(t.x, bb, ba ? pq.x : q.x, p.x);
    fsel(t.y, bb, ba ? pq.y : q.y, p.y);
    t.inf = bb ? (ba ? pq.inf : q.inf) : p.inf;
    Jac<F> n;
    jac_add_aff(n, acc, t);
    const bool take = ba || bb;
    fsel(acc.x, take, n.x, acc.x);
    fsel(acc.y, take, n.y, acc.y);
    fsel(acc.z, take, n.z, acc.z);
  }
  r = acc;
}

// madd-2007-bl without the exceptional cases, for the uniform loop below: r = p + q for p not
// infinity and p != +-q; z3 = 2 Z1 H.  (p == +-q in that loop needs the running multiple of the
// random-scalar prefix to equal the table point: probability ~2^-250, and a wrong sum only
// makes its RLC group check fail, which falls back to the exact per-share checks.)
template <class F>
HD void jac_madd_generic(Jac<F>& r, const Jac<F>& p, const F& qx, const F& qy) {
  F z1z1, u2, s2, H, HH, I, J, rr, V, t;
  fsqr(z1z1, p.z);
  fmul(u2, qx, z1z1);
  fmul(s2, qy, p.z);
  fmul(s2, s2, z1z1);
  fsub(H, u2, p.x);
  fsub(rr, s2, p.y);
  fsqr(HH, H);
  fdbl(I, HH);
  fdbl(I, I);
  fmul(J, H, I);
  fdbl(rr, rr);
  fmul(V, p.x, I);
  F x3, y3;
  fsqr(x3, rr);
  fsub(x3, x3, J);
  fdbl(t, V);
  fsub(x3, x3, t);
  fsub(t, V, x3);
  fmul(y3, rr, t);
  fmul(t, p.y, J);
  fdbl(t, t);
  fsub(y3, y3, t);
  fmul(r.z, p.z, H);
  fdbl(r.z, r.z);
  r.x = x3;
  r.y = y3;
}

// [a] d + [b] m(d) for an endomorphism m(x, y) = (c x, y) (G1: phi, c = beta; G2: -psi^2,
// c = zeta in Fq) of a point d (not infinity, in the prime-order subgroup) and 32-bit a, b: the
// uniform joint double-and-add of jac_mul2_u32_uniform specialised to an m that keeps y (the
// table is d, c x and d + m(d): 5 coordinates instead of 6) with the generic mixed addition (the
// running sum is infinity only before the first nonzero bit pair: then the table point itself
// is taken).  mx = c x.  a, b < 2^nbits (nbits = 32 or 64: the 64- / 128-bit RLC scalars).
template <class F>
HD void glv_mul_uniform(Jac<F>& r, const Aff<F>& d, const F& mx, uint64_t a, uint64_t b,
                        int nbits = 32) {
  Aff<F> pq;  // d + m(d) (never infinity: m has no eigenvalue -1)
  {
    Jac<F> s;
    jac_from_aff(s, d);
    jac_madd_generic(s, s, mx, d.y);
    F zi, zi2, zi3;
    finv_fast(zi, s.z);
    fsqr(zi2, zi);
    fmul(zi3, zi2, zi);
    fmul(pq.x, s.x, zi2);
    fmul(pq.y, s.y, zi3);
  }
  Jac<F> acc;
  jac_set_inf(acc);
#pragma unroll 1
  for (int bit = nbits - 1; bit >= 0; --bit) {
    jac_dbl(acc, acc);
    const bool ba = ((a >> bit) & 1u) != 0, bb = ((b >> bit) & 1u) != 0;
    F tx, ty;
    fsel(tx, bb, ba ? pq.x : mx, d.x);
    fsel(ty, ba && bb, pq.y, d.y);
    const bool first = jac_is_inf(acc);
    Jac<F> n;
    jac_madd_generic(n, acc, tx, ty);
    {  // the sum is still infinity (leading zero bit pairs of this lane): take the table point
      F one;
      fone(one);
      fsel(n.x, first, tx, n.x);
      fsel(n.y, first, ty, n.y);
      fsel(n.z, first, one, n.z);
    }
    const bool take = ba || bb;
    fsel(acc.x, take, n.x, acc.x);
    fsel(acc.y, take, n.y, acc.y);
    fsel(acc.z, take, n.z, acc.z);
  }
  r = acc;
}

// ---------------------------------------------------------------- x-adic RLC scalars
// The RLC scalar of an item (DESIGN.md §4 "Soundness") is r = d0 + d1 x + d2 mu + d3 mu x (mod r)
// with four digits d_j < 2^nbits (nbits = 16 or 32: 2^64 or 2^128 distinct scalars), x the BLS
// parameter and mu = -x^2 the eigenvalue of the endomorphism m(X, Y) = (c X, Y) (G1: phi, c =
// beta; G2: -psi^2, c = zeta).  For P in the prime-order group and XP = [x] P (G1: the negated
// [|x|] P the subgroup test computes anyway; G2: psi(P), free):
//     [r] P = [d0] P + [d1] XP + [d2] m(P) + [d3] m(XP)
// one joint double-and-add over nbits bits with TWO mixed additions per bit, T[d0_i, d1_i] and
// m(T[d2_i, d3_i]) from the affine table T = {P, XP, P + XP}: nbits doublings instead of the
// 2 nbits of the two-digit form [a] P + [b] m(P), for one Fq product (G1) / two (G2) per bit to
// apply m to the selected entry.  Every lane runs the same instructions (selects only).
HD void fmul_by_fq(Fq& r, const Fq& a, const Fq& c) { fq_mul(r, a, c); }
HD void fmul_by_fq(Fq2& r, const Fq2& a, const Fq& c) {
  fq_mul(r.c0, a.c0, c);
  fq_mul(r.c1, a.c1, c);
}

// acc += (tx, ty) when `take` (acc infinity: the table point itself; no exceptional cases
// otherwise, as in glv_mul_uniform below)
template <class F>
HD void uniform_add(Jac<F>& acc, const F& tx, const F& ty, bool take) {
  const bool first = jac_is_inf(acc);
  Jac<F> n;
  jac_madd_generic(n, acc, tx, ty);
  F one;
  fone(one);
  fsel(n.x, first, tx, n.x);
  fsel(n.y, first, ty, n.y);
  fsel(n.z, first, one, n.z);
  fsel(acc.x, take, n.x, acc.x);
  fsel(acc.y, take, n.y, acc.y);
  fsel(acc.z, take, n.z, acc.z);
}

// The table entries XP and P + XP (affine) from XP in Jacobian coordinates: one inversion for
// both (P + XP != O and XP != P: x != +-1 mod r).
template <class F>
HD void xadic_table(Aff<F>& xp, Aff<F>& pxp, const Aff<F>& p, const Jac<F>& xpj) {
  Jac<F> sj;
  jac_madd_generic(sj, xpj, p.x, p.y);
  F z12, inv, zi1, zi2;
  fmul(z12, xpj.z, sj.z);
  finv_fast(inv, z12);
  fmul(zi1, inv, sj.z);   // 1 / xpj.z
  fmul(zi2, inv, xpj.z);  // 1 / sj.z
  F t, t2;
  fsqr(t, zi1);
  fmul(xp.x, xpj.x, t);
  fmul(t2, t, zi1);
  fmul(xp.y, xpj.y, t2);
  xp.inf = 0;
  fsqr(t, zi2);
  fmul(pxp.x, sj.x, t);
  fmul(t2, t, zi2);
  fmul(pxp.y, sj.y, t2);
  pxp.inf = 0;
}

template <class F>
HD void xadic_mul_uniform(Jac<F>& r, const Aff<F>& p, const Aff<F>& xp, const Aff<F>& pxp,
                          const Fq& c, uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3,
                          int nbits) {
  Jac<F> acc;
  jac_set_inf(acc);
#pragma unroll 1
  for (int bit = nbits - 1; bit >= 0; --bit) {
    jac_dbl(acc, acc);
    const bool b0 = ((d0 >> bit) & 1u) != 0, b1 = ((d1 >> bit) & 1u) != 0;
    const bool b2 = ((d2 >> bit) & 1u) != 0, b3 = ((d3 >> bit) & 1u) != 0;
    F tx, ty;
    fsel(tx, b1, b0 ? pxp.x : xp.x, p.x);
    fsel(ty, b1, b0 ? pxp.y : xp.y, p.y);
    uniform_add(acc, tx, ty, b0 || b1);
    F ux, uy;
    fsel(ux, b3, b2 ? pxp.x : xp.x, p.x);
    fsel(uy, b3, b2 ? pxp.y : xp.y, p.y);
    fmul_by_fq(ux, ux, c);  // m(T[b2, b3])
    uniform_add(acc, ux, uy, b2 || b3);
  }
  r = acc;
}

// The same loop with the three table points in LDS ([entry][word][lane]: each lane reads its own
// column, conflict-free; entry 0 = P, 1 = XP, 2 = P + XP), read by a lane-dependent entry index
// instead of selects over registers: the G2 item pass (k_sig_items, one wave per SIMD) holds
// 144 dwords of table beside its accumulator and the shared product's fixed registers otherwise,
// and re-read ~53 spilled dwords per bit from scratch.
// (LANES: the lane stride of the layout -- 64 for one lane per item, 128 for a two-wave
// workgroup of lane pairs, pair.h)
template <class F, int LANES = 64>
HD void xy_lds_get_aff(F& x, F& y, const uint32_t* lds, uint32_t lane, uint32_t e) {
  constexpr int NW = (int)(sizeof(F) / 4);
  uint32_t* dx = reinterpret_cast<uint32_t*>(&x);
  uint32_t* dy = reinterpret_cast<uint32_t*>(&y);
#pragma unroll
  for (int w = 0; w < NW; ++w) dx[w] = lds[(e * 2 * NW + w) * LANES + lane];
#pragma unroll
  for (int w = 0; w < NW; ++w) dy[w] = lds[(e * 2 * NW + NW + w) * LANES + lane];
}
template <class F, int LANES = 64>
HD void xy_lds_put_aff(uint32_t* lds, uint32_t lane, uint32_t e, const Aff<F>& p) {
  constexpr int NW = (int)(sizeof(F) / 4);
  const uint32_t* sx = reinterpret_cast<const uint32_t*>(&p.x);
  const uint32_t* sy = reinterpret_cast<const uint32_t*>(&p.y);
#pragma unroll
  for (int w = 0; w < NW; ++w) lds[(e * 2 * NW + w) * LANES + lane] = sx[w];
#pragma unroll
  for (int w = 0; w < NW; ++w) lds[(e * 2 * NW + NW + w) * LANES + lane] = sy[w];
}
template <class F, int LANES = 64>
HD void xadic_mul_uniform_lds(Jac<F>& r, const uint32_t* lds, uint32_t lane, const Fq& c, uint32_t d0,
                              uint32_t d1, uint32_t d2, uint32_t d3, int nbits) {
  Jac<F> acc;
  jac_set_inf(acc);
#pragma unroll 1
  for (int bit = nbits - 1; bit >= 0; --bit) {
    jac_dbl(acc, acc);
    const bool b0 = ((d0 >> bit) & 1u) != 0, b1 = ((d1 >> bit) & 1u) != 0;
    const bool b2 = ((d2 >> bit) & 1u) != 0, b3 = ((d3 >> bit) & 1u) != 0;
    F tx, ty;
    xy_lds_get_aff<F, LANES>(tx, ty, lds, lane, b1 ? (b0 ? 2u : 1u) : 0u);
    uniform_add(acc, tx, ty, b0 || b1);
    xy_lds_get_aff<F, LANES>(tx, ty, lds, lane, b3 ? (b2 ? 2u : 1u) : 0u);
    fmul_by_fq(tx, tx, c);  // m(T[b2, b3])
    uniform_add(acc, tx, ty, b2 || b3);
  }
  r = acc;
}

// ------------------------------------------------------------ x-adic scalars: shared pieces
#ifndef HBTC_XADIC8
#define HBTC_XADIC8 1  // G1 item passes: the sign-aligned 8-entry table (xadic_mul_sac8)
#endif
template <class F>
struct XY {
  F x, y;
};
// co-Z addition of A and B (same Z): A + B, with A rescaled to the sum's Z (Z * H) in ax, ay;
// returns H
template <class F>
HD void coz_add(XY<F>& s, F& ax, F& ay, F& h, const XY<F>& b) {
  F r, hh, hhh, v, t;
  fsub(h, b.x, ax);
  fsub(r, b.y, ay);
  fsqr(hh, h);
  fmul(hhh, hh, h);
  fmul(v, ax, hh);
  fmul(ay, ay, hhh);
  ax = v;
  fsqr(s.x, r);
  fsub(s.x, s.x, hhh);
  fdbl(t, v);
  fsub(s.x, s.x, t);
  fsub(t, v, s.x);
  fmul(s.y, r, t);
  fsub(s.y, s.y, ay);
}
template <class F>
HD void scale_xy(XY<F>& p, const F& l2, const F& l3) {
  fmul(p.x, p.x, l2);
  fmul(p.y, p.y, l3);
}
// ------------------------------------------- x-adic scalars, sign-aligned 8-entry table (GLV-SAC)
// [r] P with one mixed addition per bit from EIGHT entries, small enough to stay in registers
// (AGPRs at one wave per SIMD) and be read by selects, so no per-lane indexed table in scratch.
// (Round 4's table of all fifteen digit-bit sums was indexed per lane and lived in scratch:
// 3 KB/lane; it is gone.)  Sign-aligned recoding (Faz-Hernandez, Longa, Sanchez, "Efficient and
// secure algorithms for GLV-based scalar multiplication", 2014, Alg. 1) of the digit vector
// (k0, d1, d2, d3), k0 odd: l = nbits + 1 columns with
//     k0 = sum_i s_i 2^i,  s_{l-1} = 1,  s_i = 2 bit_{i+1}(k0) - 1 in {+-1};
//     d_j = sum_i u_j[i] s_i 2^i,  u_j[i] in {0, 1}   (computed LSB first: u_j[i] = d_j mod 2,
//                                                      d_j = (d_j >> 1) + (u_j[i] && s_i < 0))
// so [r] P = sum_i 2^i s_i T[u1 + 2 u2 + 4 u3] with T[u] = P + u1 XP + u2 m(P) + u3 m(XP): every
// column adds +-one entry (the sign is a y negation), none is empty, the first one starts the sum.
// k0 = d0 | 1; an even d0 is corrected by one final addition of -P (11 Fq products of ~2,500).
// The entries are the co-Z sums U + m(V), U in {P, S = P + XP}, V in {P, XP, S} (6 co-Z
// additions) brought to one Z*: no inversion, since points sharing one Z are affine points of the
// isomorphic curve y^2 = x^3 + b Z*^6 and the a = 0 doubling / mixed-addition formulas do not
// involve b; the double-and-add runs there and the result's Z is multiplied by Z* at the end.
// Exceptional cases: none.  Before column i is added the running sum is [c] of a combination whose
// P coefficient is 2 * (an odd integer) and whose other coefficients are below 2^(nbits+2) < |x|,
// the entry's P coefficient is +-1, and such integer combinations of {1, x, mu, mu x} are distinct
// mod r (the digit-box argument): acc != +-T, acc != O.  The final correction meets
// acc == P only for the all-zero digit vector (r = 0), which is selected to infinity.
template <class F>
HD void xadic_table8(XY<F> tab[8], F& zs, const Aff<F>& p, const Jac<F>& xpj, const Fq& c) {
  XY<F> u[4];  // u[1] = P, u[2] = XP, u[3] = S = P + XP at the common Z0
  {
    F h, hh, hhh, z2, z3;
    fsqr(z2, xpj.z);
    fmul(z3, z2, xpj.z);
    fmul(u[1].x, p.x, z2);
    fmul(u[1].y, p.y, z3);
    F ax = u[1].x, ay = u[1].y;
    XY<F> s;
    F bx = xpj.x, by = xpj.y;
    coz_add(s, bx, by, h, u[1]);  // s = XP + P1, (bx, by) = XP at Z1 H
    u[3] = s;
    u[2].x = bx;
    u[2].y = by;
    fsqr(hh, h);
    fmul(hhh, hh, h);
    XY<F> p1{ax, ay};
    scale_xy(p1, hh, hhh);
    u[1] = p1;
    fmul(zs, xpj.z, h);  // Z0
  }
  // entry k = 0..5: U = (k & 1 ? S : P), V = u[k / 2 + 1]; table slot 2 (k / 2 + 1) + (k & 1)
  F hk[6], pre[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    XY<F> mv;
    fmul_by_fq(mv.x, u[k / 2 + 1].x, c);
    mv.y = u[k / 2 + 1].y;
    F ax = u[(k & 1) ? 3 : 1].x, ay = u[(k & 1) ? 3 : 1].y;
    coz_add(tab[2 * (k / 2 + 1) + (k & 1)], ax, ay, hk[k], mv);
  }
  pre[0] = hk[0];
#pragma unroll
  for (int k = 1; k < 6; ++k) fmul(pre[k], pre[k - 1], hk[k]);
  F run;
#pragma unroll
  for (int k = 5; k >= 0; --k) {
    F l, l2, l3;
    if (k == 5)
      l = pre[4];
    else if (k == 0)
      l = run;
    else
      fmul(l, pre[k - 1], run);
    if (k == 5)
      run = hk[5];
    else if (k > 0)
      fmul(run, run, hk[k]);
    fsqr(l2, l);
    fmul(l3, l2, l);
    scale_xy(tab[2 * (k / 2 + 1) + (k & 1)], l2, l3);
  }
  {
    F l2, l3;
    fsqr(l2, pre[5]);
    fmul(l3, l2, pre[5]);
    scale_xy(u[1], l2, l3);
    scale_xy(u[3], l2, l3);
    tab[0] = u[1];
    tab[1] = u[3];
    fmul(zs, zs, pre[5]);  // Z* = Z0 prod H_k
  }
}

// the sign-aligned recoding above: bit i of m[j - 1] = u_j[i] (j = 1..3), for l = nbits + 1 columns
HD void xadic_sac_recode(uint64_t m[3], uint32_t k0, uint32_t d1, uint32_t d2, uint32_t d3,
                         int nbits) {
  const uint32_t d[3] = {d1, d2, d3};
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    uint64_t k = d[j], mk = 0;
#pragma unroll 1
    for (int i = 0; i <= nbits; ++i) {
      const uint64_t odd = k & 1u;
      const uint64_t neg = (i < nbits) ? ((~(uint64_t)k0 >> (i + 1)) & 1u) : 0u;  // s_i = -1
      mk |= odd << i;
      k = (k >> 1) + (odd & neg);
    }
    m[j] = mk;
  }
}

template <class F>
HD void xy_sel(XY<F>& r, bool c, const XY<F>& a, const XY<F>& b) {  // r = c ? a : b
  fsel(r.x, c, a.x, b.x);
  fsel(r.y, c, a.y, b.y);
}

// The same eight entries for xadic_mul_sac8<LDS3>, built as a co-Z chain at a running Z instead
// of six separate co-Z sums brought to one Z by prefix / suffix products: each sum U + m(V)
// updates U to the new Z (coz_add), and every other live entry is rescaled by (h^2, h^3) at once,
// so no arrays of H_k and prefix products are live beside the table (k_rlc_items: the build's
// spills were most of its scratch).  tab[0..4] stay in registers; tab[5..7] are written to LDS
// ([entry][word][lane], as xadic_mul_sac8 reads them) when formed and rescaled there.  ~16 more
// Fq products than xadic_table8 (22 rescaled entries), the same additions (the same exceptional-
// case argument).
template <class F>
HD void xy_rescale(XY<F>& p, const F& h2, const F& h3) {
  fmul(p.x, p.x, h2);
  fmul(p.y, p.y, h3);
}
template <class F>
HD void xy_lds_put(uint32_t* lds, uint32_t lane, int e, const XY<F>& v) {
  constexpr int NWD = (int)(sizeof(XY<F>) / 4);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
  for (int w = 0; w < NWD; ++w) lds[(e * NWD + w) * 64 + lane] = src[w];
}
template <class F>
HD void xy_lds_get(XY<F>& v, const uint32_t* lds, uint32_t lane, int e) {
  constexpr int NWD = (int)(sizeof(XY<F>) / 4);
  uint32_t* dst = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
  for (int w = 0; w < NWD; ++w) dst[w] = lds[(e * NWD + w) * 64 + lane];
}
template <class F>
HD void xy_lds_rescale(uint32_t* lds, uint32_t lane, int e, const F& h2, const F& h3) {
  XY<F> v;
  xy_lds_get(v, lds, lane, e);
  xy_rescale(v, h2, h3);
  xy_lds_put(lds, lane, e, v);
}
template <class F>
HD void xadic_table8_chain(XY<F> tab[5], F& zs, const Aff<F>& p, const Jac<F>& xpj, const Fq& c,
                           uint32_t* lds, uint32_t lane) {
  XY<F>& P = tab[0];
  XY<F>& S = tab[1];
  XY<F> X;
  F h, h2, h3;
  {  // P at XP's Z; S = XP + P (co-Z), XP updated; P rescaled: all three at Z0
    F z2, z3;
    fsqr(z2, xpj.z);
    fmul(z3, z2, xpj.z);
    fmul(P.x, p.x, z2);
    fmul(P.y, p.y, z3);
    X.x = xpj.x;
    X.y = xpj.y;
    coz_add(S, X.x, X.y, h, P);
    fsqr(h2, h);
    fmul(h3, h2, h);
    xy_rescale(P, h2, h3);
    fmul(zs, xpj.z, h);
  }
  // out = U + m(V), U updated to the new Z; h2, h3 for the other entries
  auto sum = [&](XY<F>& out, XY<F>& U, const XY<F>& V) {
    XY<F> mv;
    fmul_by_fq(mv.x, V.x, c);
    mv.y = V.y;
    coz_add(out, U.x, U.y, h, mv);
    fsqr(h2, h);
    fmul(h3, h2, h);
    fmul(zs, zs, h);
  };
  // the two sums over m(XP) first, so XP is dropped after two steps: 22 rescaled entries
  sum(tab[4], P, X);  // P + m(XP)
  xy_rescale(X, h2, h3);
  xy_rescale(S, h2, h3);
  {
    XY<F> t5;
    sum(t5, S, X);  // S + m(XP); XP is not needed past here
    xy_lds_put(lds, lane, 0, t5);
  }
  xy_rescale(P, h2, h3);
  xy_rescale(tab[4], h2, h3);
  sum(tab[2], P, P);  // P + m(P)
  xy_rescale(S, h2, h3);
  xy_rescale(tab[4], h2, h3);
  xy_lds_rescale(lds, lane, 0, h2, h3);
  sum(tab[3], S, P);  // S + m(P)
  xy_rescale(P, h2, h3);
  xy_rescale(tab[2], h2, h3);
  xy_rescale(tab[4], h2, h3);
  xy_lds_rescale(lds, lane, 0, h2, h3);
  {
    XY<F> t6;
    sum(t6, P, S);  // P + m(S)
    xy_lds_put(lds, lane, 1, t6);
  }
  xy_rescale(S, h2, h3);
  xy_rescale(tab[2], h2, h3);
  xy_rescale(tab[3], h2, h3);
  xy_rescale(tab[4], h2, h3);
  xy_lds_rescale(lds, lane, 0, h2, h3);
  {
    XY<F> t7;
    const XY<F> s0 = S;
    sum(t7, S, s0);  // S + m(S)
    xy_lds_put(lds, lane, 2, t7);
  }
  xy_rescale(P, h2, h3);
  xy_rescale(tab[2], h2, h3);
  xy_rescale(tab[3], h2, h3);
  xy_rescale(tab[4], h2, h3);
  xy_lds_rescale(lds, lane, 0, h2, h3);
  xy_lds_rescale(lds, lane, 1, h2, h3);
}

template <class F, bool LDS3 = false>
HD void xadic_mul_sac8(Jac<F>& r, const Aff<F>& p, const Jac<F>& xpj, const Fq& c, uint32_t d0,
                       uint32_t d1, uint32_t d2, uint32_t d3, int nbits, uint32_t* lds = nullptr,
                       uint32_t lane = 0) {
  // LDS3: entries 5..7 live in LDS (lds: 3 x NWD x 64 words, [entry][word][lane]: each lane reads
  // its own column, conflict-free) and are read by a lane-dependent address, entries 0..4 stay in
  // registers (k_rlc_items at two waves per SIMD: 256 VGPRs hold five entries beside the loop)
  constexpr int NWD = (int)(sizeof(XY<F>) / 4);
  XY<F> tab[LDS3 ? 5 : 8];
  F zs;
  if constexpr (LDS3)
    xadic_table8_chain(tab, zs, p, xpj, c, lds, lane);
  else
    xadic_table8(tab, zs, p, xpj, c);
  const uint32_t k0 = d0 | 1u;
  uint64_t m[3];
  xadic_sac_recode(m, k0, d1, d2, d3, nbits);
  // the entry of column i, negated when s_i = -1: a select tree over the entries (constant
  // indices only, so the register entries never go to scratch)
  auto entry = [&](int i, XY<F>& t) {
    const bool b1 = ((m[0] >> i) & 1u) != 0, b2 = ((m[1] >> i) & 1u) != 0;
    const bool b3 = ((m[2] >> i) & 1u) != 0;
    XY<F> e0, e1;
    {
      XY<F> a, b;
      xy_sel(a, b1, tab[1], tab[0]);
      xy_sel(b, b1, tab[3], tab[2]);
      xy_sel(e0, b2, b, a);
    }
    if constexpr (LDS3) {
      const uint32_t j = (b1 ? 1u : 0u) + (b2 ? 2u : 0u);  // entry 4 + j
      const uint32_t li = j ? j - 1u : 0u;
      XY<F> l;
      uint32_t* dst = reinterpret_cast<uint32_t*>(&l);
#pragma unroll
      for (int w = 0; w < NWD; ++w) dst[w] = lds[(li * NWD + w) * 64 + lane];
      xy_sel(e1, j != 0, l, tab[4]);
    } else {
      XY<F> a, b;
      xy_sel(a, b1, tab[5], tab[4]);
      xy_sel(b, b1, tab[7], tab[6]);
      xy_sel(e1, b2, b, a);
    }
    xy_sel(t, b3, e1, e0);
    const bool neg = i < nbits && (((uint64_t)k0 >> (i + 1)) & 1u) == 0;
    F ny;
    fneg(ny, t.y);
    fsel(t.y, neg, ny, t.y);
  };
  Jac<F> acc;
  {
    XY<F> t;
    entry(nbits, t);  // s = +1
    acc.x = t.x;
    acc.y = t.y;
    fone(acc.z);
  }
#pragma unroll 1
  for (int i = nbits - 1; i >= 0; --i) {
    jac_dbl(acc, acc);
    XY<F> t;
    entry(i, t);
    jac_madd_generic(acc, acc, t.x, t.y);
  }
  {  // d0 even: acc - P (P = tab[0] on the isomorphic curve)
    const bool even = (d0 & 1u) == 0;
    const bool zero = (d0 | d1 | d2 | d3) == 0;
    F ny;
    fneg(ny, tab[0].y);
    Jac<F> n;
    jac_madd_generic(n, acc, tab[0].x, ny);
    fsel(acc.x, even, n.x, acc.x);
    fsel(acc.y, even, n.y, acc.y);
    fsel(acc.z, even, n.z, acc.z);
    F z0;
    fzero(z0);
    fsel(acc.z, zero, z0, acc.z);
  }
  fmul(acc.z, acc.z, zs);  // back from the isomorphic curve
  r = acc;
}

// ------------------------------------------ two-digit sign-aligned form (the small combines)
// [d0] P + [d1] XP for digits below 2^nbits (nbits <= 64) and XP = [u] P, u = |x| (G1: from the
// subgroup test's double-and-add; G2: -psi(P)), with ONE mixed addition per column from the
// two-entry table {P, P + XP} at a common Z (the first step of xadic_table8), GLV-SAC recoded
// like xadic_mul_sac8: nbits + 1 columns, k0 = d0 | 1, every column adds +-T[u1], an even d0 is
// corrected by a final addition of -P, and d0 = d1 = 0 gives infinity.
// The digits here are NOT random (base-u digits of Lagrange coefficients), so exceptional cases
// are excluded by parity instead of probability: before column i the sum is [2A + 2B u] P with
// A odd (the processed sign digits), the entry is [+-(1 + v u)] P (v in {0, 1}), both below r in
// absolute value, and 2A -+ 1 + (2B -+ v) u = 0 is impossible (odd + even, u is even); 2A + 2B u
// = 0 would make A = -B u even.  The correction meets [k0 + d1 u] P = +-P only for d0 = d1 = 0.
template <class F>
HD void sac2_mul(Jac<F>& r, const Aff<F>& p, const Jac<F>& xpj, uint64_t d0, uint64_t d1, int nbits) {
  XY<F> t0, t1;  // P and S = P + XP at the common Z0 (= zs)
  F zs;
  {
    F h, hh, hhh, z2, z3;
    fsqr(z2, xpj.z);
    fmul(z3, z2, xpj.z);
    fmul(t0.x, p.x, z2);
    fmul(t0.y, p.y, z3);
    F bx = xpj.x, by = xpj.y;
    coz_add(t1, bx, by, h, t0);  // t1 = XP + P1 at Z1 H
    fsqr(hh, h);
    fmul(hhh, hh, h);
    scale_xy(t0, hh, hhh);
    fmul(zs, xpj.z, h);
  }
  const uint64_t k0 = d0 | 1u;
  const uint64_t all = nbits >= 64 ? ~0ull : ((1ull << nbits) - 1ull);
  const uint64_t negm = ~(k0 >> 1) & all;  // bit i: s_i = -1 (columns below nbits)
  uint64_t m1 = 0, k = d1;
#pragma unroll 1
  for (int i = 0; i < nbits; ++i) {
    const uint64_t odd = k & 1u;
    m1 |= odd << i;
    k = (k >> 1) + (odd & (negm >> i) & 1u);
  }
  Jac<F> acc;  // the top column: s = +1, u1 = what is left of d1 (0 or 1)
  fsel(acc.x, k != 0, t1.x, t0.x);
  fsel(acc.y, k != 0, t1.y, t0.y);
  fone(acc.z);
#pragma unroll 1
  for (int i = nbits - 1; i >= 0; --i) {
    jac_dbl(acc, acc);
    XY<F> t;
    xy_sel(t, ((m1 >> i) & 1u) != 0, t1, t0);
    F ny;
    fneg(ny, t.y);
    fsel(t.y, ((negm >> i) & 1u) != 0, ny, t.y);
    jac_madd_generic(acc, acc, t.x, t.y);
  }
  {
    const bool even = (d0 & 1u) == 0, zero = (d0 | d1) == 0;
    F ny;
    fneg(ny, t0.y);
    Jac<F> n;
    jac_madd_generic(n, acc, t0.x, ny);
    fsel(acc.x, even, n.x, acc.x);
    fsel(acc.y, even, n.y, acc.y);
    fsel(acc.z, even, n.z, acc.z);
    F z0;
    fzero(z0);
    fsel(acc.z, zero, z0, acc.z);
  }
  fmul(acc.z, acc.z, zs);
  r = acc;
}

// Base-u digits of a canonical scalar k < r < u^4 (u = |x| = 2^16 v): k = sum_j d_j u^j, 0 <= d_j < u,
// by three exact divisions by u (16-bit long division in 64-bit registers).  The combines' GLS / GLV
// splits (hbtc_msm.hip, hbtc_comb.hip).
HD void gls_u_digits(const uint32_t* k, uint64_t d[4]) {
  constexpr uint64_t V = BLS_X_ABS >> 16;  // 0xd20100000001
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = k[i];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const uint32_t lo16 = w[0] & 0xffffu;
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = (w[i] >> 16) | (i < 7 ? w[i + 1] << 16 : 0u);
    uint64_t rem = 0;  // < V < 2^48, so rem * 2^16 + 16 bits fits 64
#pragma unroll
    for (int i = 7; i >= 0; --i) {
      uint64_t cur = (rem << 16) | (w[i] >> 16);
      const uint32_t qh = (uint32_t)(cur / V);
      rem = cur - (uint64_t)qh * V;
      cur = (rem << 16) | (w[i] & 0xffffu);
      const uint32_t ql = (uint32_t)(cur / V);
      rem = cur - (uint64_t)ql * V;
      w[i] = (qh << 16) | ql;
    }
    d[j] = (rem << 16) | lo16;
  }
  d[3] = ((uint64_t)w[1] << 32) | w[0];  // the quotient after three divisions: < u
}

// GLV endomorphism of G1: phi(x, y) = (beta x, y) = [-x^2] (x, y) on the r-order subgroup
HD void g1_phi(G1A& r, const G1A& p) {
  Fq beta;
  fq_set(beta, G1_BETA);
  fq_mul(r.x, p.x, beta);
  r.y = p.y;
  r.inf = p.inf;
}

// [k] q for a Jacobian base and 64-bit k
template <class F>
HDN void jac_mul_u64_jac(Jac<F>& r, const Jac<F>& q, uint64_t k) {
  Jac<F> acc;
  jac_set_inf(acc);
  for (int b = 63; b >= 0; --b) {
    jac_dbl(acc, acc);
    if ((k >> b) & 1ull) jac_add(acc, acc, q);
  }
  r = acc;
}

// [k] q for an NW-limb little-endian integer scalar (MSB-first double-and-add).  The limbs
// are rotated through registers (static indexing only) so the device build never puts the
// scalar in scratch memory.
template <class F, int NW>
HDN void jac_mul_limbs(Jac<F>& r, const Aff<F>& q, const Limbs<NW>& k) {
  Jac<F> acc;
  jac_set_inf(acc);
  if (q.inf) {
    r = acc;
    return;
  }
  Limbs<NW> kk = k;
  for (int w = 0; w < NW; ++w) {
    const uint32_t word = kk.v[NW - 1];
#pragma unroll
    for (int j = NW - 1; j > 0; --j) kk.v[j] = kk.v[j - 1];
    for (int b = 31; b >= 0; --b) {
      jac_dbl(acc, acc);
      if ((word >> b) & 1u) jac_add_aff(acc, acc, q);
    }
  }
  r = acc;
}

// [k] q for a canonical (non-Montgomery) 8-limb scalar
template <class F>
HD void jac_mul_fr(Jac<F>& r, const Aff<F>& q, const Fr& k) {
  jac_mul_limbs<F, 8>(r, q, k);
}

// Is the Jacobian point p equal to the affine point (ax, ay)?  (p not infinity)
template <class F>
HD bool jac_eq_aff(const Jac<F>& p, const F& ax, const F& ay) {
  F z2, z3, t;
  fsqr(z2, p.z);
  fmul(z3, z2, p.z);
  fmul(t, ax, z2);
  if (!feq(t, p.x)) return false;
  fmul(t, ay, z3);
  return feq(t, p.y);
}

template <class F>
HD bool jac_eq(const Jac<F>& p, const Jac<F>& q) {
  bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F z1z1, z2z2, a, b;
  fsqr(z1z1, p.z);
  fsqr(z2z2, q.z);
  fmul(a, p.x, z2z2);
  fmul(b, q.x, z1z1);
  if (!feq(a, b)) return false;
  fmul(a, p.y, z2z2);
  fmul(a, a, q.z);
  fmul(b, q.y, z1z1);
  fmul(b, b, p.z);
  return feq(a, b);
}

// ---------------------------------------------------------------- subgroup tests
// t1 = [|x|] P, the first half of the test (the RLC item passes reuse it: [x] P = -t1)
HDN bool g1_in_subgroup_t1(const G1A& p, G1J& t) {
  if (p.inf) {
    jac_set_inf(t);
    return true;
  }
  G1J t2;
  jac_mul_u64(t, p, BLS_X_ABS);
  jac_mul_u64_jac(t2, t, BLS_X_ABS);  // [x^2] P
  if (jac_is_inf(t2)) return false;   // phi(P) != O for P != O
  Fq bx, ny;
  Fq beta;
  fq_set(beta, G1_BETA);
  fq_mul(bx, p.x, beta);
  fq_neg(ny, p.y);  // phi(P) == -[x^2]P  <=>  (beta x, -y) == [x^2] P
  return jac_eq_aff(t2, bx, ny);
}

HDN bool g1_in_subgroup(const G1A& p) {
  if (p.inf) return true;
  G1J t, t2;
  jac_mul_u64(t, p, BLS_X_ABS);
  jac_mul_u64_jac(t2, t, BLS_X_ABS);  // [x^2] P
  if (jac_is_inf(t2)) return false;   // phi(P) != O for P != O
  Fq bx, ny;
  Fq beta;
  fq_set(beta, G1_BETA);
  fq_mul(bx, p.x, beta);
  fq_neg(ny, p.y);  // phi(P) == -[x^2]P  <=>  (beta x, -y) == [x^2] P
  return jac_eq_aff(t2, bx, ny);
}

HD void g2_psi(Fq2& rx, Fq2& ry, const G2A& p) {
  Fq2 c, k;
  fq2_conj(c, p.x);
  fq2_set(k, G2_PSI_CX);
  fq2_mul(rx, c, k);
  fq2_conj(c, p.y);
  fq2_set(k, G2_PSI_CY);
  fq2_mul(ry, c, k);
}

HDN bool g2_in_subgroup(const G2A& p) {
  if (p.inf) return true;
  G2J t;
  jac_mul_u64(t, p, BLS_X_ABS);  // [|x|] P ; [x]P = -[|x|]P
  if (jac_is_inf(t)) return false;
  Fq2 px, py, npy;
  g2_psi(px, py, p);
  fq2_neg(npy, py);  // psi(P) == -[|x|]P  <=>  (psi_x, -psi_y) == [|x|]P
  return jac_eq_aff(t, px, npy);
}

// psi on Jacobian coordinates: (conj(X) cx, conj(Y) cy, conj(Z)) (conj is a field automorphism,
// so x = X / Z^2 maps to conj(X) / conj(Z)^2)
HD void g2j_psi(G2J& r, const G2J& p) {
  Fq2 c, k;
  fq2_conj(c, p.x);
  fq2_set(k, G2_PSI_CX);
  fq2_mul(r.x, c, k);
  fq2_conj(c, p.y);
  fq2_set(k, G2_PSI_CY);
  fq2_mul(r.y, c, k);
  fq2_conj(r.z, p.z);
}

// [h2] P for any P on E'(Fq2): pairing 0.14's G2 scale_by_cofactor, the last step of G2::rand in
// hash_g2 / hash_g1_g2.  Instead of the 508-bit double-and-add by h2 (~507 doublings + ~250
// additions):
//   g(P) = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P) = [h_eff] P,  h_eff = (3x^2 - 3) h2
// (Budroni-Pintore; it kills the whole cofactor group, so g(P) is in G2), then
//   [h2] P = [s] g(P),  s = (3x^2 - 3)^-1 mod r,
// and on G2, with m = -psi^2 = (zeta x, y) (eigenvalue -x^2) and the offline decomposition
// s = c0 + c1 (-x^2) mod r, c1 = c0 + 1 (127-bit c0 = G2_CLEAR_C0, tools/gen_constants.py):
//   [s] Q = [c0] (Q + m(Q)) + m(Q).
// Two 64-bit multiplications by |x| (sparse) + 126 doublings and 42 mixed additions: about
// 2.5x fewer Fq products.  g(P) = O exactly when [h2] P = O (gcd(3x^2 - 3, r) = 1).
HD uint32_t cofactor_c0_word(int i) {  // G2_CLEAR_C0 (tools/gen_constants.py derives and checks it)
  return i == 0 ? G2_CLEAR_C0[0] : i == 1 ? G2_CLEAR_C0[1] : i == 2 ? G2_CLEAR_C0[2] : G2_CLEAR_C0[3];
}
HDN void g2_clear_cofactor(G2J& out, const G2A& p) {
  if (p.inf) {
    jac_set_inf(out);
    return;
  }
  G2J pj, t1, t2, t3;
  jac_from_aff(pj, p);
  jac_mul_u64(t1, p, BLS_X_ABS);
  jac_neg(t1, t1);  // t1 = [x] P  (x < 0)
  G2A ps;           // psi(P)
  g2_psi(ps.x, ps.y, p);
  ps.inf = 0;
  jac_dbl(t3, pj);
  g2j_psi(t3, t3);
  g2j_psi(t3, t3);  // psi^2(2P)
  {
    G2A nps;
    aff_neg(nps, ps);
    jac_add_aff(t3, t3, nps);  // psi^2(2P) - psi(P)
  }
  jac_add_aff(t2, t1, ps);        // [x] P + psi(P)
  jac_mul_u64_jac(t2, t2, BLS_X_ABS);
  jac_neg(t2, t2);                // [x^2] P + [x] psi(P)
  jac_add(t3, t3, t2);
  {
    G2J nt1;
    jac_neg(nt1, t1);
    jac_add(t3, t3, nt1);
  }
  {
    G2A np;
    aff_neg(np, p);
    jac_add_aff(t3, t3, np);  // Q = g(P)
  }
  if (jac_is_inf(t3)) {
    out = t3;
    return;
  }
  G2J mq = t3;  // m(Q) = (zeta X, Y, Z)
  {
    Fq zeta;
    fq_set(zeta, G2_ZETA);
    fq_mul(mq.x.c0, t3.x.c0, zeta);
    fq_mul(mq.x.c1, t3.x.c1, zeta);
  }
  G2J bj;
  jac_add(bj, t3, mq);  // B = Q + m(Q) = [1 - x^2] Q != O
  G2A b;
  {
    Fq2 zi, zi2, zi3;
    finv_fast(zi, bj.z);
    fsqr(zi2, zi);
    fmul(zi3, zi2, zi);
    fmul(b.x, bj.x, zi2);
    fmul(b.y, bj.y, zi3);
    b.inf = 0;
  }
  G2J acc;
  jac_from_aff(acc, b);  // bit 126 of c0
  for (int bit = 125; bit >= 0; --bit) {
    jac_dbl(acc, acc);
    if ((cofactor_c0_word(bit >> 5) >> (bit & 31)) & 1u) jac_add_aff(acc, acc, b);
  }
  jac_add(out, acc, mq);
}

// ---------------------------------------------------------------- codec
// big-endian 48 bytes (as 12 big-endian 32-bit words, first word most significant) <-> limbs
HD void fq_from_be_words(Fq& r, const uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint32_t x = w[11 - i];
    r.v[i] = (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
  }
}
HD void fq_to_be_words(uint32_t* w, const Fq& a) {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint32_t x = a.v[11 - i];
    w[i] = (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
  }
}

// Flags live in the first byte = the low byte of word 0 (little-endian load of BE bytes).
enum : uint32_t { FLAG_COMPRESSED = 0x80u, FLAG_INFINITY = 0x40u, FLAG_LARGEST = 0x20u };

// G1Compressed::into_affine.  w = the 48 input bytes as 12 little-endian-loaded words.
HDN bool g1_decompress(G1A& out, const uint32_t* w_in, bool check_subgroup = true) {
  uint32_t w[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) w[i] = w_in[i];
  const uint32_t flags = w[0] & 0xffu;
  fq_zero(out.x);
  fq_zero(out.y);
  out.inf = 0;
  if (!(flags & FLAG_COMPRESSED)) return false;
  if (flags & FLAG_INFINITY) {
    uint32_t acc = (w[0] & ~0xc0u);
#pragma unroll
    for (int i = 1; i < 12; ++i) acc |= w[i];
    out.inf = 1;
    return acc == 0;
  }
  const bool greatest = (flags & FLAG_LARGEST) != 0;
  w[0] &= ~0xe0u;
  Fq xc;
  fq_from_be_words(xc, w);
  if (!limbs_lt_const<12>(xc, FQ_P)) return false;
  Fq x, rhs, b, y;
  fq_to_mont(x, xc);
  fq_sqr(rhs, x);
  fq_mul(rhs, rhs, x);
  fq_set(b, G1_B);
  fq_add(rhs, rhs, b);
  if (!fq_sqrt(y, rhs)) return false;
  // choose y if (y < -y) ^ greatest, else -y   (pairing 0.14 get_point_from_x)
  const bool y_largest = fq_is_lex_largest(y);  // y > -y
  if (y_largest != greatest) fq_neg(y, y);
  out.x = x;
  fq_canon(out.y, y);
  fq_canon(out.x, out.x);
  return !check_subgroup || g1_in_subgroup(out);
}

// G1Compressed::into_affine returning also t1 = [|x|] P from the subgroup test (the x-adic RLC
// table: [x] P = -t1).  t1 is infinity for the point at infinity.
HDN bool g1_decompress_t1(G1A& out, G1J& t1, const uint32_t* w_in) {
  jac_set_inf(t1);
  if (!g1_decompress(out, w_in, false)) return false;
  return g1_in_subgroup_t1(out, t1);
}

HDN bool g2_decompress(G2A& out, const uint32_t* w_in, bool check_subgroup = true) {
  uint32_t w[24];
#pragma unroll
  for (int i = 0; i < 24; ++i) w[i] = w_in[i];
  const uint32_t flags = w[0] & 0xffu;
  fq2_zero(out.x);
  fq2_zero(out.y);
  out.inf = 0;
  if (!(flags & FLAG_COMPRESSED)) return false;
  if (flags & FLAG_INFINITY) {
    uint32_t acc = (w[0] & ~0xc0u);
#pragma unroll
    for (int i = 1; i < 24; ++i) acc |= w[i];
    out.inf = 1;
    return acc == 0;
  }
  const bool greatest = (flags & FLAG_LARGEST) != 0;
  w[0] &= ~0xe0u;
  Fq x1c, x0c;
  fq_from_be_words(x1c, w);       // x.c1 first
  fq_from_be_words(x0c, w + 12);  // then x.c0
  if (!limbs_lt_const<12>(x0c, FQ_P) || !limbs_lt_const<12>(x1c, FQ_P)) return false;
  Fq2 x, rhs, b, y;
  fq_to_mont(x.c0, x0c);
  fq_to_mont(x.c1, x1c);
  fq2_sqr(rhs, x);
  fq2_mul(rhs, rhs, x);
  fq2_set(b, G2_B);
  fq2_add(rhs, rhs, b);
  if (!fq2_sqrt(y, rhs)) return false;
  const bool y_largest = fq2_is_lex_largest(y);
  if (y_largest != greatest) fq2_neg(y, y);
  fq_canon(out.x.c0, x.c0);
  fq_canon(out.x.c1, x.c1);
  fq_canon(out.y.c0, y.c0);
  fq_canon(out.y.c1, y.c1);
  return !check_subgroup || g2_in_subgroup(out);
}

// G1Compressed::from_affine -> 12 words (to be stored little-endian => BE bytes)
HDN void g1_compress(uint32_t* w, const G1A& p) {
  if (p.inf) {
#pragma unroll
    for (int i = 0; i < 12; ++i) w[i] = 0;
    w[0] = 0xc0u;
    return;
  }
  Fq xc;
  fq_from_mont(xc, p.x);
  fq_to_be_words(w, xc);
  uint32_t f = FLAG_COMPRESSED;
  if (fq_is_lex_largest(p.y)) f |= FLAG_LARGEST;
  w[0] |= f;
}

HDN void g2_compress(uint32_t* w, const G2A& p) {
  if (p.inf) {
#pragma unroll
    for (int i = 0; i < 24; ++i) w[i] = 0;
    w[0] = 0xc0u;
    return;
  }
  Fq c;
  fq_from_mont(c, p.x.c1);
  fq_to_be_words(w, c);
  fq_from_mont(c, p.x.c0);
  fq_to_be_words(w + 12, c);
  uint32_t f = FLAG_COMPRESSED;
  if (fq2_is_lex_largest(p.y)) f |= FLAG_LARGEST;
  w[0] |= f;
}

// G2Uncompressed::from_affine (192 bytes = 48 words: x.c1, x.c0, y.c1, y.c0)
HD void g2_uncompress_words(uint32_t* w, const G2A& p) {
  if (p.inf) {
#pragma unroll
    for (int i = 0; i < 48; ++i) w[i] = 0;
    w[0] = 0x40u;
    return;
  }
  Fq c;
  fq_from_mont(c, p.x.c1);
  fq_to_be_words(w, c);
  fq_from_mont(c, p.x.c0);
  fq_to_be_words(w + 12, c);
  fq_from_mont(c, p.y.c1);
  fq_to_be_words(w + 24, c);
  fq_from_mont(c, p.y.c0);
  fq_to_be_words(w + 36, c);
}

// Signature::parity: popcount parity of the XOR of all 192 uncompressed bytes
HD uint32_t g2_parity(const G2A& p) {
  uint32_t w[48];
  g2_uncompress_words(w, p);
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 48; ++i) x ^= w[i];
  x ^= x >> 16;
  x ^= x >> 8;
  x &= 0xffu;
  return __builtin_popcount(x) & 1u;
}

HD uint32_t point_parity(const G1A&) { return 0; }
HD uint32_t point_parity(const G2A& p) { return g2_parity(p); }

}  // namespace hbtc
