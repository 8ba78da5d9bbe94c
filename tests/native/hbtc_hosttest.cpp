// Host build of the SAME arithmetic headers the gfx950 kernels use (hbbft_amd/csrc/*.h),
// exposed through a tiny C ABI so the CPU test suite can check the kernel arithmetic
// against the Python oracle without a GPU.  Test infrastructure only: never linked into
// the product library.
#include <cstring>

#include "pairing.h"

using namespace hbtc;

namespace {

void load_words(uint32_t* w, const uint8_t* b, int nwords) {
  for (int i = 0; i < nwords; ++i)
    w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
           ((uint32_t)b[4 * i + 3] << 24);
}
void store_words(uint8_t* b, const uint32_t* w, int nwords) {
  for (int i = 0; i < nwords; ++i) {
    b[4 * i] = (uint8_t)w[i];
    b[4 * i + 1] = (uint8_t)(w[i] >> 8);
    b[4 * i + 2] = (uint8_t)(w[i] >> 16);
    b[4 * i + 3] = (uint8_t)(w[i] >> 24);
  }
}
void fq_store_be(uint8_t* out, const Fq& a) {  // a in Montgomery form
  Fq c;
  fq_from_mont(c, a);
  uint32_t w[12];
  fq_to_be_words(w, c);
  store_words(out, w, 12);
}
void fq12_store(uint8_t* out, const Fq12& f) {
  const Fq6* s[2] = {&f.c0, &f.c1};
  int k = 0;
  for (int i = 0; i < 2; ++i) {
    const Fq2* c[3] = {&s[i]->c0, &s[i]->c1, &s[i]->c2};
    for (int j = 0; j < 3; ++j) {
      fq_store_be(out + 48 * (k++), c[j]->c0);
      fq_store_be(out + 48 * (k++), c[j]->c1);
    }
  }
}

struct HostLines {
  const Line* l;
  void load(Line& out, int j) const { out = l[j]; }
};

}  // namespace

extern "C" {

int ht_g1_decompress(const uint8_t* in48, uint8_t* out_x48, uint8_t* out_y48) {
  uint32_t w[12];
  load_words(w, in48, 12);
  G1A p;
  if (!g1_decompress(p, w)) return -1;
  if (p.inf) return 1;
  fq_store_be(out_x48, p.x);
  fq_store_be(out_y48, p.y);
  return 0;
}

int ht_g2_decompress(const uint8_t* in96, uint8_t* out192) {
  uint32_t w[24];
  load_words(w, in96, 24);
  G2A p;
  if (!g2_decompress(p, w)) return -1;
  if (p.inf) return 1;
  uint32_t u[48];
  g2_uncompress_words(u, p);
  store_words(out192, u, 48);
  return 0;
}

// decompress -> compress round trip (exercises the encoder)
int ht_g1_roundtrip(const uint8_t* in48, uint8_t* out48) {
  uint32_t w[12];
  load_words(w, in48, 12);
  G1A p;
  if (!g1_decompress(p, w)) return -1;
  g1_compress(w, p);
  store_words(out48, w, 12);
  return 0;
}
int ht_g2_roundtrip(const uint8_t* in96, uint8_t* out96) {
  uint32_t w[24];
  load_words(w, in96, 24);
  G2A p;
  if (!g2_decompress(p, w)) return -1;
  g2_compress(w, p);
  store_words(out96, w, 24);
  return 0;
}

// [k] P in G1 / G2, scalar as 32 little-endian bytes (canonical)
int ht_g1_mul(const uint8_t* in48, const uint8_t* k32, uint8_t* out48) {
  uint32_t w[12];
  load_words(w, in48, 12);
  G1A p;
  if (!g1_decompress(p, w)) return -1;
  Fr k;
  load_words(k.v, k32, 8);
  G1J r;
  jac_mul_fr(r, p, k);
  G1A a;
  jac_to_aff(a, r);
  g1_compress(w, a);
  store_words(out48, w, 12);
  return 0;
}
// [a] P + [b] phi(P) with 32-bit a, b (the RLC item's r_i d_i, hbtc_rlc.hip)
int ht_g1_mul_glv32(const uint8_t* in48, uint32_t a, uint32_t b, uint8_t* out48) {
  uint32_t w[12];
  load_words(w, in48, 12);
  G1A p;
  if (!g1_decompress(p, w)) return -1;
  G1A pp;
  g1_phi(pp, p);
  G1J r;
  jac_mul2_u32(r, p, a, pp, b);
  G1A o;
  jac_to_aff(o, r);
  g1_compress(w, o);
  store_words(out48, w, 12);
  return 0;
}
// The x-adic RLC scalar (curve.h xadic_mul_uniform): [d0 + d1 x + d2 mu + d3 mu x] P, mu = -x^2,
// digits of nbits bits; G1 with [x] P from the subgroup test, G2 with psi(P)
int ht_g1_mul_xadic(const uint8_t* in48, const uint32_t* d, int nbits, uint8_t* out48) {
  uint32_t w[12];
  load_words(w, in48, 12);
  G1A p;
  G1J t1;
  if (!g1_decompress_t1(p, t1, w)) return -1;
  jac_neg(t1, t1);
  G1A xp, pxp;
  xadic_table(xp, pxp, p, t1);
  Fq beta;
  fq_set(beta, G1_BETA);
  G1J r;
  xadic_mul_uniform(r, p, xp, pxp, beta, d[0], d[1], d[2], d[3], nbits);
  G1A o;
  jac_to_aff(o, r);
  g1_compress(w, o);
  store_words(out48, w, 12);
  return 0;
}
int ht_g2_mul_xadic(const uint8_t* in96, const uint32_t* d, int nbits, uint8_t* out96) {
  uint32_t w[24];
  load_words(w, in96, 24);
  G2A p;
  if (!g2_decompress(p, w)) return -1;
  G2A xp, pxp;
  g2_psi(xp.x, xp.y, p);
  xp.inf = 0;
  G2J xj;
  jac_from_aff(xj, xp);
  xadic_table(xp, pxp, p, xj);
  Fq zeta;
  fq_set(zeta, G2_ZETA);
  G2J r;
  xadic_mul_uniform(r, p, xp, pxp, zeta, d[0], d[1], d[2], d[3], nbits);
  G2A o;
  jac_to_aff(o, r);
  g2_compress(w, o);
  store_words(out96, w, 24);
  return 0;
}
// the same loop over the table held in an LDS-layout buffer (curve.h xadic_mul_uniform_lds:
// k_sig_items' form), lane 7 of 64
int ht_g2_mul_xadic_lds(const uint8_t* in96, const uint32_t* d, int nbits, uint8_t* out96) {
  uint32_t w[24];
  load_words(w, in96, 24);
  G2A p;
  if (!g2_decompress(p, w)) return -1;
  G2A xp, pxp;
  g2_psi(xp.x, xp.y, p);
  xp.inf = 0;
  G2J xj;
  jac_from_aff(xj, xp);
  xadic_table(xp, pxp, p, xj);
  Fq zeta;
  fq_set(zeta, G2_ZETA);
  static uint32_t lds[3 * 48 * 64];
  xy_lds_put_aff(lds, 7, 0, p);
  xy_lds_put_aff(lds, 7, 1, xp);
  xy_lds_put_aff(lds, 7, 2, pxp);
  G2J r;
  xadic_mul_uniform_lds(r, lds, 7, zeta, d[0], d[1], d[2], d[3], nbits);
  G2A o;
  jac_to_aff(o, r);
  g2_compress(w, o);
  store_words(out96, w, 24);
  return 0;
}
// the sign-aligned 8-entry form (curve.h xadic_mul_sac8) of the same scalar
int ht_g1_mul_xadic8(const uint8_t* in48, const uint32_t* d, int nbits, uint8_t* out48) {
  uint32_t w[12];
  load_words(w, in48, 12);
  G1A p;
  G1J t1;
  if (!g1_decompress_t1(p, t1, w)) return -1;
  jac_neg(t1, t1);
  Fq beta;
  fq_set(beta, G1_BETA);
  G1J r;
  xadic_mul_sac8(r, p, t1, beta, d[0], d[1], d[2], d[3], nbits);
  G1A o;
  jac_to_aff(o, r);
  g1_compress(w, o);
  store_words(out48, w, 12);
  return 0;
}
// the same with entries 5..7 in an LDS-layout buffer ([entry][word][lane], lane 5 of 64) and the
// co-Z chain build (curve.h xadic_table8_chain: k_rlc_items' form)
int ht_g1_mul_xadic8_lds(const uint8_t* in48, const uint32_t* d, int nbits, uint8_t* out48) {
  uint32_t w[12];
  load_words(w, in48, 12);
  G1A p;
  G1J t1;
  if (!g1_decompress_t1(p, t1, w)) return -1;
  jac_neg(t1, t1);
  Fq beta;
  fq_set(beta, G1_BETA);
  static uint32_t lds[3 * 24 * 64];
  G1J r;
  xadic_mul_sac8<Fq, true>(r, p, t1, beta, d[0], d[1], d[2], d[3], nbits, lds, 5);
  G1A o;
  jac_to_aff(o, r);
  g1_compress(w, o);
  store_words(out48, w, 12);
  return 0;
}
int ht_g2_mul_xadic8_lds(const uint8_t* in96, const uint32_t* d, int nbits, uint8_t* out96) {
  uint32_t w[24];
  load_words(w, in96, 24);
  G2A p;
  if (!g2_decompress(p, w)) return -1;
  G2A xp;
  g2_psi(xp.x, xp.y, p);
  xp.inf = 0;
  G2J xj;
  jac_from_aff(xj, xp);
  Fq zeta;
  fq_set(zeta, G2_ZETA);
  static uint32_t lds[3 * 48 * 64];
  G2J r;
  xadic_mul_sac8<Fq2, true>(r, p, xj, zeta, d[0], d[1], d[2], d[3], nbits, lds, 5);
  G2A o;
  jac_to_aff(o, r);
  g2_compress(w, o);
  store_words(out96, w, 24);
  return 0;
}
int ht_g2_mul_xadic8(const uint8_t* in96, const uint32_t* d, int nbits, uint8_t* out96) {
  uint32_t w[24];
  load_words(w, in96, 24);
  G2A p;
  if (!g2_decompress(p, w)) return -1;
  G2A xp;
  g2_psi(xp.x, xp.y, p);
  xp.inf = 0;
  G2J xj;
  jac_from_aff(xj, xp);
  Fq zeta;
  fq_set(zeta, G2_ZETA);
  G2J r;
  xadic_mul_sac8(r, p, xj, zeta, d[0], d[1], d[2], d[3], nbits);
  G2A o;
  jac_to_aff(o, r);
  g2_compress(w, o);
  store_words(out96, w, 24);
  return 0;
}
// the two-digit sign-aligned form of the small combines (curve.h sac2_mul): [d0] P + [d1] [u] P
int ht_g1_mul_sac2(const uint8_t* in48, uint64_t d0, uint64_t d1, uint8_t* out48) {
  uint32_t w[12];
  load_words(w, in48, 12);
  G1A p;
  if (!g1_decompress(p, w)) return -1;
  G1J xj;
  jac_mul_u64(xj, p, BLS_X_ABS);
  G1J r;
  sac2_mul(r, p, xj, d0, d1, 64);
  G1A o;
  jac_to_aff(o, r);
  g1_compress(w, o);
  store_words(out48, w, 12);
  return 0;
}
int ht_g2_mul_sac2(const uint8_t* in96, uint64_t d0, uint64_t d1, uint8_t* out96) {
  uint32_t w[24];
  load_words(w, in96, 24);
  G2A p;
  if (!g2_decompress(p, w)) return -1;
  G2A xp;
  g2_psi(xp.x, xp.y, p);
  fq2_neg(xp.y, xp.y);  // [u] P = -psi(P)
  xp.inf = 0;
  G2J xj;
  jac_from_aff(xj, xp);
  G2J r;
  sac2_mul(r, p, xj, d0, d1, 64);
  G2A o;
  jac_to_aff(o, r);
  g2_compress(w, o);
  store_words(out96, w, 24);
  return 0;
}
int ht_g2_mul(const uint8_t* in96, const uint8_t* k32, uint8_t* out96) {
  uint32_t w[24];
  load_words(w, in96, 24);
  G2A p;
  if (!g2_decompress(p, w)) return -1;
  Fr k;
  load_words(k.v, k32, 8);
  G2J r;
  jac_mul_fr(r, p, k);
  G2A a;
  jac_to_aff(a, r);
  g2_compress(w, a);
  store_words(out96, w, 24);
  return 0;
}

// Miller loop f_{|x|,Q}(P) (conjugated) via precomputed lines, and the final exponentiation
int ht_miller(const uint8_t* p48, const uint8_t* q96, uint8_t* out576) {
  uint32_t w[24];
  load_words(w, p48, 12);
  G1A P;
  if (!g1_decompress(P, w)) return -1;
  load_words(w, q96, 24);
  G2A Q;
  if (!g2_decompress(Q, w)) return -1;
  static Line lines[MILLER_STEPS];
  g2_precompute_lines(lines, Q);
  HostLines L{lines};
  Fq12 f;
  miller_loop_2(f, L, P, !P.inf && !Q.inf, L, P, false);
  fq12_store(out576, f);
  return 0;
}

int ht_pairing(const uint8_t* p48, const uint8_t* q96, uint8_t* out576) {
  uint32_t w[24];
  load_words(w, p48, 12);
  G1A P;
  if (!g1_decompress(P, w)) return -1;
  load_words(w, q96, 24);
  G2A Q;
  if (!g2_decompress(Q, w)) return -1;
  static Line lines[MILLER_STEPS];
  g2_precompute_lines(lines, Q);
  HostLines L{lines};
  Fq12 f, e;
  miller_loop_2(f, L, P, !P.inf && !Q.inf, L, P, false);
  final_exponentiation(e, f);
  fq12_store(out576, e);
  return 0;
}

// e(p1, q1) == e(p2, q2) ?   via e(p1,q1) * e(-p2,q2) == 1 with precomputed lines
int ht_pairing_eq(const uint8_t* p1, const uint8_t* q1, const uint8_t* p2, const uint8_t* q2) {
  uint32_t w[24];
  G1A P1, P2;
  G2A Q1, Q2;
  load_words(w, p1, 12);
  if (!g1_decompress(P1, w)) return -1;
  load_words(w, p2, 12);
  if (!g1_decompress(P2, w)) return -1;
  load_words(w, q1, 24);
  if (!g2_decompress(Q1, w)) return -1;
  load_words(w, q2, 24);
  if (!g2_decompress(Q2, w)) return -1;
  static Line l1[MILLER_STEPS], l2[MILLER_STEPS];
  if (!Q1.inf) g2_precompute_lines(l1, Q1);
  if (!Q2.inf) g2_precompute_lines(l2, Q2);
  G1A nP2;
  aff_neg(nP2, P2);
  Fq12 f, e;
  miller_loop_2(f, HostLines{l1}, P1, !P1.inf && !Q1.inf, HostLines{l2}, nP2, !P2.inf && !Q2.inf);
  final_exponentiation(e, f);
  return fq12_is_one(e) ? 1 : 0;
}

// same check with Q2's lines computed on the fly (signature-share kernel structure)
int ht_pairing_eq_var(const uint8_t* p1, const uint8_t* q1, const uint8_t* p2, const uint8_t* q2) {
  uint32_t w[24];
  G1A P1, P2;
  G2A Q1, Q2;
  load_words(w, p1, 12);
  if (!g1_decompress(P1, w)) return -1;
  load_words(w, p2, 12);
  if (!g1_decompress(P2, w)) return -1;
  load_words(w, q1, 24);
  if (!g2_decompress(Q1, w)) return -1;
  load_words(w, q2, 24);
  if (!g2_decompress(Q2, w)) return -1;
  static Line l1[MILLER_STEPS];
  if (!Q1.inf) g2_precompute_lines(l1, Q1);
  G1A nP2;
  aff_neg(nP2, P2);
  Fq12 f, e;
  miller_loop_fixed_var(f, HostLines{l1}, P1, !P1.inf && !Q1.inf, nP2, Q2, !P2.inf && !Q2.inf);
  final_exponentiation(e, f);
  return fq12_is_one(e) ? 1 : 0;
}

// subgroup test on an on-curve point given uncompressed (x, y) canonical BE (G1: 96 bytes)
int ht_g1_subgroup_xy(const uint8_t* xy96) {
  uint32_t w[12];
  G1A p;
  Fq c;
  load_words(w, xy96, 12);
  fq_from_be_words(c, w);
  fq_to_mont(p.x, c);
  load_words(w, xy96 + 48, 12);
  fq_from_be_words(c, w);
  fq_to_mont(p.y, c);
  p.inf = 0;
  return g1_in_subgroup(p) ? 1 : 0;
}
int ht_g2_subgroup_xy(const uint8_t* xy192) {  // x.c1, x.c0, y.c1, y.c0
  uint32_t w[12];
  G2A p;
  Fq c;
  const uint8_t* src[4] = {xy192, xy192 + 48, xy192 + 96, xy192 + 144};
  Fq* dst[4] = {&p.x.c1, &p.x.c0, &p.y.c1, &p.y.c0};
  for (int i = 0; i < 4; ++i) {
    load_words(w, src[i], 12);
    fq_from_be_words(c, w);
    fq_to_mont(*dst[i], c);
  }
  p.inf = 0;
  return g2_in_subgroup(p) ? 1 : 0;
}

// Fr helpers: r = a * b^{-1} mod r (canonical 32-byte LE)
void ht_fr_div(const uint8_t* a32, const uint8_t* b32, uint8_t* out32) {
  Fr a, b, am, bm, bi, r, rc;
  load_words(a.v, a32, 8);
  load_words(b.v, b32, 8);
  fr_to_mont(am, a);
  fr_to_mont(bm, b);
  fr_inv(bi, bm);
  fr_mul(r, am, bi);
  fr_from_mont(rc, r);
  store_words(out32, rc.v, 8);
}

}  // extern "C"
