/* threshold_crypto @ 0.1.0-rng-fix / pairing 0.14.2 restated in plain C — TEST ORACLE AND CPU
 * BASELINE ONLY.  Never linked into the product (hbbft_amd/libhbtc.so); only tests/, smoke()
 * and bench.py's cpu_baseline leg load it (via oracle/cbaseline.py).
 *
 * The crates are external to /root/reference (Cargo.toml:27,33; not vendored, no Rust
 * toolchain here), so this follows their published algorithms [EXT-UNVERIFIED]:
 *   * pairing 0.14 bls12_381: Fq as 6 x u64 Montgomery limbs (the `u128-support` feature's
 *     widening multiply), Fq2/Fq6/Fq12 tower (u^2 = -1, v^3 = u + 1, w^2 = v), G1/G2 in
 *     Jacobian coordinates, `G2Prepared` line coefficients (doubling_step / addition_step in
 *     Jacobian coordinates, Algorithms 26/27 of eprint 2010/354) evaluated with `ell` =
 *     mul_by_014, `miller_loop`, `final_exponentiation` (Fuentes-Castaneda et al. chain with
 *     generic Fq12 exponentiation by x), scalar multiplication by double-and-add, zcash codec,
 *     subgroup check [r]P == O on decode.
 *   * threshold_crypto 0.1: hash_g2 (SHA3-256 -> ChaCha20 rand 0.4 -> G2::rand), hash_g1_g2,
 *     PublicKeyShare::verify_decryption_share = two full pairings compared (called per share,
 *     hbbft src/threshold_decryption.rs:159), PublicKeySet::decrypt interpolation.
 * A completely independent restatement from the product kernels (64-bit limbs, different line
 * and final-exponentiation formulas) so that agreement is evidence, not self-consistency.
 *
 * Baseline entry points time the reference's per-call algorithm ("faithful": per share serde
 * decode + hash_g1_g2 + 2 pairings) and an optimized CPU variant (hash once per ciphertext,
 * one 2-pair multi-Miller loop + one final exponentiation), over a pthread pool.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef unsigned __int128 u128;

/* ============================================================================ Fq */
typedef struct { uint64_t v[6]; } fp; /* Montgomery form, canonical [0, p) */

static const uint64_t P[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                              0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static uint64_t PINV; /* -p^-1 mod 2^64 */
static fp FP_ONE, FP_R2, FP_ZERO;
static uint64_t EXP_PM2[6], EXP_SQRT[6], EXP_PM3_4[6], EXP_PM1_2[6], HALF_P[6];

static int ge_p(const uint64_t* a) {
  for (int i = 5; i >= 0; --i) {
    if (a[i] > P[i]) return 1;
    if (a[i] < P[i]) return 0;
  }
  return 1;
}
static void sub_p(uint64_t* a) {
  u128 b = 0;
  for (int i = 0; i < 6; ++i) {
    u128 d = (u128)a[i] - P[i] - b;
    a[i] = (uint64_t)d;
    b = (d >> 64) & 1;
  }
}
static void fp_add(fp* r, const fp* a, const fp* b) {
  u128 c = 0;
  uint64_t t[6];
  for (int i = 0; i < 6; ++i) {
    c += (u128)a->v[i] + b->v[i];
    t[i] = (uint64_t)c;
    c >>= 64;
  }
  if (ge_p(t)) sub_p(t);
  memcpy(r->v, t, 48);
}
static void fp_sub(fp* r, const fp* a, const fp* b) {
  u128 br = 0;
  uint64_t t[6];
  for (int i = 0; i < 6; ++i) {
    u128 d = (u128)a->v[i] - b->v[i] - br;
    t[i] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  if (br) {
    u128 c = 0;
    for (int i = 0; i < 6; ++i) {
      c += (u128)t[i] + P[i];
      t[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  memcpy(r->v, t, 48);
}
static void fp_dbl(fp* r, const fp* a) { fp_add(r, a, a); }
static int fp_is_zero(const fp* a) {
  return (a->v[0] | a->v[1] | a->v[2] | a->v[3] | a->v[4] | a->v[5]) == 0;
}
static int fp_eq(const fp* a, const fp* b) { return memcmp(a->v, b->v, 48) == 0; }
static void fp_neg(fp* r, const fp* a) {
  if (fp_is_zero(a)) {
    *r = *a;
    return;
  }
  fp_sub(r, &FP_ZERO, a);
}
static void fp_mul(fp* r, const fp* a, const fp* b) {
  uint64_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 6; ++i) {
    u128 c = 0;
    for (int j = 0; j < 6; ++j) {
      c += (u128)a->v[j] * b->v[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[6];
    t[6] = (uint64_t)c;
    t[7] = (uint64_t)(c >> 64);
    uint64_t m = t[0] * PINV;
    c = (u128)m * P[0] + t[0];
    c >>= 64;
    for (int j = 1; j < 6; ++j) {
      c += (u128)m * P[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[6];
    t[5] = (uint64_t)c;
    t[6] = t[7] + (uint64_t)(c >> 64);
  }
  if (t[6] || ge_p(t)) sub_p(t);
  memcpy(r->v, t, 48);
}
static void fp_sqr(fp* r, const fp* a) { fp_mul(r, a, a); }
static void fp_pow(fp* r, const fp* a, const uint64_t* e, int nlimbs) {
  fp acc = FP_ONE;
  int started = 0;
  for (int i = nlimbs - 1; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      if (started) fp_sqr(&acc, &acc);
      if ((e[i] >> b) & 1) {
        fp_mul(&acc, &acc, a);
        started = 1;
      }
    }
  *r = acc;
}
static void fp_inv(fp* r, const fp* a) { fp_pow(r, a, EXP_PM2, 6); }
static void fp_from_int(fp* r, const uint64_t* x) { /* canonical integer -> Montgomery */
  fp t;
  memcpy(t.v, x, 48);
  fp_mul(r, &t, &FP_R2);
}
static void fp_to_int(uint64_t* x, const fp* a) {
  fp one = {{1, 0, 0, 0, 0, 0}}, t;
  fp_mul(&t, a, &one);
  memcpy(x, t.v, 48);
}
static int fp_sqrt(fp* r, const fp* a) { /* p = 3 mod 4 */
  fp y, y2;
  fp_pow(&y, a, EXP_SQRT, 6);
  fp_sqr(&y2, &y);
  *r = y;
  return fp_eq(&y2, a);
}
static int int_gt(const uint64_t* a, const uint64_t* b) {
  for (int i = 5; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return 0;
}
/* pairing 0.14 Ord on canonical values: a > -a  <=>  a > (p-1)/2 */
static int fp_lex_largest(const fp* a) {
  uint64_t x[6];
  fp_to_int(x, a);
  return int_gt(x, HALF_P);
}
static void be48_to_int(uint64_t* x, const uint8_t* b) {
  for (int i = 0; i < 6; ++i) {
    uint64_t w = 0;
    for (int k = 0; k < 8; ++k) w = (w << 8) | b[8 * (5 - i) + k];
    x[i] = w;
  }
}
static void int_to_be48(uint8_t* b, const uint64_t* x) {
  for (int i = 0; i < 6; ++i)
    for (int k = 0; k < 8; ++k) b[8 * (5 - i) + k] = (uint8_t)(x[i] >> (56 - 8 * k));
}

/* ============================================================================ Fq2 */
typedef struct { fp c0, c1; } fp2;
static fp2 F2_ONE, F2_ZERO;

static void f2_add(fp2* r, const fp2* a, const fp2* b) { fp_add(&r->c0, &a->c0, &b->c0); fp_add(&r->c1, &a->c1, &b->c1); }
static void f2_sub(fp2* r, const fp2* a, const fp2* b) { fp_sub(&r->c0, &a->c0, &b->c0); fp_sub(&r->c1, &a->c1, &b->c1); }
static void f2_dbl(fp2* r, const fp2* a) { f2_add(r, a, a); }
static void f2_neg(fp2* r, const fp2* a) { fp_neg(&r->c0, &a->c0); fp_neg(&r->c1, &a->c1); }
static void f2_conj(fp2* r, const fp2* a) { r->c0 = a->c0; fp_neg(&r->c1, &a->c1); }
static int f2_is_zero(const fp2* a) { return fp_is_zero(&a->c0) && fp_is_zero(&a->c1); }
static int f2_eq(const fp2* a, const fp2* b) { return fp_eq(&a->c0, &b->c0) && fp_eq(&a->c1, &b->c1); }
static void f2_mul(fp2* r, const fp2* a, const fp2* b) {
  fp aa, bb, s, t;
  fp_mul(&aa, &a->c0, &b->c0);
  fp_mul(&bb, &a->c1, &b->c1);
  fp_add(&s, &a->c0, &a->c1);
  fp_add(&t, &b->c0, &b->c1);
  fp_mul(&s, &s, &t);
  fp_sub(&s, &s, &aa);
  fp_sub(&r->c1, &s, &bb);
  fp_sub(&r->c0, &aa, &bb);
}
static void f2_sqr(fp2* r, const fp2* a) {
  fp s, d, m;
  fp_add(&s, &a->c0, &a->c1);
  fp_sub(&d, &a->c0, &a->c1);
  fp_mul(&m, &a->c0, &a->c1);
  fp_mul(&r->c0, &s, &d);
  fp_dbl(&r->c1, &m);
}
static void f2_mul_fp(fp2* r, const fp2* a, const fp* b) { fp_mul(&r->c0, &a->c0, b); fp_mul(&r->c1, &a->c1, b); }
static void f2_mul_nr(fp2* r, const fp2* a) { /* * (u + 1) */
  fp t0, t1;
  fp_sub(&t0, &a->c0, &a->c1);
  fp_add(&t1, &a->c0, &a->c1);
  r->c0 = t0;
  r->c1 = t1;
}
static void f2_inv(fp2* r, const fp2* a) {
  fp t0, t1;
  fp_sqr(&t0, &a->c0);
  fp_sqr(&t1, &a->c1);
  fp_add(&t0, &t0, &t1);
  fp_inv(&t0, &t0);
  fp_mul(&r->c0, &a->c0, &t0);
  fp_mul(&t1, &a->c1, &t0);
  fp_neg(&r->c1, &t1);
}
static void f2_pow(fp2* r, const fp2* a, const uint64_t* e, int nl) {
  fp2 acc = F2_ONE;
  int started = 0;
  for (int i = nl - 1; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      if (started) f2_sqr(&acc, &acc);
      if ((e[i] >> b) & 1) {
        f2_mul(&acc, &acc, a);
        started = 1;
      }
    }
  *r = acc;
}
/* pairing 0.14 Fq2::sqrt (Algorithm 9, eprint 2012/685) */
static int f2_sqrt(fp2* r, const fp2* a) {
  if (f2_is_zero(a)) {
    *r = *a;
    return 1;
  }
  fp2 a1, alpha, a0, minus_one, x0;
  f2_pow(&a1, a, EXP_PM3_4, 6);
  f2_sqr(&alpha, &a1);
  f2_mul(&alpha, &alpha, a);
  f2_conj(&a0, &alpha);
  f2_mul(&a0, &a0, &alpha);
  f2_neg(&minus_one, &F2_ONE);
  if (f2_eq(&a0, &minus_one)) return 0;
  f2_mul(&x0, &a1, a);
  if (f2_eq(&alpha, &minus_one)) {
    fp2 t;
    fp_neg(&t.c0, &x0.c1);
    t.c1 = x0.c0;
    *r = t;
  } else {
    fp2 b;
    f2_add(&alpha, &alpha, &F2_ONE);
    f2_pow(&b, &alpha, EXP_PM1_2, 6);
    f2_mul(r, &b, &x0);
  }
  return 1;
}
/* pairing 0.14 Ord for Fq2: c1 first, then c0; a > -a */
static int f2_lex_largest(const fp2* a) {
  if (!fp_is_zero(&a->c1)) return fp_lex_largest(&a->c1);
  return fp_lex_largest(&a->c0);
}

/* ============================================================================ Fq6, Fq12 */
typedef struct { fp2 c0, c1, c2; } fp6;
typedef struct { fp6 c0, c1; } fp12;
static fp2 FROB6_C1[4], FROB6_C2[4], FROB12_C1[4];

static void f6_add(fp6* r, const fp6* a, const fp6* b) { f2_add(&r->c0, &a->c0, &b->c0); f2_add(&r->c1, &a->c1, &b->c1); f2_add(&r->c2, &a->c2, &b->c2); }
static void f6_sub(fp6* r, const fp6* a, const fp6* b) { f2_sub(&r->c0, &a->c0, &b->c0); f2_sub(&r->c1, &a->c1, &b->c1); f2_sub(&r->c2, &a->c2, &b->c2); }
static void f6_neg(fp6* r, const fp6* a) { f2_neg(&r->c0, &a->c0); f2_neg(&r->c1, &a->c1); f2_neg(&r->c2, &a->c2); }
static void f6_mul_nr(fp6* r, const fp6* a) { /* * v */
  fp2 t;
  f2_mul_nr(&t, &a->c2);
  r->c2 = a->c1;
  r->c1 = a->c0;
  r->c0 = t;
}
static void f6_mul(fp6* r, const fp6* a, const fp6* b) {
  fp2 a_a, b_b, c_c, t1, t2, t3, tmp;
  f2_mul(&a_a, &a->c0, &b->c0);
  f2_mul(&b_b, &a->c1, &b->c1);
  f2_mul(&c_c, &a->c2, &b->c2);
  f2_add(&t1, &b->c1, &b->c2);
  f2_add(&tmp, &a->c1, &a->c2);
  f2_mul(&t1, &t1, &tmp);
  f2_sub(&t1, &t1, &b_b);
  f2_sub(&t1, &t1, &c_c);
  f2_mul_nr(&t1, &t1);
  f2_add(&t1, &t1, &a_a);
  f2_add(&t3, &b->c0, &b->c2);
  f2_add(&tmp, &a->c0, &a->c2);
  f2_mul(&t3, &t3, &tmp);
  f2_sub(&t3, &t3, &a_a);
  f2_add(&t3, &t3, &b_b);
  f2_sub(&t3, &t3, &c_c);
  f2_add(&t2, &b->c0, &b->c1);
  f2_add(&tmp, &a->c0, &a->c1);
  f2_mul(&t2, &t2, &tmp);
  f2_sub(&t2, &t2, &a_a);
  f2_sub(&t2, &t2, &b_b);
  f2_mul_nr(&tmp, &c_c);
  f2_add(&t2, &t2, &tmp);
  r->c0 = t1;
  r->c1 = t2;
  r->c2 = t3;
}
static void f6_mul_by_1(fp6* r, const fp6* a, const fp2* c1) {
  fp2 b_b, t1, t2;
  f2_mul(&b_b, &a->c1, c1);
  f2_add(&t1, &a->c1, &a->c2);
  f2_mul(&t1, &t1, c1);
  f2_sub(&t1, &t1, &b_b);
  f2_mul_nr(&t1, &t1);
  f2_add(&t2, &a->c0, &a->c1);
  f2_mul(&t2, &t2, c1);
  f2_sub(&t2, &t2, &b_b);
  r->c0 = t1;
  r->c1 = t2;
  r->c2 = b_b;
}
static void f6_mul_by_01(fp6* r, const fp6* a, const fp2* c0, const fp2* c1) {
  fp2 a_a, b_b, t1, t2, t3, tmp;
  f2_mul(&a_a, &a->c0, c0);
  f2_mul(&b_b, &a->c1, c1);
  f2_add(&t1, &a->c1, &a->c2);
  f2_mul(&t1, &t1, c1);
  f2_sub(&t1, &t1, &b_b);
  f2_mul_nr(&t1, &t1);
  f2_add(&t1, &t1, &a_a);
  f2_add(&t3, &a->c0, &a->c2);
  f2_mul(&t3, &t3, c0);
  f2_sub(&t3, &t3, &a_a);
  f2_add(&t3, &t3, &b_b);
  f2_add(&t2, c0, c1);
  f2_add(&tmp, &a->c0, &a->c1);
  f2_mul(&t2, &t2, &tmp);
  f2_sub(&t2, &t2, &a_a);
  f2_sub(&t2, &t2, &b_b);
  r->c0 = t1;
  r->c1 = t2;
  r->c2 = t3;
}
static void f6_inv(fp6* r, const fp6* a) {
  fp2 c0, c1, c2, t, tmp;
  f2_mul_nr(&c0, &a->c2);
  f2_mul(&c0, &c0, &a->c1);
  f2_neg(&c0, &c0);
  f2_sqr(&tmp, &a->c0);
  f2_add(&c0, &c0, &tmp);
  f2_sqr(&c1, &a->c2);
  f2_mul_nr(&c1, &c1);
  f2_mul(&tmp, &a->c0, &a->c1);
  f2_sub(&c1, &c1, &tmp);
  f2_sqr(&c2, &a->c1);
  f2_mul(&tmp, &a->c0, &a->c2);
  f2_sub(&c2, &c2, &tmp);
  f2_mul(&tmp, &a->c2, &c1);
  f2_mul(&t, &a->c1, &c2);
  f2_add(&tmp, &tmp, &t);
  f2_mul_nr(&tmp, &tmp);
  f2_mul(&t, &a->c0, &c0);
  f2_add(&tmp, &tmp, &t);
  f2_inv(&tmp, &tmp);
  f2_mul(&r->c0, &c0, &tmp);
  f2_mul(&r->c1, &c1, &tmp);
  f2_mul(&r->c2, &c2, &tmp);
}
static void f6_frob(fp6* r, const fp6* a, int k) {
  fp2 c0, c1, c2;
  if (k & 1) {
    f2_conj(&c0, &a->c0);
    f2_conj(&c1, &a->c1);
    f2_conj(&c2, &a->c2);
  } else {
    c0 = a->c0;
    c1 = a->c1;
    c2 = a->c2;
  }
  f2_mul(&c1, &c1, &FROB6_C1[k]);
  f2_mul(&c2, &c2, &FROB6_C2[k]);
  r->c0 = c0;
  r->c1 = c1;
  r->c2 = c2;
}

static void f12_one(fp12* r) {
  memset(r, 0, sizeof *r);
  r->c0.c0 = F2_ONE;
}
static void f12_mul(fp12* r, const fp12* a, const fp12* b) {
  fp6 aa, bb, o, t;
  f6_mul(&aa, &a->c0, &b->c0);
  f6_mul(&bb, &a->c1, &b->c1);
  f6_add(&o, &b->c0, &b->c1);
  f6_add(&t, &a->c1, &a->c0);
  f6_mul(&t, &t, &o);
  f6_sub(&t, &t, &aa);
  f6_sub(&r->c1, &t, &bb);
  f6_mul_nr(&bb, &bb);
  f6_add(&r->c0, &bb, &aa);
}
static void f12_sqr(fp12* r, const fp12* a) {
  fp6 ab, c0c1, t;
  f6_mul(&ab, &a->c0, &a->c1);
  f6_add(&c0c1, &a->c0, &a->c1);
  f6_mul_nr(&t, &a->c1);
  f6_add(&t, &t, &a->c0);
  f6_mul(&t, &t, &c0c1);
  f6_sub(&t, &t, &ab);
  f6_mul_nr(&c0c1, &ab);
  f6_sub(&r->c0, &t, &c0c1);
  f6_add(&r->c1, &ab, &ab);
}
static void f12_conj(fp12* r, const fp12* a) {
  r->c0 = a->c0;
  f6_neg(&r->c1, &a->c1);
}
static void f12_inv(fp12* r, const fp12* a) {
  fp6 c0s, c1s;
  f6_mul(&c0s, &a->c0, &a->c0);
  f6_mul(&c1s, &a->c1, &a->c1);
  f6_mul_nr(&c1s, &c1s);
  f6_sub(&c0s, &c0s, &c1s);
  f6_inv(&c0s, &c0s);
  f6_mul(&r->c0, &a->c0, &c0s);
  f6_mul(&c1s, &a->c1, &c0s);
  f6_neg(&r->c1, &c1s);
}
static void f12_frob(fp12* r, const fp12* a, int k) {
  fp6 c0, c1;
  f6_frob(&c0, &a->c0, k);
  f6_frob(&c1, &a->c1, k);
  f2_mul(&c1.c0, &c1.c0, &FROB12_C1[k]);
  f2_mul(&c1.c1, &c1.c1, &FROB12_C1[k]);
  f2_mul(&c1.c2, &c1.c2, &FROB12_C1[k]);
  r->c0 = c0;
  r->c1 = c1;
}
/* pairing 0.14 Fq12::mul_by_014 */
static void f12_mul_by_014(fp12* f, const fp2* c0, const fp2* c1, const fp2* c4) {
  fp6 aa, bb, t;
  fp2 o;
  f6_mul_by_01(&aa, &f->c0, c0, c1);
  f6_mul_by_1(&bb, &f->c1, c4);
  f2_add(&o, c1, c4);
  f6_add(&t, &f->c1, &f->c0);
  f6_mul_by_01(&t, &t, c0, &o);
  f6_sub(&t, &t, &aa);
  f6_sub(&f->c1, &t, &bb);
  f6_mul_nr(&bb, &bb);
  f6_add(&f->c0, &bb, &aa);
}
static int f12_eq(const fp12* a, const fp12* b) { return memcmp(a, b, sizeof *a) == 0; }

/* ============================================================================ curves */
typedef struct { fp x, y; int inf; } g1a;
typedef struct { fp x, y, z; } g1j;
typedef struct { fp2 x, y; int inf; } g2a;
typedef struct { fp2 x, y, z; } g2j;
static fp B1;  /* 4 */
static fp2 B2; /* 4(u+1) */
static g1a G1GEN;
static g2a G2GEN;
static const uint64_t R_ORDER[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                                    0x73eda753299d7d48ULL};
static const uint64_t BLS_X = 0xd201000000010000ULL; /* |x|, x negative */
/* G2 cofactor h2 (pairing 0.14 scale_by_cofactor) */
static const uint64_t H2[8] = {0xcf1c38e31c7238e5ULL, 0x1616ec6e786f0c70ULL, 0x21537e293a6691aeULL,
                               0xa628f1cb4d9e82efULL, 0xa68a205b2e5a7ddfULL, 0xcd91de4547085abaULL,
                               0x91d50792876a202ULL, 0x5d543a95414e7f1ULL};

#define DEFINE_JAC(G, F, FA, FS, FM, FSQ, FD, FZ, FNEG, FONE, FZERO, FINV)                       \
  static void G##_set_inf(G##j* r) { r->x = FONE; r->y = FONE; r->z = FZERO; }                   \
  static int G##_is_inf(const G##j* p) { return FZ(&p->z); }                                      \
  static void G##_dbl(G##j* r, const G##j* p) {                                                   \
    if (G##_is_inf(p)) { *r = *p; return; }                                                       \
    __typeof__(p->x) a, b, c, d, e, f, t;                                                          \
    FSQ(&a, &p->x); FSQ(&b, &p->y); FSQ(&c, &b);                                                   \
    FA(&d, &p->x, &b); FSQ(&d, &d); FS(&d, &d, &a); FS(&d, &d, &c); FD(&d, &d);                   \
    FD(&e, &a); FA(&e, &e, &a); FSQ(&f, &e);                                                       \
    FM(&r->z, &p->z, &p->y); FD(&r->z, &r->z);                                                     \
    FD(&t, &d); FS(&r->x, &f, &t);                                                                 \
    FS(&t, &d, &r->x); FM(&r->y, &t, &e); FD(&c, &c); FD(&c, &c); FD(&c, &c);                     \
    FS(&r->y, &r->y, &c);                                                                          \
  }                                                                                                \
  static void G##_add(G##j* r, const G##j* p, const G##j* q) {                                    \
    if (G##_is_inf(p)) { *r = *q; return; }                                                       \
    if (G##_is_inf(q)) { *r = *p; return; }                                                       \
    __typeof__(p->x) z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;                               \
    FSQ(&z1z1, &p->z); FSQ(&z2z2, &q->z);                                                          \
    FM(&u1, &p->x, &z2z2); FM(&u2, &q->x, &z1z1);                                                  \
    FM(&s1, &p->y, &q->z); FM(&s1, &s1, &z2z2); FM(&s2, &q->y, &p->z); FM(&s2, &s2, &z1z1);       \
    if (FEQ(&u1, &u2)) {                                                                           \
      if (FEQ(&s1, &s2)) { G##_dbl(r, p); } else { G##_set_inf(r); }                               \
      return;                                                                                      \
    }                                                                                              \
    FS(&h, &u2, &u1); FD(&i, &h); FSQ(&i, &i); FM(&j, &h, &i);                                     \
    FS(&rr, &s2, &s1); FD(&rr, &rr); FM(&v, &u1, &i);                                              \
    __typeof__(p->x) x3, y3, z3;                                                                   \
    FSQ(&x3, &rr); FS(&x3, &x3, &j); FD(&t, &v); FS(&x3, &x3, &t);                                \
    FS(&t, &v, &x3); FM(&y3, &rr, &t); FM(&t, &s1, &j); FD(&t, &t); FS(&y3, &y3, &t);             \
    FA(&z3, &p->z, &q->z); FSQ(&z3, &z3); FS(&z3, &z3, &z1z1); FS(&z3, &z3, &z2z2);               \
    FM(&z3, &z3, &h);                                                                              \
    r->x = x3; r->y = y3; r->z = z3;                                                               \
  }                                                                                                \
  static void G##_from_aff(G##j* r, const G##a* a) {                                              \
    if (a->inf) { G##_set_inf(r); return; }                                                       \
    r->x = a->x; r->y = a->y; r->z = FONE;                                                         \
  }                                                                                                \
  static void G##_to_aff(G##a* r, const G##j* p) {                                                \
    if (G##_is_inf(p)) { r->x = FZERO; r->y = FZERO; r->inf = 1; return; }                       \
    __typeof__(p->x) zi, zi2;                                                                      \
    FINV(&zi, &p->z); FSQ(&zi2, &zi); FM(&r->x, &p->x, &zi2); FM(&zi2, &zi2, &zi);                \
    FM(&r->y, &p->y, &zi2); r->inf = 0;                                                            \
  }                                                                                                \
  /* pairing 0.14 mul_assign: double-and-add from the most significant set bit */                  \
  static void G##_mul(G##j* r, const G##a* a, const uint64_t* k, int nl) {                        \
    G##j acc, base;                                                                                \
    G##_set_inf(&acc);                                                                             \
    G##_from_aff(&base, a);                                                                        \
    for (int i_ = nl - 1; i_ >= 0; --i_)                                                           \
      for (int b_ = 63; b_ >= 0; --b_) {                                                           \
        G##_dbl(&acc, &acc);                                                                       \
        if ((k[i_] >> b_) & 1) G##_add(&acc, &acc, &base);                                         \
      }                                                                                            \
    *r = acc;                                                                                      \
  }

#define FEQ fp_eq
DEFINE_JAC(g1, fp, fp_add, fp_sub, fp_mul, fp_sqr, fp_dbl, fp_is_zero, fp_neg, FP_ONE, FP_ZERO, fp_inv)
#undef FEQ
#define FEQ f2_eq
DEFINE_JAC(g2, fp2, f2_add, f2_sub, f2_mul, f2_sqr, f2_dbl, f2_is_zero, f2_neg, F2_ONE, F2_ZERO, f2_inv)
#undef FEQ

static int g1_in_subgroup(const g1a* p) {
  g1j t;
  g1_mul(&t, p, R_ORDER, 4);
  return g1_is_inf(&t);
}
static int g2_in_subgroup(const g2a* p) {
  g2j t;
  g2_mul(&t, p, R_ORDER, 4);
  return g2_is_inf(&t);
}

/* ---- zcash codec (pairing 0.14 G1Compressed / G2Compressed) */
static int g1_from_x(g1a* r, const fp* x, int greatest) {
  fp rhs, y, ny;
  fp_sqr(&rhs, x);
  fp_mul(&rhs, &rhs, x);
  fp_add(&rhs, &rhs, &B1);
  if (!fp_sqrt(&y, &rhs)) return 0;
  fp_neg(&ny, &y);
  /* (y < -y) ^ greatest ? y : -y   (Ord on canonical values) */
  int y_lt = !fp_lex_largest(&y) && !fp_eq(&y, &ny);
  r->x = *x;
  r->y = ((y_lt ^ greatest) ? y : ny);
  r->inf = 0;
  return 1;
}
static int g2_from_x(g2a* r, const fp2* x, int greatest) {
  fp2 rhs, y, ny;
  f2_sqr(&rhs, x);
  f2_mul(&rhs, &rhs, x);
  f2_add(&rhs, &rhs, &B2);
  if (!f2_sqrt(&y, &rhs)) return 0;
  f2_neg(&ny, &y);
  int y_lt = !f2_lex_largest(&y) && !f2_eq(&y, &ny);
  r->x = *x;
  r->y = ((y_lt ^ greatest) ? y : ny);
  r->inf = 0;
  return 1;
}
int tco_g1_decompress(const uint8_t* in, g1a* out, int check_subgroup) {
  uint8_t b[48];
  memcpy(b, in, 48);
  if (!(b[0] & 0x80)) return -1;
  if (b[0] & 0x40) {
    b[0] &= 0x3f;
    for (int i = 0; i < 48; ++i)
      if (b[i]) return -1;
    out->inf = 1;
    out->x = FP_ZERO;
    out->y = FP_ZERO;
    return 0;
  }
  int greatest = (b[0] & 0x20) != 0;
  b[0] &= 0x1f;
  uint64_t xi[6];
  be48_to_int(xi, b);
  if (ge_p(xi)) return -1;
  fp x;
  fp_from_int(&x, xi);
  if (!g1_from_x(out, &x, greatest)) return -1;
  if (check_subgroup && !g1_in_subgroup(out)) return -1;
  return 0;
}
int tco_g2_decompress(const uint8_t* in, g2a* out, int check_subgroup) {
  uint8_t b[96];
  memcpy(b, in, 96);
  if (!(b[0] & 0x80)) return -1;
  if (b[0] & 0x40) {
    b[0] &= 0x3f;
    for (int i = 0; i < 96; ++i)
      if (b[i]) return -1;
    out->inf = 1;
    out->x = F2_ZERO;
    out->y = F2_ZERO;
    return 0;
  }
  int greatest = (b[0] & 0x20) != 0;
  b[0] &= 0x1f;
  uint64_t x1[6], x0[6];
  be48_to_int(x1, b);
  be48_to_int(x0, b + 48);
  if (ge_p(x1) || ge_p(x0)) return -1;
  fp2 x;
  fp_from_int(&x.c0, x0);
  fp_from_int(&x.c1, x1);
  if (!g2_from_x(out, &x, greatest)) return -1;
  if (check_subgroup && !g2_in_subgroup(out)) return -1;
  return 0;
}
static void g1_compress(uint8_t* out, const g1a* p) {
  memset(out, 0, 48);
  if (p->inf) {
    out[0] = 0xc0;
    return;
  }
  uint64_t xi[6];
  fp_to_int(xi, &p->x);
  int_to_be48(out, xi);
  if (fp_lex_largest(&p->y)) out[0] |= 0x20;
  out[0] |= 0x80;
}
static void g2_compress(uint8_t* out, const g2a* p) {
  memset(out, 0, 96);
  if (p->inf) {
    out[0] = 0xc0;
    return;
  }
  uint64_t xi[6];
  fp_to_int(xi, &p->x.c1);
  int_to_be48(out, xi);
  fp_to_int(xi, &p->x.c0);
  int_to_be48(out + 48, xi);
  if (f2_lex_largest(&p->y)) out[0] |= 0x20;
  out[0] |= 0x80;
}
static void g2_uncompressed(uint8_t* out, const g2a* p) {
  memset(out, 0, 192);
  if (p->inf) {
    out[0] = 0x40;
    return;
  }
  uint64_t xi[6];
  fp_to_int(xi, &p->x.c1);
  int_to_be48(out, xi);
  fp_to_int(xi, &p->x.c0);
  int_to_be48(out + 48, xi);
  fp_to_int(xi, &p->y.c1);
  int_to_be48(out + 96, xi);
  fp_to_int(xi, &p->y.c0);
  int_to_be48(out + 144, xi);
}

/* ============================================================================ pairing */
#define NCOEFFS 68
typedef struct { fp2 c[NCOEFFS][3]; int inf; } g2prep;

/* pairing 0.14 G2Prepared::doubling_step (Jacobian, Algorithm 26 of eprint 2010/354) */
static void doubling_step(g2j* r, fp2* o0, fp2* o1, fp2* o2) {
  fp2 tmp0, tmp1, tmp2, tmp3, tmp4, tmp5, tmp6, zsq;
  f2_sqr(&tmp0, &r->x);
  f2_sqr(&tmp1, &r->y);
  f2_sqr(&tmp2, &tmp1);
  f2_add(&tmp3, &tmp1, &r->x);
  f2_sqr(&tmp3, &tmp3);
  f2_sub(&tmp3, &tmp3, &tmp0);
  f2_sub(&tmp3, &tmp3, &tmp2);
  f2_dbl(&tmp3, &tmp3);
  f2_dbl(&tmp4, &tmp0);
  f2_add(&tmp4, &tmp4, &tmp0);
  f2_add(&tmp6, &r->x, &tmp4);
  f2_sqr(&tmp5, &tmp4);
  f2_sqr(&zsq, &r->z);
  f2_sub(&r->x, &tmp5, &tmp3);
  f2_sub(&r->x, &r->x, &tmp3);
  f2_add(&r->z, &r->z, &r->y);
  f2_sqr(&r->z, &r->z);
  f2_sub(&r->z, &r->z, &tmp1);
  f2_sub(&r->z, &r->z, &zsq);
  f2_sub(&r->y, &tmp3, &r->x);
  f2_mul(&r->y, &r->y, &tmp4);
  f2_dbl(&tmp2, &tmp2);
  f2_dbl(&tmp2, &tmp2);
  f2_dbl(&tmp2, &tmp2);
  f2_sub(&r->y, &r->y, &tmp2);
  f2_mul(&tmp3, &tmp4, &zsq);
  f2_dbl(&tmp3, &tmp3);
  f2_neg(&tmp3, &tmp3);
  f2_sqr(&tmp6, &tmp6);
  f2_sub(&tmp6, &tmp6, &tmp0);
  f2_sub(&tmp6, &tmp6, &tmp5);
  f2_dbl(&tmp1, &tmp1);
  f2_dbl(&tmp1, &tmp1);
  f2_sub(&tmp6, &tmp6, &tmp1);
  f2_mul(&tmp0, &r->z, &zsq);
  f2_dbl(&tmp0, &tmp0);
  *o0 = tmp0;
  *o1 = tmp3;
  *o2 = tmp6;
}
/* pairing 0.14 G2Prepared::addition_step (Algorithm 27 of eprint 2010/354) */
static void addition_step(g2j* r, const g2a* q, fp2* o0, fp2* o1, fp2* o2) {
  fp2 zsq, ysq, t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, ztsq;
  f2_sqr(&zsq, &r->z);
  f2_sqr(&ysq, &q->y);
  f2_mul(&t0, &zsq, &q->x);
  f2_add(&t1, &q->y, &r->z);
  f2_sqr(&t1, &t1);
  f2_sub(&t1, &t1, &ysq);
  f2_sub(&t1, &t1, &zsq);
  f2_mul(&t1, &t1, &zsq);
  f2_sub(&t2, &t0, &r->x);
  f2_sqr(&t3, &t2);
  f2_dbl(&t4, &t3);
  f2_dbl(&t4, &t4);
  f2_mul(&t5, &t4, &t2);
  f2_sub(&t6, &t1, &r->y);
  f2_sub(&t6, &t6, &r->y);
  f2_mul(&t9, &t6, &q->x);
  f2_mul(&t7, &t4, &r->x);
  f2_sqr(&r->x, &t6);
  f2_sub(&r->x, &r->x, &t5);
  f2_sub(&r->x, &r->x, &t7);
  f2_sub(&r->x, &r->x, &t7);
  f2_add(&r->z, &r->z, &t2);
  f2_sqr(&r->z, &r->z);
  f2_sub(&r->z, &r->z, &zsq);
  f2_sub(&r->z, &r->z, &t3);
  f2_add(&t10, &q->y, &r->z);
  f2_sub(&t8, &t7, &r->x);
  f2_mul(&t8, &t8, &t6);
  f2_mul(&t0, &r->y, &t5);
  f2_dbl(&t0, &t0);
  f2_sub(&r->y, &t8, &t0);
  f2_sqr(&t10, &t10);
  f2_sub(&t10, &t10, &ysq);
  f2_sqr(&ztsq, &r->z);
  f2_sub(&t10, &t10, &ztsq);
  f2_dbl(&t9, &t9);
  f2_sub(&t9, &t9, &t10);
  f2_dbl(&t10, &r->z);
  f2_neg(&t6, &t6);
  f2_dbl(&t1, &t6);
  *o0 = t10;
  *o1 = t1;
  *o2 = t9;
}
static void g2_prepare(g2prep* pr, const g2a* q) {
  pr->inf = q->inf;
  if (q->inf) return;
  g2j r;
  g2_from_aff(&r, q);
  int j = 0, found = 0;
  for (int b = 63; b >= 0; --b) {
    int bit = (BLS_X >> b) & 1;
    if (!found) {
      found = bit;
      continue;
    }
    doubling_step(&r, &pr->c[j][0], &pr->c[j][1], &pr->c[j][2]);
    ++j;
    if (bit) {
      addition_step(&r, q, &pr->c[j][0], &pr->c[j][1], &pr->c[j][2]);
      ++j;
    }
  }
}
/* ell: f *= line evaluated at p (pairing 0.14: c0 *= p.y, c1 *= p.x, mul_by_014(c2, c1, c0)) */
static void ell(fp12* f, const fp2* c, const g1a* p) {
  fp2 c0, c1;
  f2_mul_fp(&c0, &c[0], &p->y);
  f2_mul_fp(&c1, &c[1], &p->x);
  f12_mul_by_014(f, &c[2], &c1, &c0);
}
/* multi-Miller loop over n pairs (pairing 0.14 miller_loop structure) */
static void miller_loop(fp12* f, const g1a* const* ps, const g2prep* const* qs, int n) {
  f12_one(f);
  int j = 0, found = 0;
  for (int b = 63; b >= 0; --b) {
    int bit = (BLS_X >> b) & 1;
    if (!found) {
      found = bit;
      continue;
    }
    if (j > 0) f12_sqr(f, f);
    for (int k = 0; k < n; ++k)
      if (!ps[k]->inf && !qs[k]->inf) ell(f, qs[k]->c[j], ps[k]);
    ++j;
    if (bit) {
      for (int k = 0; k < n; ++k)
        if (!ps[k]->inf && !qs[k]->inf) ell(f, qs[k]->c[j], ps[k]);
      ++j;
    }
  }
  f12_conj(f, f); /* x < 0 */
}
static void exp_by_x(fp12* r, const fp12* f) {
  fp12 acc;
  f12_one(&acc);
  int started = 0;
  for (int b = 63; b >= 0; --b) {
    if (started) f12_sqr(&acc, &acc);
    if ((BLS_X >> b) & 1) {
      f12_mul(&acc, &acc, f);
      started = 1;
    }
  }
  f12_conj(r, &acc);
}
/* pairing 0.14 final_exponentiation */
static void final_exp(fp12* out, const fp12* in) {
  fp12 f1, f2, r, y0, y1, y2, y3;
  f12_conj(&f1, in);
  f12_inv(&f2, in);
  f12_mul(&r, &f1, &f2);
  f2 = r;
  f12_frob(&r, &r, 2);
  f12_mul(&r, &r, &f2);
  f12_sqr(&y0, &r);
  exp_by_x(&y1, &y0);
  /* x >> 1 */
  {
    fp12 acc;
    f12_one(&acc);
    int started = 0;
    const uint64_t xh = BLS_X >> 1;
    for (int b = 63; b >= 0; --b) {
      if (started) f12_sqr(&acc, &acc);
      if ((xh >> b) & 1) {
        f12_mul(&acc, &acc, &y1);
        started = 1;
      }
    }
    f12_conj(&y2, &acc);
  }
  f12_conj(&y3, &r);
  f12_mul(&y1, &y1, &y3);
  f12_conj(&y1, &y1);
  f12_mul(&y1, &y1, &y2);
  exp_by_x(&y2, &y1);
  exp_by_x(&y3, &y2);
  f12_conj(&y1, &y1);
  f12_mul(&y3, &y3, &y1);
  f12_conj(&y1, &y1);
  f12_frob(&y1, &y1, 3);
  f12_frob(&y2, &y2, 2);
  f12_mul(&y1, &y1, &y2);
  exp_by_x(&y2, &y3);
  f12_mul(&y2, &y2, &y0);
  f12_mul(&y2, &y2, &r);
  f12_mul(&y1, &y1, &y2);
  f12_frob(&y2, &y3, 1);
  f12_mul(out, &y1, &y2);
}
/* Bls12::pairing(p, q) */
static void pairing(fp12* out, const g1a* p, const g2a* q) {
  g2prep* pr = (g2prep*)malloc(sizeof(g2prep));
  g2_prepare(pr, q);
  const g1a* ps[1] = {p};
  const g2prep* qs[1] = {pr};
  fp12 f;
  miller_loop(&f, ps, qs, 1);
  final_exp(out, &f);
  free(pr);
}

/* ============================================================================ hashing */
static const uint64_t KECCAK_RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int KECCAK_ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
static uint64_t rol64(uint64_t x, int s) { return s ? (x << s) | (x >> (64 - s)) : x; }
static void keccak_f(uint64_t* A) {
  for (int round = 0; round < 24; ++round) {
    uint64_t C[5], D[5], Bv[25];
    for (int x = 0; x < 5; ++x) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
    for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rol64(C[(x + 1) % 5], 1);
    for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) Bv[y + 5 * ((2 * x + 3 * y) % 5)] = rol64(A[x + 5 * y], KECCAK_ROT[x + 5 * y]);
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) A[x + 5 * y] = Bv[x + 5 * y] ^ (~Bv[(x + 1) % 5 + 5 * y] & Bv[(x + 2) % 5 + 5 * y]);
    A[0] ^= KECCAK_RC[round];
  }
}
void tco_sha3_256(const uint8_t* msg, size_t len, uint8_t* out) {
  uint64_t A[25];
  memset(A, 0, sizeof A);
  const size_t rate = 136;
  uint8_t block[136];
  while (len >= rate) {
    for (size_t i = 0; i < rate / 8; ++i) {
      uint64_t w = 0;
      for (int k = 7; k >= 0; --k) w = (w << 8) | msg[8 * i + k];
      A[i] ^= w;
    }
    keccak_f(A);
    msg += rate;
    len -= rate;
  }
  memset(block, 0, rate);
  memcpy(block, msg, len);
  block[len] ^= 0x06;
  block[rate - 1] ^= 0x80;
  for (size_t i = 0; i < rate / 8; ++i) {
    uint64_t w = 0;
    for (int k = 7; k >= 0; --k) w = (w << 8) | block[8 * i + k];
    A[i] ^= w;
  }
  keccak_f(A);
  for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(A[i / 8] >> (8 * (i % 8)));
}
/* rand 0.4 ChaChaRng (20 rounds, 128-bit counter in words 12..15, next_u64 = high word first) */
typedef struct { uint32_t st[16], buf[16]; int idx; } chacha;
static uint32_t rol32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }
#define QR(a, b, c, d)                                     \
  s[a] += s[b]; s[d] = rol32(s[d] ^ s[a], 16);             \
  s[c] += s[d]; s[b] = rol32(s[b] ^ s[c], 12);             \
  s[a] += s[b]; s[d] = rol32(s[d] ^ s[a], 8);              \
  s[c] += s[d]; s[b] = rol32(s[b] ^ s[c], 7);
static void chacha_init(chacha* c, const uint32_t* key8) {
  const uint32_t k0[4] = {0x61707865, 0x3320646e, 0x79622d32, 0x6b206574};
  memcpy(c->st, k0, 16);
  memcpy(c->st + 4, key8, 32);
  memset(c->st + 12, 0, 16);
  c->idx = 16;
}
static void chacha_refill(chacha* c) {
  uint32_t s[16];
  memcpy(s, c->st, 64);
  for (int i = 0; i < 10; ++i) {
    QR(0, 4, 8, 12) QR(1, 5, 9, 13) QR(2, 6, 10, 14) QR(3, 7, 11, 15)
    QR(0, 5, 10, 15) QR(1, 6, 11, 12) QR(2, 7, 8, 13) QR(3, 4, 9, 14)
  }
  for (int i = 0; i < 16; ++i) c->buf[i] = s[i] + c->st[i];
  for (int i = 12; i < 16; ++i)
    if (++c->st[i] != 0) break;
  c->idx = 0;
}
static uint32_t chacha_u32(chacha* c) {
  if (c->idx == 16) chacha_refill(c);
  return c->buf[c->idx++];
}
static uint64_t chacha_u64(chacha* c) {
  uint64_t hi = chacha_u32(c);
  uint64_t lo = chacha_u32(c);
  return (hi << 32) | lo;
}
static void seed_from_digest(uint32_t* key, const uint8_t* d) {
  for (int i = 0; i < 8; ++i)
    key[i] = ((uint32_t)d[4 * i] << 24) | ((uint32_t)d[4 * i + 1] << 16) | ((uint32_t)d[4 * i + 2] << 8) | d[4 * i + 3];
}
/* ff_derive Rand for Fq: repr = 6 x u64 (Montgomery repr), top 3 bits masked, reject >= p */
static void fp_rand(fp* r, chacha* c) {
  for (;;) {
    uint64_t l[6];
    for (int i = 0; i < 6; ++i) l[i] = chacha_u64(c);
    l[5] &= 0xffffffffffffffffULL >> 3;
    if (!ge_p(l)) {
      memcpy(r->v, l, 48);
      return;
    }
  }
}
/* threshold_crypto hash_g2: sha3 -> ChaCha -> G2::rand (x, greatest, get_point_from_x, *h2) */
void tco_hash_g2(const uint8_t* msg, size_t len, uint8_t* out96) {
  uint8_t d[32];
  uint32_t key[8];
  tco_sha3_256(msg, len, d);
  seed_from_digest(key, d);
  chacha c;
  chacha_init(&c, key);
  for (;;) {
    fp2 x;
    fp_rand(&x.c0, &c);
    fp_rand(&x.c1, &c);
    int greatest = (chacha_u32(&c) & 1) != 0;
    g2a p;
    if (g2_from_x(&p, &x, greatest)) {
      g2j q;
      g2_mul(&q, &p, H2, 8);
      if (!g2_is_inf(&q)) {
        g2a a;
        g2_to_aff(&a, &q);
        g2_compress(out96, &a);
        return;
      }
    }
  }
}
void tco_hash_g1_g2(const uint8_t* g1_c48, const uint8_t* msg, size_t len, uint8_t* out96) {
  uint8_t* buf = (uint8_t*)malloc(len + 80);
  size_t n;
  if (len > 64) {
    tco_sha3_256(msg, len, buf);
    n = 32;
  } else {
    memcpy(buf, msg, len);
    n = len;
  }
  memcpy(buf + n, g1_c48, 48);
  tco_hash_g2(buf, n + 48, out96);
  free(buf);
}

/* ============================================================================ init */
static void int_div_small(uint64_t* q, const uint64_t* a, uint64_t d) {
  u128 rem = 0;
  for (int i = 5; i >= 0; --i) {
    u128 cur = (rem << 64) | a[i];
    q[i] = (uint64_t)(cur / d);
    rem = cur % d;
  }
}
static int g_inited = 0;
static pthread_mutex_t g_init_mu = PTHREAD_MUTEX_INITIALIZER;
void tco_init(void) {
  pthread_mutex_lock(&g_init_mu);
  if (g_inited) {
    pthread_mutex_unlock(&g_init_mu);
    return;
  }
  uint64_t inv = 1;
  for (int i = 0; i < 7; ++i) inv *= 2 - P[0] * inv;
  PINV = (uint64_t)0 - inv;
  memset(&FP_ZERO, 0, sizeof FP_ZERO);
  /* R mod p by doubling 1 384 times (plain integers), then R^2 = R * 2^384 the same way */
  uint64_t t[6] = {1, 0, 0, 0, 0, 0};
  fp tt;
  for (int k = 0; k < 768; ++k) {
    memcpy(tt.v, t, 48);
    fp_add(&tt, &tt, &tt);
    memcpy(t, tt.v, 48);
    if (k == 383) memcpy(FP_ONE.v, t, 48);
  }
  memcpy(FP_R2.v, t, 48);
  uint64_t pm[6];
  memcpy(pm, P, 48);
  pm[0] -= 2;
  memcpy(EXP_PM2, pm, 48);
  uint64_t p1[6];
  memcpy(p1, P, 48);
  p1[0] += 1; /* p + 1 (no carry: low limb is ...aaab) */
  int_div_small(EXP_SQRT, p1, 4);
  uint64_t p3[6];
  memcpy(p3, P, 48);
  p3[0] -= 3;
  int_div_small(EXP_PM3_4, p3, 4);
  uint64_t pm1[6];
  memcpy(pm1, P, 48);
  pm1[0] -= 1;
  int_div_small(EXP_PM1_2, pm1, 2);
  memcpy(HALF_P, EXP_PM1_2, 48);
  F2_ONE.c0 = FP_ONE;
  F2_ONE.c1 = FP_ZERO;
  F2_ZERO.c0 = FP_ZERO;
  F2_ZERO.c1 = FP_ZERO;
  uint64_t four[6] = {4, 0, 0, 0, 0, 0};
  fp_from_int(&B1, four);
  B2.c0 = B1;
  B2.c1 = B1;
  /* Frobenius coefficients: gamma = xi^((p-1)/3), delta = xi^((p-1)/6); k = 2, 3 by
   * gamma^(p+1) = gamma * conj(gamma), gamma^(p^2+p+1) = gamma^2 * conj(gamma) */
  fp2 xi;
  xi.c0 = FP_ONE;
  xi.c1 = FP_ONE;
  uint64_t e3[6], e6[6];
  int_div_small(e3, pm1, 3);
  int_div_small(e6, pm1, 6);
  fp2 g, dl, cg, cd;
  f2_pow(&g, &xi, e3, 6);
  f2_pow(&dl, &xi, e6, 6);
  f2_conj(&cg, &g);
  f2_conj(&cd, &dl);
  FROB6_C1[0] = F2_ONE;
  FROB12_C1[0] = F2_ONE;
  FROB6_C1[1] = g;
  f2_mul(&FROB6_C1[2], &g, &cg);
  f2_mul(&FROB6_C1[3], &g, &g);
  f2_mul(&FROB6_C1[3], &FROB6_C1[3], &cg);
  FROB12_C1[1] = dl;
  f2_mul(&FROB12_C1[2], &dl, &cd);
  f2_mul(&FROB12_C1[3], &dl, &dl);
  f2_mul(&FROB12_C1[3], &FROB12_C1[3], &cd);
  for (int k = 0; k < 4; ++k) f2_sqr(&FROB6_C2[k], &FROB6_C1[k]);
  /* generators (canonical big-endian) */
  static const uint8_t g1x[48] = {0x17, 0xf1, 0xd3, 0xa7, 0x31, 0x97, 0xd7, 0x94, 0x26, 0x95, 0x63, 0x8c, 0x4f, 0xa9, 0xac, 0x0f, 0xc3, 0x68, 0x8c, 0x4f, 0x97, 0x74, 0xb9, 0x05, 0xa1, 0x4e, 0x3a, 0x3f, 0x17, 0x1b, 0xac, 0x58, 0x6c, 0x55, 0xe8, 0x3f, 0xf9, 0x7a, 0x1a, 0xef, 0xfb, 0x3a, 0xf0, 0x0a, 0xdb, 0x22, 0xc6, 0xbb};
  static const uint8_t g1y[48] = {0x08, 0xb3, 0xf4, 0x81, 0xe3, 0xaa, 0xa0, 0xf1, 0xa0, 0x9e, 0x30, 0xed, 0x74, 0x1d, 0x8a, 0xe4, 0xfc, 0xf5, 0xe0, 0x95, 0xd5, 0xd0, 0x0a, 0xf6, 0x00, 0xdb, 0x18, 0xcb, 0x2c, 0x04, 0xb3, 0xed, 0xd0, 0x3c, 0xc7, 0x44, 0xa2, 0x88, 0x8a, 0xe4, 0x0c, 0xaa, 0x23, 0x29, 0x46, 0xc5, 0xe7, 0xe1};
  uint64_t xi6[6];
  be48_to_int(xi6, g1x);
  fp_from_int(&G1GEN.x, xi6);
  be48_to_int(xi6, g1y);
  fp_from_int(&G1GEN.y, xi6);
  G1GEN.inf = 0;
  static const uint8_t g2c[96] = {0x93, 0xe0, 0x2b, 0x60, 0x52, 0x71, 0x9f, 0x60, 0x7d, 0xac, 0xd3, 0xa0, 0x88, 0x27, 0x4f, 0x65, 0x59, 0x6b, 0xd0, 0xd0, 0x99, 0x20, 0xb6, 0x1a, 0xb5, 0xda, 0x61, 0xbb, 0xdc, 0x7f, 0x50, 0x49, 0x33, 0x4c, 0xf1, 0x12, 0x13, 0x94, 0x5d, 0x57, 0xe5, 0xac, 0x7d, 0x05, 0x5d, 0x04, 0x2b, 0x7e, 0x02, 0x4a, 0xa2, 0xb2, 0xf0, 0x8f, 0x0a, 0x91, 0x26, 0x08, 0x05, 0x27, 0x2d, 0xc5, 0x10, 0x51, 0xc6, 0xe4, 0x7a, 0xd4, 0xfa, 0x40, 0x3b, 0x02, 0xb4, 0x51, 0x0b, 0x64, 0x7a, 0xe3, 0xd1, 0x77, 0x0b, 0xac, 0x03, 0x26, 0xa8, 0x05, 0xbb, 0xef, 0xd4, 0x80, 0x56, 0xc8, 0xc1, 0x21, 0xbd, 0xb8};
  tco_g2_decompress(g2c, &G2GEN, 0);
  g_inited = 1;
  pthread_mutex_unlock(&g_init_mu);
}

/* ============================================================================ exported API */
static void scalar_from_le32(uint64_t* k, const uint8_t* s) {
  for (int i = 0; i < 4; ++i) {
    uint64_t w = 0;
    for (int b = 7; b >= 0; --b) w = (w << 8) | s[8 * i + b];
    k[i] = w;
  }
}
/* returns 0 ok, -1 decode error */
int tco_g1_mul(const uint8_t* p48, const uint8_t* k32, uint8_t* out48) {
  tco_init();
  g1a p, a;
  if (tco_g1_decompress(p48, &p, 1)) return -1;
  uint64_t k[4];
  scalar_from_le32(k, k32);
  g1j r;
  g1_mul(&r, &p, k, 4);
  g1_to_aff(&a, &r);
  g1_compress(out48, &a);
  return 0;
}
int tco_g2_mul(const uint8_t* p96, const uint8_t* k32, uint8_t* out96) {
  tco_init();
  g2a p, a;
  if (tco_g2_decompress(p96, &p, 1)) return -1;
  uint64_t k[4];
  scalar_from_le32(k, k32);
  g2j r;
  g2_mul(&r, &p, k, 4);
  g2_to_aff(&a, &r);
  g2_compress(out96, &a);
  return 0;
}
/* e(p1, q1) == e(p2, q2) with two full pairings (threshold_crypto's verify*): 1/0, -1 decode */
int tco_pairing_eq(const uint8_t* p1, const uint8_t* q1, const uint8_t* p2, const uint8_t* q2) {
  tco_init();
  g1a a1, a2;
  g2a b1, b2;
  if (tco_g1_decompress(p1, &a1, 1) || tco_g1_decompress(p2, &a2, 1) ||
      tco_g2_decompress(q1, &b1, 1) || tco_g2_decompress(q2, &b2, 1))
    return -1;
  fp12 e1, e2;
  pairing(&e1, &a1, &b1);
  pairing(&e2, &a2, &b2);
  return f12_eq(&e1, &e2);
}
/* Signature::parity of a compressed G2 signature */
int tco_sig_parity(const uint8_t* sig96) {
  tco_init();
  g2a s;
  if (tco_g2_decompress(sig96, &s, 1)) return -1;
  uint8_t u[192];
  g2_uncompressed(u, &s);
  uint8_t x = 0;
  for (int i = 0; i < 192; ++i) x ^= u[i];
  return __builtin_popcount(x) & 1;
}

/* ---- PublicKeySet::combine_signatures / decrypt interpolation (first t items; x = idx + 1) */
static const uint64_t FR_P[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL, 0x73eda753299d7d48ULL};
static void fr_mulmod(uint64_t* r, const uint64_t* a, const uint64_t* b) { /* schoolbook + slow reduction */
  uint64_t t[8] = {0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c += (u128)a[i] * b[j] + t[i + j];
      t[i + j] = (uint64_t)c;
      c >>= 64;
    }
    t[i + 4] = (uint64_t)c;
  }
  /* reduce 512-bit t mod r by shift-subtract (oracle speed is irrelevant for t <= a few k) */
  uint64_t rem[5] = {0, 0, 0, 0, 0};
  for (int bit = 511; bit >= 0; --bit) {
    /* rem = rem*2 + bit */
    uint64_t carry = (t[bit / 64] >> (bit % 64)) & 1;
    for (int i = 0; i < 5; ++i) {
      uint64_t nc = rem[i] >> 63;
      rem[i] = (rem[i] << 1) | carry;
      carry = nc;
    }
    /* if rem >= r: rem -= r */
    int ge = rem[4] != 0;
    if (!ge) {
      ge = 1;
      for (int i = 3; i >= 0; --i) {
        if (rem[i] != FR_P[i]) {
          ge = rem[i] > FR_P[i];
          break;
        }
      }
    }
    if (ge) {
      u128 br = 0;
      for (int i = 0; i < 4; ++i) {
        u128 d = (u128)rem[i] - FR_P[i] - br;
        rem[i] = (uint64_t)d;
        br = (d >> 64) & 1;
      }
      rem[4] -= (uint64_t)br;
    }
  }
  memcpy(r, rem, 32);
}
static void fr_submod(uint64_t* r, const uint64_t* a, const uint64_t* b) {
  u128 br = 0;
  uint64_t t[4];
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a[i] - b[i] - br;
    t[i] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  if (br) {
    u128 c = 0;
    for (int i = 0; i < 4; ++i) {
      c += (u128)t[i] + FR_P[i];
      t[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  memcpy(r, t, 32);
}
static void fr_inv(uint64_t* r, const uint64_t* a) {
  uint64_t e[4];
  memcpy(e, FR_P, 32);
  e[0] -= 2;
  uint64_t acc[4] = {1, 0, 0, 0};
  for (int i = 3; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      fr_mulmod(acc, acc, acc);
      if ((e[i] >> b) & 1) fr_mulmod(acc, acc, a);
    }
  memcpy(r, acc, 32);
}
/* returns 0 ok (out written), 5 NotEnoughShares, 6 DuplicateEntry, 2 decode error */
static int interpolate(int group, uint32_t n, const uint32_t* idx, const uint8_t* pts, uint32_t t,
                       uint8_t* out) {
  tco_init();
  if (n < t) return 5;
  for (uint32_t i = 0; i < t; ++i)
    for (uint32_t j = 0; j < i; ++j)
      if (idx[i] == idx[j]) return 6;
  g1j acc1;
  g2j acc2;
  g1_set_inf(&acc1);
  g2_set_inf(&acc2);
  for (uint32_t i = 0; i < t; ++i) {
    uint64_t xi[4] = {(uint64_t)idx[i] + 1, 0, 0, 0}, l0[4] = {1, 0, 0, 0};
    for (uint32_t j = 0; j < t; ++j) {
      if (j == i) continue;
      uint64_t xj[4] = {(uint64_t)idx[j] + 1, 0, 0, 0}, den[4], inv[4];
      fr_submod(den, xj, xi);
      fr_inv(inv, den);
      fr_mulmod(l0, l0, xj);
      fr_mulmod(l0, l0, inv);
    }
    if (group == 1) {
      g1a p;
      if (tco_g1_decompress(pts + 48 * i, &p, 1)) return 2;
      g1j m;
      g1_mul(&m, &p, l0, 4);
      g1_add(&acc1, &acc1, &m);
    } else {
      g2a p;
      if (tco_g2_decompress(pts + 96 * i, &p, 1)) return 2;
      g2j m;
      g2_mul(&m, &p, l0, 4);
      g2_add(&acc2, &acc2, &m);
    }
  }
  if (group == 1) {
    g1a a;
    g1_to_aff(&a, &acc1);
    g1_compress(out, &a);
  } else {
    g2a a;
    g2_to_aff(&a, &acc2);
    g2_compress(out, &a);
  }
  return 0;
}
int tco_combine_g1(uint32_t n, const uint32_t* idx, const uint8_t* pts48, uint32_t t, uint8_t* out48) {
  return interpolate(1, n, idx, pts48, t, out48);
}
int tco_combine_g2(uint32_t n, const uint32_t* idx, const uint8_t* pts96, uint32_t t, uint8_t* out96) {
  return interpolate(2, n, idx, pts96, t, out96);
}

/* ============================================================================ CPU baseline */
/* Per DecryptionShare, threshold_crypto's verify_decryption_share as hbbft calls it
 * (src/threshold_decryption.rs:152-161), including the serde decode of the share:
 *   faithful: decode(share) [on-curve + [r]P], H = hash_g1_g2(u, v), pairing(share, H) ==
 *             pairing(pk, w)                                        (two full pairings)
 *   optimized: decode(share) once, H and both G2Prepared computed once per ciphertext, one
 *             2-pair multi-Miller loop + one final exponentiation per share. */
typedef struct {
  int mode;
  const uint8_t *shares, *pk, *u, *v, *w, *H;
  size_t v_len;
  uint32_t n_shares;
  double budget_s;
  uint32_t done, accepted;
  const g2prep *prep_H, *prep_w;
  const g1a* pk_aff;
} bjob;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}
static void* bworker(void* arg) {
  bjob* j = (bjob*)arg;
  const double t0 = now_s();
  for (uint32_t i = 0; i < j->n_shares; ++i) {
    g1a s;
    if (tco_g1_decompress(j->shares + 48 * i, &s, 1) == 0) {
      int ok;
      if (j->mode == 0) {
        uint8_t H[96];
        tco_hash_g1_g2(j->u, j->v, j->v_len, H);
        g2a h, w;
        g1a pk;
        tco_g2_decompress(H, &h, 0);
        tco_g2_decompress(j->w, &w, 1);
        tco_g1_decompress(j->pk, &pk, 1);
        fp12 e1, e2;
        pairing(&e1, &s, &h);
        pairing(&e2, &pk, &w);
        ok = f12_eq(&e1, &e2);
      } else {
        g1a npk = *j->pk_aff;
        fp_neg(&npk.y, &npk.y);
        const g1a* ps[2] = {&s, &npk};
        const g2prep* qs[2] = {j->prep_H, j->prep_w};
        fp12 f, e;
        miller_loop(&f, ps, qs, 2);
        final_exp(&e, &f);
        fp12 one;
        f12_one(&one);
        ok = f12_eq(&e, &one);
      }
      j->accepted += ok;
    }
    j->done++;
    if (now_s() - t0 > j->budget_s) break;
  }
  return NULL;
}
/* Runs `threads` workers, each verifying up to n_shares shares (all against the same
 * ciphertext (u, v, w) and pk) for at most budget_s seconds.  Returns shares done; *wall_s
 * gets the wall time and *accepted the accepted count. */
uint64_t tco_bench_dec_shares(int mode, int threads, double budget_s, const uint8_t* shares48,
                              uint32_t n_shares, const uint8_t* pk48, const uint8_t* u48,
                              const uint8_t* v, size_t v_len, const uint8_t* w96, double* wall_s,
                              uint64_t* accepted) {
  tco_init();
  g2prep* ph = (g2prep*)malloc(sizeof(g2prep));
  g2prep* pw = (g2prep*)malloc(sizeof(g2prep));
  g1a pk;
  tco_g1_decompress(pk48, &pk, 1);
  if (mode == 1) {
    uint8_t H[96];
    tco_hash_g1_g2(u48, v, v_len, H);
    g2a h, w;
    tco_g2_decompress(H, &h, 0);
    tco_g2_decompress(w96, &w, 1);
    g2_prepare(ph, &h);
    g2_prepare(pw, &w);
  }
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  bjob* jobs = (bjob*)calloc(threads, sizeof(bjob));
  const double t0 = now_s();
  for (int k = 0; k < threads; ++k) {
    bjob* j = &jobs[k];
    j->mode = mode;
    j->shares = shares48;
    j->n_shares = n_shares;
    j->pk = pk48;
    j->u = u48;
    j->v = v;
    j->v_len = v_len;
    j->w = w96;
    j->budget_s = budget_s;
    j->prep_H = ph;
    j->prep_w = pw;
    j->pk_aff = &pk;
    pthread_create(&th[k], NULL, bworker, j);
  }
  uint64_t done = 0, acc = 0;
  for (int k = 0; k < threads; ++k) {
    pthread_join(th[k], NULL);
    done += jobs[k].done;
    acc += jobs[k].accepted;
  }
  *wall_s = now_s() - t0;
  if (accepted) *accepted = acc;
  free(th);
  free(jobs);
  free(ph);
  free(pw);
  return done;
}

/* Per SignatureShare, threshold_crypto's PublicKeyShare::verify as hbbft's Coin calls it
 * (src/coin.rs:151), including the serde decode of the share: decode(sig) [on-curve + [r]Q],
 * H = hash_g2(nonce) (recomputed per call, as the reference does), decode(pk_i),
 * pairing(pk_i, H) == pairing(G1, sig).  Share i uses pk48[i] (n_shares of each). */
typedef struct {
  const uint8_t *sigs, *pks, *nonce;
  size_t nonce_len;
  uint32_t n_shares, first, stride;
  double budget_s;
  uint32_t done, accepted;
} sjob;
static void* sworker(void* arg) {
  sjob* j = (sjob*)arg;
  const double t0 = now_s();
  for (uint32_t i = j->first; i < j->n_shares; i += j->stride) {
    g2a s;
    if (tco_g2_decompress(j->sigs + 96 * i, &s, 1) == 0) {
      uint8_t H[96];
      tco_hash_g2(j->nonce, j->nonce_len, H);
      g2a h;
      g1a pk, g;
      tco_g2_decompress(H, &h, 0);
      tco_g1_decompress(j->pks + 48 * i, &pk, 1);
      g = G1GEN;
      fp12 e1, e2;
      pairing(&e1, &pk, &h);
      pairing(&e2, &g, &s);
      j->accepted += f12_eq(&e1, &e2);
    }
    j->done++;
    if (now_s() - t0 > j->budget_s) break;
  }
  return NULL;
}
uint64_t tco_bench_sig_shares(int threads, double budget_s, const uint8_t* sigs96, const uint8_t* pks48,
                              uint32_t n_shares, const uint8_t* nonce, size_t nonce_len, double* wall_s,
                              uint64_t* accepted) {
  tco_init();
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  sjob* jobs = (sjob*)calloc(threads, sizeof(sjob));
  const double t0 = now_s();
  for (int k = 0; k < threads; ++k) {
    sjob* j = &jobs[k];
    j->sigs = sigs96;
    j->pks = pks48;
    j->nonce = nonce;
    j->nonce_len = nonce_len;
    j->n_shares = n_shares;
    j->first = (uint32_t)k;
    j->stride = (uint32_t)threads;
    j->budget_s = budget_s;
    pthread_create(&th[k], NULL, sworker, j);
  }
  uint64_t done = 0, acc = 0;
  for (int k = 0; k < threads; ++k) {
    pthread_join(th[k], NULL);
    done += jobs[k].done;
    acc += jobs[k].accepted;
  }
  *wall_s = now_s() - t0;
  if (accepted) *accepted = acc;
  free(th);
  free(jobs);
  return done;
}

/* G1 scalar multiplications (255-bit scalars, pairing 0.14's double-and-add) of the generator on
 * `threads` threads for budget_s seconds: the unit of BivarCommitment::evaluate, which the
 * reference runs (t+1)^2 times per Ack (src/sync_key_gen.rs:493).  Returns multiplications done. */
typedef struct {
  double budget_s;
  uint64_t seed;
  uint32_t done;
} mjob;
static void* mworker(void* arg) {
  mjob* j = (mjob*)arg;
  const double t0 = now_s();
  uint64_t s = j->seed;
  g1a base = G1GEN;
  while (now_s() - t0 < j->budget_s) {
    uint64_t k[4];
    for (int i = 0; i < 4; ++i) {
      s = s * 6364136223846793005ull + 1442695040888963407ull;
      k[i] = s;
    }
    k[3] &= 0x3fffffffffffffffull;
    g1j r;
    g1_mul(&r, &base, k, 4);
    j->done++;
  }
  return NULL;
}
uint64_t tco_bench_g1_mul(int threads, double budget_s, double* wall_s) {
  tco_init();
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  mjob* jobs = (mjob*)calloc(threads, sizeof(mjob));
  const double t0 = now_s();
  for (int k = 0; k < threads; ++k) {
    jobs[k].budget_s = budget_s;
    jobs[k].seed = 0x9e3779b97f4a7c15ull * (uint64_t)(k + 1);
    pthread_create(&th[k], NULL, mworker, &jobs[k]);
  }
  uint64_t done = 0;
  for (int k = 0; k < threads; ++k) {
    pthread_join(th[k], NULL);
    done += jobs[k].done;
  }
  *wall_s = now_s() - t0;
  free(th);
  free(jobs);
  return done;
}
