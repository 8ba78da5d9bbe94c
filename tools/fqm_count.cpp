// Counts Fq Montgomery multiplications (Fqm) per unit of work for the exact algorithms the
// gfx950 kernels run (same headers, host build with HBTC_COUNT_FQM).  Output: JSON on stdout,
// frozen into bench/roofline_constants.json by `make roofline-constants`.
//
// Units:
//   dec_share   one DecryptionShare check: G1 decode + subgroup test, 2-pair Miller loop with
//               two precomputed line tables, final exponentiation        (k_dec_verify, per item)
//   sig_share   one SignatureShare check: G2 decode + subgroup test, Miller loop with one
//               precomputed table and one on-the-fly G2 argument, final exp (k_sig_verify)
//   g2_prepare  per-instance G2 decode + 68-line precomputation           (k_g2_prepare)
//   g1_combine_item  one G1 combine term: decode + 255-bit double-and-add (the reference's
//               interpolate; kept for comparison)
//   g1_msm_combine   one G1 Lagrange combine of t = 334 verified shares as the batched
//               Pippenger kernels run it (hbtc_msm.hip, c = 6): trusted decode (no subgroup
//               test) per term, exact digit statistics of random scalars, bucket running sums,
//               segment scaling, window sums, Horner doublings, normalisation
#include <cstdio>
#include <cstring>
#include <random>

#include "pairing.h"

namespace hbtc {
unsigned long long hbtc_fqm_count = 0;
}

using namespace hbtc;

namespace {
struct HL {
  const Line* l;
  void load(Line& o, int j) const { o = l[j]; }
};

// [k] G for a random k, compressed (host build of the same code; counting disabled around it)
void rand_scalar(Fr& k, std::mt19937_64& g) {
  for (int i = 0; i < 8; ++i) k.v[i] = (uint32_t)g();
  k.v[7] &= 0x3fffffffu;
}
}  // namespace

int main() {
  std::mt19937_64 g(42);
  G1A gen1;
  fq_set(gen1.x, G1_GEN_X);
  fq_set(gen1.y, G1_GEN_Y);
  gen1.inf = 0;
  G2A gen2;
  fq2_set(gen2.x, G2_GEN_X);
  fq2_set(gen2.y, G2_GEN_Y);
  gen2.inf = 0;
  Fr k;
  rand_scalar(k, g);
  G1J pj;
  jac_mul_fr(pj, gen1, k);
  G1A share;
  jac_to_aff(share, pj);
  uint32_t w1[12];
  g1_compress(w1, share);
  G2J qj;
  jac_mul_fr(qj, gen2, k);
  G2A sig;
  jac_to_aff(sig, qj);
  uint32_t w2[24];
  g2_compress(w2, sig);
  static Line l1[MILLER_STEPS], l2[MILLER_STEPS];

  // per-instance preparation
  hbtc_fqm_count = 0;
  G2A H;
  g2_decompress(H, w2);
  g2_precompute_lines(l1, H);
  const unsigned long long prepare = hbtc_fqm_count;
  g2_precompute_lines(l2, gen2);

  // decryption share
  hbtc_fqm_count = 0;
  G1A s;
  g1_decompress(s, w1);
  const unsigned long long dec_decode = hbtc_fqm_count;
  G1A npk;
  aff_neg(npk, gen1);
  Fq12 f, e;
  hbtc_fqm_count = 0;
  miller_loop_2(f, HL{l1}, s, true, HL{l2}, npk, true);
  const unsigned long long ml2 = hbtc_fqm_count;
  hbtc_fqm_count = 0;
  final_exponentiation(e, f);
  const unsigned long long fe = hbtc_fqm_count;

  // signature share
  hbtc_fqm_count = 0;
  G2A sg;
  g2_decompress(sg, w2);
  const unsigned long long sig_decode = hbtc_fqm_count;
  hbtc_fqm_count = 0;
  miller_loop_fixed_var(f, HL{l1}, gen1, true, npk, sg, true);
  const unsigned long long mlfv = hbtc_fqm_count;

  // combine term (G1): decode + 255-bit scalar mult + accumulate
  hbtc_fqm_count = 0;
  G1A cp;
  g1_decompress(cp, w1);
  G1J m, acc;
  jac_mul_fr(m, cp, k);
  jac_add(acc, pj, m);
  const unsigned long long comb1 = hbtc_fqm_count;
  hbtc_fqm_count = 0;
  G2A cq;
  g2_decompress(cq, w2);
  G2J m2, acc2;
  jac_mul_fr(m2, cq, k);
  jac_add(acc2, qj, m2);
  const unsigned long long comb2 = hbtc_fqm_count;

  // RLC item (k_rlc_items): decode (the subgroup test yields [|x|] d), r*d by xadic_mul_sac8
  // (the sign-aligned 8-entry common-Z table, one mixed addition per digit bit, plus the even-d0
  // correction, computed by every lane) over nbits = 16 (64-bit RLC)
  // or 32 (128-bit) digit bits, r*pk from the fixed-base table (4 nbits / 8 mixed additions, half
  // of them with phi), and the item's share of the plain + position-weighted reduction tree of
  // its tile: per side 3 * 63 Jacobian additions and 57 doublings, two sides, over 64 items
  const uint32_t dg[4] = {0xa5a55a5au, 0x5a5aa5a5u, 0x3c3cc3c3u, 0xc3c33c3cu};
  G1J rd;  // a generic accumulator, for the tree costs below
  unsigned long long rlc_item = 0, rlc_item_128 = 0, jadd = 0, jdbl = 0;
  {
    G1J pj2;
    jac_dbl(pj2, pj);
    hbtc_fqm_count = 0;
    G1J ts;
    jac_add(ts, pj, pj2);
    jadd = hbtc_fqm_count;
    hbtc_fqm_count = 0;
    jac_dbl(ts, ts);
    jdbl = hbtc_fqm_count;
  }
  const unsigned long long tree1 = (2 * (189 * jadd + 57 * jdbl) + 63) / 64;
  for (int nb : {16, 32}) {
    hbtc_fqm_count = 0;
    G1A d2;
    G1J t1;
    g1_decompress_t1(d2, t1, w1);
    jac_neg(t1, t1);
    Fq beta;
    fq_set(beta, G1_BETA);
    const uint32_t m = nb == 32 ? 0xffffffffu : 0xffffu;
#if HBTC_XADIC8
    // k_rlc_items' form: the co-Z chain table build, three entries in LDS (xadic_table8_chain)
    static uint32_t lds[3 * 24 * 64];
    xadic_mul_sac8<Fq, true>(rd, d2, t1, beta, dg[0] & m, dg[1] & m, dg[2] & m, dg[3] & m, nb, lds, 0);
#else
    G1A xp, pxp;
    xadic_table(xp, pxp, d2, t1);
    xadic_mul_uniform(rd, d2, xp, pxp, beta, dg[0] & m, dg[1] & m, dg[2] & m, dg[3] & m, nb);
#endif
    G1J rp;
    jac_set_inf(rp);
    jac_add_aff(rp, rp, gen1);
    for (int a = 1; a < nb / 2; ++a) {  // 4 nb / 8 table additions, half with phi
      G1A q = gen1;
      if (a & 1) g1_phi(q, gen1);
      jac_add_aff(rp, rp, q);
    }
    (nb == 16 ? rlc_item : rlc_item_128) = hbtc_fqm_count + tree1;
  }
  // SignatureShare RLC item (k_sig_items): G2 decode + subgroup test, r*sigma by the
  // two-addition x-adic loop in G2 ([x] s = psi(s), m = -psi^2 = (zeta x, y)), r*pk from the
  // fixed-base table, and the item's share of the G2 and G1 plain + weighted tile trees
  unsigned long long sig_item[2] = {};  // [nb == 32]
  for (int nb : {16, 32}) {
    hbtc_fqm_count = 0;
    G2A s2;
    g2_decompress(s2, w2);
    G2A xp;
    g2_psi(xp.x, xp.y, s2);
    xp.inf = 0;
    G2J xj;
    jac_from_aff(xj, xp);
    Fq zeta;
    fq_set(zeta, G2_ZETA);
    const uint32_t m = nb == 32 ? 0xffffffffu : 0xffffu;
    G2J r2;
    G2A pxp;
    xadic_table(xp, pxp, s2, xj);
    xadic_mul_uniform(r2, s2, xp, pxp, zeta, dg[0] & m, dg[1] & m, dg[2] & m, dg[3] & m, nb);
    G1J rp;
    jac_set_inf(rp);
    jac_add_aff(rp, rp, gen1);
    for (int a = 1; a < nb / 2; ++a) {
      G1A q = gen1;
      if (a & 1) g1_phi(q, gen1);
      jac_add_aff(rp, rp, q);
    }
    const unsigned long long mults = hbtc_fqm_count;
    hbtc_fqm_count = 0;
    G2J t2;
    jac_add(t2, r2, qj);
    const unsigned long long jadd2 = hbtc_fqm_count;
    hbtc_fqm_count = 0;
    jac_dbl(t2, t2);
    const unsigned long long jdbl2 = hbtc_fqm_count;
    sig_item[nb == 32] =
        mults + (2 * (189 * jadd2 + 57 * jdbl2) / 2 + 2 * (189 * jadd + 57 * jdbl) / 2 + 63) / 64;
  }
  G1J rp = rd;
  // group check: two normalisations + 2-pair Miller loop + final exponentiation
  hbtc_fqm_count = 0;
  G1A sa, pa;
  jac_to_aff(sa, rd);
  jac_to_aff(pa, rp);
  aff_neg(pa, pa);
  miller_loop_2(f, HL{l1}, sa, true, HL{l2}, pa, true);
  final_exponentiation(e, f);
  const unsigned long long rlc_group = hbtc_fqm_count;

  // Pippenger combine (t = 334, c = 6, W = 43, B = 32, S = 4), exact digit counts
  unsigned long long msm_combine = 0;
  {
    const int t = 334, c = 6, W = (256 + c - 1) / c, B = 1 << (c - 1), S = B / 8;
    hbtc_fqm_count = 0;
    G1A dp;
    g1_decompress(dp, w1, false);
    const unsigned long long dec_trusted = hbtc_fqm_count;
    hbtc_fqm_count = 0;
    G1J tj = pj;
    jac_add_aff(tj, tj, gen1);
    const unsigned long long madd = hbtc_fqm_count;
    hbtc_fqm_count = 0;
    G1A na;
    jac_to_aff(na, pj);
    const unsigned long long norm = hbtc_fqm_count;
    unsigned long long n_madd = 0;
    for (int i = 0; i < t; ++i) {
      Fr kk;
      rand_scalar(kk, g);
      uint32_t carry = 0;
      for (int w = 0; w < W; ++w) {
        const int bit = w * c;
        uint64_t two = 0;
        const int wi = bit >> 5, sh = bit & 31;
        two = ((uint64_t)(wi + 1 < 8 ? kk.v[wi + 1] : 0) << 32) | kk.v[wi];
        uint32_t v = (uint32_t)(two >> sh) & ((1u << c) - 1u);
        v += carry;
        int d;
        if (v > (uint32_t)B) { d = (int)v - (1 << c); carry = 1; } else { d = (int)v; carry = 0; }
        n_madd += d != 0;
      }
    }
    // per window: B running-sum closes + S segment adds of [base] run (base = B - 8s - 8 with
    // its bits as doublings and popcount adds), S-1 window-sum adds; then W-1 Horner steps
    unsigned long long seg = 0;
    for (int s2 = 0; s2 < S; ++s2) {
      const uint32_t base = B - 8 * s2 - 8;
      if (!base) continue;
      const int bits = 32 - __builtin_clz(base);
      seg += bits * jdbl + (__builtin_popcount(base) + 1) * jadd;
    }
    msm_combine = t * dec_trusted + n_madd * madd +
                  W * (B * jadd + seg + (S - 1) * jadd) + (W - 1) * (c * jdbl + jadd) + norm;
  }

  printf("{\n");
  printf("  \"unit\": \"Fqm (12x32-bit-limb CIOS Montgomery multiplications; 288 v_mad_u64_u32 + 12 v_mul_lo_u32 each)\",\n");
  printf("  \"mul32_per_fqm\": 300,\n  \"mad_u64_u32_per_fqm\": 288,\n");
  printf("  \"g2_prepare\": %llu,\n", prepare);
  printf("  \"dec_share\": {\"decode\": %llu, \"miller_loop_2\": %llu, \"final_exp\": %llu, \"total\": %llu},\n",
         dec_decode, ml2, fe, dec_decode + ml2 + fe);
  printf("  \"sig_share\": {\"decode\": %llu, \"miller_loop_fixed_var\": %llu, \"final_exp\": %llu, \"total\": %llu},\n",
         sig_decode, mlfv, fe, sig_decode + mlfv + fe);
  printf("  \"g1_combine_item\": %llu,\n  \"g2_combine_item\": %llu,\n", comb1, comb2);
  printf("  \"g1_msm_combine\": %llu,\n", msm_combine);
  // k_sig_items runs the two-addition loop only since round 5 (the G2 table is gone)
  printf("  \"rlc_item\": %llu,\n  \"rlc_item_128\": %llu,\n  \"sig_rlc_item\": %llu,\n"
         "  \"sig_rlc_item_128\": %llu,\n  \"rlc_group_check\": %llu\n}\n", rlc_item,
         rlc_item_128, sig_item[0], sig_item[1], rlc_group);
  return 0;
}
