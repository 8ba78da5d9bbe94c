// Random-linear-combination batch verification of pairing equalities with a per-item G2
// argument:  e(A_i, Q_i) == e(G1, W_i)  for every item i of a batch.  It is the fast path of
//   hbtc_verify_ciphertexts / hbtc_decrypt: Ciphertext::verify, e(G1, w) == e(u, H) with
//       H = hash_g1_g2(u, v) (A = u, Q = H, W = w; SecretKey::decrypt of the SyncKeyGen rows and
//       Ack values, /root/reference/src/sync_key_gen.rs:358,481-484), and
//   hbtc_verify_sigs: PublicKey::verify, e(pk, H) == e(G1, sigma) (A = pk, Q = H, W = sigma;
//       src/coin.rs:192-197, dynamic_honey_badger/votes.rs:154).
// The reference evaluates two full pairings per item.  Here, for a group G of consecutive items
// and ChaCha20 scalars r_i drawn per call (hbtc_rlc.hip explains the scalars and the bounds):
//     every item valid  =>  prod_G e(r_i A_i, Q_i) * e(-G1, sum_G r_i W_i) == 1
// one multi-Miller loop of |G| + 1 pairs and ONE final exponentiation per group, instead of
// |G| pairs of pairings.  Groups are 64-item tiles, then the 8-item sub-tiles of failing tiles,
// then exact per-item checks (k_pair_verify) of failing sub-tiles.
//
// Every pair has an affine G1 point and a G2 argument that varies, so every line table is
// projective (A, B, C per Miller step, pairing.h g2_proj_lines): k_pb_lines builds the table of
// each item's Q_i, k_plines (hbtc_sig.hip, modes 3 / 4) those of the groups' W sums; k_pb_ml
// (Miller partials per 8-item sub-tile) and k_pb_fe (group products, final exponentiations) in
// hbtc_check.hip evaluate them on the cooperative GT arithmetic of gt6.h.
#include "rlc_common.h"

namespace hbtc {

#ifndef HBTC_PB_ITEMS_WAVES
#define HBTC_PB_ITEMS_WAVES 1  // the G1 half and the decodes (the G2 half: k_pb_wsum_pair)
#endif

// One lane per item: decode A (G1, subgroup check; null = the G1 generator), W and Q (G2,
// subgroup checks; Q trusted = our own hash output, in the subgroup by construction: on-curve
// decode only), draw r_i, store r_i A_i (affine), the decoded Q_i and W_i.  An item that fails to
// decode gets DECODE_ERR and contributes nothing.  r_i W_i and its tile / sub-tile sums follow on
// lane pairs (k_pb_wsum_pair, hbtc_sig.hip).
__global__ void __launch_bounds__(64, HBTC_PB_ITEMS_WAVES) k_pb_items(uint32_t n, const uint8_t* __restrict__ a_c48,
                                                    const uint8_t* __restrict__ q_c96, bool q_trusted,
                                                    const uint8_t* __restrict__ w_c96, RlcKey key,
                                                    G1A* __restrict__ rA, G2A* __restrict__ Qdec,
                                                    G2A* __restrict__ Wdec,
                                                    int32_t* __restrict__ status,
                                                    G1A* __restrict__ adec) {
  const uint32_t lane = threadIdx.x;
  const uint32_t i = blockIdx.x * 64u + lane;
  if (i < n) {
    uint32_t w[24];
    G1A A;
    G1J t1;  // [|x|] A (the subgroup test's first half): [x] A = -t1 for the x-adic table
    G2A Q, W;
    bool ok = true;
    if (a_c48) {
      rlc_load_words(w, a_c48, i, 12);
      ok = g1_decompress_t1(A, t1, w);
    } else {
      fq_set(A.x, G1_GEN_X);
      fq_set(A.y, G1_GEN_Y);
      A.inf = 0;
      jac_mul_u64(t1, A, BLS_X_ABS);
    }
    rlc_load_words(w, q_c96, i, 24);
    ok = g2_decompress(Q, w, !q_trusted) && ok;
    rlc_load_words(w, w_c96, i, 24);
    ok = g2_decompress(W, w) && ok;
    G1A ra;
    ra.inf = 1;
    if (ok) {
      // the x-adic scalar r_i (rlc_common.h rlc_digits), the same for A_i (G1: [x] A = -t1, m =
      // phi) and W_i (G2: [x] W = psi(W), m = -psi^2): both endomorphism pairs have the
      // eigenvalues x and mu = -x^2
      const XDigits xd = rlc_digits(key, i);
      if (!A.inf && !Q.inf) {  // r A, affine (one binary-Euclid inversion)
        jac_neg(t1, t1);
        Fq beta;
        fq_set(beta, G1_BETA);
        G1J t;
#if HBTC_XADIC8
        xadic_mul_sac8(t, A, t1, beta, xd.d[0], xd.d[1], xd.d[2], xd.d[3], xd.nbits);
#else
        G1A xp, pxp;
        xadic_table(xp, pxp, A, t1);
        xadic_mul_uniform(t, A, xp, pxp, beta, xd.d[0], xd.d[1], xd.d[2], xd.d[3], xd.nbits);
#endif
        if (!jac_is_inf(t)) {
          Fq zi, zi2, zi3;
          finv_fast(zi, t.z);
          fq_sqr(zi2, zi);
          fq_mul(zi3, zi2, zi);
          fq_mul(ra.x, t.x, zi2);
          fq_mul(ra.y, t.y, zi3);
          ra.inf = 0;
        }
      }
    }
    rA[i] = ra;
    Qdec[i] = Q;
    Wdec[i] = W;  // r W and the tile sums: k_pb_wsum_pair (hbtc_sig.hip), on lane pairs
    if (adec) adec[i] = A;  // the decoded A for the caller (hbtc_decrypt's g = sk u)
    status[i] = ok ? HBTC_RLC_PENDING : HBTC_DECODE_ERR;
  }
}

// The projective line table of every pending item's Q_i (one lane per item).
__global__ void __launch_bounds__(64) k_pb_lines(uint32_t n, const G2A* __restrict__ Qdec,
                                                 const int32_t* __restrict__ status,
                                                 Fq2* __restrict__ tables) {
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  if (i >= n || status[i] != HBTC_RLC_PENDING) return;
  const G2A Q = Qdec[i];
  if (Q.inf) return;  // the pair is unused (e(A, O) = 1)
  g2_proj_lines(tables + (size_t)i * PLINES_FQ2, Q);
}

// The items of a failing sub-tile, gathered for the exact checks (pb_exact_list): list[0, n).
__global__ void __launch_bounds__(64) k_pb_gather(uint32_t n, const uint32_t* __restrict__ list,
                                                  const uint8_t* __restrict__ a, const uint8_t* __restrict__ q,
                                                  const uint8_t* __restrict__ w, uint8_t* __restrict__ ga,
                                                  uint8_t* __restrict__ gq, uint8_t* __restrict__ gw) {
  const uint32_t g = blockIdx.x * 64u + threadIdx.x;
  if (g >= n) return;
  const size_t i = list[g];
  const uint4* sa = reinterpret_cast<const uint4*>(a + 48 * i);
  const uint4* sq = reinterpret_cast<const uint4*>(q + 96 * i);
  const uint4* sw = reinterpret_cast<const uint4*>(w + 96 * i);
  uint4* da = reinterpret_cast<uint4*>(ga + (size_t)48 * g);
  uint4* dq = reinterpret_cast<uint4*>(gq + (size_t)96 * g);
  uint4* dw = reinterpret_cast<uint4*>(gw + (size_t)96 * g);
  for (int j = 0; j < 3; ++j) da[j] = sa[j];
  for (int j = 0; j < 6; ++j) {
    dq[j] = sq[j];
    dw[j] = sw[j];
  }
}
__global__ void __launch_bounds__(64) k_pb_scatter(uint32_t n, const uint32_t* __restrict__ list,
                                                   const int32_t* __restrict__ gst, int32_t* __restrict__ st) {
  const uint32_t g = blockIdx.x * 64u + threadIdx.x;
  if (g < n) st[list[g]] = gst[g];
}
hipError_t launch_pb_gather(hipStream_t s, uint32_t n, const uint32_t* list, const uint8_t* a,
                            const uint8_t* q, const uint8_t* w, uint8_t* ga, uint8_t* gq, uint8_t* gw) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pb_gather, dim3((n + 63) / 64), dim3(64), 0, s, n, list, a, q, w, ga, gq, gw);
  return hipGetLastError();
}
hipError_t launch_pb_scatter(hipStream_t s, uint32_t n, const uint32_t* list, const int32_t* gst,
                             int32_t* st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pb_scatter, dim3((n + 63) / 64), dim3(64), 0, s, n, list, gst, st);
  return hipGetLastError();
}

hipError_t launch_pb_items(hipStream_t s, uint32_t n, const uint8_t* a_c48, const uint8_t* q_c96,
                           bool q_trusted, const uint8_t* w_c96, RlcKey key, G1A* rA, G2A* Qdec,
                           G2A* Wdec, SigTileSums* sums, int32_t* status, G1A* adec) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pb_items, dim3((n + 63) / 64), dim3(64), 0, s, n, a_c48, q_c96, q_trusted, w_c96,
                     key, rA, Qdec, Wdec, status, adec);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_pb_wsum(s, n, key, Wdec, status, sums);
}

// g_i = [k] A_i for the ACCEPTed items of a pair batch (hbtc_decrypt: g = sk u), from the decoded
// A_i and the host's split k = k0 + k1 x^2 (k0 < x^2, k1 < 2^128): [k] A = [k0] A + [k1] m(A)
// with m(A) = -phi(A) = (beta x, -y) = [x^2] A on G1 -- a joint 128-bit double-and-add whose
// bits are the same on every lane (no divergence) over {A, m(A), A + m(A)}, instead of a fresh
// decode and a 255-bit double-and-add (k_point_mul).  Other items: zero bytes.
__global__ void __launch_bounds__(64) k_pb_mul_glv(uint32_t n, const G1A* __restrict__ adec,
                                                   const int32_t* __restrict__ status,
                                                   Limbs<4> k0, Limbs<4> k1,
                                                   uint32_t* __restrict__ out_w) {
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  if (i >= n) return;
  uint32_t w[12];
  for (int j = 0; j < 12; ++j) w[j] = 0;
  if (status[i] == HBTC_ACCEPT) {
    const G1A A = adec[i];
    G1A m, am;
    {
      Fq beta;
      fq_set(beta, G1_BETA);
      fq_mul(m.x, A.x, beta);
      fq_neg(m.y, A.y);
      m.inf = A.inf;
      G1J s;
      jac_from_aff(s, A);
      jac_add_aff(s, s, m);  // [1 + x^2] A: O only for A = O
      am.inf = jac_is_inf(s) ? 1u : 0u;
      if (!am.inf) {
        Fq zi, zi2, zi3;
        finv_fast(zi, s.z);
        fq_sqr(zi2, zi);
        fq_mul(zi3, zi2, zi);
        fq_mul(am.x, s.x, zi2);
        fq_mul(am.y, s.y, zi3);
      }
    }
    G1J acc;
    jac_set_inf(acc);
#pragma unroll 1
    for (int bit = 127; bit >= 0; --bit) {
      jac_dbl(acc, acc);
      const bool ba = ((k0.v[bit >> 5] >> (bit & 31)) & 1u) != 0;
      const bool bb = ((k1.v[bit >> 5] >> (bit & 31)) & 1u) != 0;
      if (ba && bb)
        jac_add_aff(acc, acc, am);
      else if (ba)
        jac_add_aff(acc, acc, A);
      else if (bb)
        jac_add_aff(acc, acc, m);
    }
    G1A g;
    g.inf = jac_is_inf(acc) ? 1u : 0u;
    if (!g.inf) {
      Fq zi, zi2, zi3;
      finv_fast(zi, acc.z);
      fq_sqr(zi2, zi);
      fq_mul(zi3, zi2, zi);
      fq_mul(g.x, acc.x, zi2);
      fq_mul(g.y, acc.y, zi3);
    } else {
      fq_zero(g.x);
      fq_zero(g.y);
    }
    g1_compress(w, g);
  }
  uint4* o = reinterpret_cast<uint4*>(out_w + 12 * (size_t)i);
  for (int k = 0; k < 3; ++k) o[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}

hipError_t launch_pb_mul_glv(hipStream_t s, uint32_t n, const G1A* adec, const int32_t* status,
                             const uint32_t* k0, const uint32_t* k1, uint8_t* out_c48) {
  if (n == 0) return hipSuccess;
  Limbs<4> a, b;
  for (int j = 0; j < 4; ++j) {
    a.v[j] = k0[j];
    b.v[j] = k1[j];
  }
  hipLaunchKernelGGL(k_pb_mul_glv, dim3((n + 63) / 64), dim3(64), 0, s, n, adec, status, a, b,
                     reinterpret_cast<uint32_t*>(out_c48));
  return hipGetLastError();
}

hipError_t launch_pb_lines(hipStream_t s, uint32_t n, const G2A* Qdec, const int32_t* status,
                           Fq2* tables) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pb_lines, dim3((n + 63) / 64), dim3(64), 0, s, n, Qdec, status, tables);
  return hipGetLastError();
}

}  // namespace hbtc
