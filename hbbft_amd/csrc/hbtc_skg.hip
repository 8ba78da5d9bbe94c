// SyncKeyGen checks on gfx950 (reference src/sync_key_gen.rs:338-498).
//
// A node handling a Part checks `row.commitment() != commit.row(our_idx + 1)` (:366) and, per
// Ack, `commit.evaluate(our_idx + 1, sender_idx + 1) != G1Affine::one().mul(val)` (:493).
// BivarCommitment stores the (t+1)(t+2)/2 coefficients C_ij (i <= j) of a symmetric bivariate
// polynomial at coeff_pos(i, j) = j(j+1)/2 + i.  Both checks become ONE Pippenger MSM per Part
// over those points (hbtc_msm.hip), with the scalar of the stored C_ij
//
//     s_ij = U_i V_j + U_j V_i   (i < j),      s_ii = U_i V_i,
//
// plus one extra generator term carrying the right-hand side, so the check is "MSM == O":
//   * Part (A10 + A11): U = rho (random, fresh per call), V = (x^j): sum_i rho_i row_i(x) ==
//     [sum_i rho_i a_i] G1 — all t+1 row coefficients at once, error probability <= 1/r;
//   * Acks of one Part (A12): U = (x^i), V = Y with Y_j = sum_a rho_a y_a^j: the random linear
//     combination of that Part's Ack equations; a failing combination falls back to one exact
//     MSM per Ack (Y_j = y_a^j).
// k_skg_ack_rows is the exact shortcut for Parts whose row this node has verified: then
// commit.row(x) == [a_j] G1 coefficient-wise, so evaluate(x, y) == [row(y)] G1 and the Ack check
// is the scalar equation val == row(y) (identical decision, no curve arithmetic).
#include "hbtc_kernels.h"

#ifndef HBTC_PART
#define HBTC_PART 0
#endif
#define HBTC_IN_PART(n) (HBTC_PART == 0 || HBTC_PART == (n))

namespace hbtc {

#if HBTC_IN_PART(10)
// out[p][q] (canonical) for q < M from the packed (i | j << 16) table, out[p][M] = tail[p].
// U, V are Montgomery Fr with per-part strides (0: shared by all parts).
__global__ void __launch_bounds__(256) k_skg_sym_scalars(uint32_t n_parts, uint32_t M,
                                                         const Fr* __restrict__ U,
                                                         uint32_t u_stride,
                                                         const Fr* __restrict__ V,
                                                         uint32_t v_stride,
                                                         const uint32_t* __restrict__ ij,
                                                         const Fr* __restrict__ tail,
                                                         Fr* __restrict__ out) {
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t per = (uint64_t)M + 1;
  if (g >= (uint64_t)n_parts * per) return;
  const uint64_t p = g / per;
  const uint32_t q = (uint32_t)(g % per);
  if (q == M) {
    out[g] = tail[p];
    return;
  }
  const uint32_t i = ij[q] & 0xffffu, j = ij[q] >> 16;
  const Fr* u = U + p * u_stride;
  const Fr* v = V + p * v_stride;
  Fr a;
  fr_mul(a, u[i], v[j]);
  if (i != j) {
    Fr b;
    fr_mul(b, u[j], v[i]);
    fr_add(a, a, b);
  }
  Fr c;
  fr_from_mont(c, a);
  out[g] = c;
}

// Ack value check against a verified row: val == row(sender + 1) (Horner over Montgomery Fr).
__global__ void __launch_bounds__(256) k_skg_ack_rows(uint32_t n_acks, uint32_t t1,
                                                      const Fr* __restrict__ rows,
                                                      const uint32_t* __restrict__ ack_part,
                                                      const uint32_t* __restrict__ ack_sender,
                                                      const Fr* __restrict__ vals,
                                                      int32_t* __restrict__ status) {
  const uint32_t a = blockIdx.x * 256 + threadIdx.x;
  if (a >= n_acks) return;
  const Fr* row = rows + (size_t)ack_part[a] * t1;
  Fr y, acc;
  fr_from_u64(y, (uint64_t)ack_sender[a] + 1);
  acc = row[t1 - 1];
  for (int j = (int)t1 - 2; j >= 0; --j) {
    fr_mul(acc, acc, y);
    fr_add(acc, acc, row[j]);
  }
  Fr c;
  fr_from_mont(c, acc);
  const Fr v = vals[a];
  uint32_t diff = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) diff |= c.v[k] ^ v.v[k];
  status[a] = diff ? HBTC_REJECT : HBTC_ACCEPT;
}

static inline uint32_t skg_blocks(uint64_t n, uint32_t bs) { return (uint32_t)((n + bs - 1) / bs); }

hipError_t launch_skg_sym_scalars(hipStream_t s, uint32_t n_parts, uint32_t M, const Fr* U,
                                  uint32_t u_stride, const Fr* V, uint32_t v_stride,
                                  const uint32_t* ij, const Fr* tail, Fr* out) {
  const uint64_t n = (uint64_t)n_parts * (M + 1);
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_skg_sym_scalars, dim3(skg_blocks(n, 256)), dim3(256), 0, s, n_parts, M, U,
                     u_stride, V, v_stride, ij, tail, out);
  return hipGetLastError();
}

hipError_t launch_skg_ack_rows(hipStream_t s, uint32_t n_acks, uint32_t t1, const Fr* rows,
                               const uint32_t* ack_part, const uint32_t* ack_sender,
                               const Fr* vals, int32_t* status) {
  if (n_acks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_skg_ack_rows, dim3(skg_blocks(n_acks, 256)), dim3(256), 0, s, n_acks, t1,
                     rows, ack_part, ack_sender, vals, status);
  return hipGetLastError();
}
#endif  // part 10

}  // namespace hbtc
