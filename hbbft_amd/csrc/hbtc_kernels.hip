// gfx950 kernels of the batched threshold-crypto verifier (C ABI in include/hbtc.h, host side
// in hbtc_api.hip).
//
// Replaces, per item, threshold_crypto's pairing checks and combines as called by hbbft
// (SURVEY.md §8a): PublicKeyShare::verify (src/coin.rs:151), verify_decryption_share
// (src/threshold_decryption.rs:159), PublicKey::verify (src/coin.rs:196), Ciphertext::verify
// (src/threshold_decryption.rs:98), combine_signatures / decrypt (src/coin.rs:190,
// src/threshold_decryption.rs:184) and the zcash point codec of their serde impls.
//
// Data layout in HBM:
//   * compressed items exactly as on hbbft's wire, item-major (G1 48 B, G2 96 B), read with
//     16-byte loads as little-endian words of the big-endian byte string (curve.h's codec
//     works on those words directly);
//   * decoded points G1A / G2A (canonical Montgomery limbs + infinity flag);
//   * per-instance line tables: 68 Lines (2 Fq2 = 192 B) per fixed G2 argument.  A wave only
//     ever verifies items of ONE instance (a Tile = up to 64 consecutive items), so every lane
//     reads the same line: the loads are wave-uniform and go through the scalar cache into
//     SGPRs, which the multiplies consume directly as operands.
#include "hbtc_kernels.h"

// The file is compiled once per kernel group (Makefile: -DHBTC_PART=1..5) so the groups,
// each minutes of register allocation, build in parallel; HBTC_PART=0 builds all of them.
#ifndef HBTC_PART
#define HBTC_PART 0
#endif
#define HBTC_IN_PART(n) (HBTC_PART == 0 || HBTC_PART == (n))

namespace hbtc {

// ------------------------------------------------------------------------------ helpers
__device__ __forceinline__ void load_words(uint32_t* w, const uint8_t* base, size_t item,
                                           int nwords) {
  const uint4* q = reinterpret_cast<const uint4*>(base + item * (size_t)(nwords * 4));
  for (int i = 0; i < nwords / 4; ++i) {
    const uint4 v = q[i];
    w[4 * i] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
}

__device__ __forceinline__ void store_words(uint8_t* base, size_t item, const uint32_t* w,
                                            int nwords) {
  uint4* q = reinterpret_cast<uint4*>(base + item * (size_t)(nwords * 4));
  for (int i = 0; i < nwords / 4; ++i) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

struct TableLines {
  const Line* __restrict__ l;
  __device__ __forceinline__ void load(Line& out, int j) const { out = l[j]; }
};

__device__ __forceinline__ void neg_g1_generator(G1A& g) {
  fq_set(g.x, G1_GEN_X);
  Fq y;
  fq_set(y, G1_GEN_Y);
  fq_neg(g.y, y);
  g.inf = 0;
}

__device__ __forceinline__ void g1_generator(G1A& g) {
  fq_set(g.x, G1_GEN_X);
  fq_set(g.y, G1_GEN_Y);
  g.inf = 0;
}

HD bool pt_decompress(G1A& p, const uint32_t* w) { return g1_decompress(p, w); }
HD bool pt_decompress(G2A& p, const uint32_t* w) { return g2_decompress(p, w); }
HD void pt_compress(uint32_t* w, const G1A& p) { g1_compress(w, p); }
HD void pt_compress(uint32_t* w, const G2A& p) { g2_compress(w, p); }

#if HBTC_IN_PART(1)
// ------------------------------------------------------------------------------ decode / prepare
__global__ void __launch_bounds__(64) k_g1_decode(const uint8_t* __restrict__ in, uint32_t n,
                                                  G1A* __restrict__ out,
                                                  int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  uint32_t w[12];
  load_words(w, in, i, 12);
  G1A p;
  const bool ok = g1_decompress(p, w);
  out[i] = p;
  status[i] = ok ? HBTC_ACCEPT : HBTC_DECODE_ERR;
}

// Decode the fixed per-instance G2 arguments (H = hash_g2(nonce), and w for ciphertexts) and
// walk their Miller-loop steps: one lane per argument, both argument sets in ONE launch
// (in0: n0 items, in1: n1 items; outputs [0, n0) then [n0, n0 + n1)).  The 68 projective
// lines (A, B, C) go to the workspace; k_g2_norm scales them affine in parallel.
__global__ void __launch_bounds__(64) k_g2_steps(const uint8_t* __restrict__ in0, uint32_t n0,
                                                 const uint8_t* __restrict__ in1, uint32_t n1,
                                                 G2A* __restrict__ aff, Fq2* __restrict__ ws,
                                                 int32_t* __restrict__ status) {
  HBTC_LATENCY_PRIO();
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (g >= n0 + n1) return;
  uint32_t w[24];
  load_words(w, g < n0 ? in0 : in1, g < n0 ? g : g - n0, 24);
  G2A q;
  // the subgroup test (psi(Q) == -[|x|] Q, curve.h g2_in_subgroup) reuses the Miller loop's own
  // double-and-add: after the 68 steps T = [|x|] Q
  bool ok = g2_decompress(q, w, false);
  aff[g] = q;
  if (!ok || q.inf) {
    status[g] = ok ? HBTC_ACCEPT : HBTC_DECODE_ERR;
    return;
  }
  Fq2* out = ws + (size_t)g * 3 * MILLER_STEPS;
  G2J T;
  jac_from_aff(T, q);
  int j = 0;
  for (int bit = 62; bit >= 0; --bit) {
    Fq2 A, B, C;
    g2_dbl_line(T, A, B, C);
    out[3 * j] = A;
    out[3 * j + 1] = B;
    out[3 * j + 2] = C;
    ++j;
    if ((BLS_X_ABS >> bit) & 1ull) {
      g2_add_step(T, q, A, B, C);
      out[3 * j] = A;
      out[3 * j + 1] = B;
      out[3 * j + 2] = C;
      ++j;
    }
  }
  Fq2 px, py, npy;
  g2_psi(px, py, q);
  fq2_neg(npy, py);
  ok = !jac_is_inf(T) && jac_eq_aff(T, px, npy);
  status[g] = ok ? HBTC_ACCEPT : HBTC_DECODE_ERR;
}

// One lane per (argument, step): the affine-normalised line (A / C, B / C) (pairing.h Line).
__global__ void __launch_bounds__(64) k_g2_norm(uint32_t n, const G2A* __restrict__ aff,
                                                const int32_t* __restrict__ status,
                                                const Fq2* __restrict__ ws,
                                                Line* __restrict__ lines) {
  HBTC_LATENCY_PRIO();
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (g >= n * MILLER_STEPS) return;
  const uint32_t a = g / MILLER_STEPS;
  if (status[a] != HBTC_ACCEPT || aff[a].inf) return;  // never read: the pair is unused
  const Fq2* in = ws + (size_t)g * 3;
  // 1 / C = conj(C) / (c0^2 + c1^2), the Fq inversion by binary extended Euclid (field.h)
  Fq2 ci;
  {
    Fq n0, n1, ni;
    fq_sqr(n0, in[2].c0);
    fq_sqr(n1, in[2].c1);
    fq_add(n0, n0, n1);
    fq_inv_binary(ni, n0);
    fq_mul(ci.c0, in[2].c0, ni);
    fq_mul(n1, in[2].c1, ni);
    fq_neg(ci.c1, n1);
  }
  Line l;
  fq2_mul(l.a, in[0], ci);
  fq2_mul(l.b, in[1], ci);
  lines[g] = l;
}

// Fixed-base tables of the key set (PK_TAB_WIN windows of 8 bits): one lane per (share i,
// window w) walks v * B for B = 2^(8w) pk_i, v = 1..255, in Jacobian coordinates and
// normalises the 255 points with one batched inversion (ws: 512 Fq per lane).
__global__ void __launch_bounds__(64) k_pk_table(const G1A* __restrict__ pk,
                                                 const int32_t* __restrict__ pk_status,
                                                 uint32_t n, PtXY* __restrict__ tab,
                                                 Fq* __restrict__ ws) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (g >= n * PK_TAB_WIN) return;
  const uint32_t i = g / PK_TAB_WIN, win = g % PK_TAB_WIN;
  PtXY* out = tab + (size_t)g * 256;
  Fq* zs = ws + (size_t)g * 512;  // [0, 256): Z_v, [256, 512): prefix products
  const G1A p = pk[i];
  if (pk_status[i] != HBTC_ACCEPT || p.inf) return;  // never read (items check pk first)
  // windows 0..3: multiples of pk; 4..7: of [x] pk = -[|x|] pk (the x-adic RLC digits d1, d3)
  G1J b;
  if (win < 4) {
    jac_from_aff(b, p);
  } else {
    jac_mul_u64(b, p, BLS_X_ABS);
    jac_neg(b, b);
  }
  for (uint32_t j = 0; j < 8 * (win & 3u); ++j) jac_dbl(b, b);
  G1A base;
  jac_to_aff(base, b);
  G1J acc;
  jac_set_inf(acc);
  Fq pre;
  fq_one(pre);
  for (int v = 1; v < 256; ++v) {
    jac_add_aff(acc, acc, base);  // v B != O: v 2^(8w) < r
    out[v].x = acc.x;
    out[v].y = acc.y;
    zs[v] = acc.z;
    fq_mul(pre, pre, acc.z);
    zs[256 + v] = pre;
  }
  Fq inv;
  fq_inv(inv, pre);
  for (int v = 255; v >= 1; --v) {
    Fq zi, zi2, t;
    if (v > 1)
      fq_mul(zi, inv, zs[256 + v - 1]);
    else
      zi = inv;
    fq_mul(inv, inv, zs[v]);
    fq_sqr(zi2, zi);
    PtXY e = out[v];
    fq_mul(t, e.x, zi2);
    fq_canon(e.x, t);
    fq_mul(zi2, zi2, zi);
    fq_mul(t, e.y, zi2);
    fq_canon(e.y, t);
    out[v] = e;
  }
  fq_zero(out[0].x);
  fq_zero(out[0].y);
}

#endif  // part 1

// ------------------------------------------------------------------------------ share checks
#if HBTC_IN_PART(2)
// DecryptionShare: e(share_i, H_k) == e(pk_idx, w_k)  <=>  e(share_i, H_k) e(-pk_idx, w_k) == 1.
// Both G2 arguments are per-ciphertext constants: two precomputed line tables, one Fq12
// squaring chain, one final exponentiation per item.
__global__ void __launch_bounds__(64) k_dec_verify(
    const Tile* __restrict__ tiles, const uint32_t* __restrict__ idx,
    const uint8_t* __restrict__ shares, const G1A* __restrict__ pk,
    const int32_t* __restrict__ pk_status, uint32_t n_pk, const G2A* __restrict__ h_aff,
    const int32_t* __restrict__ h_status, const Line* __restrict__ h_lines,
    const G2A* __restrict__ w_aff, const int32_t* __restrict__ w_status,
    const Line* __restrict__ w_lines, int32_t* __restrict__ status) {
  const Tile tile = tiles[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  if (lane >= tile.count) return;
  const size_t item = (size_t)tile.first + lane;
  const uint32_t k = tile.inst;
  if (h_status[k] != HBTC_ACCEPT || w_status[k] != HBTC_ACCEPT) {
    status[item] = HBTC_INSTANCE_ERR;
    return;
  }
  const uint32_t id = idx[item];
  if (id >= n_pk) {
    status[item] = HBTC_UNKNOWN_SENDER;
    return;
  }
  if (pk_status[id] != HBTC_ACCEPT) {
    status[item] = HBTC_DECODE_ERR;
    return;
  }
  uint32_t w[12];
  load_words(w, shares, item, 12);
  G1A s;
  if (!g1_decompress(s, w)) {
    status[item] = HBTC_DECODE_ERR;
    return;
  }
  G1A npk;
  aff_neg(npk, pk[id]);
  const bool h_inf = h_aff[k].inf != 0, w_inf = w_aff[k].inf != 0;
  Fq12 f, e;
  miller_loop_2(f, TableLines{h_lines + (size_t)k * MILLER_STEPS}, s, !s.inf && !h_inf,
                TableLines{w_lines + (size_t)k * MILLER_STEPS}, npk, !npk.inf && !w_inf);
  final_exponentiation(e, f);
  status[item] = fq12_is_one(e) ? HBTC_ACCEPT : HBTC_REJECT;
}

#endif  // part 2

#if HBTC_IN_PART(3)
// SignatureShare: e(pk_idx, H_k) == e(G1, sig_i)  <=>  e(pk_idx, H_k) e(-G1, sig_i) == 1.
// H_k's lines are precomputed per instance; sig_i's lines are computed on the fly.
__global__ void __launch_bounds__(64) k_sig_verify(
    const Tile* __restrict__ tiles, const uint32_t* __restrict__ idx,
    const uint8_t* __restrict__ sigs, const G1A* __restrict__ pk,
    const int32_t* __restrict__ pk_status, uint32_t n_pk, const G2A* __restrict__ h_aff,
    const int32_t* __restrict__ h_status, const Line* __restrict__ h_lines,
    int32_t* __restrict__ status) {
  const Tile tile = tiles[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  if (lane >= tile.count) return;
  const size_t item = (size_t)tile.first + lane;
  const uint32_t k = tile.inst;
  if (h_status[k] != HBTC_ACCEPT) {
    status[item] = HBTC_INSTANCE_ERR;
    return;
  }
  const uint32_t id = idx[item];
  if (id >= n_pk) {
    status[item] = HBTC_UNKNOWN_SENDER;
    return;
  }
  if (pk_status[id] != HBTC_ACCEPT) {
    status[item] = HBTC_DECODE_ERR;
    return;
  }
  uint32_t w[24];
  load_words(w, sigs, item, 24);
  G2A sg;
  if (!g2_decompress(sg, w)) {
    status[item] = HBTC_DECODE_ERR;
    return;
  }
  const G1A P = pk[id];
  G1A ng;
  neg_g1_generator(ng);
  const bool h_inf = h_aff[k].inf != 0;
  Fq12 f, e;
  miller_loop_fixed_var(f, TableLines{h_lines + (size_t)k * MILLER_STEPS}, P,
                        !P.inf && !h_inf, ng, sg, !sg.inf);
  final_exponentiation(e, f);
  status[item] = fq12_is_one(e) ? HBTC_ACCEPT : HBTC_REJECT;
}

#endif  // part 3

#if HBTC_IN_PART(4)
// Generic e(a1, a2) == e(b1, b2) with every argument per item; a null G1 pointer means the
// G1 generator.  verify_sigs: (pk, H) vs (G1, sig).  verify_ciphertexts: (G1, w) vs (u, H).
// With `count` non-null: only the *count items list[0 ..) (the exact checks behind a failing
// pair-batch group, hbtc_pb.hip).
__global__ void __launch_bounds__(64) k_pair_verify(uint32_t n, const uint8_t* __restrict__ a1,
                                                    const uint8_t* __restrict__ a2,
                                                    const uint8_t* __restrict__ b1,
                                                    const uint8_t* __restrict__ b2,
                                                    int32_t* __restrict__ status,
                                                    const uint32_t* __restrict__ list,
                                                    const uint32_t* __restrict__ count) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (count) n = *count;
  if (g >= n) return;
  const uint32_t i = count ? list[g] : g;
  uint32_t w[24];
  G1A A1, B1;
  G2A A2, B2;
  bool ok = true;
  if (a1) {
    load_words(w, a1, i, 12);
    ok &= g1_decompress(A1, w);
  } else {
    g1_generator(A1);
  }
  if (b1) {
    load_words(w, b1, i, 12);
    ok &= g1_decompress(B1, w);
  } else {
    g1_generator(B1);
  }
  load_words(w, a2, i, 24);
  ok &= g2_decompress(A2, w);
  load_words(w, b2, i, 24);
  ok &= g2_decompress(B2, w);
  if (!ok) {
    status[i] = HBTC_DECODE_ERR;
    return;
  }
  G1A nB1;
  aff_neg(nB1, B1);
  Fq12 f, e;
  miller_loop_var_var(f, A1, A2, !A1.inf && !A2.inf, nB1, B2, !nB1.inf && !B2.inf);
  final_exponentiation(e, f);
  status[i] = fq12_is_one(e) ? HBTC_ACCEPT : HBTC_REJECT;
}

#endif  // part 4

#if HBTC_IN_PART(1)
// ------------------------------------------------------------------------------ scalar mult
template <class F, int NW>
__global__ void __launch_bounds__(64) k_point_mul(uint32_t n, const uint8_t* __restrict__ base,
                                                  uint32_t base_stride,
                                                  const uint8_t* __restrict__ scalars,
                                                  uint32_t scalar_stride,
                                                  uint8_t* __restrict__ out,
                                                  int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  uint32_t w[NW];
  load_words(w, base, (size_t)i * base_stride, NW);
  Aff<F> p;
  if (!pt_decompress(p, w)) {
    status[i] = HBTC_DECODE_ERR;
    for (int j = 0; j < NW; ++j) w[j] = 0;
    store_words(out, i, w, NW);
    return;
  }
  Fr k;
  load_words(k.v, scalars, (size_t)i * scalar_stride, 8);
  Jac<F> r;
  jac_mul_fr(r, p, k);
  Aff<F> a;
  jac_to_aff(a, r);
  pt_compress(w, a);
  store_words(out, i, w, NW);
  status[i] = HBTC_ACCEPT;
}

template __global__ void k_point_mul<Fq, 12>(uint32_t, const uint8_t*, uint32_t, const uint8_t*,
                                             uint32_t, uint8_t*, int32_t*);
template __global__ void k_point_mul<Fq2, 24>(uint32_t, const uint8_t*, uint32_t,
                                              const uint8_t*, uint32_t, uint8_t*, int32_t*);

#endif  // part 1


// ------------------------------------------------------------------------------ launchers
static inline uint32_t blocks_for(uint64_t n, uint32_t bs) { return (uint32_t)((n + bs - 1) / bs); }

#if HBTC_IN_PART(1)
hipError_t launch_g1_decode(hipStream_t s, const uint8_t* in, uint32_t n, G1A* out,
                            int32_t* status) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_g1_decode, dim3(blocks_for(n, 64)), dim3(64), 0, s, in, n, out, status);
  return hipGetLastError();
}

hipError_t launch_pk_table(hipStream_t s, const G1A* pk, const int32_t* pk_status, uint32_t n,
                           PtXY* tab, Fq* ws) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pk_table, dim3(blocks_for((uint64_t)n * PK_TAB_WIN, 64)), dim3(64), 0, s, pk,
                     pk_status, n, tab, ws);
  return hipGetLastError();
}

hipError_t launch_g2_prepare(hipStream_t s, const uint8_t* in0, uint32_t n0, const uint8_t* in1,
                             uint32_t n1, G2A* aff, Line* lines, Fq2* ws, int32_t* status) {
  const uint32_t n = n0 + n1;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_g2_steps, dim3(blocks_for(n, 64)), dim3(64), 0, s, in0, n0, in1, n1, aff, ws,
                     status);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_g2_norm, dim3(blocks_for((uint64_t)n * MILLER_STEPS, 64)), dim3(64), 0, s, n,
                     aff, status, ws, lines);
  return hipGetLastError();
}

#endif  // part 1

#if HBTC_IN_PART(2)
hipError_t launch_dec_verify(hipStream_t s, uint32_t n_tiles, const Tile* tiles,
                             const uint32_t* idx, const uint8_t* shares, const G1A* pk,
                             const int32_t* pk_status, uint32_t n_pk, const G2A* h_aff,
                             const int32_t* h_status, const Line* h_lines, const G2A* w_aff,
                             const int32_t* w_status, const Line* w_lines, int32_t* status) {
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_dec_verify, dim3(n_tiles), dim3(64), 0, s, tiles, idx, shares, pk,
                     pk_status, n_pk, h_aff, h_status, h_lines, w_aff, w_status, w_lines, status);
  return hipGetLastError();
}

#endif  // part 2

#if HBTC_IN_PART(3)
hipError_t launch_sig_verify(hipStream_t s, uint32_t n_tiles, const Tile* tiles,
                             const uint32_t* idx, const uint8_t* sigs, const G1A* pk,
                             const int32_t* pk_status, uint32_t n_pk, const G2A* h_aff,
                             const int32_t* h_status, const Line* h_lines, int32_t* status) {
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sig_verify, dim3(n_tiles), dim3(64), 0, s, tiles, idx, sigs, pk,
                     pk_status, n_pk, h_aff, h_status, h_lines, status);
  return hipGetLastError();
}

#endif  // part 3

#if HBTC_IN_PART(4)
hipError_t launch_pair_verify(hipStream_t s, uint32_t n, const uint8_t* a1, const uint8_t* a2,
                              const uint8_t* b1, const uint8_t* b2, int32_t* status,
                              const uint32_t* list, const uint32_t* count) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pair_verify, dim3(blocks_for(n, 64)), dim3(64), 0, s, n, a1, a2, b1, b2,
                     status, list, count);
  return hipGetLastError();
}

#endif  // part 4

#if HBTC_IN_PART(1)
hipError_t launch_point_mul(hipStream_t s, int group, uint32_t n, const uint8_t* base,
                            uint32_t base_stride, const uint8_t* scalars, uint32_t scalar_stride,
                            uint8_t* out, int32_t* status) {
  if (n == 0) return hipSuccess;
  if (group == 1)
    hipLaunchKernelGGL((k_point_mul<Fq, 12>), dim3(blocks_for(n, 64)), dim3(64), 0, s, n, base,
                       base_stride, scalars, scalar_stride, out, status);
  else
    hipLaunchKernelGGL((k_point_mul<Fq2, 24>), dim3(blocks_for(n, 64)), dim3(64), 0, s, n, base,
                       base_stride, scalars, scalar_stride, out, status);
  return hipGetLastError();
}

#endif  // part 1


}  // namespace hbtc
