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
#include "pair.h"

// Kernel groups are selected by -DHBTC_PART (one group left since round 5: the per-item exact
// kernels k_dec_verify / k_sig_verify / k_pair_verify, a whole Fq12 tower per lane and ~6 KB of
// scratch per lane, are gone -- the per-share modes take the cooperative exact leaf checks).
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

#ifndef HBTC_G2STEPS_PAIR
#define HBTC_G2STEPS_PAIR 1  // k_g2_steps on lane pairs (pair.h): the 68 steps at half the latency
#endif
#if !HBTC_G2STEPS_PAIR  // the one-lane form (variant builds only)
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
#endif

#if HBTC_G2STEPS_PAIR
// k_g2_steps on lane pairs: argument g on lanes (2g, 2g + 1).  The decode (square roots) runs on
// both lanes in one-lane form, the 68 line steps and the psi test in pair form.
__global__ void __launch_bounds__(64) k_g2_steps_pair(const uint8_t* __restrict__ in0, uint32_t n0,
                                                      const uint8_t* __restrict__ in1, uint32_t n1,
                                                      G2A* __restrict__ aff, Fq2* __restrict__ ws,
                                                      int32_t* __restrict__ status) {
  HBTC_LATENCY_PRIO();
  const uint32_t g = (blockIdx.x * 64 + threadIdx.x) >> 1;
  const bool even = (threadIdx.x & 1u) == 0;
  if (g >= n0 + n1) return;  // pair-uniform
  uint32_t w[24];
  load_words(w, g < n0 ? in0 : in1, g < n0 ? g : g - n0, 24);
  G2A q;
  bool ok = g2_decompress(q, w, false);
  if (even) aff[g] = q;
  if (ok && !q.inf) {
    G2Ap Q;
    g2p_from_full(Q, q);
    G2Jp T;
    g2p_walk_lines(ws + (size_t)g * 3 * MILLER_STEPS, T, Q);
    ok = g2p_psi_test(T, Q);
  }
  if (even) status[g] = ok ? HBTC_ACCEPT : HBTC_DECODE_ERR;
}
#endif

// Prepared G2 tables (hbtc.h hbtc_prepare_g2): entry i copied from slot ss[i] to slot ds[i]
// (null: i) -- the decoded point, its status and its 68 affine lines, one lane per (entry, line).
__global__ void __launch_bounds__(64) k_g2_tab_copy(uint32_t n, const uint32_t* __restrict__ ss,
                                                    const uint32_t* __restrict__ ds,
                                                    const G2A* __restrict__ saff, const int32_t* __restrict__ sst,
                                                    const Line* __restrict__ sl, G2A* __restrict__ daff,
                                                    int32_t* __restrict__ dst, Line* __restrict__ dl) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (g >= n * MILLER_STEPS) return;
  const uint32_t i = g / MILLER_STEPS, j = g % MILLER_STEPS;
  const uint32_t s = ss ? ss[i] : i, d = ds ? ds[i] : i;
  dl[(size_t)d * MILLER_STEPS + j] = sl[(size_t)s * MILLER_STEPS + j];
  if (j == 0) {
    daff[d] = saff[s];
    dst[d] = sst[s];
  }
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

hipError_t launch_g2_tab_copy(hipStream_t s, uint32_t n, const uint32_t* ss, const uint32_t* ds, const G2A* saff,
                              const int32_t* sst, const Line* sl, G2A* daff, int32_t* dst, Line* dl) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_g2_tab_copy, dim3(blocks_for((uint64_t)n * MILLER_STEPS, 64)), dim3(64), 0, s, n, ss, ds,
                     saff, sst, sl, daff, dst, dl);
  return hipGetLastError();
}

hipError_t launch_g2_prepare(hipStream_t s, const uint8_t* in0, uint32_t n0, const uint8_t* in1,
                             uint32_t n1, G2A* aff, Line* lines, Fq2* ws, int32_t* status) {
  const uint32_t n = n0 + n1;
  if (n == 0) return hipSuccess;
#if HBTC_G2STEPS_PAIR
  hipLaunchKernelGGL(k_g2_steps_pair, dim3(blocks_for(2 * (uint64_t)n, 64)), dim3(64), 0, s, in0, n0, in1,
                     n1, aff, ws, status);
#else
  hipLaunchKernelGGL(k_g2_steps, dim3(blocks_for(n, 64)), dim3(64), 0, s, in0, n0, in1, n1, aff, ws,
                     status);
#endif
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_g2_norm, dim3(blocks_for((uint64_t)n * MILLER_STEPS, 64)), dim3(64), 0, s, n,
                     aff, status, ws, lines);
  return hipGetLastError();
}

#endif  // part 1


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
