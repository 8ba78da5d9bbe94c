// Batched Pippenger multi-scalar multiplication on gfx950, and the Lagrange combines built on it.
//
// Replaces threshold_crypto's `interpolate` as called by PublicKeySet::combine_signatures
// (src/coin.rs:190) and PublicKeySet::decrypt (src/threshold_decryption.rs:184): the reference
// computes sum_i lambda_i * P_i with t independent 255-bit double-and-add multiplications
// (≈ 383 group operations per term).  Here every combine is one MSM of t terms, and a batch of
// combines (one per coin instance / ciphertext) is one launch sequence:
//
//   k_select     first t items of each instance (optionally: the first t ACCEPTED items, i.e.
//                the shares hbbft would hold in its verified-share map)         1 wave / instance
//   k_lagrange   lambda_i at 0 over the selected abscissae x = idx + 1, duplicate detection
//   k_msm_decode decode the selected compressed points to affine (subgroup check skipped for
//                items the verifier already accepted: it decoded and checked them)
//   k_msm_recode signed c-bit digits of every scalar (digits in [-2^(c-1), 2^(c-1)])
//   k_msm_sort   per (msm, window): counting sort of the terms by |digit| (bucket), largest
//                bucket first; LDS histogram + scan, one workgroup per (msm, window)
//   k_msm_buckets per (msm, window, 8-bucket segment): running-sum bucket reduction over the
//                sorted list (mixed additions of affine points), = sum_b b * B_b restricted to
//                the segment
//   k_msm_wsum   per (msm, window): sum of its segments
//   k_msm_final  per msm: Horner over the windows (c doublings per window), normalise, encode,
//                instance status (+ Signature::parity for G2)
//
// Cost per MSM of n terms: ceil(256/c) * (n mixed adds + 2^(c-1) full adds) + 255 doublings;
// c is chosen on the host to minimise it (n = 334: c = 6, ≈ 17k adds instead of ≈ 128k).
// Work is spread over (msm, window, segment) threads, so a batch of 1000 combines of 334
// terms runs ≈ 172k independent lanes.
//
// Data layout in HBM (all per batch, dense):
//   pts    [m][i]         Aff<F> (canonical Montgomery x, y, infinity flag)
//   digits [m][w][i]      int16
//   list   [m][w][pos]    u32: term index | sign << 31, grouped by bucket, largest first
//   roff   [m][w][r]      u32 start of bucket rank r (rank 0 = bucket 2^(c-1)), r = 0..B
//   part   [m][w][s]      Jac<F> segment partial sums;  wsum [m][w] Jac<F>
#include "hbtc_kernels.h"
#include "pair.h"

#ifndef HBTC_PART
#define HBTC_PART 0
#endif
#define HBTC_IN_PART(n) (HBTC_PART == 0 || HBTC_PART == (n))

namespace hbtc {

namespace {
__device__ __forceinline__ void msm_load_words(uint32_t* w, const uint8_t* base, size_t item,
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
__device__ __forceinline__ void msm_store_words(uint8_t* base, size_t item, const uint32_t* w,
                                                int nwords) {
  uint4* q = reinterpret_cast<uint4*>(base + item * (size_t)(nwords * 4));
  for (int i = 0; i < nwords / 4; ++i)
    q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}
__device__ __forceinline__ bool msm_decompress(G1A& p, const uint32_t* w, bool chk) {
  return g1_decompress(p, w, chk);
}
__device__ __forceinline__ bool msm_decompress(G2A& p, const uint32_t* w, bool chk) {
  return g2_decompress(p, w, chk);
}
__device__ __forceinline__ void msm_compress(uint32_t* w, const G1A& p) { g1_compress(w, p); }
__device__ __forceinline__ void msm_compress(uint32_t* w, const G2A& p) { g2_compress(w, p); }
__device__ __forceinline__ uint32_t msm_parity(const G1A&) { return 0; }
__device__ __forceinline__ uint32_t msm_parity(const G2A& p) { return g2_parity(p); }

// [k] p for a small k (< 2^16), Jacobian base, MSB-first
template <class F>
__device__ __forceinline__ void jac_mul_small(Jac<F>& r, const Jac<F>& p, uint32_t k) {
  Jac<F> acc;
  jac_set_inf(acc);
  const int top = k ? 31 - __builtin_clz(k) : -1;
  for (int b = top; b >= 0; --b) {
    jac_dbl(acc, acc);
    if ((k >> b) & 1u) jac_add(acc, acc, p);
  }
  r = acc;
}
}  // namespace

#if HBTC_IN_PART(8)
// ------------------------------------------------------------------ selection + Lagrange
// The first t items of instance k in item order (the caller orders items by node index, as
// hbbft's BTreeMap iteration does); with `status`, only items whose status is ACCEPT count.
__global__ void __launch_bounds__(64) k_select(const uint32_t* __restrict__ offsets,
                                               uint32_t t, const int32_t* __restrict__ status,
                                               const uint32_t* __restrict__ idx,
                                               uint32_t* __restrict__ sel_pos,
                                               uint32_t* __restrict__ sel_idx,
                                               uint32_t* __restrict__ sel_cnt) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  const uint32_t k = blockIdx.x, lane = threadIdx.x;
  const uint32_t a = offsets[k], b = offsets[k + 1];
  const size_t o = (size_t)k * t;
  uint32_t found = 0;
  for (uint32_t base = a; base < b && found < t; base += 64) {
    const uint32_t i = base + lane;
    const bool ok = i < b && (!status || status[i] == HBTC_ACCEPT);
    const uint64_t mask = __ballot(ok);
    const uint32_t slot = found + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
    if (ok && slot < t) {
      sel_pos[o + slot] = i;
      sel_idx[o + slot] = idx[i];
    }
    found += (uint32_t)__popcll(mask);
  }
  const uint32_t cnt = found < t ? found : t;
  for (uint32_t s = cnt + lane; s < t; s += 64) {
    sel_pos[o + s] = 0xffffffffu;
    sel_idx[o + s] = 0xffffffffu - s;  // distinct fillers: no spurious duplicate flag
  }
  if (lane == 0) sel_cnt[k] = cnt;
}

// Lagrange coefficients at 0 of the selected x_i = idx_i + 1 (Montgomery Fr), three passes:
//   k_lagrange_x    x_i in Montgomery form (one lane per term)
//   k_lagrange_den  q_i = x_i * prod_{j != i} (x_j - x_i): O(t) per term, one lane per term;
//                   x_j == x_i for j != i is a DuplicateEntry (threshold_crypto interpolate)
//   k_lagrange_inv  one workgroup per instance: P = prod_j x_j and a batched inversion of the
//                   q_i (chunk products, one inversion, backward walk), lambda_i = P / q_i
// (round 1 spent ~1,500 Fr products per coefficient: a conversion inside the O(t) loop and a
// Fermat inversion per coefficient).
__global__ void __launch_bounds__(256) k_lagrange_x(uint64_t n, const uint32_t* __restrict__ sel_idx,
                                                    Fr* __restrict__ x) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= n) return;
  Fr v;
  fr_from_u64(v, (uint64_t)sel_idx[g] + 1);
  x[g] = v;
}

__global__ void __launch_bounds__(256) k_lagrange_den(uint32_t n_inst, uint32_t t,
                                                      const Fr* __restrict__ x,
                                                      Fr* __restrict__ q,
                                                      uint32_t* __restrict__ dup,
                                                      const uint32_t* __restrict__ done) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= (uint64_t)n_inst * t) return;
  const uint32_t k = (uint32_t)(g / t), i = (uint32_t)(g % t);
  if (done && done[k]) return;  // k_lagrange_fact has the coefficients
  const Fr* xk = x + (size_t)k * t;
  const Fr xi = xk[i];
  Fr den;
  limbs_set_const<8>(den, FR_ONE);
  bool is_dup = false;
  for (uint32_t j = 0; j < t; ++j) {
    if (j == i) continue;
    const Fr xj = xk[j];
    is_dup |= limbs_eq<8>(xj, xi);
    Fr d;
    fr_sub(d, xj, xi);
    fr_mul(den, den, d);
  }
  if (is_dup) atomicOr(&dup[k], 1u);
  Fr qi;
  fr_mul(qi, xi, den);
  q[g] = qi;
}

constexpr uint32_t LG_BS = 256;
__global__ void __launch_bounds__(LG_BS) k_lagrange_inv(uint32_t t, Fr* __restrict__ x,
                                                        Fr* __restrict__ q_lambda,
                                                        const uint32_t* __restrict__ done) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  if (done && done[blockIdx.x]) return;  // block-uniform: k_lagrange_fact has the coefficients
  __shared__ Fr C[LG_BS];   // product of q over chunk u
  __shared__ Fr E[LG_BS];   // product of q over the chunks before u
  __shared__ Fr IE[LG_BS];  // (E[u] * C[u])^-1
  __shared__ Fr X[LG_BS];   // product of x over chunk u; X[0] then holds P = prod x
  const uint32_t tid = threadIdx.x;
  Fr* q = q_lambda + (size_t)blockIdx.x * t;
  Fr* xw = x + (size_t)blockIdx.x * t;
  const uint32_t chunk = (t + LG_BS - 1) / LG_BS;
  const uint32_t lo = min(t, tid * chunk), hi = min(t, lo + chunk);
  Fr pq, px;
  limbs_set_const<8>(pq, FR_ONE);
  limbs_set_const<8>(px, FR_ONE);
  for (uint32_t i = lo; i < hi; ++i) {
    fr_mul(px, px, xw[i]);
    xw[i] = pq;  // x_i is no longer needed: keep q's in-chunk exclusive prefix instead
    fr_mul(pq, pq, q[i]);
  }
  // prefix products of the chunk products (q in C, x in X) and the suffix products of q (in
  // IE) by log-step scans: 8 products deep instead of the 3 * 256 of one thread's walk
  C[tid] = pq;
  X[tid] = px;
  IE[tid] = pq;
  __syncthreads();
  Fr cp = pq, xp = px, sp = pq;
  for (uint32_t off = 1; off < LG_BS; off <<= 1) {
    Fr a, b, d;
    const bool lo_ok = tid >= off, hi_ok = tid + off < LG_BS;
    if (lo_ok) {
      a = C[tid - off];
      b = X[tid - off];
    }
    if (hi_ok) d = IE[tid + off];
    __syncthreads();
    if (lo_ok) {
      fr_mul(cp, cp, a);
      fr_mul(xp, xp, b);
      C[tid] = cp;
      X[tid] = xp;
    }
    if (hi_ok) {
      fr_mul(sp, sp, d);
      IE[tid] = sp;
    }
    __syncthreads();
  }
  // C[u]: q over chunks 0..u;  X[LG_BS - 1]: P;  IE[u]: q over chunks u..LG_BS-1
  Fr e_excl, s_excl;
  limbs_set_const<8>(e_excl, FR_ONE);
  limbs_set_const<8>(s_excl, FR_ONE);
  if (tid > 0) e_excl = C[tid - 1];
  if (tid + 1 < LG_BS) s_excl = IE[tid + 1];
  __shared__ Fr INV_TOTAL;
  if (tid == 0) fr_inv(INV_TOTAL, C[LG_BS - 1]);  // the one inversion
  __syncthreads();
  E[tid] = e_excl;
  fr_mul(IE[tid], INV_TOTAL, s_excl);  // (q over chunks 0..tid)^-1
  if (tid == 0) X[0] = X[LG_BS - 1];
  __syncthreads();
  const Fr P = X[0], e = E[tid];
  Fr inv_incl = IE[tid];  // inverse of the prefix of q through item i (starting at the chunk end)
  for (uint32_t i = hi; i-- > lo;) {
    Fr excl, qi_inv, l, lc;
    fr_mul(excl, e, xw[i]);          // prefix of q before item i
    fr_mul(qi_inv, inv_incl, excl);  // 1 / q_i
    fr_mul(inv_incl, inv_incl, q[i]);
    fr_mul(l, P, qi_inv);            // prod_{j != i} x_j / prod_{j != i} (x_j - x_i)
    fr_from_mont(lc, l);
    q[i] = lc;
  }
}

// ---------------------------------------------------- Lagrange through factorials (round 5)
// The selected abscissae of a combine are the first t ACCEPTed shares in node order, so they are
// strictly increasing and fill [1, M] but for the few rejected / missing nodes R = [1, M] \ S
// (|R| = M - t).  Then
//   prod_{j in S, j != i} x_j          = M! / (prod_R r * x_i)
//   prod_{j in S, j != i} (x_j - x_i)  = (-1)^(x_i - 1) (x_i - 1)! (M - x_i)! / prod_R (r - x_i)
// so lambda_i = (-1)^(x_i - 1) M! Q_i / (prod_R r) / x_i! / (M - x_i)!,  Q_i = prod_R (r - x_i):
// |R| + 5 products per term and no inversion (1/r = (r - 1)! / r! from the tables), against
// O(t) products per term and a batched inversion (k_lagrange_den / k_lagrange_inv).  Instances
// whose x are not strictly increasing (a duplicate: DUPLICATE_ENTRY), with M past the tables or
// with |R| > LG_FACT_RMAX are left to those kernels (done[k] = 0).
__global__ void __launch_bounds__(256) k_fact_chunks(uint32_t n, Fr* __restrict__ part) {
  // part[c] = prod_{i in chunk c} i, chunks of 256 of [1, n]
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c * 256u >= n + 1) return;
  Fr acc, v;
  limbs_set_const<8>(acc, FR_ONE);
  for (uint32_t i = c * 256u; i < min(n + 1, c * 256u + 256u); ++i) {
    if (i == 0) continue;
    fr_from_u64(v, i);
    fr_mul(acc, acc, v);
  }
  part[c] = acc;
}
__global__ void __launch_bounds__(256) k_fact_fill(uint32_t n, const Fr* __restrict__ part,
                                                   Fr* __restrict__ fact, Fr* __restrict__ inv_fact) {
  // fact[i] = i! (Montgomery), inv_fact[i] = 1 / i!
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i > n) return;
  Fr acc, v;
  limbs_set_const<8>(acc, FR_ONE);
  for (uint32_t c = 0; c < i / 256u; ++c) fr_mul(acc, acc, part[c]);
  for (uint32_t j = (i / 256u) * 256u; j <= i; ++j) {
    if (j == 0) continue;
    fr_from_u64(v, j);
    fr_mul(acc, acc, v);
  }
  fact[i] = acc;
  Fr inv;
  fr_inv(inv, acc);
  inv_fact[i] = inv;
}

constexpr uint32_t LG_FACT_RMAX = 256;
constexpr uint32_t LG_FACT_TMAX = 4096;
__global__ void __launch_bounds__(256) k_lagrange_fact(uint32_t t, const uint32_t* __restrict__ sel_idx,
                                                       const uint32_t* __restrict__ sel_cnt,
                                                       uint32_t n_fact, const Fr* __restrict__ fact,
                                                       const Fr* __restrict__ inv_fact,
                                                       Fr* __restrict__ lambda, uint32_t* __restrict__ done) {
  HBTC_LATENCY_PRIO();
  __shared__ uint32_t xs[LG_FACT_TMAX];
  __shared__ uint32_t rs[LG_FACT_RMAX];
  __shared__ uint32_t s_ok, s_nr;
  __shared__ Fr s_c;  // M! / prod_R r
  const uint32_t k = blockIdx.x, tid = threadIdx.x;
  const uint32_t* sx = sel_idx + (size_t)k * t;
  if (tid == 0) s_ok = sel_cnt[k] == t ? 1u : 0u;
  __syncthreads();
  if (!s_ok) {  // NOT_ENOUGH_SHARES: the coefficients are never used
    if (tid == 0) done[k] = 1;
    return;
  }
  for (uint32_t j = tid; j < t; j += 256) xs[j] = sx[j] + 1u;
  __syncthreads();
  for (uint32_t j = tid; j + 1 < t; j += 256)
    if (xs[j + 1] <= xs[j] || xs[j] == 0) s_ok = 0;  // not strictly increasing (x = 0: idx wrap)
  __syncthreads();
  const uint32_t M = xs[t - 1];
  if (tid == 0 && (xs[0] == 0 || M > n_fact || M - t > LG_FACT_RMAX)) s_ok = 0;
  __syncthreads();
  if (!s_ok) {
    if (tid == 0) done[k] = 0;
    return;
  }
  if (tid == 0) {  // R: the gaps of S in [1, M]
    uint32_t nr = 0, prev = 0;
    for (uint32_t j = 0; j < t; ++j) {
      for (uint32_t r = prev + 1; r < xs[j]; ++r) rs[nr++] = r;
      prev = xs[j];
    }
    s_nr = nr;
    Fr c = fact[M], q;
    for (uint32_t j = 0; j < nr; ++j) {  // 1 / r = (r - 1)! / r!
      fr_mul(q, fact[rs[j] - 1], inv_fact[rs[j]]);
      fr_mul(c, c, q);
    }
    s_c = c;
  }
  __syncthreads();
  const uint32_t nr = s_nr;
  const Fr c = s_c;
  for (uint32_t i = tid; i < t; i += 256) {
    const uint32_t x = xs[i];
    Fr q, d, l, lc;
    fr_mul(q, inv_fact[x], inv_fact[M - x]);
    fr_mul(q, q, c);
    for (uint32_t j = 0; j < nr; ++j) {
      const uint32_t r = rs[j];
      fr_from_u64(d, r > x ? r - x : x - r);
      if (r < x) {
        Fr z;
        limbs_zero<8>(z);
        fr_sub(d, z, d);
      }
      fr_mul(q, q, d);
    }
    if (!(x & 1u)) {  // (-1)^(x - 1)
      Fr z;
      limbs_zero<8>(z);
      fr_sub(q, z, q);
    }
    l = q;
    fr_from_mont(lc, l);
    lambda[(size_t)k * t + i] = lc;
  }
  if (tid == 0) done[k] = 1;
}

// ------------------------------------------------------------------ digits and buckets
// Signed c-bit digits of every (canonical, < 2^255) scalar: W = ceil(256 / c) windows,
// digit_w in [-2^(c-1), 2^(c-1)], sum_w digit_w 2^(cw) = k.
__global__ void __launch_bounds__(256) k_msm_recode(uint64_t n_terms, uint32_t n, uint32_t c,
                                                    uint32_t W, const uint32_t* __restrict__ sc,
                                                    int16_t* __restrict__ digits) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= n_terms) return;
  const uint64_t m = g / n, i = g % n;
  const uint32_t* k = sc + g * 8;
  uint32_t kw[9];
#pragma unroll
  for (int j = 0; j < 8; ++j) kw[j] = k[j];
  kw[8] = 0;
  const uint32_t mask = (1u << c) - 1u, half = 1u << (c - 1);
  uint32_t carry = 0;
  int16_t* out = digits + (m * W) * n + i;
  for (uint32_t w = 0; w < W; ++w) {
    const uint32_t bit = w * c, wi = bit >> 5, sh = bit & 31;
    uint64_t two = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j)  // static indexing: kw stays in registers
      if ((uint32_t)j == wi) two = ((uint64_t)kw[j + 1] << 32) | kw[j];
    uint32_t v = (uint32_t)(two >> sh) & mask;
    v += carry;
    int32_t d;
    if (v > half) {
      d = (int32_t)v - (int32_t)(1u << c);
      carry = 1;
    } else {
      d = (int32_t)v;
      carry = 0;
    }
    out[(size_t)w * n] = (int16_t)d;
  }
}

// Counting sort of one (msm, window)'s n digits by bucket |d| (rank r = B - |d|), 256 threads.
constexpr uint32_t MSM_SORT_BS = 256;
__global__ void __launch_bounds__(MSM_SORT_BS) k_msm_sort(uint32_t n, uint32_t c,
                                                          const int16_t* __restrict__ digits,
                                                          uint32_t* __restrict__ list,
                                                          uint32_t* __restrict__ roff) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  extern __shared__ uint32_t cnt[];  // B counters, then MSM_SORT_BS chunk sums
  uint32_t* part = cnt + (1u << (c - 1));
  const uint32_t B = 1u << (c - 1), tid = threadIdx.x;
  const size_t mw = blockIdx.x;
  const int16_t* d = digits + mw * n;
  for (uint32_t r = tid; r < B; r += MSM_SORT_BS) cnt[r] = 0;
  __syncthreads();
  for (uint32_t i = tid; i < n; i += MSM_SORT_BS) {
    const int32_t v = d[i];
    if (v) atomicAdd(&cnt[B - (uint32_t)(v < 0 ? -v : v)], 1u);
  }
  __syncthreads();
  // exclusive scan: thread tid owns ranks [tid*ch, (tid+1)*ch)
  const uint32_t ch = (B + MSM_SORT_BS - 1) / MSM_SORT_BS;
  const uint32_t r0 = tid * ch, r1 = min(B, r0 + ch);
  uint32_t s = 0;
  for (uint32_t r = r0; r < r1; ++r) s += cnt[r];
  part[tid] = s;
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (uint32_t j = 0; j < MSM_SORT_BS; ++j) {
      const uint32_t v = part[j];
      part[j] = acc;
      acc += v;
    }
  }
  __syncthreads();
  uint32_t* ro = roff + mw * (B + 1);
  uint32_t acc = part[tid];
  for (uint32_t r = r0; r < r1; ++r) {
    const uint32_t v = cnt[r];
    cnt[r] = acc;  // becomes the scatter cursor
    ro[r] = acc;
    acc += v;
  }
  if (tid == MSM_SORT_BS - 1) ro[B] = acc;  // last chunk ends at the total (empty chunks: part)
  __syncthreads();
  uint32_t* L = list + mw * n;
  for (uint32_t i = tid; i < n; i += MSM_SORT_BS) {
    const int32_t v = d[i];
    if (v) {
      const uint32_t pos = atomicAdd(&cnt[B - (uint32_t)(v < 0 ? -v : v)], 1u);
      L[pos] = i | (v < 0 ? 0x80000000u : 0u);
    }
  }
}
#endif  // part 8

// ------------------------------------------------------------------ group kernels
#if HBTC_IN_PART(8) || HBTC_IN_PART(9)
__device__ __forceinline__ void msm_generator(G1A& p) {
  fq_set(p.x, G1_GEN_X);
  fq_set(p.y, G1_GEN_Y);
  p.inf = 0;
}
__device__ __forceinline__ void msm_generator(G2A& p) {
  fq2_set(p.x, G2_GEN_X);
  fq2_set(p.y, G2_GEN_Y);
  p.inf = 0;
}

// Term i of MSM k: the selected item sel_pos[k*t+i] (combines), else item k*stride+i of the
// compressed array; terms i >= stride are the group generator (SyncKeyGen checks fold the
// right-hand side [v]G into the MSM as one extra term).
// G1: at most 256 VGPRs so two waves share a SIMD (uncapped, the fully inlined Fq product took
// 256 + 2 AGPRs: one wave per SIMD for the 56 M commitment points of a SyncKeyGen era)
#ifndef HBTC_MSM_DECODE_WAVES
#define HBTC_MSM_DECODE_WAVES 2
#endif
// the G1 bucket walk likewise (256 + 15 AGPRs uncapped)
#ifndef HBTC_MSM_BUCKET_WAVES
#define HBTC_MSM_BUCKET_WAVES 2
#endif
template <class F, int NW>
__global__ void __launch_bounds__(64, (sizeof(F) == sizeof(Fq) ? HBTC_MSM_DECODE_WAVES : 1))
    k_msm_decode(uint32_t n_inst, uint32_t t, uint32_t stride,
                                                   const uint8_t* __restrict__ pts,
                                                   const uint32_t* __restrict__ sel_pos,
                                                   const uint32_t* __restrict__ sel_cnt,
                                                   const int32_t* __restrict__ status,
                                                   const Aff<F>* __restrict__ dec,
                                                   Aff<F>* __restrict__ out,
                                                   uint32_t* __restrict__ bad) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  const uint64_t g = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (g >= (uint64_t)n_inst * t) return;
  const uint32_t k = (uint32_t)(g / t), i = (uint32_t)(g % t);
  Aff<F> p;
  fzero(p.x);
  fzero(p.y);
  p.inf = 1;
  if (!sel_pos && i >= stride) {
    msm_generator(p);
  } else if (i < sel_cnt[k]) {
    const uint64_t pos = sel_pos ? (uint64_t)sel_pos[g] : (uint64_t)k * stride + i;
    // an item the verifier accepted was decoded and subgroup-checked by it; with its decoded
    // form at hand (the RLC item pass keeps it) nothing is decoded again
    const bool accepted = status && status[pos] == HBTC_ACCEPT;
    if (accepted && dec) {
      p = dec[pos];
    } else {
      uint32_t w[NW];
      msm_load_words(w, pts, pos, NW);
      if (!msm_decompress(p, w, !accepted)) {
        atomicOr(&bad[k], 1u);
        p.inf = 1;
      }
    }
  }
  out[g] = p;
}

#if HBTC_IN_PART(8)
// The selected terms of a combine over VERIFIED items whose decoded form the verification kept
// (k_rlc_items / k_sig_items): a plain gather, no decode and no subgroup check.
template <class A>
__global__ void __launch_bounds__(256) k_msm_gather(uint32_t n_inst, uint32_t t,
                                                    const uint32_t* __restrict__ sel_pos,
                                                    const uint32_t* __restrict__ sel_cnt,
                                                    const A* __restrict__ dec,
                                                    A* __restrict__ out) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= (uint64_t)n_inst * t) return;
  const uint32_t k = (uint32_t)(g / t), i = (uint32_t)(g % t);
  A p;
  if (i < sel_cnt[k]) {
    p = dec[sel_pos[g]];
  } else {
    fzero(p.x);
    fzero(p.y);
    p.inf = 1;
  }
  out[g] = p;
}
template __global__ void k_msm_gather<G1A>(uint32_t, uint32_t, const uint32_t*, const uint32_t*,
                                           const G1A*, G1A*);
template __global__ void k_msm_gather<G2A>(uint32_t, uint32_t, const uint32_t*, const uint32_t*,
                                           const G2A*, G2A*);
#endif  // part 8

// Rank whose bucket holds sorted position p: the largest r < B with ro[r] <= p (ro[0] = 0 and
// p < ro[B]).
__device__ __forceinline__ uint32_t msm_rank(const uint32_t* ro, uint32_t B, uint32_t p) {
  uint32_t lo = 0, hi = B;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ro[mid] <= p) lo = mid;
    else hi = mid;
  }
  return lo;
}

// One lane per (msm, window, segment): S = B/8 segments split the window's sorted nonzero terms
// into equal slices of the LIST (not of the buckets), so a window whose digits crowd into a few
// buckets (the top window: k < 2^255 leaves it only a few bits) is shared by all S lanes instead
// of serialising n additions on one.  Running-sum reduction over the slice's ranks
// [r_lo, r_hi): tot = sum_r (r_hi - r) B'_r, run = sum_r B'_r (B'_r = the slice's part of
// bucket rank r, bucket b = B - r), so the slice's share of sum_b b B_b is tot + [B - r_hi] run.
template <class F>
__global__ void __launch_bounds__(64, (sizeof(F) == sizeof(Fq) ? HBTC_MSM_BUCKET_WAVES : 1))
    k_msm_buckets(uint64_t n_lanes, uint32_t n, uint32_t c,
                                                    uint32_t W, const Aff<F>* __restrict__ pts,
                                                    const uint32_t* __restrict__ list,
                                                    const uint32_t* __restrict__ roff,
                                                    const uint32_t* __restrict__ pts_map,
                                                    Jac<F>* __restrict__ part) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  const uint64_t g = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (g >= n_lanes) return;
  const uint32_t B = 1u << (c - 1), S = B / 8;
  const uint32_t s = (uint32_t)(g % S);
  const uint64_t mw = g / S;
  const uint32_t* ro = roff + mw * (B + 1);
  const uint32_t* L = list + mw * n;
  // pts_map: MSMs sharing one decoded point set (several Ack equations over one commitment)
  const uint64_t blk = pts_map ? (uint64_t)pts_map[mw / W] : mw / W;
  const Aff<F>* P = pts + blk * n;
  Jac<F> run, tot;
  jac_set_inf(run);
  jac_set_inf(tot);
  const uint32_t total = ro[B];
  const uint32_t p0 = (uint32_t)((uint64_t)total * s / S);
  const uint32_t p1 = (uint32_t)((uint64_t)total * (s + 1) / S);
  if (p0 < p1) {
    const uint32_t r_last = msm_rank(ro, B, p1 - 1);
    uint32_t e = p0;
    for (uint32_t r = msm_rank(ro, B, p0); r <= r_last; ++r) {
      const uint32_t end = min(ro[r + 1], p1);
      for (; e < end; ++e) {
        const uint32_t v = L[e];
        Aff<F> q = P[v & 0x7fffffffu];
        if (v >> 31) fneg(q.y, q.y);
        jac_add_aff(run, run, q);
      }
      jac_add(tot, tot, run);
    }
    const uint32_t base = B - r_last - 1;
    if (base) {
      Jac<F> m;
      jac_mul_small(m, run, base);
      jac_add(tot, tot, m);
    }
  }
  part[g] = tot;
}

template <class F>
__global__ void __launch_bounds__(64) k_msm_wsum(uint64_t n_mw, uint32_t S,
                                                 const Jac<F>* __restrict__ part,
                                                 Jac<F>* __restrict__ wsum) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  const uint64_t g = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (g >= n_mw) return;
  const Jac<F>* p = part + g * S;
  Jac<F> acc = p[0];
  for (uint32_t s = 1; s < S; ++s) jac_add(acc, acc, p[s]);
  wsum[g] = acc;
}

// Horner over the windows, normalise and encode.  Combine mode (sel_cnt != nullptr): the
// instance status (NOT_ENOUGH_SHARES > DECODE_ERR > DUPLICATE_ENTRY > ACCEPT), zero bytes for a
// failed instance and the parity bit.  MSM mode: status DECODE_ERR if any term failed to decode.
template <class F, int NW>
__global__ void __launch_bounds__(64) k_msm_final(uint32_t n_msm, uint32_t c, uint32_t W,
                                                  const Jac<F>* __restrict__ wsum,
                                                  const uint32_t* __restrict__ sel_cnt,
                                                  uint32_t t, const uint32_t* __restrict__ bad,
                                                  const uint32_t* __restrict__ dup,
                                                  int32_t* __restrict__ status,
                                                  uint8_t* __restrict__ out,
                                                  uint8_t* __restrict__ parity) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  const uint32_t m = blockIdx.x * 64 + threadIdx.x;
  if (m >= n_msm) return;
  const Jac<F>* ws = wsum + (size_t)m * W;
  Jac<F> acc = ws[W - 1];
  for (int w = (int)W - 2; w >= 0; --w) {
    for (uint32_t j = 0; j < c; ++j) jac_dbl(acc, acc);
    jac_add(acc, acc, ws[w]);
  }
  int32_t st = HBTC_ACCEPT;
  if (sel_cnt && sel_cnt[m] < t)
    st = HBTC_NOT_ENOUGH_SHARES;
  else if (bad[m])
    st = HBTC_DECODE_ERR;
  else if (dup && dup[m])
    st = HBTC_DUPLICATE_ENTRY;
  status[m] = st;
  Aff<F> a;
  jac_to_aff(a, acc);
  uint32_t w[NW];
  msm_compress(w, a);
  if (st != HBTC_ACCEPT)
    for (int j = 0; j < NW; ++j) w[j] = 0;
  msm_store_words(out, m, w, NW);
  if (parity) parity[m] = (st == HBTC_ACCEPT) ? (uint8_t)msm_parity(a) : 0;
}
#endif

#if HBTC_IN_PART(8)
template __global__ void k_msm_decode<Fq, 12>(uint32_t, uint32_t, uint32_t, const uint8_t*,
                                              const uint32_t*, const uint32_t*, const int32_t*,
                                              const G1A*, G1A*, uint32_t*);
template __global__ void k_msm_buckets<Fq>(uint64_t, uint32_t, uint32_t, uint32_t, const G1A*,
                                           const uint32_t*, const uint32_t*, const uint32_t*,
                                           G1J*);
template __global__ void k_msm_wsum<Fq>(uint64_t, uint32_t, const G1J*, G1J*);
template __global__ void k_msm_final<Fq, 12>(uint32_t, uint32_t, uint32_t, const G1J*,
                                             const uint32_t*, uint32_t, const uint32_t*,
                                             const uint32_t*, int32_t*, uint8_t*, uint8_t*);
#endif
#ifndef HBTC_MSM_G2_PAIR
#define HBTC_MSM_G2_PAIR 1  // the G2 bucket / window / final passes on lane pairs (pair.h)
#endif
#if HBTC_IN_PART(9)
template __global__ void k_msm_decode<Fq2, 24>(uint32_t, uint32_t, uint32_t, const uint8_t*,
                                               const uint32_t*, const uint32_t*, const int32_t*,
                                               const G2A*, G2A*, uint32_t*);
#if !HBTC_MSM_G2_PAIR  // the one-lane G2 passes (variant builds only)
template __global__ void k_msm_buckets<Fq2>(uint64_t, uint32_t, uint32_t, uint32_t, const G2A*,
                                            const uint32_t*, const uint32_t*, const uint32_t*,
                                            G2J*);
template __global__ void k_msm_wsum<Fq2>(uint64_t, uint32_t, const G2J*, G2J*);
template __global__ void k_msm_final<Fq2, 24>(uint32_t, uint32_t, uint32_t, const G2J*,
                                              const uint32_t*, uint32_t, const uint32_t*,
                                              const uint32_t*, int32_t*, uint8_t*, uint8_t*);
#endif
#endif

#ifndef HBTC_MSM_G2P_WAVES
#define HBTC_MSM_G2P_WAVES 2
#endif
#ifndef HBTC_MSM_G2P_BUCKET_WAVES
// one wave: no scratch (two: 324 B/lane); C4 6.069 / 6.062 M shares/s and C2 1.111 / 1.091 M at
// one / two waves (profiles/r06/run12/)
#define HBTC_MSM_G2P_BUCKET_WAVES 1
#endif
#if HBTC_IN_PART(9) && HBTC_MSM_G2_PAIR
// The three G2 reduction passes above on lane pairs (round 6): unit g (one (msm, window,
// segment) slice, one window sum, one MSM) on lanes 2g, 2g + 1, lane 2g + e holding component e
// of every Fq2 (pair.h): each Fq2 product is one fused two-product per lane, half the one-lane
// chain's latency, and the state fits two waves per SIMD where the one-lane form runs one.  All
// control flow depends on g only (pair-uniform).  Same outputs as k_msm_buckets / k_msm_wsum /
// k_msm_final<Fq2, 24>.
__global__ void __launch_bounds__(64, HBTC_MSM_G2P_BUCKET_WAVES)
    k_msm_buckets_g2p(uint64_t n_lanes, uint32_t n, uint32_t c, uint32_t W,
                      const G2A* __restrict__ pts, const uint32_t* __restrict__ list,
                      const uint32_t* __restrict__ roff, const uint32_t* __restrict__ pts_map,
                      G2J* __restrict__ part) {
  HBTC_LATENCY_PRIO();
  const uint64_t g = ((uint64_t)blockIdx.x * 64 + threadIdx.x) >> 1;
  if (g >= n_lanes) return;  // pair-uniform
  const uint32_t B = 1u << (c - 1), S = B / 8;
  const uint32_t s = (uint32_t)(g % S);
  const uint64_t mw = g / S;
  const uint32_t* ro = roff + mw * (B + 1);
  const uint32_t* L = list + mw * n;
  const uint64_t blk = pts_map ? (uint64_t)pts_map[mw / W] : mw / W;
  const G2A* P = pts + blk * n;
  G2Jp run, tot;
  jac_set_inf(run);
  jac_set_inf(tot);
  const uint32_t total = ro[B];
  const uint32_t p0 = (uint32_t)((uint64_t)total * s / S);
  const uint32_t p1 = (uint32_t)((uint64_t)total * (s + 1) / S);
  if (p0 < p1) {
    const uint32_t r_last = msm_rank(ro, B, p1 - 1);
    uint32_t e = p0;
    for (uint32_t r = msm_rank(ro, B, p0); r <= r_last; ++r) {
      const uint32_t end = min(ro[r + 1], p1);
      for (; e < end; ++e) {
        const uint32_t v = L[e];
        G2Ap q;
        g2p_load_aff(q, P + (v & 0x7fffffffu));
        if (v >> 31) fneg(q.y, q.y);
        jac_add_aff(run, run, q);
      }
      jac_add(tot, tot, run);
    }
    const uint32_t base = B - r_last - 1;
    if (base) {
      G2Jp m;
      jac_mul_small(m, run, base);
      jac_add(tot, tot, m);
    }
  }
  g2p_store_jac(part + g, tot);
}

__global__ void __launch_bounds__(64, HBTC_MSM_G2P_WAVES)
    k_msm_wsum_g2p(uint64_t n_mw, uint32_t S, const G2J* __restrict__ part,
                   G2J* __restrict__ wsum) {
  HBTC_LATENCY_PRIO();
  const uint64_t g = ((uint64_t)blockIdx.x * 64 + threadIdx.x) >> 1;
  if (g >= n_mw) return;
  const G2J* p = part + g * S;
  G2Jp acc, x;
  g2p_load_jac(acc, p);
  for (uint32_t s = 1; s < S; ++s) {
    g2p_load_jac(x, p + s);
    jac_add(acc, acc, x);
  }
  g2p_store_jac(wsum + g, acc);
}

__global__ void __launch_bounds__(64, HBTC_MSM_G2P_WAVES)
    k_msm_final_g2p(uint32_t n_msm, uint32_t c, uint32_t W, const G2J* __restrict__ wsum,
                    const uint32_t* __restrict__ sel_cnt, uint32_t t,
                    const uint32_t* __restrict__ bad, const uint32_t* __restrict__ dup,
                    int32_t* __restrict__ status, uint8_t* __restrict__ out,
                    uint8_t* __restrict__ parity) {
  HBTC_LATENCY_PRIO();
  const uint32_t m = (blockIdx.x * 64 + threadIdx.x) >> 1;
  if (m >= n_msm) return;
  const G2J* ws = wsum + (size_t)m * W;
  G2Jp acc, x;
  g2p_load_jac(acc, ws + (W - 1));
  for (int w = (int)W - 2; w >= 0; --w) {
    for (uint32_t j = 0; j < c; ++j) jac_dbl(acc, acc);
    g2p_load_jac(x, ws + w);
    jac_add(acc, acc, x);
  }
  int32_t st = HBTC_ACCEPT;
  if (sel_cnt && sel_cnt[m] < t)
    st = HBTC_NOT_ENOUGH_SHARES;
  else if (bad[m])
    st = HBTC_DECODE_ERR;
  else if (dup && dup[m])
    st = HBTC_DUPLICATE_ENTRY;
  const bool si = jac_is_inf(acc);
  G2Ap ap;
  jac_to_aff(ap, acc);
  Fq px, py;  // the partner's components: the even lane assembles the Fq2 point
  fq_xchg(px, ap.x.v);
  fq_xchg(py, ap.y.v);
  if (pair_odd()) return;
  status[m] = st;
  G2A a;
  a.x.c0 = ap.x.v;
  a.x.c1 = px;
  a.y.c0 = ap.y.v;
  a.y.c1 = py;
  a.inf = si ? 1u : 0u;
  uint32_t w[24];
  msm_compress(w, a);
  if (st != HBTC_ACCEPT)
    for (int j = 0; j < 24; ++j) w[j] = 0;
  msm_store_words(out, m, w, 24);
  if (parity) parity[m] = (st == HBTC_ACCEPT) ? (uint8_t)msm_parity(a) : 0;
}
#endif

// ------------------------------------------------------------------ launchers
static inline uint32_t msm_blocks(uint64_t n, uint32_t bs) { return (uint32_t)((n + bs - 1) / bs); }

#if HBTC_IN_PART(8)
hipError_t launch_select(hipStream_t s, uint32_t n_inst, const uint32_t* offsets, uint32_t t,
                         const int32_t* status, const uint32_t* idx, uint32_t* sel_pos,
                         uint32_t* sel_idx, uint32_t* sel_cnt) {
  if (n_inst == 0) return hipSuccess;
  hipLaunchKernelGGL(k_select, dim3(n_inst), dim3(64), 0, s, offsets, t, status, idx, sel_pos,
                     sel_idx, sel_cnt);
  return hipGetLastError();
}

hipError_t launch_fact_tables(hipStream_t s, uint32_t n, Fr* part, Fr* fact, Fr* inv_fact) {
  hipLaunchKernelGGL(k_fact_chunks, dim3(msm_blocks(n / 256 + 1, 256)), dim3(256), 0, s, n, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_fact_fill, dim3(msm_blocks((uint64_t)n + 1, 256)), dim3(256), 0, s, n, part, fact,
                     inv_fact);
  return hipGetLastError();
}

hipError_t launch_lagrange_sel(hipStream_t s, uint32_t n_inst, uint32_t t, const uint32_t* sel_idx,
                               Fr* lambda, Fr* ws, uint32_t* dup, const LagrangeFact* lf) {
  const uint64_t n = (uint64_t)n_inst * t;
  if (n == 0) return hipSuccess;
  hipError_t e;
  const uint32_t* done = nullptr;
  if (lf && lf->fact && t <= LG_FACT_TMAX) {
    hipLaunchKernelGGL(k_lagrange_fact, dim3(n_inst), dim3(256), 0, s, t, sel_idx, lf->sel_cnt, lf->n,
                       lf->fact, lf->inv_fact, lambda, lf->done);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    done = lf->done;
  }
  hipLaunchKernelGGL(k_lagrange_x, dim3(msm_blocks(n, 256)), dim3(256), 0, s, n, sel_idx, ws);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_lagrange_den, dim3(msm_blocks(n, 256)), dim3(256), 0, s, n_inst, t, ws, lambda,
                     dup, done);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_lagrange_inv, dim3(n_inst), dim3(LG_BS), 0, s, t, ws, lambda, done);
  return hipGetLastError();
}

hipError_t launch_msm_digits(hipStream_t s, const MsmPlan& p, const uint32_t* scalars,
                             int16_t* digits, uint32_t* list, uint32_t* roff) {
  const uint64_t terms = (uint64_t)p.n_msm * p.n;
  if (terms == 0) return hipSuccess;
  hipLaunchKernelGGL(k_msm_recode, dim3(msm_blocks(terms, 256)), dim3(256), 0, s, terms, p.n, p.c,
                     p.W, scalars, digits);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t lds = ((size_t)(1u << (p.c - 1)) + MSM_SORT_BS) * 4;
  hipLaunchKernelGGL(k_msm_sort, dim3((uint32_t)((uint64_t)p.n_msm * p.W)), dim3(MSM_SORT_BS), lds,
                     s, p.n, p.c, (const int16_t*)digits, list, roff);
  return hipGetLastError();
}
#endif

template <class F, int NW>
static hipError_t launch_msm_reduce(hipStream_t s, const MsmPlan& p, const Aff<F>* pts,
                                    const uint32_t* pts_map, const uint32_t* list,
                                    const uint32_t* roff, Jac<F>* part,
                                    Jac<F>* wsum, const uint32_t* sel_cnt, uint32_t t,
                                    const uint32_t* bad, const uint32_t* dup, int32_t* status,
                                    uint8_t* out, uint8_t* parity) {
  const uint32_t S = (1u << (p.c - 1)) / 8;
  const uint64_t lanes = (uint64_t)p.n_msm * p.W * S;
  hipLaunchKernelGGL((k_msm_buckets<F>), dim3(msm_blocks(lanes, 64)), dim3(64), 0, s, lanes, p.n,
                     p.c, p.W, pts, list, roff, pts_map, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint64_t n_mw = (uint64_t)p.n_msm * p.W;
  hipLaunchKernelGGL((k_msm_wsum<F>), dim3(msm_blocks(n_mw, 64)), dim3(64), 0, s, n_mw, S,
                     (const Jac<F>*)part, wsum);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_msm_final<F, NW>), dim3(msm_blocks(p.n_msm, 64)), dim3(64), 0, s, p.n_msm,
                     p.c, p.W, (const Jac<F>*)wsum, sel_cnt, t, bad, dup, status, out, parity);
  return hipGetLastError();
}

#if HBTC_IN_PART(8)
template <class A>
static hipError_t launch_msm_gather(hipStream_t s, uint32_t n_inst, uint32_t t,
                                    const uint32_t* sel_pos, const uint32_t* sel_cnt, const A* dec,
                                    A* pts) {
  const uint64_t terms = (uint64_t)n_inst * t;
  if (terms == 0) return hipSuccess;
  hipLaunchKernelGGL((k_msm_gather<A>), dim3(msm_blocks(terms, 256)), dim3(256), 0, s, n_inst, t,
                     sel_pos, sel_cnt, dec, pts);
  return hipGetLastError();
}
hipError_t launch_msm_gather_g1(hipStream_t s, uint32_t n_inst, uint32_t t, const uint32_t* sel_pos,
                                const uint32_t* sel_cnt, const G1A* dec, G1A* pts) {
  return launch_msm_gather(s, n_inst, t, sel_pos, sel_cnt, dec, pts);
}
hipError_t launch_msm_gather_g2(hipStream_t s, uint32_t n_inst, uint32_t t, const uint32_t* sel_pos,
                                const uint32_t* sel_cnt, const G2A* dec, G2A* pts) {
  return launch_msm_gather(s, n_inst, t, sel_pos, sel_cnt, dec, pts);
}

// GLS split of a G2 combine (ψ acts on G2 as [x], x = -u, u = |x| = 2^16 v): every term
// λ P with λ < r < u^4 becomes four 64-bit terms
//     λ P = d0 P + d1 [u]P + d2 [u^2]P + d3 [u^3]P,   λ = sum_j d_j u^j,  0 <= d_j < u,
// [u]P = -ψ(P) = (ψ_x, -ψ_y), [u^2]P = ψ^2(P), [u^3]P = -ψ^3(P) -- so the Pippenger pass runs
// over 65-bit windows (a Horner chain of ~64 doublings in k_msm_final instead of ~255) and the
// result is the same point.  Term k of msm m goes to positions m * 4n + 4k + j; scalars are
// written in the 8-word canonical layout k_msm_recode reads.
__global__ void __launch_bounds__(64) k_msm_gls_g2(uint64_t terms, uint32_t n,
                                                   const uint32_t* __restrict__ lambda,
                                                   const G2A* __restrict__ pts,
                                                   uint32_t* __restrict__ sc4, G2A* __restrict__ pts4) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  const uint64_t g = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (g >= terms) return;
  uint64_t d[4];
  gls_u_digits(lambda + g * 8, d);
  const G2A p = pts[g];
  G2A q[4];
  q[0] = p;
  Fq2 x1, y1, x2, y2, x3, y3;
  g2_psi(x1, y1, p);
  G2A t1;
  t1.x = x1;
  t1.y = y1;
  t1.inf = p.inf;
  g2_psi(x2, y2, t1);
  G2A t2;
  t2.x = x2;
  t2.y = y2;
  t2.inf = p.inf;
  g2_psi(x3, y3, t2);
  q[1].x = x1;
  fq2_neg(q[1].y, y1);  // [u]P = -ψ(P)
  q[2] = t2;            // [u^2]P = ψ^2(P)
  q[3].x = x3;
  fq2_neg(q[3].y, y3);  // [u^3]P = -ψ^3(P)
  q[1].inf = q[2].inf = q[3].inf = p.inf;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    pts4[4 * g + j] = q[j];
    uint32_t* o = sc4 + (4 * g + j) * 8;
    o[0] = (uint32_t)d[j];
    o[1] = (uint32_t)(d[j] >> 32);
#pragma unroll
    for (int i = 2; i < 8; ++i) o[i] = 0u;
  }
}

// GLV split of a G1 combine (φ = [-x^2] = [-u^2] on G1): λ P = e0 P + e1 [u^2]P with
// λ = e0 + e1 u^2, 0 <= e_j < u^2 < 2^128 (the base-u digits paired: e0 = d0 + d1 u,
// e1 = d2 + d3 u), [u^2]P = -φ(P) = (β x, -y).  Term k of msm m goes to 2k + j.
__global__ void __launch_bounds__(64) k_msm_glv_g1(uint64_t terms, const uint32_t* __restrict__ lambda,
                                                   const G1A* __restrict__ pts,
                                                   uint32_t* __restrict__ sc2, G1A* __restrict__ pts2) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  const uint64_t g = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (g >= terms) return;
  uint64_t d[4];
  gls_u_digits(lambda + g * 8, d);
  const G1A p = pts[g];
  G1A q = p;
  Fq beta;
  fq_set(beta, G1_BETA);
  fq_mul(q.x, p.x, beta);
  fq_neg(q.y, p.y);
  pts2[2 * g] = p;
  pts2[2 * g + 1] = q;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    // e = d_lo + d_hi * u  (< u^2 < 2^128)
    const uint64_t lo = d[2 * j], hi = d[2 * j + 1];
    const uint64_t m_lo = hi * BLS_X_ABS, m_hi = __umul64hi(hi, BLS_X_ABS);
    const uint64_t e_lo = m_lo + lo, e_hi = m_hi + (e_lo < lo ? 1u : 0u);
    uint32_t* o = sc2 + (2 * g + j) * 8;
    o[0] = (uint32_t)e_lo;
    o[1] = (uint32_t)(e_lo >> 32);
    o[2] = (uint32_t)e_hi;
    o[3] = (uint32_t)(e_hi >> 32);
#pragma unroll
    for (int i = 4; i < 8; ++i) o[i] = 0u;
  }
}

hipError_t launch_msm_glv_g1(hipStream_t s, uint32_t n_msm, uint32_t n, const uint32_t* lambda,
                             const G1A* pts, uint32_t* sc2, G1A* pts2) {
  const uint64_t terms = (uint64_t)n_msm * n;
  if (terms == 0) return hipSuccess;
  hipLaunchKernelGGL(k_msm_glv_g1, dim3(msm_blocks(terms, 64)), dim3(64), 0, s, terms, lambda, pts, sc2,
                     pts2);
  return hipGetLastError();
}

hipError_t launch_msm_gls_g2(hipStream_t s, uint32_t n_msm, uint32_t n, const uint32_t* lambda,
                             const G2A* pts, uint32_t* sc4, G2A* pts4) {
  const uint64_t terms = (uint64_t)n_msm * n;
  if (terms == 0) return hipSuccess;
  hipLaunchKernelGGL(k_msm_gls_g2, dim3(msm_blocks(terms, 64)), dim3(64), 0, s, terms, n, lambda, pts,
                     sc4, pts4);
  return hipGetLastError();
}
hipError_t launch_msm_decode_g1(hipStream_t s, uint32_t n_msm, uint32_t n, uint32_t stride,
                                const uint8_t* pts_c, const uint32_t* sel_pos,
                                const uint32_t* sel_cnt, const int32_t* item_status,
                                const G1A* dec, G1A* pts, uint32_t* bad) {
  const uint64_t terms = (uint64_t)n_msm * n;
  if (terms == 0) return hipSuccess;
  hipLaunchKernelGGL((k_msm_decode<Fq, 12>), dim3(msm_blocks(terms, 64)), dim3(64), 0, s, n_msm, n,
                     stride, pts_c, sel_pos, sel_cnt, item_status, dec, pts, bad);
  return hipGetLastError();
}
hipError_t launch_msm_reduce_g1(hipStream_t s, const MsmPlan& p, const G1A* pts,
                                const uint32_t* pts_map, const uint32_t* list, const uint32_t* roff, G1J* part, G1J* wsum,
                                const uint32_t* sel_cnt, uint32_t t, const uint32_t* bad,
                                const uint32_t* dup, int32_t* status, uint8_t* out) {
  if (p.n_msm == 0) return hipSuccess;
  return launch_msm_reduce<Fq, 12>(s, p, pts, pts_map, list, roff, part, wsum, sel_cnt, t, bad, dup, status,
                                   out, nullptr);
}
#endif
#if HBTC_IN_PART(9)
hipError_t launch_msm_decode_g2(hipStream_t s, uint32_t n_msm, uint32_t n, uint32_t stride,
                                const uint8_t* pts_c, const uint32_t* sel_pos,
                                const uint32_t* sel_cnt, const int32_t* item_status,
                                const G2A* dec, G2A* pts, uint32_t* bad) {
  const uint64_t terms = (uint64_t)n_msm * n;
  if (terms == 0) return hipSuccess;
  hipLaunchKernelGGL((k_msm_decode<Fq2, 24>), dim3(msm_blocks(terms, 64)), dim3(64), 0, s, n_msm,
                     n, stride, pts_c, sel_pos, sel_cnt, item_status, dec, pts, bad);
  return hipGetLastError();
}
hipError_t launch_msm_reduce_g2(hipStream_t s, const MsmPlan& p, const G2A* pts,
                                const uint32_t* pts_map, const uint32_t* list, const uint32_t* roff, G2J* part, G2J* wsum,
                                const uint32_t* sel_cnt, uint32_t t, const uint32_t* bad,
                                const uint32_t* dup, int32_t* status, uint8_t* out,
                                uint8_t* parity) {
  if (p.n_msm == 0) return hipSuccess;
#if HBTC_MSM_G2_PAIR
  const uint32_t S = (1u << (p.c - 1)) / 8;
  const uint64_t lanes = (uint64_t)p.n_msm * p.W * S;
  hipLaunchKernelGGL(k_msm_buckets_g2p, dim3(msm_blocks(2 * lanes, 64)), dim3(64), 0, s, lanes, p.n,
                     p.c, p.W, pts, list, roff, pts_map, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint64_t n_mw = (uint64_t)p.n_msm * p.W;
  hipLaunchKernelGGL(k_msm_wsum_g2p, dim3(msm_blocks(2 * n_mw, 64)), dim3(64), 0, s, n_mw, S,
                     (const G2J*)part, wsum);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_msm_final_g2p, dim3(msm_blocks(2 * (uint64_t)p.n_msm, 64)), dim3(64), 0, s,
                     p.n_msm, p.c, p.W, (const G2J*)wsum, sel_cnt, t, bad, dup, status, out, parity);
  return hipGetLastError();
#else
  return launch_msm_reduce<Fq2, 24>(s, p, pts, pts_map, list, roff, part, wsum, sel_cnt, t, bad, dup, status,
                                    out, parity);
#endif
}
#endif

}  // namespace hbtc
