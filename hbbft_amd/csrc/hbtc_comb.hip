// Small Lagrange combines (t <= 64 shares per instance) in ONE launch: PublicKeySet::
// combine_signatures (src/coin.rs:185-191: a coin instance combines t = f + 1 SignatureShares, 4 at
// N = 10, 34 at N = 100) and PublicKeySet::decrypt (src/threshold_decryption.rs:181-185) for
// networks of up to ~190 validators.
//
// The Pippenger chain of hbtc_msm.hip (select -> Lagrange x / den / inv -> GLV/GLS split ->
// decode -> recode -> sort -> buckets -> segment sums -> Horner) is nine dependent launches whose
// per-lane chains are long for a handful of terms (C2's 100 x 34-share G2 combines: 11.7 ms in the
// bucket pass alone).  Here one workgroup of 128 lanes takes one instance:
//   wave 0     the first t ACCEPTed items in item order (hbbft's verified-share map order);
//   lane pair  (2i, 2i + 1) for selected share i: its Lagrange coefficient at 0,
//              lambda_i = prod_{j != i} x_j / prod_{j != i} (x_j - x_i) (x = idx + 1, one Fr
//              inversion per lane), split into base-u digits lambda = d0 + d1 u + d2 u^2 + d3 u^3
//              (u = |x|); lane h computes [d_2h] P + [d_2h+1] [u] P by the two-digit sign-aligned
//              double-and-add (curve.h sac2_mul: 64 doublings + 65 mixed additions), and lane 1
//              applies [u^2] (G1: -phi = (beta X, -Y); G2: psi^2 = (zeta X, -Y)) to its half;
//   tree       the 128 partial points summed in LDS, then normalised, compressed, the
//              instance status (NOT_ENOUGH_SHARES > DECODE_ERR > DUPLICATE_ENTRY > ACCEPT, as
//              k_msm_final) and Signature::parity (G2).
// [u] P: G2 -psi(P) (free); G1 [|x|] P by 64 doublings (jac_mul_u64).  Shares the verification
// decoded are gathered, never decoded again (as k_msm_decode); others are decoded with the
// subgroup check unless their status says the verifier accepted them.
#include "hbtc_kernels.h"
#include "pair.h"

namespace hbtc {

namespace {
__device__ __forceinline__ bool comb_decode(G1A& p, const uint32_t* w, bool chk) {
  return g1_decompress(p, w, chk);
}
__device__ __forceinline__ bool comb_decode(G2A& p, const uint32_t* w, bool chk) {
  return g2_decompress(p, w, chk);
}
// [u] P (u = |x|)
__device__ __forceinline__ void comb_upoint(G1J& r, const G1A& p) { jac_mul_u64(r, p, BLS_X_ABS); }
__device__ __forceinline__ void comb_upoint(G2J& r, const G2A& p) {
  G2A q;
  g2_psi(q.x, q.y, p);  // psi = [x] = [-u] on G2
  fq2_neg(q.y, q.y);
  q.inf = 0;
  jac_from_aff(r, q);
}
// [u] pk from the key set's fixed-base table: -([x] pk) (G1 only; G2 has no table)
__device__ __forceinline__ void comb_upoint_tab(G1J& r, const PtXY* tab, uint32_t node) {
  const PtXY e = tab[((size_t)node * PK_TAB_WIN + 4) * 256 + 1];
  r.x = e.x;
  fq_neg(r.y, e.y);
  fq_one(r.z);
}
__device__ __forceinline__ void comb_upoint_tab(G2J&, const PtXY*, uint32_t) {}
// r <- [u^2] r (Jacobian): G1 -phi(X, Y, Z) = (beta X, -Y, Z); G2 psi^2 = -(-psi^2) = (zeta X, -Y, Z)
__device__ __forceinline__ void comb_u2(G1J& r) {
  Fq c;
  fq_set(c, G1_BETA);
  fq_mul(r.x, r.x, c);
  fq_neg(r.y, r.y);
}
__device__ __forceinline__ void comb_u2(G2J& r) {
  Fq c;
  fq_set(c, G2_ZETA);
  fmul_by_fq(r.x, r.x, c);
  fq2_neg(r.y, r.y);
}
__device__ __forceinline__ void comb_store(uint8_t* out, size_t k, const uint32_t* w, int nw) {
  uint32_t* o = reinterpret_cast<uint32_t*>(out + k * (size_t)(nw * 4));
  for (int j = 0; j < nw; ++j) o[j] = w[j];
}
__device__ __forceinline__ void comb_load(uint32_t* w, const uint8_t* base, size_t item, int nw) {
  const uint4* q = reinterpret_cast<const uint4*>(base + item * (size_t)(nw * 4));
  for (int i = 0; i < nw / 4; ++i) {
    const uint4 v = q[i];
    w[4 * i] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
}
__device__ __forceinline__ void comb_compress(uint32_t* w, const G1A& p) { g1_compress(w, p); }
__device__ __forceinline__ void comb_compress(uint32_t* w, const G2A& p) { g2_compress(w, p); }
__device__ __forceinline__ uint32_t comb_parity(const G1A&) { return 0; }
__device__ __forceinline__ uint32_t comb_parity(const G2A& p) { return g2_parity(p); }
}  // namespace

template <class F, int NW>
__global__ void __launch_bounds__(COMB_SMALL_BS, 1) k_comb_small(CombSmallArgs A) {
  HBTC_LATENCY_PRIO();  // a latency chain beside the item passes: win the issue arbitration
  __shared__ uint32_t s_pos[COMB_SMALL_T];
  __shared__ Fr s_x[COMB_SMALL_T];
  __shared__ uint32_t s_cnt, s_bad, s_dup;
  __shared__ Jac<F> s_red[COMB_SMALL_BS];
  const uint32_t k = blockIdx.x, tid = threadIdx.x;
  if (A.only && !A.only[k]) return;  // block-uniform
  const uint32_t t = A.t;
  // speculative subsets (gridDim.y > 1): block j leaves out the instance's j-th item
  const uint32_t skip = gridDim.y > 1 ? blockIdx.y : 0xffffffffu;
  const size_t o = (size_t)k * gridDim.y + blockIdx.y;  // output slot
  if (tid < 64) {  // wave 0: the first t items whose status is ACCEPT (all items without status)
    const uint32_t a = A.offsets[k], b = A.offsets[k + 1];
    uint32_t found = 0;
    for (uint32_t base = a; base < b && found < t; base += 64) {
      const uint32_t i = base + tid;
      const bool ok = i < b && i - a != skip && (!A.item_status || A.item_status[i] == HBTC_ACCEPT);
      const uint64_t mask = __ballot(ok);
      const uint32_t slot = found + (uint32_t)__popcll(mask & ((1ull << tid) - 1ull));
      if (ok && slot < t) s_pos[slot] = i;
      found += (uint32_t)__popcll(mask);
    }
    if (tid == 0) {
      s_cnt = found < t ? found : t;
      s_bad = 0;
      s_dup = 0;
    }
  }
  __syncthreads();
  const uint32_t cnt = s_cnt;
  const uint32_t pi = tid >> 1, h = tid & 1u;
  const bool live = cnt == t && pi < cnt;
  if (live && h == 0) {
    Fr x;
    fr_from_u64(x, (uint64_t)A.idx[s_pos[pi]] + 1);
    s_x[pi] = x;
  }
  __syncthreads();
  Jac<F> R;
  jac_set_inf(R);
  if (live) {
    // lambda_i at 0 (Montgomery Fr), then canonical for the digit split
    const Fr xi = s_x[pi];
    Fr num, den;
    limbs_set_const<8>(num, FR_ONE);
    limbs_set_const<8>(den, FR_ONE);
    bool dup = false;
    for (uint32_t j = 0; j < cnt; ++j) {
      if (j == pi) continue;
      const Fr xj = s_x[j];
      dup |= limbs_eq<8>(xj, xi);
      Fr d;
      fr_sub(d, xj, xi);
      fr_mul(den, den, d);
      fr_mul(num, num, xj);
    }
    if (dup) atomicOr(&s_dup, 1u);
    Fr inv, l, lc;
    fr_inv(inv, den);  // den = 0 only for a duplicate: the instance fails, the value is unused
    fr_mul(l, num, inv);
    fr_from_mont(lc, l);
    uint64_t d[4];
    gls_u_digits(lc.v, d);
    // the point: a key-set entry (by node), the verification's decoded share, or decoded here
    const uint32_t pos = s_pos[pi];
    const Aff<F>* dec = static_cast<const Aff<F>*>(A.dec);
    Aff<F> P;
    if (A.by_node) {
      const uint32_t id = A.idx[pos];
      if (id < A.n_nodes) {
        P = dec[id];
      } else {  // an unknown sender (its share is never ACCEPTed: only speculative subsets get here)
        atomicOr(&s_bad, 1u);
        P.inf = 1;
      }
    } else {
      const bool accepted = A.item_status && A.item_status[pos] == HBTC_ACCEPT;
      if (accepted && dec) {
        P = dec[pos];
      } else {
        uint32_t w[NW];
        comb_load(w, A.pts, pos, NW);
        if (!comb_decode(P, w, !accepted && !A.nocheck)) {
          atomicOr(&s_bad, 1u);
          P.inf = 1;
        }
      }
    }
    if (!P.inf) {
      Jac<F> XP;
      if (A.xtab && A.by_node)
        comb_upoint_tab(XP, A.xtab, A.idx[pos]);
      else
        comb_upoint(XP, P);
      sac2_mul(R, P, XP, h ? d[2] : d[0], h ? d[3] : d[1], 64);
      if (h) comb_u2(R);
    }
  }
  s_red[tid] = R;
  __syncthreads();
  for (uint32_t s = COMB_SMALL_BS / 2; s >= 1; s >>= 1) {
    if (tid < s) {
      Jac<F> a = s_red[tid];
      const Jac<F> b = s_red[tid + s];
      jac_add(a, a, b);
      s_red[tid] = a;
    }
    __syncthreads();
  }
  if (tid == 0) {
    int32_t st = HBTC_ACCEPT;
    if (cnt < t)
      st = HBTC_NOT_ENOUGH_SHARES;
    else if (s_bad)
      st = HBTC_DECODE_ERR;
    else if (s_dup)
      st = HBTC_DUPLICATE_ENTRY;
    const Jac<F> sum = s_red[0];
    if (A.cmp) {  // compare with a point instead of encoding the sum
      const Aff<F> q = *static_cast<const Aff<F>*>(A.cmp);
      const bool si = jac_is_inf(sum);
      const bool eq = (si || q.inf) ? (si && q.inf) : jac_eq_aff(sum, q.x, q.y);
      A.inst_status[o] = st != HBTC_ACCEPT ? st : (eq ? HBTC_ACCEPT : HBTC_REJECT);
      return;
    }
    A.inst_status[o] = st;
    Aff<F> a;
    jac_to_aff(a, sum);
    uint32_t w[NW];
    comb_compress(w, a);
    if (st != HBTC_ACCEPT)
      for (int j = 0; j < NW; ++j) w[j] = 0;
    comb_store(A.out, o, w, NW);
    if (A.parity) A.parity[o] = (st == HBTC_ACCEPT) ? (uint8_t)comb_parity(a) : 0;
  }
}

#ifndef HBTC_COMB_G2_PAIR
#define HBTC_COMB_G2_PAIR 1  // G2 combines in lane-pair form (pair.h): four lanes per share
#endif
#if HBTC_COMB_G2_PAIR
// The G2 form of k_comb_small on lane pairs (round 6): share i on lanes 4i .. 4i + 3, lane
// (4i + 2h + e) holding component e of the digit-half h chain [d_2h] P + [d_2h+1] [u] P, so every
// Fq2 product of the 64-doubling chain is one fused two-product per lane (pair.h) instead of three
// products on one lane: half the chain's latency.  Selection, Lagrange coefficients and statuses
// as k_comb_small (every lane of a share computes its coefficient); the tree sums the 128 pair
// units in LDS; the final point is assembled on lane 0 for the encoding and the parity.
constexpr uint32_t COMB_G2P_BS = 4 * COMB_SMALL_T;
__global__ void __launch_bounds__(COMB_G2P_BS, 1) k_comb_small_g2p(CombSmallArgs A) {
  HBTC_LATENCY_PRIO();
  __shared__ uint32_t s_pos[COMB_SMALL_T];
  __shared__ Fr s_x[COMB_SMALL_T];
  __shared__ uint32_t s_cnt, s_bad, s_dup;
  __shared__ uint32_t s_red[36 * COMB_G2P_BS];  // [word][lane]
  const uint32_t k = blockIdx.x, tid = threadIdx.x;
  if (A.only && !A.only[k]) return;  // block-uniform
  const uint32_t t = A.t;
  const uint32_t skip = gridDim.y > 1 ? blockIdx.y : 0xffffffffu;
  const size_t o = (size_t)k * gridDim.y + blockIdx.y;
  if (tid < 64) {  // wave 0: the first t items whose status is ACCEPT (all items without status)
    const uint32_t a = A.offsets[k], b = A.offsets[k + 1];
    uint32_t found = 0;
    for (uint32_t base = a; base < b && found < t; base += 64) {
      const uint32_t i = base + tid;
      const bool ok = i < b && i - a != skip && (!A.item_status || A.item_status[i] == HBTC_ACCEPT);
      const uint64_t mask = __ballot(ok);
      const uint32_t slot = found + (uint32_t)__popcll(mask & ((1ull << tid) - 1ull));
      if (ok && slot < t) s_pos[slot] = i;
      found += (uint32_t)__popcll(mask);
    }
    if (tid == 0) {
      s_cnt = found < t ? found : t;
      s_bad = 0;
      s_dup = 0;
    }
  }
  __syncthreads();
  const uint32_t cnt = s_cnt;
  const uint32_t pi = tid >> 2, h = (tid >> 1) & 1u;
  const bool live = cnt == t && pi < cnt;
  if (live && (tid & 3u) == 0) {
    Fr x;
    fr_from_u64(x, (uint64_t)A.idx[s_pos[pi]] + 1);
    s_x[pi] = x;
  }
  __syncthreads();
  G2Jp R;
  jac_set_inf(R);
  if (live) {
    const Fr xi = s_x[pi];
    Fr num, den;
    limbs_set_const<8>(num, FR_ONE);
    limbs_set_const<8>(den, FR_ONE);
    bool dup = false;
    for (uint32_t j = 0; j < cnt; ++j) {
      if (j == pi) continue;
      const Fr xj = s_x[j];
      dup |= limbs_eq<8>(xj, xi);
      Fr d;
      fr_sub(d, xj, xi);
      fr_mul(den, den, d);
      fr_mul(num, num, xj);
    }
    if (dup) atomicOr(&s_dup, 1u);
    Fr inv, l, lc;
    fr_inv(inv, den);
    fr_mul(l, num, inv);
    fr_from_mont(lc, l);
    uint64_t d[4];
    gls_u_digits(lc.v, d);
    const uint32_t pos = s_pos[pi];
    const G2A* dec = static_cast<const G2A*>(A.dec);
    G2Ap P;
    P.inf = 1;
    if (A.by_node) {
      const uint32_t id = A.idx[pos];
      if (id < A.n_nodes)
        g2p_load_aff(P, dec + id);
      else
        atomicOr(&s_bad, 1u);  // an unknown sender (only speculative subsets get here)
    } else {
      const bool accepted = A.item_status && A.item_status[pos] == HBTC_ACCEPT;
      if (accepted && dec) {
        g2p_load_aff(P, dec + pos);
      } else {  // decoded on every lane of the pair (one-lane code), then split
        uint32_t w[24];
        comb_load(w, A.pts, pos, 24);
        G2A f;
        if (!comb_decode(f, w, !accepted && !A.nocheck)) {
          atomicOr(&s_bad, 1u);
        } else {
          const bool odd = pair_odd();
          P.x.v = odd ? f.x.c1 : f.x.c0;
          P.y.v = odd ? f.y.c1 : f.y.c0;
          P.inf = f.inf;
        }
      }
    }
    if (!P.inf) {
      G2Ap xp;  // [u] P = -psi(P)
      g2p_psi(xp.x, xp.y, P);
      fneg(xp.y, xp.y);
      xp.inf = 0;
      G2Jp XP;
      jac_from_aff(XP, xp);
      sac2_mul(R, P, XP, h ? d[2] : d[0], h ? d[3] : d[1], 64);
      if (h) {  // [u^2] = psi^2 = (zeta X, -Y)
        Fq c;
        fq_set(c, G2_ZETA);
        fmul_by_fq(R.x, R.x, c);
        fneg(R.y, R.y);
      }
    }
  }
  auto put = [&](uint32_t unit, const G2Jp& x) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&x);
    const uint32_t l = 2 * unit + (tid & 1u);
#pragma unroll
    for (int w = 0; w < 36; ++w) s_red[w * COMB_G2P_BS + l] = src[w];
  };
  auto get = [&](G2Jp& x, uint32_t unit) {
    uint32_t* dst = reinterpret_cast<uint32_t*>(&x);
    const uint32_t l = 2 * unit + (tid & 1u);
#pragma unroll
    for (int w = 0; w < 36; ++w) dst[w] = s_red[w * COMB_G2P_BS + l];
  };
  const uint32_t unit = tid >> 1;
  put(unit, R);
  __syncthreads();
  for (uint32_t s = COMB_G2P_BS / 4; s >= 1; s >>= 1) {
    if (unit < s) {
      G2Jp a, b;
      get(a, unit);
      get(b, unit + s);
      jac_add_lean(a, b);
      put(unit, a);
    }
    __syncthreads();
  }
  if (tid < 2) {
    int32_t st = HBTC_ACCEPT;
    if (cnt < t)
      st = HBTC_NOT_ENOUGH_SHARES;
    else if (s_bad)
      st = HBTC_DECODE_ERR;
    else if (s_dup)
      st = HBTC_DUPLICATE_ENTRY;
    G2Jp sum;
    get(sum, 0);
    const bool si = jac_is_inf(sum);
    if (A.cmp) {  // compare with a point instead of encoding the sum
      G2Ap q;
      g2p_load_aff(q, static_cast<const G2A*>(A.cmp));
      const bool eq = (si || q.inf) ? (si && q.inf) : jac_eq_aff(sum, q.x, q.y);
      if (tid == 0) A.inst_status[o] = st != HBTC_ACCEPT ? st : (eq ? HBTC_ACCEPT : HBTC_REJECT);
      return;
    }
    G2Ap ap;
    jac_to_aff(ap, sum);
    Fq px, py;  // the partner's components: lane 0 assembles the Fq2 point
    fq_xchg(px, ap.x.v);
    fq_xchg(py, ap.y.v);
    if (tid == 0) {
      A.inst_status[o] = st;
      G2A a;
      a.x.c0 = ap.x.v;
      a.x.c1 = px;
      a.y.c0 = ap.y.v;
      a.y.c1 = py;
      a.inf = si ? 1u : 0u;
      uint32_t w[24];
      comb_compress(w, a);
      if (st != HBTC_ACCEPT)
        for (int j = 0; j < 24; ++j) w[j] = 0;
      comb_store(A.out, o, w, 24);
      if (A.parity) A.parity[o] = (st == HBTC_ACCEPT) ? (uint8_t)comb_parity(a) : 0;
    }
  }
}
#endif

hipError_t launch_comb_small(hipStream_t s, int group, uint32_t n_inst, uint32_t n_sub,
                             const CombSmallArgs& a) {
  if (n_inst == 0) return hipSuccess;
  if (a.t == 0 || a.t > COMB_SMALL_T || n_sub == 0) return hipErrorInvalidValue;
  if (group == 1)
    hipLaunchKernelGGL((k_comb_small<Fq, 12>), dim3(n_inst, n_sub), dim3(COMB_SMALL_BS), 0, s, a);
  else
#if HBTC_COMB_G2_PAIR
    hipLaunchKernelGGL(k_comb_small_g2p, dim3(n_inst, n_sub), dim3(COMB_G2P_BS), 0, s, a);
#else
    hipLaunchKernelGGL((k_comb_small<Fq2, 24>), dim3(n_inst, n_sub), dim3(COMB_SMALL_BS), 0, s, a);
#endif
  return hipGetLastError();
}

// ---------------------------------------------------------------- coin calls: commit
// One thread per coin instance, after its shares' verification: the speculative subset whose
// selection equals the verified one -- the first t items when they are all ACCEPTed (subset t,
// which leaves out item t), or the first t + 1 minus the one non-ACCEPTed item j < t (subset j)
// -- has its signature, parity, combine status and master check copied to the outputs; any
// other pattern (two or more rejected among the first t + 1, fewer than t + 1 items with a
// rejection, fewer than t items) is flagged for the status-driven combine (redo).
__global__ void __launch_bounds__(64) k_coin_commit(uint32_t n_inst, uint32_t t, const uint32_t* __restrict__ offsets,
                                                    const int32_t* __restrict__ item_status, uint32_t n_sub,
                                                    const int32_t* __restrict__ spec_cst,
                                                    const uint8_t* __restrict__ spec_sig,
                                                    const uint8_t* __restrict__ spec_par,
                                                    const int32_t* __restrict__ spec_master,
                                                    int32_t* __restrict__ cst, uint8_t* __restrict__ sig,
                                                    uint8_t* __restrict__ par, int32_t* __restrict__ master,
                                                    uint32_t* __restrict__ redo) {
  const uint32_t k = blockIdx.x * 64 + threadIdx.x;
  if (k >= n_inst) return;
  const uint32_t a = offsets[k], c = offsets[k + 1] - a;
  uint32_t choice = 0xffffffffu;
  if (c >= t) {
    const uint32_t m = c < t + 1 ? c : t + 1;
    uint32_t nrej = 0, rej = 0;
    for (uint32_t i = 0; i < m; ++i)
      if (item_status[a + i] != HBTC_ACCEPT) {
        ++nrej;
        rej = i;
      }
    if (nrej == 0 || (nrej == 1 && rej == t))
      choice = t;  // the first t are ACCEPTed
    else if (nrej == 1 && c >= t + 1)
      choice = rej;
  }
  if (choice == 0xffffffffu) {
    redo[k] = 1;
    return;
  }
  redo[k] = 0;
  const size_t o = (size_t)k * n_sub + choice;
  cst[k] = spec_cst[o];
  master[k] = spec_master[o];
  par[k] = spec_par[o];
  const uint4* src = reinterpret_cast<const uint4*>(spec_sig + o * 96);
  uint4* dst = reinterpret_cast<uint4*>(sig + (size_t)k * 96);
  for (int j = 0; j < 6; ++j) dst[j] = src[j];
}

hipError_t launch_coin_commit(hipStream_t s, uint32_t n_inst, uint32_t t, const uint32_t* offsets,
                              const int32_t* item_status, uint32_t n_sub, const int32_t* spec_cst,
                              const uint8_t* spec_sig, const uint8_t* spec_par,
                              const int32_t* spec_master, int32_t* cst, uint8_t* sig, uint8_t* par,
                              int32_t* master, uint32_t* redo) {
  if (n_inst == 0) return hipSuccess;
  hipLaunchKernelGGL(k_coin_commit, dim3((n_inst + 63) / 64), dim3(64), 0, s, n_inst, t, offsets,
                     item_status, n_sub, spec_cst, spec_sig, spec_par, spec_master, cst, sig, par,
                     master, redo);
  return hipGetLastError();
}

}  // namespace hbtc
