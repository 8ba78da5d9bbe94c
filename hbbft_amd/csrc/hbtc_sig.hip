// Random-linear-combination batch verification of SignatureShares — the fast path behind
// hbtc_verify_sig_shares (PublicKeyShare::verify, /root/reference/src/coin.rs:151, called once
// per share by the reference; every share of a coin instance signs the same nonce, so
// H = hash_g2(nonce) is one G2 point per instance: SURVEY.md §3.1's batching lever).
//
// Share i of instance k is valid iff E_i = e(pk_i, H) e(-G1, sigma_i) == 1.  For a group G:
//     every share valid  =>  e(sum_G r_i pk_i, H) * e(-G1, sum_G r_i sigma_i) == prod E_i^r_i == 1
// with r_i = a_i + b_i mu drawn as in hbtc_rlc.hip (mu = -x^2 mod r, the eigenvalue of phi on
// G1 and of -psi^2 on G2, so r_i pk_i comes from the fixed-base table and r_i sigma_i =
// [a] sigma + [b] (-psi^2(sigma)) is a joint 32-bit double-and-add in G2).  Location of a single
// wrong share (position-weighted sums), the 64 -> 8 -> 1 split and the probability bounds are
// those of the DecryptionShare path.
//
// The G2 argument of the second pair varies per group, so its Miller-loop lines are computed
// per group (k_plines: one lane walks the 68 steps of the affine sum, projective (A, B, C) per
// step) and evaluated at the fixed point -G1 by the cooperative check (gt6.h miller2_t<true>).
#include "gt6.h"
#include "pair.h"
#include "rlc_common.h"

namespace hbtc {

#ifndef HBTC_SIG_SPLIT
#define HBTC_SIG_SPLIT 1
#endif
#ifndef HBTC_SIG_TAB_LDS
#define HBTC_SIG_TAB_LDS 1  // k_sig_items: the x-adic table's three points in LDS
#endif
#ifndef HBTC_SIG_DEC_WAVES
#define HBTC_SIG_DEC_WAVES 2
#endif
// Round 6 defaults: the lane-pair kernels.  The one-lane kernels they replace are compiled only
// into variant builds that switch them back (tools/build_variant.sh), so the library holds no
// unused one-lane G2 kernel.  HBTC_SIGDEC_PAIR=0 goes on both objects (hbtc_sig.s1 defines the
// one-lane decode that s2 launches).
#ifndef HBTC_SIG_PAIR
#define HBTC_SIG_PAIR 1  // k_sig_items in lane-pair form (pair.h; 0: the one-lane kernel)
#endif
#ifndef HBTC_SIGDEC_PAIR
#define HBTC_SIGDEC_PAIR 1  // k_sig_decode with its psi chains on lane pairs (k_sig_decode_pair)
#endif
// The file is compiled twice (Makefile): part 1 = the decode half with the Fq product inlined
// (its loops then run without scratch: the shared subroutine's 102 fixed VGPRs left the G2
// doubling loop re-reading ~150 spilled dwords per bit at two waves), part 2 = the rest with the
// product as the shared subroutine.
#ifndef HBTC_SIG_PART
#define HBTC_SIG_PART 0
#endif
#define HBTC_SIG_IN(n) (HBTC_SIG_PART == 0 || HBTC_SIG_PART == (n))
#if HBTC_SIG_SPLIT && HBTC_SIG_IN(1) && !HBTC_SIGDEC_PAIR
// The decode half of the SignatureShare item pass, a kernel of its own so it runs at two waves per
// SIMD (432 B/lane of scratch; in one kernel with the scalar half the G2 state needs one wave per
// SIMD): zcash G2 decode with the psi subgroup test into dec, DECODE_ERR into status (every other
// item: RLC_PENDING, decided by k_sig_items).
__global__ void __launch_bounds__(64, HBTC_SIG_DEC_WAVES) k_sig_decode(
    const Tile* __restrict__ tiles, const uint32_t* __restrict__ idx, const uint8_t* __restrict__ sigs,
    const int32_t* __restrict__ pk_status, uint32_t n_pk, G2A* __restrict__ dec,
    int32_t* __restrict__ status) {
  const Tile tile = tiles[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  if (lane >= tile.count) return;
  const size_t item = (size_t)tile.first + lane;
  const uint32_t id = idx[item];
  int32_t st = HBTC_RLC_PENDING;
  if (id < n_pk && pk_status[id] == HBTC_ACCEPT) {
    uint32_t w[24];
    rlc_load_words(w, sigs, item, 24);
    G2A sg;
    if (!g2_decompress(sg, w, false)) {
      st = HBTC_DECODE_ERR;
    } else {
      // for the scalar half, the exact leaf checks and the combine; then the psi subgroup test
      // (curve.h g2_in_subgroup: psi(P) == -[|x|] P) with P parked there: the double-and-add
      // re-reads it for each of its five additions and for the final comparison, so the
      // doublings run with only the accumulator live (772 -> 588 B/lane with the shared-
      // subroutine product, 432 with it inlined -- this part's build -- and no scratch access in
      // any loop; one wave per SIMD instead, 0 B/lane, loses: C4 126 vs 131 ms,
      // profiles/r05/run21/)
      dec[item] = sg;
      if (!sg.inf) {
        G2J t;
        jac_from_aff(t, sg);  // bit 63 of |x|
#pragma unroll 1
        for (int b = 62; b >= 0; --b) {
          jac_dbl(t, t);
          if ((BLS_X_ABS >> b) & 1ull) {
            __asm__ volatile("" ::: "memory");  // P is re-read, not kept in registers
            const G2A q = dec[item];
            jac_add_aff(t, t, q);
          }
        }
        __asm__ volatile("" ::: "memory");
        const G2A q = dec[item];
        Fq2 px, py, npy;
        g2_psi(px, py, q);
        fq2_neg(npy, py);
        if (jac_is_inf(t) || !jac_eq_aff(t, px, npy)) st = HBTC_DECODE_ERR;
      }
    }
  }
  status[item] = st;
}
hipError_t launch_sig_decode(hipStream_t s, uint32_t n_tiles, const Tile* tiles, const uint32_t* idx,
                             const uint8_t* sigs, const int32_t* pk_status, uint32_t n_pk, G2A* dec,
                             int32_t* status) {
  hipLaunchKernelGGL(k_sig_decode, dim3(n_tiles), dim3(64), 0, s, tiles, idx, sigs, pk_status, n_pk, dec,
                     status);
  return hipGetLastError();
}
#endif

#if HBTC_SIG_IN(2)
hipError_t launch_sig_decode(hipStream_t s, uint32_t n_tiles, const Tile* tiles, const uint32_t* idx,
                             const uint8_t* sigs, const int32_t* pk_status, uint32_t n_pk, G2A* dec,
                             int32_t* status);
#ifndef HBTC_SIGDEC_WAVES
#define HBTC_SIGDEC_WAVES 2
#endif
#if HBTC_SIGDEC_PAIR
// The decode half of the SignatureShare item pass with the subgroup test's chain on lane pairs:
// every lane decodes one share (the square roots, one-lane form: no redundant work), then each lane
// pair runs the psi test of its two shares one after the other in pair form ([|x|] P: 63 doublings
// and 5 additions, the point exchanged from its lane by DPP), so the chain's state is 36 + 24
// registers per lane instead of 72 + 48 and the kernel runs more waves per SIMD.
__global__ void __launch_bounds__(64, HBTC_SIGDEC_WAVES) k_sig_decode_pair(
    const Tile* __restrict__ tiles, const uint32_t* __restrict__ idx, const uint8_t* __restrict__ sigs,
    const int32_t* __restrict__ pk_status, uint32_t n_pk, G2A* __restrict__ dec,
    int32_t* __restrict__ status) {
  const Tile tile = tiles[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  const size_t item = (size_t)tile.first + lane;
  const bool in = lane < tile.count;
  int32_t st = HBTC_RLC_PENDING;
  bool test = false;  // decoded, not infinity: needs the subgroup test
  G2A sg;
  fq2_zero(sg.x);
  fq2_zero(sg.y);
  sg.inf = 1;
  if (in) {
    const uint32_t id = idx[item];
    if (id < n_pk && pk_status[id] == HBTC_ACCEPT) {
      uint32_t w[24];
      rlc_load_words(w, sigs, item, 24);
      if (!g2_decompress(sg, w, false)) {
        st = HBTC_DECODE_ERR;
      } else {
        dec[item] = sg;
        test = !sg.inf;
      }
    }
  }
  const bool odd = (lane & 1u) != 0;
#pragma unroll 1
  for (uint32_t k = 0; k < 2; ++k) {
    // the pair's share k (held by lane 2j + k): each lane takes its component of it
    const bool holder = (odd ? 1u : 0u) == k;
    G2Ap P;
    {
      Fq sx, sy, rx, ry;
      fq_sel(sx, odd, sg.x.c0, sg.x.c1);  // what the partner needs: the other component
      fq_sel(sy, odd, sg.y.c0, sg.y.c1);
      fq_xchg(rx, sx);
      fq_xchg(ry, sy);
      Fq ox, oy;
      fq_sel(ox, odd, sg.x.c1, sg.x.c0);  // the own component of the own share
      fq_sel(oy, odd, sg.y.c1, sg.y.c0);
      fq_sel(P.x.v, holder, ox, rx);
      fq_sel(P.y.v, holder, oy, ry);
      P.inf = 0;
    }
    const uint32_t t_other = pair_xchg(test ? 1u : 0u);
    const bool run = holder ? test : t_other != 0u;  // pair-uniform
    if (run) {
      G2Jp t;
      jac_from_aff(t, P);  // bit 63 of |x|
#pragma unroll 1
      for (int b = 62; b >= 0; --b) {
        jac_dbl(t, t);
        if ((BLS_X_ABS >> b) & 1ull) jac_add_aff(t, t, P);
      }
      const bool ok = g2p_psi_test(t, P);
      if (holder && !ok) st = HBTC_DECODE_ERR;
    }
  }
  if (in) status[item] = st;
}
#endif
#if !(HBTC_SIG_PAIR && HBTC_SIG_SPLIT)
// One wave per tile: decode every SignatureShare (zcash compressed G2 + subgroup check), r_i,
// r_i sigma_i, r_i pk_i, then the plain and weighted tile / sub-tile sums in both groups.  One
// wave per SIMD (256 VGPRs + 256 AGPRs).  No kernel keeps a multi-KB private segment any more:
// the runtime reserves a kernel's scratch per hardware queue, and with 16 queues such segments
// aborted queues in round 3 (HSA_STATUS_ERROR_OUT_OF_RESOURCES).
__global__ void __launch_bounds__(64, 1) k_sig_items(
    const Tile* __restrict__ tiles, const uint32_t* __restrict__ idx,
    const uint8_t* __restrict__ sigs, const G1A* __restrict__ pk,
    const int32_t* __restrict__ pk_status, const PtXY* __restrict__ pk_tab, uint32_t n_pk,
    RlcKey key, Suspects sus, SigTileSums* __restrict__ sums, G2A* __restrict__ dec,
    int32_t* __restrict__ status) {
  __shared__ G2J red2[2][64];  // reused for the G1 reduction
  G1J* red1 = reinterpret_cast<G1J*>(&red2[0][0]);
  const Tile tile = tiles[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  const size_t item = (size_t)tile.first + lane;
  G2J S;
  G1J P;
  jac_set_inf(S);
  jac_set_inf(P);
  bool leaf = false;
  if (lane < tile.count) {
    int32_t st = HBTC_RLC_PENDING;
    const uint32_t id = idx[item];
    if (id >= n_pk) {
      st = HBTC_UNKNOWN_SENDER;
    } else if (pk_status[id] != HBTC_ACCEPT) {
      st = HBTC_DECODE_ERR;
    } else {
      G2A sg;
#if HBTC_SIG_SPLIT
      const bool dec_ok = status[item] != HBTC_DECODE_ERR;  // k_sig_decode ran first
      if (dec_ok) sg = dec[item];
#else
      uint32_t w[24];
      rlc_load_words(w, sigs, item, 24);
      const bool dec_ok = g2_decompress(sg, w);
#endif
      if (!dec_ok) {
        st = HBTC_DECODE_ERR;
      } else {
#if !HBTC_SIG_SPLIT
        dec[item] = sg;  // for the exact leaf checks and the combine (no second decode)
#endif
        if (is_suspect(sus, id)) {
          st = HBTC_RLC_LEAF;  // straight to an exact check, outside the group sums
        } else {
          // the x-adic scalar (rlc_common.h rlc_digits): [x] sigma = psi(sigma) on G2 (free), m =
          // -psi^2 = (zeta x, y) of eigenvalue mu = -x^2
          const XDigits xd = rlc_digits(key, item);
          if (!sg.inf) {
            G2A xp;
            g2_psi(xp.x, xp.y, sg);
            xp.inf = 0;
            G2J xj;
            jac_from_aff(xj, xp);
            Fq zeta;
            fq_set(zeta, G2_ZETA);
            G2A pxp;
            xadic_table(xp, pxp, sg, xj);
#if HBTC_SIG_TAB_LDS
            // the three table points in the reduction's LDS (idle until the loop is over: one
            // wave per block)
            uint32_t* tl = reinterpret_cast<uint32_t*>(&red2[0][0]);
            xy_lds_put_aff(tl, lane, 0, sg);
            xy_lds_put_aff(tl, lane, 1, xp);
            xy_lds_put_aff(tl, lane, 2, pxp);
            xadic_mul_uniform_lds(S, tl, lane, zeta, xd.d[0], xd.d[1], xd.d[2], xd.d[3], xd.nbits);
#else
            xadic_mul_uniform(S, sg, xp, pxp, zeta, xd.d[0], xd.d[1], xd.d[2], xd.d[3], xd.nbits);
#endif
          }
          if (!pk[id].inf) rlc_pk_mul_x(P, pk_tab + (size_t)id * PK_TAB_WIN * 256, xd);
        }
      }
    }
    status[item] = st;
    leaf = st == HBTC_RLC_LEAF;
  }
  rlc_list_leaf(sus, leaf, (uint32_t)item, tile.inst, lane);
  SigTileSums* ts = sums + blockIdx.x;
  rlc_reduce<Fq2>(red2[0], red2[1], S, lane, ts->S, ts->SW);
  rlc_reduce<Fq>(red1, red1 + 64, P, lane, ts->P, ts->PW);
}

#endif  // one-lane k_sig_items

#ifndef HBTC_SIGP_WAVES
#define HBTC_SIGP_WAVES 2  // k_sig_items_pair: minimum waves per SIMD of the register allocation
#endif
// The wave-local form of a __syncthreads between LDS writes and reads of ONE wave: a wave's LDS
// operations execute in order, so only the compiler's reordering and the outstanding counters
// need fencing.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// r pk_i of the x-adic scalar on a lane pair: lane e takes digits e and e + 2 (the pk window of
// digit e, then the phi window of digit e + 2: the beta product is on the same iteration for
// both lanes), 8 of the 16 mixed additions; the pair's halves are then added (both lanes hold
// the sum).
__device__ __forceinline__ void rlc_pk_mul_x_pair(G1J& r, const PtXY* __restrict__ tab, const XDigits& x) {
  const uint32_t e = pair_odd() ? 1u : 0u;
  jac_set_inf(r);
  const int nwin = x.nbits / 8;
#pragma unroll 1
  for (int i = 0; i < 2; ++i) {
    const uint32_t j = e + 2u * (uint32_t)i;
    const uint32_t dj = x.d[0] * (j == 0) + x.d[1] * (j == 1) + x.d[2] * (j == 2) + x.d[3] * (j == 3);
    const int tw = (j & 1u) ? 4 : 0;  // d1, d3: the [x] pk windows
#pragma unroll 1
    for (int w = 0; w < nwin; ++w) {
      const uint32_t v = (dj >> (8 * w)) & 0xffu;
      if (!v) continue;
      const PtXY en = tab[(tw + w) * 256 + v];
      G1A q;
      q.y = en.y;
      q.inf = 0;
      if (i == 1) {  // digits 2, 3: phi
        Fq beta;
        fq_set(beta, G1_BETA);
        fq_mul(q.x, en.x, beta);
      } else {
        q.x = en.x;
      }
      jac_add_aff(r, r, q);
    }
  }
  G1J o;
  fq_xchg(o.x, r.x);
  fq_xchg(o.y, r.y);
  fq_xchg(o.z, r.z);
  jac_add(r, r, o);
}

// LDS layouts of the two reductions: word w of item m's G2 point component e at
// w * 128 + 2 m + e (36 words), of its G1 point at w * 64 + m -- a wave's stores are conflict-free.
__device__ __forceinline__ void g2p_lds_put(uint32_t* lds, uint32_t m, const G2Jp& a) {
  const uint32_t o = 2 * m + (pair_odd() ? 1u : 0u);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&a);
#pragma unroll
  for (int w = 0; w < 36; ++w) lds[w * 128 + o] = src[w];
}
__device__ __forceinline__ void g2p_lds_get(G2Jp& a, const uint32_t* lds, uint32_t m) {
  const uint32_t o = 2 * m + (pair_odd() ? 1u : 0u);
  uint32_t* dst = reinterpret_cast<uint32_t*>(&a);
#pragma unroll
  for (int w = 0; w < 36; ++w) dst[w] = lds[w * 128 + o];
}
__device__ __forceinline__ void g1_lds_put(uint32_t* lds, uint32_t m, const G1J& a) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&a);
#pragma unroll
  for (int w = 0; w < 36; ++w) lds[w * 64 + m] = src[w];
}
__device__ __forceinline__ void g1_lds_get(G1J& a, const uint32_t* lds, uint32_t m) {
  uint32_t* dst = reinterpret_cast<uint32_t*>(&a);
#pragma unroll
  for (int w = 0; w < 36; ++w) dst[w] = lds[w * 64 + m];
}
template <class J>
__device__ __forceinline__ void shfl_words(J& r, const J& x, uint32_t src) {
  const uint32_t* xs = reinterpret_cast<const uint32_t*>(&x);
  uint32_t* rs = reinterpret_cast<uint32_t*>(&r);
  const int addr = (int)((src & 63u) << 2);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(J) / 4); ++i) rs[i] = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)xs[i]);
}

// 36 words of one lane at w * 64 + l (the B area of the G2 tree)
template <class J>
__device__ __forceinline__ void g1w_put36(uint32_t* lds, uint32_t l, const J& x) {
  static_assert(sizeof(J) == 144, "36 words");
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&x);
#pragma unroll
  for (int w = 0; w < 36; ++w) lds[w * 64 + l] = src[w];
}
template <class J>
__device__ __forceinline__ void g1w_get36(J& x, const uint32_t* lds, uint32_t l) {
  static_assert(sizeof(J) == 144, "36 words");
  uint32_t* dst = reinterpret_cast<uint32_t*>(&x);
#pragma unroll
  for (int w = 0; w < 36; ++w) dst[w] = lds[w * 64 + l];
}

// The tile's G2 tree (rlc_reduce's merges: A = A_l + A_r, B = 2 (B_l + B_r) + A_r) on ONE wave of
// 32 lane pairs: pair j owns node m = 2 j.  A and B both in LDS (B at w * 64 + lane: the right
// node's B is the one of pair j + s / 2, i.e. lane + s), so at most two points are live beside the
// product's fixed registers (B in registers left a 848 B/lane frame).
__device__ __forceinline__ void rlc_reduce_g2p(uint32_t* lds, uint32_t* ldsB, uint32_t lane, G2J* outA, G2J* outB) {
  const uint32_t j = lane >> 1, m = 2 * j;
  {  // level 1: the leaves' B are infinity, so B = A_r
    G2Jp a, ar;
    g2p_lds_get(ar, lds, m + 1);
    g1w_put36(ldsB, lane, ar);
    g2p_lds_get(a, lds, m);
    jac_add_lean(a, ar);
    g2p_lds_put(lds, m, a);
    wave_lds_sync();
  }
#pragma unroll 1
  for (uint32_t s = 2; s < 64; s <<= 1) {
    if ((j & (s - 1)) == 0) {  // active pairs read only inactive pairs' entries besides their own
      G2Jp b, x;
      g1w_get36(b, ldsB, lane);
      g1w_get36(x, ldsB, lane + s);
      jac_add_lean(b, x);
      jac_dbl(b, b);
      g2p_lds_get(x, lds, m + s);  // A_r
      jac_add_lean(b, x);
      g1w_put36(ldsB, lane, b);
      g2p_lds_get(b, lds, m);
      jac_add_lean(b, x);
      g2p_lds_put(lds, m, b);
    }
    wave_lds_sync();
    if (s == 4 && (j & 3u) == 0) {
      G2Jp x;
      g2p_lds_get(x, lds, m);
      g2p_store_jac(outA + (m >> 3), x);
      g1w_get36(x, ldsB, lane);
      g2p_store_jac(outB + (m >> 3), x);
    }
  }
  if (j == 0) {
    G2Jp x;
    g2p_lds_get(x, lds, 0);
    g2p_store_jac(outA + 8, x);
    g1w_get36(x, ldsB, lane);
    g2p_store_jac(outB + 8, x);
  }
}

// The tile's G1 tree, one lane per item on ONE wave (rlc_reduce1 without workgroup barriers).
__device__ __forceinline__ void rlc_reduce_g1w(uint32_t* lds, uint32_t lane, G1J* outA, G1J* outB) {
  G1J b;
  jac_set_inf(b);
  for (uint32_t s = 1; s < 64; s <<= 1) {
    const bool active = (lane & (2 * s - 1)) == 0;
    {
      G1J br;
      shfl_words(br, b, lane + s);
      if (active) jac_add(b, b, br);
    }
    if (active) {
      G1J ar, a;
      g1_lds_get(ar, lds, lane + s);
      jac_dbl(b, b);
      jac_add(b, b, ar);
      g1_lds_get(a, lds, lane);
      jac_add(a, a, ar);
      g1_lds_put(lds, lane, a);
    }
    wave_lds_sync();
    if (s == 4 && (lane & 7u) == 0) {
      G1J a;
      g1_lds_get(a, lds, lane);
      outA[lane >> 3] = a;
      outB[lane >> 3] = b;
    }
  }
  if (lane == 0) {
    G1J a;
    g1_lds_get(a, lds, 0);
    outA[8] = a;
    outB[8] = b;
  }
}

#if HBTC_SIG_PAIR
// k_sig_items in lane-pair form: one workgroup of two waves per 64-share tile, share i on lanes
// (2i, 2i + 1).  r_i sigma_i by the x-adic two-addition loop in pair arithmetic (table in
// registers: 72 per lane), r_i pk_i split over the pair (rlc_pk_mul_x_pair), then the two trees
// side by side: the G2 tree on wave 0 (pair form), the G1 tree on wave 1 (one lane per share).
__global__ void __launch_bounds__(128, HBTC_SIGP_WAVES) k_sig_items_pair(
    const Tile* __restrict__ tiles, const uint32_t* __restrict__ idx,
    const uint8_t* __restrict__ sigs, const G1A* __restrict__ pk,
    const int32_t* __restrict__ pk_status, const PtXY* __restrict__ pk_tab, uint32_t n_pk,
    RlcKey key, Suspects sus, SigTileSums* __restrict__ sums, G2A* __restrict__ dec,
    int32_t* __restrict__ status) {
#ifndef HBTC_SIGP_TAB_LDS
#define HBTC_SIGP_TAB_LDS 1  // the x-adic table's three points in LDS (72 words per lane)
#endif
  // the table ([entry][word][lane], 36 KB) while the scalars run, then the two trees' arrays
  // (G2 A 18 KB, G1 A 9 KB, G2 B 9 KB)
  __shared__ uint32_t lds[72 * 128];
  uint32_t* lds2 = lds;
  uint32_t* lds1 = lds + 36 * 128;
  uint32_t* ldsB = lds + 36 * 128 + 36 * 64;  // the G2 tree's B: 36 words x 64 lanes of wave 0
  const Tile tile = tiles[blockIdx.x];
  const uint32_t m = threadIdx.x >> 1;  // the share's position in the tile
  const bool even = (threadIdx.x & 1u) == 0;
  const size_t item = (size_t)tile.first + m;
  G2Jp S;
  G1J P;
  jac_set_inf(S);
  jac_set_inf(P);
  bool leaf = false;
  if (m < tile.count) {
    int32_t st = HBTC_RLC_PENDING;
    const uint32_t id = idx[item];
    if (id >= n_pk) {
      st = HBTC_UNKNOWN_SENDER;
    } else if (pk_status[id] != HBTC_ACCEPT) {
      st = HBTC_DECODE_ERR;
    } else if (status[item] == HBTC_DECODE_ERR) {  // k_sig_decode ran first
      st = HBTC_DECODE_ERR;
    } else if (is_suspect(sus, id)) {
      st = HBTC_RLC_LEAF;  // straight to an exact check, outside the group sums
    } else {
      const XDigits xd = rlc_digits(key, item);
      G2Ap sg;
      g2p_load_aff(sg, dec + item);
      if (!sg.inf) {
        // [x] sigma = psi(sigma), m = -psi^2 = (zeta x, y)
        G2Ap xp, pxp;
        g2p_psi(xp.x, xp.y, sg);
        xp.inf = 0;
        G2Jp xj;
        jac_from_aff(xj, xp);
        xadic_table(xp, pxp, sg, xj);
        Fq zeta;
        fq_set(zeta, G2_ZETA);
#if HBTC_SIGP_TAB_LDS
        xy_lds_put_aff<Fq2p, 128>(lds, threadIdx.x, 0, sg);
        xy_lds_put_aff<Fq2p, 128>(lds, threadIdx.x, 1, xp);
        xy_lds_put_aff<Fq2p, 128>(lds, threadIdx.x, 2, pxp);
        xadic_mul_uniform_lds<Fq2p, 128>(S, lds, threadIdx.x, zeta, xd.d[0], xd.d[1], xd.d[2], xd.d[3],
                                         xd.nbits);
#else
        xadic_mul_uniform(S, sg, xp, pxp, zeta, xd.d[0], xd.d[1], xd.d[2], xd.d[3], xd.nbits);
#endif
      }
      if (!pk[id].inf) rlc_pk_mul_x_pair(P, pk_tab + (size_t)id * PK_TAB_WIN * 256, xd);
    }
    if (even) status[item] = st;
    leaf = even && st == HBTC_RLC_LEAF;
  }
  rlc_list_leaf(sus, leaf, (uint32_t)item, tile.inst, threadIdx.x & 63u);
#if HBTC_SIGP_TAB_LDS
  __syncthreads();  // every lane's table reads are over before the trees' arrays are written
#endif
  g2p_lds_put(lds2, m, S);
  if (even) g1_lds_put(lds1, m, P);
  __syncthreads();
  SigTileSums* ts = sums + blockIdx.x;
  if (threadIdx.x < 64)
    rlc_reduce_g2p(lds2, ldsB, threadIdx.x, ts->S, ts->SW);
  else
    rlc_reduce_g1w(lds1, threadIdx.x - 64, ts->P, ts->PW);
}
#endif

// The G2 half of the pair-batch item pass (hbtc_pb.hip: PublicKey::verify's sigma /
// Ciphertext::verify's w, DESIGN.md §4 "Pair batches") in lane-pair form: item i of the chunk on
// lanes (2i, 2i + 1) of its tile's workgroup, r_i W_i by the same x-adic loop as
// k_sig_items_pair (r_i from the same key and index as k_pb_items' G1 half), then the tile's G2
// tree on wave 0.  The pair batches use the plain sums S only (the weighted SW are written
// too, unused).  k_pb_items decoded W_i (wdec) and set the status: PENDING items count.
__global__ void __launch_bounds__(128, HBTC_SIGP_WAVES) k_pb_wsum_pair(
    uint32_t n, RlcKey key, const G2A* __restrict__ wdec, const int32_t* __restrict__ status,
    SigTileSums* __restrict__ sums) {
  __shared__ uint32_t lds[72 * 128];
  uint32_t* ldsB = lds + 36 * 128 + 36 * 64;
  const uint32_t m = threadIdx.x >> 1;
  const uint32_t i = blockIdx.x * 64u + m;
  G2Jp S;
  jac_set_inf(S);
  if (i < n && status[i] == HBTC_RLC_PENDING) {  // pair-uniform
    G2Ap W;
    g2p_load_aff(W, wdec + i);
    if (!W.inf) {  // r W, m = -psi^2: (x, y) -> (zeta x, y)
      const XDigits xd = rlc_digits(key, i);
      G2Ap xp, pxp;
      g2p_psi(xp.x, xp.y, W);
      xp.inf = 0;
      G2Jp xj;
      jac_from_aff(xj, xp);
      xadic_table(xp, pxp, W, xj);
      Fq zeta;
      fq_set(zeta, G2_ZETA);
      xy_lds_put_aff<Fq2p, 128>(lds, threadIdx.x, 0, W);
      xy_lds_put_aff<Fq2p, 128>(lds, threadIdx.x, 1, xp);
      xy_lds_put_aff<Fq2p, 128>(lds, threadIdx.x, 2, pxp);
      xadic_mul_uniform_lds<Fq2p, 128>(S, lds, threadIdx.x, zeta, xd.d[0], xd.d[1], xd.d[2], xd.d[3],
                                       xd.nbits);
    }
  }
  __syncthreads();  // every lane's table reads are over before the tree's arrays are written
  g2p_lds_put(lds, m, S);
  __syncthreads();
  if (threadIdx.x < 64) {
    SigTileSums* ts = sums + blockIdx.x;
    rlc_reduce_g2p(lds, ldsB, threadIdx.x, ts->S, ts->SW);
  }
}
hipError_t launch_pb_wsum(hipStream_t s, uint32_t n, RlcKey key, const G2A* wdec, const int32_t* status,
                          SigTileSums* sums) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pb_wsum_pair, dim3((n + 63) / 64), dim3(128), 0, s, n, key, wdec, status, sums);
  return hipGetLastError();
}

#if HBTC_SIG_PAIR
// The exact small-call path in ONE kernel (round 6): per SignatureShare on a lane pair, the zcash
// decode (square roots, one-lane form on both lanes), the leaf listing (every decodable share of a
// known sender), then its 68 projective Miller lines straight into the leaf's table (pair form,
// g2p_walk_lines), whose double-and-add ends at [|x|] sigma: the psi subgroup test needs no chain
// of its own.  A share failing that test is DECODE_ERR (k_sigchk_leaves skips it).  Replaces
// k_sig_decode (decode + a separate psi chain), k_sig_items (the listing) and k_plines (an
// inversion and the 68 steps on one lane): three dependent launches of c1's chain.
__global__ void __launch_bounds__(64) k_sig_exact(uint32_t n, const uint32_t* __restrict__ idx,
                                                  const uint8_t* __restrict__ sigs,
                                                  const int32_t* __restrict__ pk_status, uint32_t n_pk,
                                                  const Tile* __restrict__ tiles, uint32_t n_tiles,
                                                  uint32_t* __restrict__ leaf_count, uint32_t* __restrict__ leaves,
                                                  G2A* __restrict__ dec, Fq2* __restrict__ tables,
                                                  uint32_t* __restrict__ inf, int32_t* __restrict__ status) {
  HBTC_LATENCY_PRIO();
  const uint32_t item = (blockIdx.x * 64 + threadIdx.x) >> 1;
  const bool even = (threadIdx.x & 1u) == 0;
  const bool in = item < n;
  int32_t st = HBTC_DECODE_ERR;
  bool leaf = false;
  G2A sg;
  sg.inf = 1;
  uint32_t inst = 0;
  if (in) {
    const uint32_t id = idx[item];
    uint32_t lo = 0, hi = n_tiles;  // the last tile starting at or before the item
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (tiles[mid].first <= item) lo = mid; else hi = mid;
    }
    inst = tiles[lo].inst;
    if (id >= n_pk) {
      st = HBTC_UNKNOWN_SENDER;
    } else if (pk_status[id] == HBTC_ACCEPT) {
      uint32_t w[24];
      rlc_load_words(w, sigs, item, 24);
      if (g2_decompress(sg, w, false)) {
        st = HBTC_RLC_LEAF;
        leaf = true;
        if (even) dec[item] = sg;
      }
    }
  }
  // the leaf position: one atomic per wave over the even lanes, then to the odd lane
  const uint64_t m = __ballot(leaf && even);
  uint32_t base = 0;
  if (m && (threadIdx.x & 63u) == 0) base = atomicAdd(leaf_count, (uint32_t)__popcll(m));
  base = __shfl(base, 0);
  const uint32_t mine = base + (uint32_t)__popcll(m & ((1ull << (threadIdx.x & 63u)) - 1ull));
  const uint32_t other = pair_xchg(mine);  // odd lanes hold no bit of m: the even lane's slot
  const uint32_t pos = even ? mine : other;
  if (leaf) {
    if (even) {
      leaves[2 * pos] = item;
      leaves[2 * pos + 1] = inst;
      inf[pos] = sg.inf;
    }
    if (!sg.inf) {
      G2Ap Q;
      g2p_from_full(Q, sg);
      G2Jp T;
      g2p_walk_lines(tables + (size_t)pos * PLINES_FQ2, T, Q);
      if (!g2p_psi_test(T, Q)) st = HBTC_DECODE_ERR;
    }
  }
  if (in && even) status[item] = st;
}
#endif

// Projective line table of one G2 sum: affine (one Fq2 inversion) then the 68 steps.
__device__ __forceinline__ void g2j_plines(Fq2* out, uint32_t* inf, const G2J& S) {
  if (jac_is_inf(S)) {
    *inf = 1;
    return;
  }
  *inf = 0;
  Fq nrm, t, ni;
  fq_sqr(nrm, S.z.c0);
  fq_sqr(t, S.z.c1);
  fq_add(nrm, nrm, t);
  fq_inv_binary(ni, nrm);
  Fq2 zi, zi2, zi3;
  fq_mul(zi.c0, S.z.c0, ni);
  fq_mul(t, S.z.c1, ni);
  fq_neg(zi.c1, t);
  fq2_sqr(zi2, zi);
  fq2_mul(zi3, zi2, zi);
  G2A Q;
  fq2_mul(Q.x, S.x, zi2);
  fq2_mul(Q.y, S.y, zi3);
  Q.inf = 0;
  g2_proj_lines(out, Q);
}

__global__ void __launch_bounds__(64) k_plines(int mode, uint32_t max_groups, uint32_t base,
                                               const uint32_t* __restrict__ count,
                                               const uint32_t* __restrict__ list,
                                               const Tile* __restrict__ tiles,
                                               const SigTileSums* __restrict__ sums,
                                               const G2A* __restrict__ dec,
                                               Fq2* __restrict__ tables,
                                               uint32_t* __restrict__ inf) {
  HBTC_LATENCY_PRIO();
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  // mode 2: leaves [base, base + max_groups) of the list (chunks keep the tables bounded);
  // modes 3 / 4 (pair-batch path, hbtc_pb.hip): the plain sum of every tile / of the 8 sub-tiles
  // of the listed tiles
  const uint32_t c = (mode == 0 || mode == 3) ? 0u : *count;
  const uint32_t n = (mode == 0 || mode == 3) ? max_groups
                   : mode == 1 ? c * 16u
                   : mode == 4 ? c * 8u
                               : (c > base ? min(c - base, max_groups) : 0u);
  if (g >= n) return;
  G2J S;
  if (mode == 3) {
    S = sums[g].S[8];
  } else if (mode == 4) {
    S = sums[list[g >> 3]].S[g & 7u];
  } else if (mode == 0) {
    const uint32_t t = g >> 1;
    S = (g & 1u) ? sums[t].SW[8] : sums[t].S[8];
  } else if (mode == 1) {
    const uint32_t t = list[g >> 4], sub = (g >> 1) & 7u;
    const Tile tile = tiles[t];
    if (sub * 8u >= tile.count)
      jac_set_inf(S);
    else
      S = (g & 1u) ? sums[t].SW[sub] : sums[t].S[sub];
  } else {
    jac_from_aff(S, dec[list[2 * (base + g)]]);
  }
  g2j_plines(tables + (size_t)g * PLINES_FQ2, inf + g, S);
}

#ifndef HBTC_PLINES_PAIR
#define HBTC_PLINES_PAIR HBTC_SIG_PAIR
#endif
#if HBTC_PLINES_PAIR
// k_plines on lane pairs: group g on lanes (2g, 2g + 1); the affine normalisation (one binary-GCD
// inversion of the norm) and the 68 projective steps in pair form (g2p_walk_lines).
#ifndef HBTC_PLINES_WAVES
#define HBTC_PLINES_WAVES 2
#endif
__global__ void __launch_bounds__(64, HBTC_PLINES_WAVES) k_plines_pair(int mode, uint32_t max_groups, uint32_t base,
                                                    const uint32_t* __restrict__ count,
                                                    const uint32_t* __restrict__ list,
                                                    const Tile* __restrict__ tiles,
                                                    const SigTileSums* __restrict__ sums,
                                                    const G2A* __restrict__ dec,
                                                    Fq2* __restrict__ tables,
                                                    uint32_t* __restrict__ inf) {
  HBTC_LATENCY_PRIO();
  const uint32_t g = (blockIdx.x * 64 + threadIdx.x) >> 1;
  const bool even = (threadIdx.x & 1u) == 0;
  const uint32_t c = (mode == 0 || mode == 3) ? 0u : *count;
  const uint32_t n = (mode == 0 || mode == 3) ? max_groups
                   : mode == 1 ? c * 16u
                   : mode == 4 ? c * 8u
                               : (c > base ? min(c - base, max_groups) : 0u);
  if (g >= n) return;  // pair-uniform
  G2Jp S;
  if (mode == 3) {
    g2p_load_jac(S, &sums[g].S[8]);
  } else if (mode == 4) {
    g2p_load_jac(S, &sums[list[g >> 3]].S[g & 7u]);
  } else if (mode == 0) {
    const uint32_t t = g >> 1;
    g2p_load_jac(S, (g & 1u) ? &sums[t].SW[8] : &sums[t].S[8]);
  } else if (mode == 1) {
    const uint32_t t = list[g >> 4], sub = (g >> 1) & 7u;
    const Tile tile = tiles[t];
    if (sub * 8u >= tile.count)
      jac_set_inf(S);
    else
      g2p_load_jac(S, (g & 1u) ? &sums[t].SW[sub] : &sums[t].S[sub]);
  } else {
    G2Ap a;
    g2p_load_aff(a, dec + list[2 * (base + g)]);
    jac_from_aff(S, a);
  }
  if (jac_is_inf(S)) {
    if (even) inf[g] = 1;
    return;
  }
  if (even) inf[g] = 0;
  G2Ap Q;
  {
    Fq2p zi, zi2, zi3;
    finv_fast(zi, S.z);
    fsqr(zi2, zi);
    fmul(zi3, zi2, zi);
    fmul(Q.x, S.x, zi2);
    fmul(Q.y, S.y, zi3);
    Q.inf = 0;
  }
  G2Jp T;
  g2p_walk_lines(tables + (size_t)g * PLINES_FQ2, T, Q);
}
#endif

static inline uint32_t sig_blocks(uint64_t n, uint32_t bs) { return (uint32_t)((n + bs - 1) / bs); }

hipError_t launch_sig_items(hipStream_t s, uint32_t n_tiles, const Tile* tiles, const uint32_t* idx,
                            const uint8_t* sigs, const G1A* pk, const int32_t* pk_status,
                            const PtXY* pk_tab, uint32_t n_pk, RlcKey key, Suspects sus,
                            SigTileSums* sums, G2A* dec, int32_t* status) {
  if (n_tiles == 0) return hipSuccess;
#if HBTC_SIG_SPLIT
#if HBTC_SIGDEC_PAIR
  hipLaunchKernelGGL(k_sig_decode_pair, dim3(n_tiles), dim3(64), 0, s, tiles, idx, sigs, pk_status, n_pk, dec,
                     status);
  const hipError_t e = hipGetLastError();
#else
  const hipError_t e = launch_sig_decode(s, n_tiles, tiles, idx, sigs, pk_status, n_pk, dec, status);
#endif
  if (e != hipSuccess) return e;
#endif
#if HBTC_SIG_PAIR && HBTC_SIG_SPLIT
  hipLaunchKernelGGL(k_sig_items_pair, dim3(n_tiles), dim3(128), 0, s, tiles, idx, sigs, pk, pk_status,
                     pk_tab, n_pk, key, sus, sums, dec, status);
#else
  hipLaunchKernelGGL(k_sig_items, dim3(n_tiles), dim3(64), 0, s, tiles, idx, sigs, pk, pk_status,
                     pk_tab, n_pk, key, sus, sums, dec, status);
#endif
  return hipGetLastError();
}

bool sig_exact_built() { return HBTC_SIG_PAIR != 0; }

hipError_t launch_sig_exact(hipStream_t s, uint32_t n, const uint32_t* idx, const uint8_t* sigs,
                            const int32_t* pk_status, uint32_t n_pk, const Tile* tiles, uint32_t n_tiles,
                            uint32_t* leaf_count, uint32_t* leaves, G2A* dec, Fq2* tables, uint32_t* inf,
                            int32_t* status) {
#if HBTC_SIG_PAIR
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sig_exact, dim3(sig_blocks(2 * (uint64_t)n, 64)), dim3(64), 0, s, n, idx, sigs, pk_status,
                     n_pk, tiles, n_tiles, leaf_count, leaves, dec, tables, inf, status);
  return hipGetLastError();
#else
  return hipErrorNotSupported;
#endif
}

hipError_t launch_plines(hipStream_t s, int mode, uint32_t max_groups, uint32_t base,
                         const uint32_t* count, const uint32_t* list, const Tile* tiles,
                         const SigTileSums* sums, const G2A* dec, Fq2* tables, uint32_t* inf) {
  if (max_groups == 0) return hipSuccess;
#if HBTC_PLINES_PAIR
  hipLaunchKernelGGL(k_plines_pair, dim3(sig_blocks(2 * (uint64_t)max_groups, 64)), dim3(64), 0, s, mode,
                     max_groups, base, count, list, tiles, sums, dec, tables, inf);
#else
  hipLaunchKernelGGL(k_plines, dim3(sig_blocks(max_groups, 64)), dim3(64), 0, s, mode, max_groups,
                     base, count, list, tiles, sums, dec, tables, inf);
#endif
  return hipGetLastError();
}
#endif  // part 2

}  // namespace hbtc
