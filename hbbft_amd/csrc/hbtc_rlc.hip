// Random-linear-combination (RLC) batch verification of DecryptionShares with hierarchical
// fallback and single-error location — the fast path behind hbtc_verify_dec_shares
// (PublicKeyShare::verify_decryption_share, /root/reference/src/threshold_decryption.rs:159,
// called once per share by the reference).
//
// For a group G of shares of ONE ciphertext (u, v, w), H = hash_g1_g2(u, v), and
// E_i = e(d_i, H) / e(pk_i, w) (E_i == 1 iff share i is valid):
//     every share valid  =>  e(sum_G r_i d_i, H) * e(-sum_G r_i pk_i, w) == prod E_i^r_i == 1
// and, for r_i drawn uniformly from a set of 2^64 scalars AFTER the shares are fixed (a ChaCha20
// stream under a fresh 256-bit host key per call), an invalid share makes the equation fail
// except with probability <= 2^-64 per check (every point is in the prime-order subgroup: decode
// checks it, so E_i has order 1 or r).
//
// Single-error location.  Next to the plain sum the item pass also forms the position-weighted
// sum (weights = the share's position p_i inside its group), so each group yields
//     T = prod E_i^r_i      and      T_w = prod E_i^(p_i r_i).
// If exactly one share b is wrong, T_w == T^(p_b): the search over p = 0..|G|-1 finds it with
// |G|-1 GT multiplications instead of per-share pairings, and the rest of the group is valid.
// With two or more wrong shares, T_w == T^p holds for some p only if prod_i E_i^(r_i (p_i - p))
// == 1 with a nonzero exponent on a wrong share, i.e. with probability <= 2^-64 per p (the same
// argument as the plain check), <= |G| 2^-64 <= 2^-58 per located group; such groups are split.
//
// Levels:
//     k_rlc_check_groups  ciphertext checks + (plain, weighted) checks of every 64-share tile;
//                         a failing tile with one wrong share is located right there
//     k_rlc_triage        failing, unlocated tiles -> compact list
//     k_rlc_sub           (plain, weighted) checks of their 8-share sub-tiles, located likewise
//     k_rlc_leaves        the exact per-share check for sub-tiles with >= 2 wrong shares
// Work per share in the honest case: decode + r_i d_i (a joint 32-bit double-and-add through
// the GLV endomorphism) + r_i pk_i (8 mixed additions from the key set's fixed-base table) + a
// share of the wave's reduction tree; the pairing work is per group.
#include "hbtc_kernels.h"

#ifndef HBTC_PART
#define HBTC_PART 0
#endif
#define HBTC_IN_PART(n) (HBTC_PART == 0 || HBTC_PART == (n))

namespace hbtc {

__device__ __forceinline__ void rlc_load_words(uint32_t* w, const uint8_t* base, size_t item,
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

// ChaCha20 block (RFC 8439 layout: constants, 8 key words, counter, 3 nonce words) -> the
// two 32-bit words [2j, 2j+1] of block `ctr`, combined into the 64-bit scalar r_i.
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }
__device__ uint64_t rlc_scalar(const RlcKey& key, uint64_t item) {
  uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                     key.k[0], key.k[1], key.k[2], key.k[3], key.k[4], key.k[5], key.k[6], key.k[7],
                     (uint32_t)(item >> 3), (uint32_t)(item >> 35), 0x68626266u, 0x72726c63u};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = st[i];
#define QR(a, b, c, d)                 \
  x[a] += x[b];                        \
  x[d] = rotl32(x[d] ^ x[a], 16);      \
  x[c] += x[d];                        \
  x[b] = rotl32(x[b] ^ x[c], 12);      \
  x[a] += x[b];                        \
  x[d] = rotl32(x[d] ^ x[a], 8);       \
  x[c] += x[d];                        \
  x[b] = rotl32(x[b] ^ x[c], 7);
#pragma unroll 1
  for (int r = 0; r < 10; ++r) {
    QR(0, 4, 8, 12) QR(1, 5, 9, 13) QR(2, 6, 10, 14) QR(3, 7, 11, 15)
    QR(0, 5, 10, 15) QR(1, 6, 11, 12) QR(2, 7, 8, 13) QR(3, 4, 9, 14)
  }
#undef QR
  const int j = (int)(item & 7);
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i == j) {
      lo = x[2 * i] + st[2 * i];
      hi = x[2 * i + 1] + st[2 * i + 1];
    }
  return ((uint64_t)hi << 32) | lo;
}

struct RlcTableLines {
  const Line* l;
  __device__ __forceinline__ void load(Line& out, int j) const { out = l[j]; }
};

#ifndef HBTC_CHECK_WAVES
#define HBTC_CHECK_WAVES 1  // minimum waves per SIMD for the pairing-check kernels
#endif

#if HBTC_IN_PART(7)
// T = e(S, H) * e(-P, w) for aggregated Jacobian S, P (per-lane instance: vector line loads);
// returns T == 1.
__device__ bool rlc_pair_value(Fq12& e, const G1J& S, const G1J& P, const Line* hl, bool h_inf,
                               const Line* wl, bool w_inf) {
  G1A s, p;
  jac_to_aff(s, S);
  jac_to_aff(p, P);
  const bool use1 = !s.inf && !h_inf, use2 = !p.inf && !w_inf;
  if (!use1 && !use2) {
    fq12_one(e);
    return true;
  }
  G1A np;
  aff_neg(np, p);
  Fq12 f;
  miller_loop_2(f, RlcTableLines{hl}, s, use1, RlcTableLines{wl}, np, use2);
  final_exponentiation(e, f);
  return fq12_is_one(e);
}

// Exchange a GT value with the partner lane (lane ^ 1) of the wave.
__device__ __forceinline__ void fq_shfl_xor1(Fq& r, const Fq& a) {
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = (uint32_t)__shfl_xor((int)a.v[i], 1);
}
__device__ __forceinline__ void fq12_shfl_xor1(Fq12& r, const Fq12& a) {
  fq_shfl_xor1(r.c0.c0.c0, a.c0.c0.c0);
  fq_shfl_xor1(r.c0.c0.c1, a.c0.c0.c1);
  fq_shfl_xor1(r.c0.c1.c0, a.c0.c1.c0);
  fq_shfl_xor1(r.c0.c1.c1, a.c0.c1.c1);
  fq_shfl_xor1(r.c0.c2.c0, a.c0.c2.c0);
  fq_shfl_xor1(r.c0.c2.c1, a.c0.c2.c1);
  fq_shfl_xor1(r.c1.c0.c0, a.c1.c0.c0);
  fq_shfl_xor1(r.c1.c0.c1, a.c1.c0.c1);
  fq_shfl_xor1(r.c1.c1.c0, a.c1.c1.c0);
  fq_shfl_xor1(r.c1.c1.c1, a.c1.c1.c1);
  fq_shfl_xor1(r.c1.c2.c0, a.c1.c2.c0);
  fq_shfl_xor1(r.c1.c2.c1, a.c1.c2.c1);
}

// Smallest p < count with Tw == T^p, or -1 (T != 1: the group failed).
__device__ __attribute__((noinline)) int32_t rlc_locate(const Fq12& T, const Fq12& Tw,
                                                        uint32_t count) {
  Fq12 acc;
  fq12_one(acc);
  for (uint32_t p = 0; p < count; ++p) {
    if (fq12_eq(acc, Tw)) return (int32_t)p;
    fq12_mul(acc, acc, T);
  }
  return -1;
}
#endif  // part 7

#if HBTC_IN_PART(6)
// ------------------------------------------------------------------------------ per item
// Tree reduction of the per-lane points q over the wave (lane = position in the tile): the sum
// A and the position-weighted sum B of every aligned group of 8 (-> outA/outB[0..7]) and of the
// tile (-> [8]).  Merging halves of size s:  A = A_l + A_r,  B = B_l + B_r + s A_r.
__device__ void rlc_reduce(G1J* redA, G1J* redB, const G1J& q, uint32_t lane, G1J* outA,
                           G1J* outB) {
  G1J z;
  jac_set_inf(z);
  redA[lane] = q;
  redB[lane] = z;
  __syncthreads();
  for (uint32_t s = 1; s < 64; s <<= 1) {
    if ((lane & (2 * s - 1)) == 0) {
      G1J a = redA[lane], ar = redA[lane + s];
      G1J b = redB[lane], br = redB[lane + s];
      jac_add(b, b, br);
      G1J sa = ar;
      for (uint32_t d = 1; d < s; d <<= 1) jac_dbl(sa, sa);
      jac_add(b, b, sa);
      jac_add(a, a, ar);
      redA[lane] = a;
      redB[lane] = b;
    }
    __syncthreads();
    if (s == 4 && (lane & 7) == 0) {
      outA[lane >> 3] = redA[lane];
      outB[lane >> 3] = redB[lane];
    }
  }
  if (lane == 0) {
    outA[8] = redA[0];
    outB[8] = redB[0];
  }
  __syncthreads();  // the arrays are reused by the next reduction
}

// [a] pk + [b] phi(pk) from the key set's fixed-base table (8 mixed additions, no doublings).
__device__ void rlc_pk_mul(G1J& r, const PtXY* __restrict__ tab, uint32_t a, uint32_t b) {
  jac_set_inf(r);
#pragma unroll
  for (int w = 0; w < PK_TAB_WIN; ++w) {
    const uint32_t va = (a >> (8 * w)) & 0xffu, vb = (b >> (8 * w)) & 0xffu;
    if (va) {
      const PtXY e = tab[w * 256 + va];
      G1A q;
      q.x = e.x;
      q.y = e.y;
      q.inf = 0;
      jac_add_aff(r, r, q);
    }
    if (vb) {
      const PtXY e = tab[w * 256 + vb];
      G1A q, pq;
      q.x = e.x;
      q.y = e.y;
      q.inf = 0;
      g1_phi(pq, q);
      jac_add_aff(r, r, pq);
    }
  }
}

// One wave per tile: decode every share, draw r_i = a_i + b_i mu (a_i, b_i the two 32-bit
// halves of a ChaCha20 word, mu the eigenvalue of the GLV endomorphism phi: 2^64 distinct
// residues mod r), compute r_i d_i = [a] d + [b] phi(d) (joint 32-bit
// double-and-add) and r_i pk_i from the fixed-base table, then the plain and weighted group
// sums.  Items that cannot be checked (decode error, unknown sender) get their final status
// here and contribute the identity; a ciphertext whose own H / w failed to decode is resolved
// by k_rlc_finalize.  Needs nothing from the per-ciphertext preparation, so it runs
// concurrently with k_g2_prepare on another stream.
#ifndef HBTC_ITEMS_WAVES
#define HBTC_ITEMS_WAVES 2  // minimum waves per SIMD the register allocation must allow (1: 153 ms, 2: 86 ms, 3: 161 ms per C3 launch)
#endif
__global__ void __launch_bounds__(64, HBTC_ITEMS_WAVES) k_rlc_items(
    const Tile* __restrict__ tiles, const uint32_t* __restrict__ idx,
    const uint8_t* __restrict__ shares, const G1A* __restrict__ pk,
    const int32_t* __restrict__ pk_status, const PtXY* __restrict__ pk_tab, uint32_t n_pk,
    RlcKey key, TileSums* __restrict__ sums, int32_t* __restrict__ status) {
  __shared__ G1J redA[64];
  __shared__ G1J redB[64];
  const Tile tile = tiles[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  const size_t item = (size_t)tile.first + lane;
  G1J S, P;
  jac_set_inf(S);
  jac_set_inf(P);
  if (lane < tile.count) {
    int32_t st = HBTC_RLC_PENDING;
    const uint32_t id = idx[item];
    if (id >= n_pk) {
      st = HBTC_UNKNOWN_SENDER;
    } else if (pk_status[id] != HBTC_ACCEPT) {
      st = HBTC_DECODE_ERR;
    } else {
      uint32_t w[12];
      rlc_load_words(w, shares, item, 12);
      G1A d;
      if (!g1_decompress(d, w)) {
        st = HBTC_DECODE_ERR;
      } else {
        const uint64_t r = rlc_scalar(key, item);
        const uint32_t ra = (uint32_t)r, rb = (uint32_t)(r >> 32);
        G1A pd;
        g1_phi(pd, d);
        jac_mul2_u32(S, d, ra, pd, rb);
        if (!pk[id].inf) rlc_pk_mul(P, pk_tab + (size_t)id * PK_TAB_WIN * 256, ra, rb);
      }
    }
    status[item] = st;
  }
  TileSums* ts = sums + blockIdx.x;
  rlc_reduce(redA, redB, S, lane, ts->S, ts->SW);
  rlc_reduce(redA, redB, P, lane, ts->P, ts->PW);
}
#endif  // part 6

#if HBTC_IN_PART(7)
// ------------------------------------------------------------------------------ group checks
// Lanes [0, 2 n_tiles): tile g/2, plain (g even) and weighted (g odd) sums — partners in one
// wave.  Lanes [2 n_tiles, 2 n_tiles + n_inst): ciphertext-level checks (sum of the tile sums).
// All run in one launch (one round of pairing latency); a tile whose ciphertext passes is
// resolved by the ciphertext verdict in k_rlc_triage.
__global__ void __launch_bounds__(64, HBTC_CHECK_WAVES) k_rlc_check_groups(
    uint32_t n_inst, uint32_t n_tiles, const Tile* __restrict__ tiles,
    const uint32_t* __restrict__ inst_tiles, const TileSums* __restrict__ sums,
    const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    const G2A* __restrict__ w_aff, const Line* __restrict__ w_lines,
    const int32_t* __restrict__ h_status, const int32_t* __restrict__ w_status,
    uint8_t* __restrict__ inst_pass, uint8_t* __restrict__ tile_pass,
    int32_t* __restrict__ tile_loc) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  const uint32_t n_tl = 2 * n_tiles;
  const bool active = g < n_tl + n_inst;
  const bool is_tile = g < n_tl;
  const bool weighted = (g & 1u) != 0;
  const uint32_t t = g >> 1;
  uint32_t k = 0, count = 0;
  bool inst_ok = false;
  G1J S, P;
  jac_set_inf(S);
  jac_set_inf(P);
  if (active) {
    if (is_tile) {
      const Tile tile = tiles[t];
      k = tile.inst;
      count = tile.count;
    } else {
      k = g - n_tl;
    }
    inst_ok = h_status[k] == HBTC_ACCEPT && w_status[k] == HBTC_ACCEPT;
    if (inst_ok) {
      if (is_tile) {
        S = weighted ? sums[t].SW[8] : sums[t].S[8];
        P = weighted ? sums[t].PW[8] : sums[t].P[8];
      } else {
        for (uint32_t u = inst_tiles[k]; u < inst_tiles[k + 1]; ++u) {
          jac_add(S, S, sums[u].S[8]);
          jac_add(P, P, sums[u].P[8]);
        }
      }
    }
  }
  Fq12 e;
  bool ok = true;
  if (active && inst_ok)
    ok = rlc_pair_value(e, S, P, h_lines + (size_t)k * MILLER_STEPS, h_aff[k].inf != 0,
                        w_lines + (size_t)k * MILLER_STEPS, w_aff[k].inf != 0);
  else
    fq12_one(e);
  Fq12 ew;
  fq12_shfl_xor1(ew, e);  // the plain lane receives its partner's weighted value
  if (!active) return;
  // undecodable H / w: no group work; k_rlc_finalize marks the items INSTANCE_ERR
  if (!is_tile) {
    inst_pass[k] = (ok || !inst_ok) ? 1 : 0;
    return;
  }
  if (weighted) return;
  tile_pass[t] = (ok || !inst_ok) ? 1 : 0;
  tile_loc[t] = (ok || !inst_ok) ? -1 : rlc_locate(e, ew, count);
}

// One lane per tile: a tile whose ciphertext AND tile checks failed either had its single
// wrong share located (REJECT it; the rest of the tile is valid) or goes to the sub-tile list.
__global__ void __launch_bounds__(64) k_rlc_triage(
    uint32_t n_tiles, const Tile* __restrict__ tiles, const uint8_t* __restrict__ inst_pass,
    const uint8_t* __restrict__ tile_pass, const int32_t* __restrict__ tile_loc,
    int32_t* __restrict__ status, uint32_t* __restrict__ sub_count,
    uint32_t* __restrict__ sub_list) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  if (t >= n_tiles) return;
  const Tile tile = tiles[t];
  if (inst_pass[tile.inst] || tile_pass[t]) return;
  const int32_t loc = tile_loc[t];
  if (loc >= 0 && status[tile.first + loc] == HBTC_RLC_PENDING) {
    status[tile.first + loc] = HBTC_REJECT;
    return;
  }
  sub_list[atomicAdd(sub_count, 1u)] = t;
}

// 16 lanes per listed tile: its 8 sub-tiles x (plain, weighted).  A failing sub-tile with one
// wrong share is located; one with more appends its pending items to the leaf list.
__global__ void __launch_bounds__(64, HBTC_CHECK_WAVES) k_rlc_sub(
    const uint32_t* __restrict__ sub_count, const uint32_t* __restrict__ sub_list,
    const Tile* __restrict__ tiles, const TileSums* __restrict__ sums,
    const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    const G2A* __restrict__ w_aff, const Line* __restrict__ w_lines,
    int32_t* __restrict__ status, uint32_t* __restrict__ leaf_count,
    uint32_t* __restrict__ leaves) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  const uint32_t entry = g >> 4, sub = (g >> 1) & 7u;
  const bool weighted = (g & 1u) != 0;
  bool active = entry < *sub_count;
  uint32_t k = 0, lo = 0, hi = 0;
  G1J S, P;
  jac_set_inf(S);
  jac_set_inf(P);
  if (active) {
    const uint32_t t = sub_list[entry];
    const Tile tile = tiles[t];
    k = tile.inst;
    lo = tile.first + sub * 8;
    hi = min(tile.first + tile.count, lo + 8);
    active = lo < hi;
    if (active) {
      S = weighted ? sums[t].SW[sub] : sums[t].S[sub];
      P = weighted ? sums[t].PW[sub] : sums[t].P[sub];
    }
  }
  Fq12 e;
  bool ok = true;
  if (active)
    ok = rlc_pair_value(e, S, P, h_lines + (size_t)k * MILLER_STEPS, h_aff[k].inf != 0,
                        w_lines + (size_t)k * MILLER_STEPS, w_aff[k].inf != 0);
  else
    fq12_one(e);
  Fq12 ew;
  fq12_shfl_xor1(ew, e);
  if (!active || weighted || ok) return;
  const int32_t loc = rlc_locate(e, ew, hi - lo);
  if (loc >= 0 && status[lo + loc] == HBTC_RLC_PENDING) {
    status[lo + loc] = HBTC_REJECT;
    return;
  }
  for (uint32_t i = lo; i < hi; ++i)
    if (status[i] == HBTC_RLC_PENDING) {
      const uint32_t pos = atomicAdd(leaf_count, 1u);
      leaves[2 * pos] = i;
      leaves[2 * pos + 1] = k;
    }
}

// Exact per-share check for the compacted leaf list (items of sub-tiles with >= 2 wrong
// shares): the same arithmetic as k_dec_verify, with per-lane instance (vector line loads).
__global__ void __launch_bounds__(64, HBTC_CHECK_WAVES) k_rlc_leaves(
    const uint32_t* __restrict__ leaf_count, const uint32_t* __restrict__ leaves,
    const uint32_t* __restrict__ idx, const uint8_t* __restrict__ shares,
    const G1A* __restrict__ pk, const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    const G2A* __restrict__ w_aff, const Line* __restrict__ w_lines,
    int32_t* __restrict__ status) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (g >= *leaf_count) return;
  const uint32_t item = leaves[2 * g], k = leaves[2 * g + 1];
  uint32_t w[12];
  rlc_load_words(w, shares, item, 12);
  G1A s;
  g1_decompress(s, w);  // decoded fine in k_rlc_items
  G1A npk;
  aff_neg(npk, pk[idx[item]]);
  const bool h_inf = h_aff[k].inf != 0, w_inf = w_aff[k].inf != 0;
  Fq12 f, e;
  miller_loop_2(f, RlcTableLines{h_lines + (size_t)k * MILLER_STEPS}, s, !s.inf && !h_inf,
                RlcTableLines{w_lines + (size_t)k * MILLER_STEPS}, npk, !npk.inf && !w_inf);
  final_exponentiation(e, f);
  status[item] = fq12_is_one(e) ? HBTC_ACCEPT : HBTC_REJECT;
}
#endif  // part 7

#if HBTC_IN_PART(6)
// Every item still pending passed some group check: ACCEPT.  Items of a ciphertext whose own
// H / w failed to decode: INSTANCE_ERR.
__global__ void __launch_bounds__(64) k_rlc_finalize(const Tile* __restrict__ tiles,
                                                     const int32_t* __restrict__ h_status,
                                                     const int32_t* __restrict__ w_status,
                                                     int32_t* __restrict__ status) {
  const Tile tile = tiles[blockIdx.x];
  if (threadIdx.x >= tile.count) return;
  const uint32_t i = tile.first + threadIdx.x;
  if (h_status[tile.inst] != HBTC_ACCEPT || w_status[tile.inst] != HBTC_ACCEPT)
    status[i] = HBTC_INSTANCE_ERR;
  else if (status[i] == HBTC_RLC_PENDING)
    status[i] = HBTC_ACCEPT;
}
#endif  // part 6

// ------------------------------------------------------------------------------ launchers
static inline uint32_t rlc_blocks(uint64_t n, uint32_t bs) { return (uint32_t)((n + bs - 1) / bs); }

#if HBTC_IN_PART(6)
hipError_t launch_rlc_items(hipStream_t s, uint32_t n_tiles, const Tile* tiles, const uint32_t* idx,
                            const uint8_t* shares, const G1A* pk, const int32_t* pk_status,
                            const PtXY* pk_tab, uint32_t n_pk, RlcKey key, TileSums* sums,
                            int32_t* status) {
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rlc_items, dim3(n_tiles), dim3(64), 0, s, tiles, idx, shares, pk, pk_status,
                     pk_tab, n_pk, key, sums, status);
  return hipGetLastError();
}
hipError_t launch_rlc_finalize(hipStream_t s, uint32_t n_tiles, const Tile* tiles,
                               const int32_t* h_status, const int32_t* w_status, int32_t* status) {
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rlc_finalize, dim3(n_tiles), dim3(64), 0, s, tiles, h_status, w_status,
                     status);
  return hipGetLastError();
}
#endif  // part 6

#if HBTC_IN_PART(7)
hipError_t launch_rlc_check_groups(hipStream_t s, uint32_t n_inst, uint32_t n_tiles,
                                   const Tile* tiles, const uint32_t* inst_tiles,
                                   const TileSums* sums, const G2A* h_aff, const Line* h_lines,
                                   const G2A* w_aff, const Line* w_lines, const int32_t* h_status,
                                   const int32_t* w_status, uint8_t* inst_pass,
                                   uint8_t* tile_pass, int32_t* tile_loc) {
  const uint64_t n = 2 * (uint64_t)n_tiles + n_inst;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rlc_check_groups, dim3(rlc_blocks(n, 64)), dim3(64), 0, s, n_inst, n_tiles,
                     tiles, inst_tiles, sums, h_aff, h_lines, w_aff, w_lines, h_status, w_status,
                     inst_pass, tile_pass, tile_loc);
  return hipGetLastError();
}
hipError_t launch_rlc_triage(hipStream_t s, uint32_t n_tiles, const Tile* tiles,
                             const uint8_t* inst_pass, const uint8_t* tile_pass,
                             const int32_t* tile_loc, int32_t* status, uint32_t* sub_count,
                             uint32_t* sub_list) {
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rlc_triage, dim3(rlc_blocks(n_tiles, 64)), dim3(64), 0, s, n_tiles, tiles,
                     inst_pass, tile_pass, tile_loc, status, sub_count, sub_list);
  return hipGetLastError();
}
hipError_t launch_rlc_sub(hipStream_t s, uint32_t max_tiles, const uint32_t* sub_count,
                          const uint32_t* sub_list, const Tile* tiles, const TileSums* sums,
                          const G2A* h_aff, const Line* h_lines, const G2A* w_aff,
                          const Line* w_lines, int32_t* status, uint32_t* leaf_count,
                          uint32_t* leaves) {
  if (max_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rlc_sub, dim3(rlc_blocks((uint64_t)max_tiles * 16, 64)), dim3(64), 0, s,
                     sub_count, sub_list, tiles, sums, h_aff, h_lines, w_aff, w_lines, status,
                     leaf_count, leaves);
  return hipGetLastError();
}
hipError_t launch_rlc_leaves(hipStream_t s, uint32_t max_leaves, const uint32_t* leaf_count,
                             const uint32_t* leaves, const uint32_t* idx, const uint8_t* shares,
                             const G1A* pk, const G2A* h_aff, const Line* h_lines,
                             const G2A* w_aff, const Line* w_lines, int32_t* status) {
  if (max_leaves == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rlc_leaves, dim3(rlc_blocks(max_leaves, 64)), dim3(64), 0, s, leaf_count,
                     leaves, idx, shares, pk, h_aff, h_lines, w_aff, w_lines, status);
  return hipGetLastError();
}
#endif  // part 7

}  // namespace hbtc
