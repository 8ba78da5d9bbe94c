// Random-linear-combination (RLC) batch verification of DecryptionShares with hierarchical
// fallback — the fast path behind hbtc_verify_dec_shares (PublicKeyShare::
// verify_decryption_share, /root/reference/src/threshold_decryption.rs:159, called once per
// share by the reference).
//
// For a group G of shares of ONE ciphertext (u, v, w), H = hash_g1_g2(u, v):
//     every share valid  =>  e(sum_G r_i d_i, H) == e(sum_G r_i pk_i, w)
// and, for r_i drawn uniformly from [0, 2^64) AFTER the shares are fixed (a ChaCha20 stream
// under a fresh 256-bit host key per call), an invalid share makes the equation fail except
// with probability <= 2^-64 per check (all points are in the prime-order subgroup: decode
// checks it).  Decisions therefore equal the per-share decisions of the reference except with
// probability <= 2^-64 per check; every group that fails is split, down to single shares, which
// get the exact per-share check of k_dec_verify.  Levels:
//     ciphertext (all its shares) -> tile (<= 64 shares, one wave) -> sub-tile (8) -> share
// Work per share in the honest case: decode + two 64-bit scalar multiplications in G1
// (r_i d_i, r_i pk_i) + a share of the wave's reduction tree; the pairing work is per group.
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

// e(S, H) * e(-P, w) == 1 for aggregated Jacobian S, P (per-lane instance: vector line loads)
__device__ bool rlc_pair_check(const G1J& S, const G1J& P, const Line* hl, bool h_inf,
                               const Line* wl, bool w_inf) {
  G1A s, p;
  jac_to_aff(s, S);
  jac_to_aff(p, P);
  const bool use1 = !s.inf && !h_inf, use2 = !p.inf && !w_inf;
  if (!use1 && !use2) return true;
  G1A np;
  aff_neg(np, p);
  Fq12 f, e;
  miller_loop_2(f, RlcTableLines{hl}, s, use1, RlcTableLines{wl}, np, use2);
  final_exponentiation(e, f);
  return fq12_is_one(e);
}

#if HBTC_IN_PART(6)
// ------------------------------------------------------------------------------ per item
// One wave per tile: decode every share, draw r_i, compute r_i d_i and r_i pk_i (64-bit
// double-and-add on G1, Jacobian), then reduce across the wave in LDS: 8 sub-tile sums (groups
// of 8 lanes) and the tile sum.  Items that cannot be checked (decode error, unknown sender)
// get their final status here and contribute the identity; a ciphertext whose own H / w failed
// to decode is resolved by k_rlc_finalize.  Needs nothing from the per-ciphertext preparation,
// so it runs concurrently with k_g2_prepare on another stream.
__global__ void __launch_bounds__(64) k_rlc_items(
    const Tile* __restrict__ tiles, const uint32_t* __restrict__ idx,
    const uint8_t* __restrict__ shares, const G1A* __restrict__ pk,
    const int32_t* __restrict__ pk_status, uint32_t n_pk, RlcKey key,
    TileSums* __restrict__ sums, int32_t* __restrict__ status) {
  __shared__ G1J redS[64];
  __shared__ G1J redP[64];
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
        jac_mul_u64(S, d, r);
        jac_mul_u64(P, pk[id], r);
      }
    }
    status[item] = st;
  }
  redS[lane] = S;
  redP[lane] = P;
  __syncthreads();
  // groups of 8 -> sub-tile sums
  for (uint32_t s = 1; s < 8; s <<= 1) {
    if ((lane & (2 * s - 1)) == 0) {
      G1J a = redS[lane], b = redS[lane + s];
      jac_add(a, a, b);
      redS[lane] = a;
      G1J c = redP[lane], d = redP[lane + s];
      jac_add(c, c, d);
      redP[lane] = c;
    }
    __syncthreads();
  }
  TileSums* ts = sums + blockIdx.x;
  if ((lane & 7) == 0) {
    ts->S[lane >> 3] = redS[lane];
    ts->P[lane >> 3] = redP[lane];
  }
  for (uint32_t s = 8; s < 64; s <<= 1) {
    if ((lane & (2 * s - 1)) == 0) {
      G1J a = redS[lane], b = redS[lane + s];
      jac_add(a, a, b);
      redS[lane] = a;
      G1J c = redP[lane], d = redP[lane + s];
      jac_add(c, c, d);
      redP[lane] = c;
    }
    __syncthreads();
  }
  if (lane == 0) {
    ts->S[8] = redS[0];
    ts->P[8] = redP[0];
  }
}
#endif  // part 6

#if HBTC_IN_PART(7)
// ------------------------------------------------------------------------------ group checks
// Lanes [0, n_inst): ciphertext-level checks (sum of the instance's tile sums).
// Lanes [n_inst, n_inst + n_tiles): tile-level checks — run together with the ciphertext level
// (one round of pairing latency instead of two); a tile whose ciphertext passes is resolved
// by the ciphertext verdict in k_rlc_sub.
__global__ void __launch_bounds__(64) k_rlc_check_groups(
    uint32_t n_inst, uint32_t n_tiles, const Tile* __restrict__ tiles,
    const uint32_t* __restrict__ inst_tiles, const TileSums* __restrict__ sums,
    const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    const G2A* __restrict__ w_aff, const Line* __restrict__ w_lines,
    const int32_t* __restrict__ h_status, const int32_t* __restrict__ w_status,
    uint8_t* __restrict__ inst_pass, uint8_t* __restrict__ tile_pass) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (g >= n_inst + n_tiles) return;
  G1J S, P;
  uint32_t k = g < n_inst ? g : tiles[g - n_inst].inst;
  if (h_status[k] != HBTC_ACCEPT || w_status[k] != HBTC_ACCEPT) {
    // undecodable H / w: no group work; k_rlc_finalize marks the items INSTANCE_ERR
    if (g < n_inst)
      inst_pass[g] = 1;
    else
      tile_pass[g - n_inst] = 1;
    return;
  }
  if (g < n_inst) {
    jac_set_inf(S);
    jac_set_inf(P);
    for (uint32_t t = inst_tiles[k]; t < inst_tiles[k + 1]; ++t) {
      jac_add(S, S, sums[t].S[8]);
      jac_add(P, P, sums[t].P[8]);
    }
  } else {
    const uint32_t t = g - n_inst;
    S = sums[t].S[8];
    P = sums[t].P[8];
  }
  const bool ok = rlc_pair_check(S, P, h_lines + (size_t)k * MILLER_STEPS, h_aff[k].inf != 0,
                                 w_lines + (size_t)k * MILLER_STEPS, w_aff[k].inf != 0);
  if (g < n_inst)
    inst_pass[g] = ok;
  else
    tile_pass[g - n_inst] = ok;
}

// One lane per (tile, sub-tile) of tiles whose ciphertext AND tile checks failed: check the
// sub-tile sum; a failing sub-tile appends its pending items to the leaf list.
__global__ void __launch_bounds__(64) k_rlc_sub(
    uint32_t n_tiles, const Tile* __restrict__ tiles, const TileSums* __restrict__ sums,
    const uint8_t* __restrict__ inst_pass, const uint8_t* __restrict__ tile_pass,
    const G2A* __restrict__ h_aff, const Line* __restrict__ h_lines,
    const G2A* __restrict__ w_aff, const Line* __restrict__ w_lines,
    const int32_t* __restrict__ status, uint32_t* __restrict__ leaf_count,
    uint32_t* __restrict__ leaves) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (g >= n_tiles * 8) return;
  const uint32_t t = g >> 3, sub = g & 7;
  const Tile tile = tiles[t];
  if (inst_pass[tile.inst] || tile_pass[t]) return;
  if (sub * 8 >= tile.count) return;
  const uint32_t k = tile.inst;
  const bool ok = rlc_pair_check(sums[t].S[sub], sums[t].P[sub], h_lines + (size_t)k * MILLER_STEPS,
                                 h_aff[k].inf != 0, w_lines + (size_t)k * MILLER_STEPS,
                                 w_aff[k].inf != 0);
  if (ok) return;
  const uint32_t lo = tile.first + sub * 8;
  const uint32_t hi = min(tile.first + tile.count, lo + 8);
  for (uint32_t i = lo; i < hi; ++i)
    if (status[i] == HBTC_RLC_PENDING) {
      const uint32_t pos = atomicAdd(leaf_count, 1u);
      leaves[2 * pos] = i;
      leaves[2 * pos + 1] = k;
    }
}

// Exact per-share check for the compacted leaf list (items of failing sub-tiles): the same
// arithmetic as k_dec_verify, with per-lane instance (vector line loads).
__global__ void __launch_bounds__(64) k_rlc_leaves(
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
                            uint32_t n_pk, RlcKey key, TileSums* sums, int32_t* status) {
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rlc_items, dim3(n_tiles), dim3(64), 0, s, tiles, idx, shares, pk, pk_status,
                     n_pk, key, sums, status);
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
                                   uint8_t* tile_pass) {
  const uint64_t n = (uint64_t)n_inst + n_tiles;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rlc_check_groups, dim3(rlc_blocks(n, 64)), dim3(64), 0, s, n_inst, n_tiles,
                     tiles, inst_tiles, sums, h_aff, h_lines, w_aff, w_lines, h_status, w_status,
                     inst_pass, tile_pass);
  return hipGetLastError();
}
hipError_t launch_rlc_sub(hipStream_t s, uint32_t n_tiles, const Tile* tiles, const TileSums* sums,
                          const uint8_t* inst_pass, const uint8_t* tile_pass, const G2A* h_aff,
                          const Line* h_lines, const G2A* w_aff, const Line* w_lines,
                          const int32_t* status, uint32_t* leaf_count, uint32_t* leaves) {
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rlc_sub, dim3(rlc_blocks((uint64_t)n_tiles * 8, 64)), dim3(64), 0, s, n_tiles,
                     tiles, sums, inst_pass, tile_pass, h_aff, h_lines, w_aff, w_lines, status,
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
