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
// This file holds the per-item pass (k_rlc_items: decode, r_i, the tile and sub-tile sums)
// and the final decision (k_rlc_finalize); the pairing-product checks of those sums run on
// the cooperative GT arithmetic in hbtc_check.hip:
//     k_chk_tiles   (plain, weighted) checks of every 64-share tile; a failing tile with one
//                   wrong share is located right there, the others are listed
//     k_chk_subs    the 8-share sub-tiles of listed tiles, located likewise
//     k_chk_leaves  the exact per-share check for sub-tiles with >= 2 wrong shares
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
    RlcKey key, TileSums* __restrict__ sums, G1A* __restrict__ dec,
    int32_t* __restrict__ status) {
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
        dec[item] = d;  // for the exact leaf checks and the combine (no second decode)
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
                            G1A* dec, int32_t* status) {
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rlc_items, dim3(n_tiles), dim3(64), 0, s, tiles, idx, shares, pk, pk_status,
                     pk_tab, n_pk, key, sums, dec, status);
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

}  // namespace hbtc
