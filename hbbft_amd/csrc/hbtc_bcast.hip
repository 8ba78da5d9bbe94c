// Reliable Broadcast coding path of hbbft (/root/reference/src/broadcast/) on gfx950: the
// Reed-Solomon erasure code over GF(2^8) and the SHA3-256 Merkle trees / proofs every node
// builds and checks for every proposer's value.
//
//   k_gf_apply        out_row[r] = sum_j M[r][j] * in_row[j] for a batch of instances: the
//                     parity rows of ReedSolomon::encode (broadcast.rs:183-185, :433-441) and the
//                     missing rows of ReedSolomon::reconstruct_shards (:444-458)
//   k_merkle_tree     MerkleTree::from_vec (merkle.rs:19-32): every level of one instance's
//                     tree per workgroup
//   k_merkle_validate Proof::validate (merkle.rs:82-102): one proof per lane pair, the N^2 Echo
//                     proofs of an epoch (broadcast.rs:255 validate_proof)
//
// Byte work, HBM / latency bound, no pairings.  GF(2^8) products by a constant use the nibble
// method: c*x = T_lo[x & 15] ^ T_hi[x >> 4] with two 16-entry tables per coefficient, looked up
// four bytes at a time with v_perm_b32 (the byte permute: 8 table bytes per instruction, the
// high half of each table selected by bit 3 of the nibble with v_bfi_b32).  The tables of a
// plan (one per matrix coefficient: 8 dwords) are built on the host with the matrices
// (reed-solomon-erasure 3.1's build_matrix and inverse, see hbtc_api.hip) and read with
// wave-uniform loads.
#include "hbtc_kernels.h"

namespace hbtc {
namespace {

// ------------------------------------------------------------------ Keccak-f[1600], SHA3-256
// Bit-interleaved over a lane PAIR: lane e (= lane & 1) of the pair holds the bits of parity e of
// each of the 25 64-bit lanes as one 32-bit word (e = 0: bits 0, 2, .., 62; e = 1: bits 1, .., 63).
// A 64-bit rotation by 2k is a 32-bit rotation by k of both halves; by 2k + 1 it swaps them:
// E' = rotl(O, k + 1), O' = rotl(E, k), i.e. rotl(partner's half, k + 1 - e) after one DPP
// exchange inside the pair.  Theta, chi and iota are half-local.  Per lane a round is ~115
// 32-bit ops instead of ~290 for the 64-bit lanes of one thread, over twice the lanes: the
// N^2 Echo proofs of an epoch are one wave per SIMD at one proof per lane, and a lone wave
// issues every 4 cycles (MI355X_MICROARCH.md, constants table), so the pair form is ~2.5x
// faster per proof.
constexpr uint64_t KRC64[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

constexpr uint32_t parity_bits(uint64_t v, int e) {
  uint32_t r = 0;
  for (int i = 0; i < 32; ++i) r |= (uint32_t)((v >> (2 * i + e)) & 1u) << i;
  return r;
}
struct KeccakRc2 {
  uint32_t v[2][24];
};
constexpr KeccakRc2 make_rc2() {
  KeccakRc2 r{};
  for (int i = 0; i < 24; ++i)
    for (int e = 0; e < 2; ++e) r.v[e][i] = parity_bits(KRC64[i], e);
  return r;
}
__constant__ KeccakRc2 KRC2 = make_rc2();

// the partner lane's value (quad_perm [1, 0, 3, 2]); both lanes of a pair are always active
__device__ __forceinline__ uint32_t pair_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t rotl32(uint32_t x, uint32_t s) {
  return __builtin_amdgcn_alignbit(x, x, (32u - s) & 31u);
}
__device__ __forceinline__ uint32_t even_bits(uint32_t x) {  // bits 0, 2, .., 30 -> 0 .. 15
  x &= 0x55555555u;
  x = (x | (x >> 1)) & 0x33333333u;
  x = (x | (x >> 2)) & 0x0f0f0f0fu;
  x = (x | (x >> 4)) & 0x00ff00ffu;
  return (x | (x >> 8)) & 0x0000ffffu;
}
__device__ __forceinline__ uint32_t spread_bits(uint32_t x) {  // bits 0 .. 15 -> 0, 2, .., 30
  x &= 0xffffu;
  x = (x | (x << 8)) & 0x00ff00ffu;
  x = (x | (x << 4)) & 0x0f0f0f0fu;
  x = (x | (x << 2)) & 0x33333333u;
  return (x | (x << 1)) & 0x55555555u;
}
// this lane's half of a 64-bit word
__device__ __forceinline__ uint32_t half_of(uint64_t w, uint32_t e) {
  return even_bits((uint32_t)w >> e) | (even_bits((uint32_t)(w >> 32) >> e) << 16);
}
// the 64-bit word of this lane's half and the partner's (both lanes get it)
__device__ __forceinline__ uint64_t word_of(uint32_t h, uint32_t e) {
  const uint32_t q = pair_swap(h);
  const uint32_t ev = e ? q : h, od = e ? h : q;
  const uint32_t lo = spread_bits(ev) | (spread_bits(od) << 1);
  const uint32_t hi = spread_bits(ev >> 16) | (spread_bits(od >> 16) << 1);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void keccak_f2(uint32_t* a, uint32_t e) {
  constexpr int ROT[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                           25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};
#pragma unroll 1
  for (int round = 0; round < 24; ++round) {
    uint32_t c[5], d[5], b[25];
#pragma unroll
    for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
#pragma unroll
    for (int x = 0; x < 5; ++x) d[x] = c[(x + 4) % 5] ^ rotl32(pair_swap(c[(x + 1) % 5]), 1u - e);
    // theta, then rho + pi: b[y, 2x + 3y] = rot(a[x, y] ^ d[x])
#pragma unroll
    for (int x = 0; x < 5; ++x)
#pragma unroll
      for (int y = 0; y < 5; ++y) {
        const uint32_t v = a[x + 5 * y] ^ d[x];
        const int r = ROT[x + 5 * y];
        b[y + 5 * ((2 * x + 3 * y) % 5)] =
            (r & 1) ? rotl32(pair_swap(v), (uint32_t)(r >> 1) + 1u - e) : (r ? rotl32(v, (uint32_t)(r >> 1)) : v);
      }
#pragma unroll
    for (int y = 0; y < 25; y += 5)
#pragma unroll
      for (int x = 0; x < 5; ++x) a[y + x] = b[y + x] ^ (~b[y + (x + 1) % 5] & b[y + (x + 2) % 5]);
    a[0] ^= e ? KRC2.v[1][round] : KRC2.v[0][round];
  }
}

constexpr int RATE = 136;  // SHA3-256 rate in bytes (17 lanes)
constexpr int RATE_DW = RATE / 4 + 1;  // aligned dwords covering a block at any byte offset

// One rate block at an arbitrary byte address: the aligned dwords that hold its bytes (only
// those: none past the dword of the last wanted byte is touched), funnel-shifted by the
// misalignment with v_alignbyte_b32.  Bytes at block offsets >= n read as zero.
__device__ __forceinline__ void load_block(const uint8_t* p, uint32_t n, uint64_t w[RATE / 8]) {
  const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3u);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p - s);  // stays a global pointer
  uint32_t dw[RATE_DW];
#pragma unroll
  for (int i = 0; i < RATE_DW; ++i) dw[i] = (4u * i < s + n) ? q[i] : 0u;
#pragma unroll
  for (int j = 0; j < RATE / 8; ++j) {
    const uint32_t lo = __builtin_amdgcn_alignbyte(dw[2 * j + 1], dw[2 * j], s);
    const uint32_t hi = __builtin_amdgcn_alignbyte(dw[2 * j + 2], dw[2 * j + 1], s);
    uint64_t v = ((uint64_t)hi << 32) | lo;
    const int keep = (int)n - 8 * j;  // bytes of this word inside the message
    if (keep < 8) v = keep <= 0 ? 0 : v & ((1ull << (8 * keep)) - 1);
    w[j] = v;
  }
}

// SHA3-256 of a byte string in global memory (any alignment), by a lane pair: out = this lane's
// halves of the 4 digest words.
__device__ void sha3_mem2(const uint8_t* msg, uint32_t len, uint32_t out[4], uint32_t e) {
  uint32_t a[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) a[i] = 0;
  uint32_t off = 0;
  uint64_t w[RATE / 8];
  while (len - off >= (uint32_t)RATE) {
    load_block(msg + off, RATE, w);
#pragma unroll
    for (int i = 0; i < RATE / 8; ++i) a[i] ^= half_of(w[i], e);
    keccak_f2(a, e);
    off += RATE;
  }
  // last block: the remaining bytes, the SHA3 domain bits 0x06 and the final 0x80
  const uint32_t rem = len - off;
  load_block(msg + off, rem, w);
#pragma unroll
  for (int i = 0; i < RATE / 8; ++i) {
    const int lo = 8 * i;
    uint64_t v = w[i];
    if ((uint32_t)lo <= rem && rem < (uint32_t)lo + 8) v ^= (uint64_t)0x06 << (8 * (rem - lo));
    if (i == RATE / 8 - 1) v ^= 0x80ull << 56;
    a[i] ^= half_of(v, e);
  }
  keccak_f2(a, e);
#pragma unroll
  for (int i = 0; i < 4; ++i) out[i] = a[i];
}

// SHA3-256 of the 64-byte concatenation x || y of two digests (one block), in halves.
__device__ __forceinline__ void sha3_pair2(const uint32_t x[4], const uint32_t y[4], uint32_t out[4],
                                           uint32_t e) {
  uint32_t a[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) a[i] = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = x[i];
    a[4 + i] = y[i];
  }
  a[8] = e ? parity_bits(0x06, 1) : parity_bits(0x06, 0);
  a[16] = e ? parity_bits(0x80ull << 56, 1) : parity_bits(0x80ull << 56, 0);
  keccak_f2(a, e);
#pragma unroll
  for (int i = 0; i < 4; ++i) out[i] = a[i];
}

__device__ __forceinline__ void ld_digest(uint64_t d[4], const uint8_t* p) {
  const uint2* q = reinterpret_cast<const uint2*>(p);  // digests are 8-byte aligned
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint2 v = q[i];
    d[i] = ((uint64_t)v.y << 32) | v.x;
  }
}
__device__ __forceinline__ void st_digest(uint8_t* p, const uint64_t d[4]) {
  uint2* q = reinterpret_cast<uint2*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = make_uint2((uint32_t)d[i], (uint32_t)(d[i] >> 32));
}

// a digest in memory as this lane's halves, and back (lane e = 0 of the pair stores)
__device__ __forceinline__ void ld_digest2(uint32_t h[4], const uint8_t* p, uint32_t e) {
  uint64_t d[4];
  ld_digest(d, p);
#pragma unroll
  for (int i = 0; i < 4; ++i) h[i] = half_of(d[i], e);
}
__device__ __forceinline__ void st_digest2(uint8_t* p, const uint32_t h[4], uint32_t e) {
  uint64_t d[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = word_of(h[i], e);
  if (e == 0) st_digest(p, d);
}

// ------------------------------------------------------------------ GF(2^8) by a constant
// t[0..3]: T_lo (c * x for x = 0..15, four entries per dword, little-endian), t[4..7]: T_hi
// (c * 16x).  Four products per call: x holds four data bytes.
__device__ __forceinline__ uint32_t nib_lookup(uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3,
                                               uint32_t n7, uint32_t m8) {
  const uint32_t lo = __builtin_amdgcn_perm(t1, t0, n7);  // entries 0..7
  const uint32_t hi = __builtin_amdgcn_perm(t3, t2, n7);  // entries 8..15
  return (hi & m8) | (lo & ~m8);                           // v_bfi_b32
}

}  // namespace

// One workgroup = R output rows of one instance; each thread one 4-byte column of those rows at
// a time, looping over the shard.  grid.x: (job, row block).  Rows are shard indices inside an
// instance's block of (k + p) shards of `len` bytes (shards[inst * stride + row * len]).  The
// block's tables (R x n_in coefficients, 32 bytes each) and input rows are staged in LDS once
// and read with broadcast ds_read_b128 (wave-uniform scalar loads of them were issued and
// waited for one row at a time: 4x slower).
constexpr int GF_R = 8;
constexpr int GF_J = 8;  // input rows whose loads are in flight together
constexpr uint32_t GF_BS_MAX = 256;
__global__ void __launch_bounds__(GF_BS_MAX) k_gf_apply(uint32_t n_jobs, const uint32_t* __restrict__ jobs,
                                                        uint8_t* __restrict__ shards, uint64_t stride,
                                                        uint32_t len, uint32_t n_out,
                                                        const uint32_t* __restrict__ out_rows, uint32_t n_in,
                                                        const uint32_t* __restrict__ in_rows,
                                                        const uint32_t* __restrict__ tabs) {
  extern __shared__ uint4 gf_lds[];  // [GF_R][n_in_p] x {T_lo, T_hi}, then the input rows
  const uint32_t row_blocks = (n_out + GF_R - 1) / GF_R;
  const uint32_t job = blockIdx.x / row_blocks, rb = blockIdx.x % row_blocks;
  if (job >= n_jobs) return;
  const uint32_t inst = jobs ? jobs[job] : job;
  const uint32_t r0 = rb * GF_R;
  // input rows padded to a multiple of GF_J with zero tables (and the last row's data)
  const uint32_t n_in_p = (n_in + GF_J - 1) / GF_J * GF_J;
  uint32_t* lrow = reinterpret_cast<uint32_t*>(gf_lds + GF_R * n_in_p * 2);
  const uint4* gtab = reinterpret_cast<const uint4*>(tabs);
  for (uint32_t i = threadIdx.x; i < GF_R * n_in_p * 2; i += blockDim.x) {
    const uint32_t r = i / (n_in_p * 2), c = i - r * n_in_p * 2;
    const uint32_t row = min(r0 + r, n_out - 1);  // rows past n_out repeat the last (not stored)
    gf_lds[i] = c < n_in * 2 ? gtab[(size_t)row * n_in * 2 + c] : make_uint4(0, 0, 0, 0);
  }
  for (uint32_t i = threadIdx.x; i < n_in_p; i += blockDim.x) lrow[i] = in_rows[min(i, n_in - 1)];
  __syncthreads();
  uint8_t* base = shards + inst * stride;
  const uint32_t n_words = (len + 3) / 4;
  for (uint32_t w = threadIdx.x; w < n_words; w += blockDim.x) {
    const uint32_t b0 = 4 * w;
    const bool full = b0 + 4 <= len;
    const uint32_t nb = full ? 4u : len - b0;
    uint32_t acc[GF_R];
#pragma unroll
    for (int r = 0; r < GF_R; ++r) acc[r] = 0;
    // rows are len bytes apart, so most start off a dword boundary (the misalignment is the
    // same for the whole wave): the aligned dwords holding bytes [b0, b0 + nb), funnel-shifted
    // (v_alignbyte_b32); the second dword is read only when it holds one of those bytes.  Input
    // rows go in groups of GF_J, their loads issued together.
    const uint32_t tail_mask = full ? ~0u : (1u << (8 * nb)) - 1u;
#pragma unroll 1
    for (uint32_t j0 = 0; j0 < n_in_p; j0 += GF_J) {
      uint32_t xa[GF_J], xb[GF_J], sh[GF_J];
#pragma unroll
      for (int u = 0; u < GF_J; ++u) {
        const uint8_t* src = base + (size_t)lrow[j0 + u] * len + b0;
        sh[u] = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 3u);
        const uint32_t* q = reinterpret_cast<const uint32_t*>(src - sh[u]);
        xa[u] = q[0];
        xb[u] = q[(sh[u] + nb > 4u) ? 1 : 0];
      }
#pragma unroll
      for (int u = 0; u < GF_J; ++u) {
        const uint32_t j = j0 + u;
        const uint32_t x = __builtin_amdgcn_alignbyte(xb[u], xa[u], sh[u]) & tail_mask;
        const uint32_t lo = x & 0x0f0f0f0fu, hi = (x >> 4) & 0x0f0f0f0fu;
        const uint32_t lo7 = lo & 0x07070707u, hi7 = hi & 0x07070707u;
        const uint32_t mlo = ((lo >> 3) & 0x01010101u) * 0xffu, mhi = ((hi >> 3) & 0x01010101u) * 0xffu;
#pragma unroll
        for (int r = 0; r < GF_R; ++r) {
          const uint4 tl = gf_lds[(r * n_in_p + j) * 2], th = gf_lds[(r * n_in_p + j) * 2 + 1];
          acc[r] ^= nib_lookup(tl.x, tl.y, tl.z, tl.w, lo7, mlo) ^ nib_lookup(th.x, th.y, th.z, th.w, hi7, mhi);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < GF_R; ++r) {
      if (r0 + r >= n_out) break;
      uint8_t* dst = base + (size_t)out_rows[r0 + r] * len + b0;
      if (full && ((reinterpret_cast<uintptr_t>(dst) & 3u) == 0)) {
        *reinterpret_cast<uint32_t*>(dst) = acc[r];
      } else if (full) {
#pragma unroll
        for (int i = 0; i < 4; ++i) dst[i] = (uint8_t)(acc[r] >> (8 * i));
      } else {
        for (uint32_t i = 0; i < nb; ++i) dst[i] = (uint8_t)(acc[r] >> (8 * i));
      }
    }
  }
}

// One workgroup per instance: the n leaf digests, then each level's pair digests (an odd last
// digest is carried up), into out[inst * n_dig ...]: level 0 (n), level 1 (ceil(n / 2)), ...,
// the root last.  Each digest is computed by a lane pair (bit-interleaved Keccak).
constexpr uint32_t MK_BS = 256;
constexpr uint32_t MK_PAIRS = MK_BS / 2;
__global__ void __launch_bounds__(MK_BS) k_merkle_tree(uint32_t n, uint32_t leaf_len,
                                                       const uint8_t* __restrict__ leaves,
                                                       uint64_t stride, uint32_t n_dig,
                                                       uint8_t* __restrict__ out) {
  const uint32_t inst = blockIdx.x;
  const uint32_t e = threadIdx.x & 1u, pr = threadIdx.x >> 1;
  const uint8_t* lv = leaves + inst * stride;
  uint8_t* o = out + (size_t)inst * n_dig * 32;
  for (uint32_t i = pr; i < n; i += MK_PAIRS) {
    uint32_t d[4];
    sha3_mem2(lv + (size_t)i * leaf_len, leaf_len, d, e);
    st_digest2(o + (size_t)i * 32, d, e);
  }
  uint32_t cur = 0, m = n;
  while (m > 1) {
    __syncthreads();
    const uint32_t nxt = cur + m, half = (m + 1) / 2;
    for (uint32_t i = pr; i < half; i += MK_PAIRS) {
      if (2 * i + 1 < m) {
        uint32_t x[4], y[4], r[4];
        ld_digest2(x, o + (size_t)(cur + 2 * i) * 32, e);
        ld_digest2(y, o + (size_t)(cur + 2 * i + 1) * 32, e);
        sha3_pair2(x, y, r, e);
        st_digest2(o + (size_t)(nxt + i) * 32, r, e);
      } else if (e == 0) {
        uint64_t x[4];
        ld_digest(x, o + (size_t)(cur + 2 * i) * 32);
        st_digest(o + (size_t)(nxt + i) * 32, x);
      }
    }
    cur = nxt;
    m = half;
  }
}

// Proof::validate(n_nodes) of proof i: value bytes [voff[i], voff[i+1]), index idx[i], digests
// [doff[i], doff[i+1]) (32 bytes each), root roots[i].  status: HBTC_ACCEPT / HBTC_REJECT.  One
// lane pair per proof (every branch below depends on the proof only, so a pair stays together).
__global__ void __launch_bounds__(64) k_merkle_validate(uint32_t n, uint32_t n_nodes,
                                                        const uint64_t* __restrict__ voff,
                                                        const uint8_t* __restrict__ values,
                                                        const uint32_t* __restrict__ idx,
                                                        const uint32_t* __restrict__ doff,
                                                        const uint8_t* __restrict__ digests,
                                                        const uint8_t* __restrict__ roots,
                                                        int32_t* __restrict__ status) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  const uint32_t p = t >> 1, e = t & 1u;
  if (p >= n) return;
  uint32_t d[4];
  sha3_mem2(values + voff[p], (uint32_t)(voff[p + 1] - voff[p]), d, e);
  uint32_t i = idx[p], m = n_nodes, it = doff[p];
  const uint32_t end = doff[p + 1];
  bool ok = true;
  while (m > 1) {
    if ((i ^ 1u) < m) {
      if (it >= end) {
        ok = false;
        break;
      }
      uint32_t sib[4], r[4];
      ld_digest2(sib, digests + (size_t)it * 32, e);
      ++it;
      if (i & 1u)
        sha3_pair2(sib, d, r, e);
      else
        sha3_pair2(d, sib, r, e);
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = r[q];
    }
    i >>= 1;
    m = (m + 1) >> 1;
  }
  if (ok && it != end) ok = false;  // too many levels in the proof
  if (ok) {
    uint32_t rt[4];
    ld_digest2(rt, roots + (size_t)p * 32, e);
#pragma unroll
    for (int q = 0; q < 4; ++q) ok = ok && rt[q] == d[q];
  }
  // both halves must match: the pair's verdict
  const uint32_t both = (uint32_t)ok & pair_swap((uint32_t)ok);
  if (e == 0) status[p] = both ? HBTC_ACCEPT : HBTC_REJECT;
}

// ------------------------------------------------------------------ launchers
hipError_t launch_gf_apply(hipStream_t s, uint32_t n_jobs, const uint32_t* jobs, uint8_t* shards,
                           uint64_t stride, uint32_t len, uint32_t n_out, const uint32_t* out_rows,
                           uint32_t n_in, const uint32_t* in_rows, const uint32_t* tabs) {
  if (n_jobs == 0 || n_out == 0 || len == 0) return hipSuccess;
  if (n_in > 256) return hipErrorInvalidValue;  // GF(2^8) codes have at most 256 shards
  const uint32_t row_blocks = (n_out + GF_R - 1) / GF_R;
  const uint32_t words = (len + 3) / 4;
  const uint32_t bs = min(GF_BS_MAX, (words + 63) / 64 * 64);
  const uint32_t n_in_p = (n_in + GF_J - 1) / GF_J * GF_J;
  const size_t lds = (size_t)GF_R * n_in_p * 32 + (size_t)n_in_p * 4;
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gf_apply),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_gf_apply, dim3(n_jobs * row_blocks), dim3(bs), lds, s, n_jobs, jobs, shards,
                     stride, len, n_out, out_rows, n_in, in_rows, tabs);
  return hipGetLastError();
}

hipError_t launch_merkle_tree(hipStream_t s, uint32_t n_inst, uint32_t n, uint32_t leaf_len,
                              const uint8_t* leaves, uint64_t stride, uint32_t n_dig, uint8_t* out) {
  if (n_inst == 0 || n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_merkle_tree, dim3(n_inst), dim3(MK_BS), 0, s, n, leaf_len, leaves, stride,
                     n_dig, out);
  return hipGetLastError();
}

hipError_t launch_merkle_validate(hipStream_t s, uint32_t n, uint32_t n_nodes, const uint64_t* voff,
                                  const uint8_t* values, const uint32_t* idx, const uint32_t* doff,
                                  const uint8_t* digests, const uint8_t* roots, int32_t* status) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_merkle_validate, dim3((2 * (uint64_t)n + 63) / 64), dim3(64), 0, s, n, n_nodes, voff, values,
                     idx, doff, digests, roots, status);
  return hipGetLastError();
}

}  // namespace hbtc
