// Reliable Broadcast coding path of hbbft (/root/reference/src/broadcast/) on gfx950: the
// Reed-Solomon erasure code over GF(2^8) and the SHA3-256 Merkle trees / proofs every node
// builds and checks for every proposer's value.
//
//   k_gf_apply        out_row[r] = sum_j M[r][j] * in_row[j] for a batch of instances: the
//                     parity rows of ReedSolomon::encode (broadcast.rs:183-185, :433-441) and the
//                     missing rows of ReedSolomon::reconstruct_shards (:444-458)
//   k_merkle_tree     MerkleTree::from_vec (merkle.rs:19-32): every level of one instance's
//                     tree per workgroup
//   k_merkle_validate Proof::validate (merkle.rs:82-102): one proof per lane, the N^2 Echo
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
// Register-resident: the 25 lanes are named variables (fully unrolled rounds, static indices).
__device__ __forceinline__ uint64_t rol(uint64_t v, int c) { return (v << c) | (v >> (64 - c)); }

__constant__ uint64_t KRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

__device__ __forceinline__ void keccak_f(uint64_t* a) {
#pragma unroll 1
  for (int round = 0; round < 24; ++round) {
    uint64_t c[5], d[5], b[25];
#pragma unroll
    for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
#pragma unroll
    for (int x = 0; x < 5; ++x) d[x] = c[(x + 4) % 5] ^ rol(c[(x + 1) % 5], 1);
    // theta, then rho + pi: b[y, 2x + 3y] = rot(a[x, y] ^ d[x])
    constexpr int ROT[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                             25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};
#pragma unroll
    for (int x = 0; x < 5; ++x)
#pragma unroll
      for (int y = 0; y < 5; ++y) {
        const uint64_t v = a[x + 5 * y] ^ d[x];
        const int r = ROT[x + 5 * y];
        b[y + 5 * ((2 * x + 3 * y) % 5)] = r ? rol(v, r) : v;
      }
#pragma unroll
    for (int y = 0; y < 25; y += 5)
#pragma unroll
      for (int x = 0; x < 5; ++x) a[y + x] = b[y + x] ^ (~b[y + (x + 1) % 5] & b[y + (x + 2) % 5]);
    a[0] ^= KRC[round];
  }
}

constexpr int RATE = 136;  // SHA3-256 rate in bytes (17 lanes)

// little-endian 64-bit word of p[0..n) (n <= 8), zero-extended
__device__ __forceinline__ uint64_t load_le(const uint8_t* p, int n) {
  uint64_t v = 0;
  for (int i = 0; i < n; ++i) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

// SHA3-256 of a byte string in global memory.
__device__ void sha3_mem(const uint8_t* msg, uint32_t len, uint64_t out[4]) {
  uint64_t a[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) a[i] = 0;
  uint32_t off = 0;
  while (len - off >= (uint32_t)RATE) {
#pragma unroll
    for (int i = 0; i < RATE / 8; ++i) a[i] ^= load_le(msg + off + 8 * i, 8);
    keccak_f(a);
    off += RATE;
  }
  // last block: the remaining bytes, the SHA3 domain bits 0x06 and the final 0x80
  const uint32_t rem = len - off;
#pragma unroll
  for (int i = 0; i < RATE / 8; ++i) {
    const int lo = 8 * i;
    uint64_t w = 0;
    if ((uint32_t)lo < rem) w = load_le(msg + off + lo, (int)min(8u, rem - (uint32_t)lo));
    if ((uint32_t)lo <= rem && rem < (uint32_t)lo + 8) w ^= (uint64_t)0x06 << (8 * (rem - lo));
    if (i == RATE / 8 - 1) w ^= 0x80ull << 56;
    a[i] ^= w;
  }
  keccak_f(a);
#pragma unroll
  for (int i = 0; i < 4; ++i) out[i] = a[i];
}

// SHA3-256 of the 64-byte concatenation x || y of two digests (one block).
__device__ __forceinline__ void sha3_pair(const uint64_t x[4], const uint64_t y[4], uint64_t out[4]) {
  uint64_t a[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) a[i] = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = x[i];
    a[4 + i] = y[i];
  }
  a[8] = 0x06;
  a[16] = 0x80ull << 56;
  keccak_f(a);
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

// One thread = one 4-byte column of R output rows of one instance.  grid.x: (job, row block),
// grid.y: column blocks of 64 words.  Rows are shard indices inside an instance's block of
// (k + p) shards of `len` bytes (shards[inst * stride + row * len]); the tail word of a shard
// whose length is not a multiple of 4 is read and written bytewise.
constexpr int GF_R = 8;
__global__ void __launch_bounds__(64) k_gf_apply(uint32_t n_jobs, const uint32_t* __restrict__ jobs,
                                                 uint8_t* __restrict__ shards, uint64_t stride,
                                                 uint32_t len, uint32_t n_out,
                                                 const uint32_t* __restrict__ out_rows, uint32_t n_in,
                                                 const uint32_t* __restrict__ in_rows,
                                                 const uint32_t* __restrict__ tabs) {
  const uint32_t row_blocks = (n_out + GF_R - 1) / GF_R;
  const uint32_t job = blockIdx.x / row_blocks, rb = blockIdx.x % row_blocks;
  if (job >= n_jobs) return;
  const uint32_t inst = jobs ? jobs[job] : job;
  const uint32_t w = blockIdx.y * 64 + threadIdx.x;  // word (column) index
  const uint32_t n_words = (len + 3) / 4;
  if (w >= n_words) return;
  const uint32_t b0 = 4 * w;
  const bool full = b0 + 4 <= len;
  const uint32_t nb = full ? 4u : len - b0;
  uint8_t* base = shards + inst * stride;
  uint32_t acc[GF_R];
#pragma unroll
  for (int r = 0; r < GF_R; ++r) acc[r] = 0;
  const uint32_t r0 = rb * GF_R;
#pragma unroll 1
  for (uint32_t j = 0; j < n_in; ++j) {
    const uint8_t* src = base + (size_t)in_rows[j] * len + b0;
    uint32_t x;
    if (full && ((reinterpret_cast<uintptr_t>(src) & 3u) == 0)) {
      x = *reinterpret_cast<const uint32_t*>(src);
    } else {
      x = 0;
      for (uint32_t i = 0; i < nb; ++i) x |= (uint32_t)src[i] << (8 * i);
    }
    const uint32_t lo = x & 0x0f0f0f0fu, hi = (x >> 4) & 0x0f0f0f0fu;
    const uint32_t lo7 = lo & 0x07070707u, hi7 = hi & 0x07070707u;
    const uint32_t mlo = ((lo >> 3) & 0x01010101u) * 0xffu, mhi = ((hi >> 3) & 0x01010101u) * 0xffu;
#pragma unroll
    for (int r = 0; r < GF_R; ++r) {
      if (r0 + r < n_out) {
        const uint32_t* t = tabs + ((size_t)(r0 + r) * n_in + j) * 8;  // wave-uniform
        acc[r] ^= nib_lookup(t[0], t[1], t[2], t[3], lo7, mlo) ^ nib_lookup(t[4], t[5], t[6], t[7], hi7, mhi);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < GF_R; ++r) {
    if (r0 + r >= n_out) break;
    uint8_t* dst = base + (size_t)out_rows[r0 + r] * len + b0;
    if (full && ((reinterpret_cast<uintptr_t>(dst) & 3u) == 0)) {
      *reinterpret_cast<uint32_t*>(dst) = acc[r];
    } else {
      for (uint32_t i = 0; i < nb; ++i) dst[i] = (uint8_t)(acc[r] >> (8 * i));
    }
  }
}

// One workgroup per instance: the n leaf digests, then each level's pair digests (an odd last
// digest is carried up), into out[inst * n_dig ...]: level 0 (n), level 1 (ceil(n / 2)), ...,
// the root last.
constexpr uint32_t MK_BS = 256;
__global__ void __launch_bounds__(MK_BS) k_merkle_tree(uint32_t n, uint32_t leaf_len,
                                                       const uint8_t* __restrict__ leaves,
                                                       uint64_t stride, uint32_t n_dig,
                                                       uint8_t* __restrict__ out) {
  const uint32_t inst = blockIdx.x;
  const uint8_t* lv = leaves + inst * stride;
  uint8_t* o = out + (size_t)inst * n_dig * 32;
  for (uint32_t i = threadIdx.x; i < n; i += MK_BS) {
    uint64_t d[4];
    sha3_mem(lv + (size_t)i * leaf_len, leaf_len, d);
    st_digest(o + (size_t)i * 32, d);
  }
  uint32_t cur = 0, m = n;
  while (m > 1) {
    __syncthreads();
    const uint32_t nxt = cur + m, half = (m + 1) / 2;
    for (uint32_t i = threadIdx.x; i < half; i += MK_BS) {
      uint64_t x[4], r[4];
      ld_digest(x, o + (size_t)(cur + 2 * i) * 32);
      if (2 * i + 1 < m) {
        uint64_t y[4];
        ld_digest(y, o + (size_t)(cur + 2 * i + 1) * 32);
        sha3_pair(x, y, r);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) r[q] = x[q];
      }
      st_digest(o + (size_t)(nxt + i) * 32, r);
    }
    cur = nxt;
    m = half;
  }
}

// Proof::validate(n_nodes) of proof i: value bytes [voff[i], voff[i+1]), index idx[i], digests
// [doff[i], doff[i+1]) (32 bytes each), root roots[i].  status: HBTC_ACCEPT / HBTC_REJECT.
__global__ void __launch_bounds__(64) k_merkle_validate(uint32_t n, uint32_t n_nodes,
                                                        const uint64_t* __restrict__ voff,
                                                        const uint8_t* __restrict__ values,
                                                        const uint32_t* __restrict__ idx,
                                                        const uint32_t* __restrict__ doff,
                                                        const uint8_t* __restrict__ digests,
                                                        const uint8_t* __restrict__ roots,
                                                        int32_t* __restrict__ status) {
  const uint32_t p = blockIdx.x * 64 + threadIdx.x;
  if (p >= n) return;
  uint64_t d[4];
  sha3_mem(values + voff[p], (uint32_t)(voff[p + 1] - voff[p]), d);
  uint32_t i = idx[p], m = n_nodes, it = doff[p];
  const uint32_t end = doff[p + 1];
  bool ok = true;
  while (m > 1) {
    if ((i ^ 1u) < m) {
      if (it >= end) {
        ok = false;
        break;
      }
      uint64_t s[4], r[4];
      ld_digest(s, digests + (size_t)it * 32);
      ++it;
      if (i & 1u)
        sha3_pair(s, d, r);
      else
        sha3_pair(d, s, r);
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = r[q];
    }
    i >>= 1;
    m = (m + 1) >> 1;
  }
  if (ok && it != end) ok = false;  // too many levels in the proof
  if (ok) {
    uint64_t rt[4];
    ld_digest(rt, roots + (size_t)p * 32);
#pragma unroll
    for (int q = 0; q < 4; ++q) ok = ok && rt[q] == d[q];
  }
  status[p] = ok ? HBTC_ACCEPT : HBTC_REJECT;
}

// ------------------------------------------------------------------ launchers
hipError_t launch_gf_apply(hipStream_t s, uint32_t n_jobs, const uint32_t* jobs, uint8_t* shards,
                           uint64_t stride, uint32_t len, uint32_t n_out, const uint32_t* out_rows,
                           uint32_t n_in, const uint32_t* in_rows, const uint32_t* tabs) {
  if (n_jobs == 0 || n_out == 0 || len == 0) return hipSuccess;
  const uint32_t row_blocks = (n_out + GF_R - 1) / GF_R;
  const uint32_t col_blocks = ((len + 3) / 4 + 63) / 64;
  hipLaunchKernelGGL(k_gf_apply, dim3(n_jobs * row_blocks, col_blocks), dim3(64), 0, s, n_jobs, jobs,
                     shards, stride, len, n_out, out_rows, n_in, in_rows, tabs);
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
  hipLaunchKernelGGL(k_merkle_validate, dim3((n + 63) / 64), dim3(64), 0, s, n, n_nodes, voff, values,
                     idx, doff, digests, roots, status);
  return hipGetLastError();
}

}  // namespace hbtc
