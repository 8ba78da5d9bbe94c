// Device helpers shared by the RLC item passes of DecryptionShares (hbtc_rlc.hip) and
// SignatureShares (hbtc_sig.hip): the per-call ChaCha20 scalars, the wave tree sums of a tile,
// the fixed-base multiplication by a key-set share.  See hbtc_rlc.hip for the method.
#pragma once
#include "hbtc_kernels.h"

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

// The scalar r_i = a + b mu of item i from a ChaCha20 block (RFC 8439 layout: constants, 8 key
// words, counter, 3 nonce words).  64-bit mode (key.bits = 64): a and b are the 32-bit words
// [2j, 2j+1] of block i / 8 (j = i mod 8); 128-bit mode: a and b are the 64-bit pairs of words
// [4j, 4j+1], [4j+2, 4j+3] of block i / 4 (j = i mod 4), under a different nonce word.
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }
static __device__ void rlc_scalar(const RlcKey& key, uint64_t item, uint64_t& a, uint64_t& b) {
  const bool wide = key.bits == 128;
  const uint64_t blk = wide ? item >> 2 : item >> 3;
  uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                     key.k[0], key.k[1], key.k[2], key.k[3], key.k[4], key.k[5], key.k[6], key.k[7],
                     (uint32_t)blk, (uint32_t)(blk >> 32), 0x68626266u, wide ? 0x32313172u : 0x72726c63u};
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
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] += st[i];
  if (wide) {
    const int j = (int)(item & 3);
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i == j) {
        w0 = x[4 * i];
        w1 = x[4 * i + 1];
        w2 = x[4 * i + 2];
        w3 = x[4 * i + 3];
      }
    a = ((uint64_t)w1 << 32) | w0;
    b = ((uint64_t)w3 << 32) | w2;
  } else {
    const int j = (int)(item & 7);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i == j) {
        lo = x[2 * i];
        hi = x[2 * i + 1];
      }
    a = lo;
    b = hi;
  }
}

// Append the wave's tracked-sender items to the leaf list: one atomic per wave.  Called by all
// 64 lanes (wave-uniform control flow).
__device__ __forceinline__ void rlc_list_leaf(const Suspects& sus, bool leaf, uint32_t item,
                                              uint32_t inst, uint32_t lane) {
  const uint64_t m = __ballot(leaf);
  if (!m) return;
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(sus.leaf_count, (uint32_t)__popcll(m));
  base = __shfl(base, 0);
  if (leaf) {
    const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    sus.leaves[2 * pos] = item;
    sus.leaves[2 * pos + 1] = inst;
  }
}

// Tree reduction of the per-lane points q over the wave (lane = position in the tile): the sum
// A and the position-weighted sum B of every aligned group of 8 (-> outA/outB[0..7]) and of the
// tile (-> [8]).  Merging halves:  A = A_l + A_r,  B = 2 (B_l + B_r) + A_r, so share i of a group
// of 2^k carries the weight bitrev_k(i) (one doubling per level instead of log2(s) for the
// positional weights B_l + B_r + s A_r; hbtc_check.hip maps a located weight back).
template <class F>
__device__ void rlc_reduce(Jac<F>* redA, Jac<F>* redB, const Jac<F>& q, uint32_t lane,
                           Jac<F>* outA, Jac<F>* outB) {
  Jac<F> z;
  jac_set_inf(z);
  redA[lane] = q;
  redB[lane] = z;
  __syncthreads();
  for (uint32_t s = 1; s < 64; s <<= 1) {
    if ((lane & (2 * s - 1)) == 0) {  // one merge at a time (register pressure, as below)
      Jac<F> b = redB[lane];
      {
        const Jac<F> br = redB[lane + s];
        jac_add(b, b, br);
      }
      const Jac<F> ar = redA[lane + s];
      jac_dbl(b, b);
      jac_add(b, b, ar);
      redB[lane] = b;
      Jac<F> a = redA[lane];
      jac_add(a, a, ar);
      redA[lane] = a;
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

// Plain tree sum of the per-lane points over the wave: out[0..7] the aligned groups of 8, out[8]
// the whole wave (no position-weighted sums: the pair-batch path locates by splitting).
template <class F>
__device__ void rlc_reduce_plain(Jac<F>* red, const Jac<F>& q, uint32_t lane, Jac<F>* out) {
  red[lane] = q;
  __syncthreads();
#pragma unroll 1
  for (uint32_t s = 1; s < 64; s <<= 1) {
    if ((lane & (2 * s - 1)) == 0) {
      Jac<F> a = red[lane];
      const Jac<F> b = red[lane + s];
      jac_add(a, a, b);
      red[lane] = a;
    }
    __syncthreads();
    if (s == 4 && (lane & 7u) == 0) out[lane >> 3] = red[lane];
  }
  if (lane == 0) out[8] = red[0];
  __syncthreads();
}

// The same reduction with ONE LDS array (the plain sums A; the weighted sums B travel between
// lanes by ds_bpermute): half the LDS of rlc_reduce, so a G2 tile (216-byte points) leaves room
// for two waves per SIMD.  All 64 lanes run every exchange (converged control flow).
template <class F>
__device__ __forceinline__ void jac_shfl(Jac<F>& r, const Jac<F>& x, uint32_t src) {
  const uint32_t* xs = reinterpret_cast<const uint32_t*>(&x);
  uint32_t* rs = reinterpret_cast<uint32_t*>(&r);
  const int addr = (int)((src & 63u) << 2);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(Jac<F>) / 4); ++i)
    rs[i] = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)xs[i]);
}
template <class F>
__device__ void rlc_reduce1(Jac<F>* red, const Jac<F>& q, uint32_t lane, Jac<F>* outA, Jac<F>* outB) {
  Jac<F> b;
  jac_set_inf(b);
  red[lane] = q;
  __syncthreads();
  for (uint32_t s = 1; s < 64; s <<= 1) {
    const bool active = (lane & (2 * s - 1)) == 0;
    {
      Jac<F> br;
      jac_shfl(br, b, lane + s);
      if (active) jac_add(b, b, br);
    }
    if (active) {
      jac_dbl(b, b);  // B = 2 (B_l + B_r) + A_r (bit-reversed weights, as rlc_reduce)
      jac_add(b, b, red[lane + s]);
      Jac<F> a = red[lane];
      const Jac<F> ar = red[lane + s];
      jac_add(a, a, ar);
      red[lane] = a;  // active lanes read only inactive entries besides their own
    }
    __syncthreads();
    if (s == 4 && (lane & 7u) == 0) {
      outA[lane >> 3] = red[lane];
      outB[lane >> 3] = b;
    }
  }
  if (lane == 0) {
    outA[8] = red[0];
    outB[8] = b;
  }
  __syncthreads();  // the array is reused by the next reduction
}

// The two G1 sums of a DecryptionShare tile (S = sum r_i d_i, P = sum r_i pk_i), each with its
// position-weighted sum, in ONE tree with every level's S and P merges on different lanes.
// Level 1 pairs lanes (2m, 2m+1) in registers: the even lane forms the S pair, the odd lane the
// P pair (A = left + right, B = right).  From then on LDS entry 2m holds an S group and entry
// 2m+1 a P group; at level s the lanes with lane mod 2s in {0, 1} merge entry `lane` with entry
// `lane + s` (A = A_l + A_r, B = 2 (B_l + B_r) + A_r).  Outputs as rlc_reduce: [0..7] the aligned
// groups of 8, [8] the tile; plus the two halves and the left quarter of each half.  Half the
// sequential merge chain of two separate reductions.
__device__ __forceinline__ void rlc_reduce_sp(G1J* redA, G1J* redB, const G1J& S, const G1J& P,
                                              uint32_t lane, G1J* outS, G1J* outSW, G1J* outP,
                                              G1J* outPW, G1J* outSH, G1J* outSHW, G1J* outPH,
                                              G1J* outPHW, G1J* outSQ, G1J* outSQW, G1J* outPQ,
                                              G1J* outPQW) {
  const bool odd = (lane & 1u) != 0;
  // selects by value (a reference chosen between S and P would put both in scratch)
  G1J x, y;  // x: the value the neighbour lane needs
  fsel(x.x, odd, S.x, P.x);
  fsel(x.y, odd, S.y, P.y);
  fsel(x.z, odd, S.z, P.z);
  {
    const uint32_t* xs = reinterpret_cast<const uint32_t*>(&x);
    uint32_t* ys = reinterpret_cast<uint32_t*>(&y);
    const int addr = (int)((lane ^ 1u) << 2);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(G1J) / 4); ++i)
      ys[i] = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)xs[i]);
  }
  G1J a, l, r;
  fsel(l.x, odd, y.x, S.x);
  fsel(l.y, odd, y.y, S.y);
  fsel(l.z, odd, y.z, S.z);
  fsel(r.x, odd, P.x, y.x);
  fsel(r.y, odd, P.y, y.y);
  fsel(r.z, odd, P.z, y.z);
  jac_add(a, l, r);
  redA[lane] = a;
  redB[lane] = r;
  __syncthreads();
  for (uint32_t s = 2; s < 64; s <<= 1) {
    if ((lane & (2 * s - 1)) < 2) {
      // one merge at a time, so at most three points are live (register pressure: the active
      // lanes only read entries of inactive ones besides their own, so the writes cannot race)
      G1J bl = redB[lane];
      {
        const G1J br = redB[lane + s];
        jac_add(bl, bl, br);
      }
      const G1J ar = redA[lane + s];
      jac_dbl(bl, bl);
      jac_add(bl, bl, ar);
      redB[lane] = bl;
      G1J al = redA[lane];
      jac_add(al, al, ar);
      redA[lane] = al;
    }
    __syncthreads();
    if (s == 4 && (lane & 7u) < 2) {
      if ((lane & 7u) == 0) {
        outS[lane >> 3] = redA[lane];
        outSW[lane >> 3] = redB[lane];
      } else {
        outP[lane >> 3] = redA[lane];
        outPW[lane >> 3] = redB[lane];
      }
    }
    if (s == 8 && (lane & 31u) < 2) {  // the left 16-share quarter of each half
      if ((lane & 31u) == 0) {
        outSQ[lane >> 5] = redA[lane];
        outSQW[lane >> 5] = redB[lane];
      } else {
        outPQ[lane >> 5] = redA[lane];
        outPQW[lane >> 5] = redB[lane];
      }
    }
    if (s == 16 && (lane & 31u) < 2) {  // the 32-share halves
      if ((lane & 31u) == 0) {
        outSH[lane >> 5] = redA[lane];
        outSHW[lane >> 5] = redB[lane];
      } else {
        outPH[lane >> 5] = redA[lane];
        outPHW[lane >> 5] = redB[lane];
      }
    }
  }
  if (lane == 0) {
    outS[8] = redA[0];
    outSW[8] = redB[0];
  } else if (lane == 1) {
    outP[8] = redA[1];
    outPW[8] = redB[1];
  }
  __syncthreads();
}

// The four x-adic digits of item i's scalar (curve.h xadic_mul_uniform): the halves (a, b) of
// rlc_scalar split in two, d = (a_lo, a_hi, b_lo, b_hi), each key.bits / 4 bits.  r = d0 + d1 x +
// d2 mu + d3 mu x (mod r) is injective on the digit box: for digits below 2^33 < |x| the integer
// d0 + d1 x - d2 x^2 - d3 x^3 has absolute value < r, and it is 0 only for all-zero digits
// (reduce mod x digit by digit), so the 2^key.bits digit vectors give 2^key.bits residues.
struct XDigits {
  uint32_t d[4];
  int nbits;
};
__device__ __forceinline__ XDigits rlc_digits(const RlcKey& key, uint64_t item) {
  uint64_t a, b;
  rlc_scalar(key, item, a, b);
  XDigits x;
  if (key.bits == 128) {
    x.d[0] = (uint32_t)a;
    x.d[1] = (uint32_t)(a >> 32);
    x.d[2] = (uint32_t)b;
    x.d[3] = (uint32_t)(b >> 32);
    x.nbits = 32;
  } else {
    x.d[0] = (uint32_t)a & 0xffffu;
    x.d[1] = (uint32_t)(a >> 16) & 0xffffu;
    x.d[2] = (uint32_t)b & 0xffffu;
    x.d[3] = (uint32_t)(b >> 16) & 0xffffu;
    x.nbits = 16;
  }
  return x;
}

// [r] pk for the x-adic scalar from the key set's fixed-base table (hbtc_kernels.h PK_TAB_WIN:
// windows 0..3 multiples of pk, 4..7 of [x] pk): [d0] pk + [d1] xpk + [d2] phi(pk) + [d3]
// phi(xpk), 4 nbits / 8 mixed additions and no doublings.
static __device__ void rlc_pk_mul_x(G1J& r, const PtXY* __restrict__ tab, const XDigits& x) {
  jac_set_inf(r);
  const int nwin = x.nbits / 8;
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    const uint32_t dj = x.d[0] * (j == 0) + x.d[1] * (j == 1) + x.d[2] * (j == 2) + x.d[3] * (j == 3);
    const int tw = (j & 1) ? 4 : 0;  // d1, d3: the [x] pk windows
#pragma unroll 1
    for (int w = 0; w < nwin; ++w) {
      const uint32_t v = (dj >> (8 * w)) & 0xffu;
      if (!v) continue;
      const PtXY e = tab[(tw + w) * 256 + v];
      G1A q;
      q.y = e.y;
      q.inf = 0;
      if (j >= 2) {  // wave-uniform
        Fq beta;
        fq_set(beta, G1_BETA);
        fq_mul(q.x, e.x, beta);
      } else {
        q.x = e.x;
      }
      jac_add_aff(r, r, q);
    }
  }
}

// [a] pk + [b] phi(pk) from the key set's fixed-base table (2 nwin mixed additions, no
// doublings; nwin = 4 for 32-bit a, b, 8 for 64-bit).
static __device__ void rlc_pk_mul(G1J& r, const PtXY* __restrict__ tab, uint64_t a, uint64_t b,
                                  int nwin) {
  jac_set_inf(r);
#pragma unroll 1
  for (int w = 0; w < nwin; ++w) {
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

}  // namespace hbtc
