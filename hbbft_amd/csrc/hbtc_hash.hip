// Host-side hash_g2 / hash_g1_g2 of threshold_crypto @ 0.1.0-rng-fix: the
// per-instance hash that hbbft's coin nonce (src/coin.rs:151 via PublicKeyShare::verify) and
// every ciphertext (src/threshold_decryption.rs:159 via verify_decryption_share) go through.
// The GPU path receives H; this computes it once per instance on the host, as the north star
// asks.  Algorithm (restated, [EXT-UNVERIFIED] like oracle/rand04.py, which it must match
// byte for byte — tests/test_hash.py):
//   seed   = sha3_256(msg) read as 8 big-endian u32 words
//   rng    = rand 0.4 ChaChaRng::from_seed(seed): 20 rounds, key = seed, 128-bit block counter
//            in words 12..15 from 0, output words in order; next_u64 = (first << 32) | second
//   G2::rand: loop { x = Fq2 { c0: Fq::rand, c1: Fq::rand }  (6 u64 limbs, top 3 bits masked,
//            rejected if >= p, the limbs ARE the Montgomery form); greatest = next_u32 & 1;
//            p = get_point_from_x(x, greatest); if some: q = [h2] p; if q != O: return q }
//   hash_g1_g2(g1, msg) = hash_g2((len(msg) > 64 ? sha3_256(msg) : msg) || compressed(g1))
// The 384-bit Montgomery radix of pairing 0.14 (6 x 64) equals this library's (12 x 32), so
// the drawn limbs are used as the Montgomery representation directly.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "hbtc.h"
#include "hbtc_kernels.h"
#include "pair.h"

namespace hbtc {
namespace {

// ------------------------------------------------------------------ SHA3-256 (FIPS 202)
// Host + device: the GPU candidate kernel (k_hash_cand) runs the same code as the host path.
#define HASH_HD __host__ __device__ inline
HASH_HD uint64_t keccak_rc(int i) {
  const uint64_t RC[24] = {
      0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
      0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
      0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
      0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
      0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
      0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
  return RC[i];
}

HASH_HD uint64_t rotl64(uint64_t v, int c) { return c ? (v << c) | (v >> (64 - c)) : v; }

HASH_HD void keccak_f(uint64_t a[25]) {
  const int ROT[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                       25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};
  for (int round = 0; round < 24; ++round) {
    uint64_t c[5], b[25];
    for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    for (int x = 0; x < 5; ++x) {
      const uint64_t d = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
      for (int y = 0; y < 25; y += 5) a[y + x] ^= d;
    }
    // rho + pi: b[y, 2x + 3y] = rot(a[x, y])
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(a[x + 5 * y], ROT[x + 5 * y]);
    for (int y = 0; y < 25; y += 5)
      for (int x = 0; x < 5; ++x) a[y + x] = b[y + x] ^ (~b[y + (x + 1) % 5] & b[y + (x + 2) % 5]);
    a[0] ^= keccak_rc(round);
  }
}

// SHA3-256 of the concatenation p1 || p2, absorbed byte by byte (no buffer).
struct Sha3 {
  uint64_t a[25];
  int pos;
  HASH_HD Sha3() : pos(0) {
    for (int i = 0; i < 25; ++i) a[i] = 0;
  }
  HASH_HD void absorb(const uint8_t* p, size_t len) {
    for (size_t i = 0; i < len; ++i) {
      a[pos >> 3] ^= (uint64_t)p[i] << (8 * (pos & 7));
      if (++pos == 136) {
        keccak_f(a);
        pos = 0;
      }
    }
  }
  HASH_HD void finish(uint8_t out[32]) {
    a[pos >> 3] ^= (uint64_t)0x06 << (8 * (pos & 7));
    a[135 >> 3] ^= (uint64_t)0x80 << (8 * (135 & 7));
    keccak_f(a);
    for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(a[i / 8] >> (8 * (i % 8)));
  }
};

HASH_HD void sha3_256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  Sha3 h;
  h.absorb(msg, len);
  h.finish(out);
}

// ------------------------------------------------------------------ rand 0.4 ChaChaRng
struct ChaCha04 {
  uint32_t state[16], buf[16];
  int index = 16;
  HASH_HD explicit ChaCha04(const uint32_t seed[8]) {
    state[0] = 0x61707865u;
    state[1] = 0x3320646eu;
    state[2] = 0x79622d32u;
    state[3] = 0x6b206574u;
    for (int i = 0; i < 8; ++i) state[4 + i] = seed[i];
    for (int i = 12; i < 16; ++i) state[i] = 0;
  }
  static HASH_HD uint32_t rotl(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }
  static HASH_HD void qr(uint32_t* s, int a, int b, int c, int d) {
    s[a] += s[b]; s[d] = rotl(s[d] ^ s[a], 16);
    s[c] += s[d]; s[b] = rotl(s[b] ^ s[c], 12);
    s[a] += s[b]; s[d] = rotl(s[d] ^ s[a], 8);
    s[c] += s[d]; s[b] = rotl(s[b] ^ s[c], 7);
  }
  HASH_HD void refill() {
    uint32_t s[16];
    for (int i = 0; i < 16; ++i) s[i] = state[i];
    for (int i = 0; i < 10; ++i) {
      qr(s, 0, 4, 8, 12); qr(s, 1, 5, 9, 13); qr(s, 2, 6, 10, 14); qr(s, 3, 7, 11, 15);
      qr(s, 0, 5, 10, 15); qr(s, 1, 6, 11, 12); qr(s, 2, 7, 8, 13); qr(s, 3, 4, 9, 14);
    }
    for (int i = 0; i < 16; ++i) buf[i] = s[i] + state[i];
    index = 0;
    for (int i = 12; i < 16; ++i)  // 128-bit block counter
      if (++state[i] != 0) break;
  }
  HASH_HD uint32_t next_u32() {
    if (index == 16) refill();
    return buf[index++];
  }
  HASH_HD uint64_t next_u64() {  // rand 0.4's default: the first word is the high half
    const uint64_t hi = next_u32();
    return (hi << 32) | next_u32();
  }
};

// ff_derive Rand for Fq: the drawn limbs are the Montgomery representation
HASH_HD void fq_rand(Fq& r, ChaCha04& rng) {
  for (;;) {
    uint64_t l[6];
    for (int i = 0; i < 6; ++i) l[i] = rng.next_u64();
    l[5] &= 0xffffffffffffffffull >> 3;
    for (int i = 0; i < 6; ++i) {
      r.v[2 * i] = (uint32_t)l[i];
      r.v[2 * i + 1] = (uint32_t)(l[i] >> 32);
    }
    if (limbs_lt_const<12>(r, FQ_P)) return;
  }
}

// One draw of G2::rand's loop: x, greatest, get_point_from_x.  False if x^3 + b is not a square
// (the loop draws again).
HASH_HD bool g2_rand_candidate(G2A& p, ChaCha04& rng) {
  Fq2 x;
  fq_rand(x.c0, rng);
  fq_rand(x.c1, rng);
  const bool greatest = (rng.next_u32() & 1u) != 0;
  Fq2 rhs, b, y;
  fq2_sqr(rhs, x);
  fq2_mul(rhs, rhs, x);
  fq2_set(b, G2_B);
  fq2_add(rhs, rhs, b);
  if (!fq2_sqrt(y, rhs)) return false;
  if (fq2_is_lex_largest(y) != greatest) fq2_neg(y, y);
  fq_canon(p.x.c0, x.c0);
  fq_canon(p.x.c1, x.c1);
  fq_canon(p.y.c0, y.c0);
  fq_canon(p.y.c1, y.c1);
  p.inf = 0;
  return true;
}

// pairing 0.14 G2::rand over the seeded ChaChaRng
void g2_rand(G2A& out, ChaCha04& rng) {
  for (;;) {
    G2A p;
    if (!g2_rand_candidate(p, rng)) continue;
    G2J q;
    g2_clear_cofactor(q, p);  // scale_by_cofactor (full h2, curve.h)
    if (jac_is_inf(q)) continue;
    jac_to_aff(out, q);
    return;
  }
}

void store_le_words(uint8_t* b, const uint32_t* w, int nwords) {
  for (int i = 0; i < nwords; ++i)
    for (int j = 0; j < 4; ++j) b[4 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

HASH_HD void seed_of_digest(const uint8_t d[32], uint32_t seed[8]) {
  for (int i = 0; i < 8; ++i)
    seed[i] = ((uint32_t)d[4 * i] << 24) | ((uint32_t)d[4 * i + 1] << 16) |
              ((uint32_t)d[4 * i + 2] << 8) | d[4 * i + 3];
}

void seed_of(const uint8_t* msg, size_t len, uint32_t seed[8]) {
  uint8_t d[32];
  sha3_256(msg, len, d);
  seed_of_digest(d, seed);
}

}  // namespace

void hash_g2_c96(const uint8_t* msg, size_t len, uint8_t* out96) {
  uint32_t seed[8];
  seed_of(msg, len, seed);
  ChaCha04 rng(seed);
  G2A h;
  g2_rand(h, rng);
  uint32_t w[24];
  g2_compress(w, h);
  store_le_words(out96, w, 24);  // little-endian words of the big-endian encoding
}

void g1_g2_message(const uint8_t* g1_c48, const uint8_t* msg, size_t len,
                   std::vector<uint8_t>& m) {
  if (len > 64) {
    m.resize(32);
    sha3_256(msg, len, m.data());
  } else {
    m.assign(msg, msg + len);
  }
  m.insert(m.end(), g1_c48, g1_c48 + 48);
}

void hash_g1_g2_c96(const uint8_t* g1_c48, const uint8_t* msg, size_t len, uint8_t* out96) {
  std::vector<uint8_t> m;
  g1_g2_message(g1_c48, msg, len, m);
  hash_g2_c96(m.data(), m.size(), out96);
}

// threshold_crypto's hash_bytes(g, len): ChaChaRng seeded with sha3_256(compressed g), one
// byte per draw (rand 0.4's u8: the low byte of next_u32).
void hash_bytes(const uint8_t* g1_c48, size_t len, uint8_t* out) {
  uint32_t seed[8];
  seed_of(g1_c48, 48, seed);
  ChaCha04 rng(seed);
  for (size_t i = 0; i < len; ++i) out[i] = (uint8_t)rng.next_u32();
}

// The first on-curve candidate of hash_g2(msg) (before [h2]); the GPU clears the cofactor.
void hash_g2_candidate(const uint8_t* msg, size_t len, G2A& p) {
  uint32_t seed[8];
  seed_of(msg, len, seed);
  ChaCha04 rng(seed);
  while (!g2_rand_candidate(p, rng)) {
  }
}

// Items [0, n) over the host's cores (a work counter; each item is independent).
void parallel_items(uint32_t n, const std::function<void(uint32_t)>& f) {
  uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
  if (const char* e = getenv("OMP_NUM_THREADS")) {  // the process's CPU share, when given
    const long v = strtol(e, nullptr, 10);
    if (v > 0) hw = std::min<uint32_t>(hw, (uint32_t)v);
  }
  const uint32_t nt = std::min<uint32_t>(std::min<uint32_t>(hw, 64u), n);
  std::atomic<uint32_t> next{0};
  auto worker = [&] {
    for (uint32_t i; (i = next.fetch_add(1)) < n;) f(i);
  };
  std::vector<std::thread> pool;
  for (uint32_t t = 1; t < nt; ++t) pool.emplace_back(worker);
  worker();
  for (auto& th : pool) th.join();
}

bool hash_offsets_ok(uint32_t n, const uint32_t* offsets) {
  if (offsets[0] != 0) return false;
  for (uint32_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i]) return false;
  return true;
}

// GPU candidates of hash_g2 / hash_g1_g2 (one lane per message): the seed, the ChaCha stream
// and G2::rand's draw loop before [h2] — the host path's code (k_g2_clear_cofactor finishes).
// g1_c48 != null: hash_g1_g2(u_i, v_i), the seed message (|v| > 64 ? sha3(v) : v) || u_i.
#ifndef HBTC_HASH_CAND_WAVES
#define HBTC_HASH_CAND_WAVES 2
#endif
// two waves per SIMD (256 VGPRs + spills; uncapped 256 + 61 AGPRs ran one)
__global__ void __launch_bounds__(64, HBTC_HASH_CAND_WAVES) k_hash_cand(uint32_t n, const uint8_t* __restrict__ g1_c48,
                                                  const uint8_t* __restrict__ msgs,
                                                  const uint32_t* __restrict__ offsets,
                                                  G2A* __restrict__ cand) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const uint8_t* v = msgs + offsets[i];
  const size_t len = offsets[i + 1] - offsets[i];
  uint8_t d[32];
  Sha3 h;
  if (g1_c48 && len > 64) {
    uint8_t inner[32];
    sha3_256(v, len, inner);
    h.absorb(inner, 32);
  } else {
    h.absorb(v, len);
  }
  if (g1_c48) h.absorb(g1_c48 + 48 * (size_t)i, 48);
  h.finish(d);
  uint32_t seed[8];
  seed_of_digest(d, seed);
  ChaCha04 rng(seed);
  G2A p;
  while (!g2_rand_candidate(p, rng)) {
  }
  cand[i] = p;
}

// The first n words of rand 0.4's ChaChaRng::from_seed(seed) on the device: the keystream code
// k_hash_cand runs, exposed for the ChaCha20 known-answer tests (tests/test_chacha_kat.py).
struct Seed8 {
  uint32_t w[8];
};
__global__ void __launch_bounds__(64) k_chacha04_words(Seed8 seed, uint32_t n, uint32_t* __restrict__ out) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  ChaCha04 rng(seed.w);
  for (uint32_t i = 0; i < n; ++i) out[i] = rng.next_u32();
}

hipError_t launch_chacha04_words(hipStream_t s, const uint32_t* seed8, uint32_t n, uint32_t* out) {
  if (n == 0) return hipSuccess;
  Seed8 sd;
  for (int i = 0; i < 8; ++i) sd.w[i] = seed8[i];
  hipLaunchKernelGGL(k_chacha04_words, dim3(1), dim3(64), 0, s, sd, n, out);
  return hipGetLastError();
}

hipError_t launch_hash_cand(hipStream_t s, uint32_t n, const uint8_t* g1_c48, const uint8_t* msgs,
                            const uint32_t* offsets, G2A* cand) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_hash_cand, dim3((n + 63) / 64), dim3(64), 0, s, n, g1_c48, msgs, offsets, cand);
  return hipGetLastError();
}

// bincode framing of wire points: item i = u64 LE length || `size` bytes.  Copies
// the point to the 16-aligned item array the verifiers read; a frame whose length is not
// `size` gets a zero compression flag, so the decoder reports HBTC_DECODE_ERR for it (serde
// refused the message).
__global__ void __launch_bounds__(64) k_unframe(uint32_t n, uint32_t size, const uint32_t* __restrict__ framed,
                                                uint32_t* __restrict__ items) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const uint32_t words = size / 4, stride = words + 2;
  const uint32_t* f = framed + (size_t)i * stride;
  const bool ok = f[0] == size && f[1] == 0u;
  uint32_t* o = items + (size_t)i * words;
  for (uint32_t w = 0; w < words; ++w) {
    uint32_t v = f[2 + w];
    if (w == 0 && !ok) v &= ~0x80u;  // first byte's compression flag
    o[w] = v;
  }
}

hipError_t launch_unframe(hipStream_t s, uint32_t n, uint32_t size, const uint8_t* framed, uint8_t* items) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_unframe, dim3((n + 63) / 64), dim3(64), 0, s, n, size,
                     reinterpret_cast<const uint32_t*>(framed), reinterpret_cast<uint32_t*>(items));
  return hipGetLastError();
}

// Host stage -> device workspace copy as a kernel on the caller's stream (the pinned stage is
// device-visible): a DMA-engine copy would queue behind copies of other streams that are still
// waiting on their own dependencies, stalling this stream with them.
__global__ void __launch_bounds__(256) k_stage_copy(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                    size_t n16, const uint8_t* __restrict__ src_b,
                                                    uint8_t* __restrict__ dst_b, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) dst[i] = src[i];
  const size_t tail = n - 16 * n16;
  if (i < tail) dst_b[16 * n16 + i] = src_b[16 * n16 + i];
}

hipError_t launch_stage_copy(hipStream_t s, const void* src, void* dst, size_t bytes) {
  if (bytes == 0) return hipSuccess;
  const size_t n16 = bytes / 16, work = n16 > 16 ? n16 : 16;
  hipLaunchKernelGGL(k_stage_copy, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s,
                     static_cast<const uint4*>(src), static_cast<uint4*>(dst), n16,
                     static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), bytes);
  return hipGetLastError();
}

// Zero n words on the caller's stream (the runtime's fill runs as a blit that can wait on other
// streams' work; this is an ordinary kernel of ours).
__global__ void __launch_bounds__(256) k_zero_u32(uint32_t* __restrict__ p, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = 0u;
}

hipError_t launch_zero_u32(hipStream_t s, uint32_t* p, size_t n) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_zero_u32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, n);
  return hipGetLastError();
}

// [h2] P for candidates P -> compressed G2 words; st = 1 if [h2] P = O (the host then continues
// G2::rand's loop itself).  Lane pairs (pair.h g2p_clear_cofactor): candidate i on lanes 2i,
// 2i + 1; the even lane assembles the affine point for the encoding.  One wave per SIMD: no
// scratch (two: 500 B/lane; the one-lane form kept 760 B at one); hash batches are small.
__global__ void __launch_bounds__(64, 1) k_g2_clear_cofactor(uint32_t n, const G2A* __restrict__ in,
                                                             uint32_t* __restrict__ out_w,
                                                             int32_t* __restrict__ st) {
  const uint32_t i = (blockIdx.x * 64 + threadIdx.x) >> 1;
  if (i >= n) return;  // pair-uniform
  G2Ap p;
  g2p_load_aff(p, in + i);
  G2Jp q;
  g2p_clear_cofactor(q, p);
  if (jac_is_inf(q)) {
    if (!pair_odd()) st[i] = 1;
    return;
  }
  G2Ap ap;
  jac_to_aff(ap, q);
  Fq px, py;
  fq_xchg(px, ap.x.v);
  fq_xchg(py, ap.y.v);
  if (pair_odd()) return;
  G2A a;
  a.x.c0 = ap.x.v;
  a.x.c1 = px;
  a.y.c0 = ap.y.v;
  a.y.c1 = py;
  a.inf = 0;
  uint32_t w[24];
  g2_compress(w, a);
  uint4* o = reinterpret_cast<uint4*>(out_w + 24 * (size_t)i);
  for (int k = 0; k < 6; ++k) o[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  st[i] = 0;
}

hipError_t launch_g2_clear_cofactor(hipStream_t s, uint32_t n, const G2A* in, uint8_t* out_c96,
                                    int32_t* st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_g2_clear_cofactor, dim3((2 * n + 63) / 64), dim3(64), 0, s, n, in,
                     reinterpret_cast<uint32_t*>(out_c96), st);
  return hipGetLastError();
}

}  // namespace hbtc

extern "C" {

int hbtc_sha3_256(const uint8_t* msg, size_t len, uint8_t* out32) {
  if ((!msg && len) || !out32) return HBTC_ERR_ARG;
  hbtc::sha3_256(msg, len, out32);
  return HBTC_OK;
}

int hbtc_hash_g2(const uint8_t* msg, size_t len, uint8_t* out_c96) {
  if ((!msg && len) || !out_c96) return HBTC_ERR_ARG;
  hbtc::hash_g2_c96(msg, len, out_c96);
  return HBTC_OK;
}

int hbtc_hash_g1_g2(const uint8_t* g1_c48, const uint8_t* msg, size_t len, uint8_t* out_c96) {
  if (!g1_c48 || (!msg && len) || !out_c96) return HBTC_ERR_ARG;
  hbtc::hash_g1_g2_c96(g1_c48, msg, len, out_c96);
  return HBTC_OK;
}

int hbtc_chacha04_words(const uint32_t* seed8, uint32_t n, uint32_t* out) {
  if (!seed8 || (!out && n)) return HBTC_ERR_ARG;
  hbtc::ChaCha04 rng(seed8);
  for (uint32_t i = 0; i < n; ++i) out[i] = rng.next_u32();
  return HBTC_OK;
}

int hbtc_hash_bytes(const uint8_t* g1_c48, size_t len, uint8_t* out) {
  if (!g1_c48 || (!out && len)) return HBTC_ERR_ARG;
  hbtc::hash_bytes(g1_c48, len, out);
  return HBTC_OK;
}

int hbtc_xor_hash_bytes_batch(uint32_t n, const uint8_t* g1_c48, const uint8_t* msgs,
                              const uint32_t* offsets, uint8_t* out) {
  if (n == 0) return HBTC_OK;
  if (!g1_c48 || !offsets || (!msgs && offsets[n]) || (!out && offsets[n]) ||
      !hbtc::hash_offsets_ok(n, offsets))
    return HBTC_ERR_ARG;
  hbtc::parallel_items(n, [&](uint32_t i) {
    const size_t len = offsets[i + 1] - offsets[i];
    uint8_t* o = out + offsets[i];
    hbtc::hash_bytes(g1_c48 + 48 * (size_t)i, len, o);
    for (size_t j = 0; j < len; ++j) o[j] ^= msgs[offsets[i] + j];
  });
  return HBTC_OK;
}

int hbtc_hash_g2_batch(uint32_t n, const uint8_t* msgs, const uint32_t* offsets,
                       uint8_t* out_c96) {
  if (n == 0) return HBTC_OK;
  if (!offsets || !out_c96 || (!msgs && offsets[n]) || !hbtc::hash_offsets_ok(n, offsets))
    return HBTC_ERR_ARG;
  hbtc::parallel_items(n, [&](uint32_t i) {
    hbtc::hash_g2_c96(msgs + offsets[i], offsets[i + 1] - offsets[i], out_c96 + 96 * (size_t)i);
  });
  return HBTC_OK;
}

int hbtc_hash_g1_g2_batch(uint32_t n, const uint8_t* g1_c48, const uint8_t* msgs,
                          const uint32_t* offsets, uint8_t* out_c96) {
  if (n == 0) return HBTC_OK;
  if (!g1_c48 || !offsets || !out_c96 || (!msgs && offsets[n]) || !hbtc::hash_offsets_ok(n, offsets))
    return HBTC_ERR_ARG;
  hbtc::parallel_items(n, [&](uint32_t i) {
    hbtc::hash_g1_g2_c96(g1_c48 + 48 * (size_t)i, msgs + offsets[i], offsets[i + 1] - offsets[i],
                         out_c96 + 96 * (size_t)i);
  });
  return HBTC_OK;
}

}  // extern "C"
