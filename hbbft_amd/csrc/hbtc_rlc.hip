// Random-linear-combination (RLC) batch verification of DecryptionShares with hierarchical
// fallback and single-error location — the fast path behind hbtc_verify_dec_shares
// (PublicKeyShare::verify_decryption_share, /root/reference/src/threshold_decryption.rs:159,
// called once per share by the reference).
//
// For a group G of shares of ONE ciphertext (u, v, w), H = hash_g1_g2(u, v), and
// E_i = e(d_i, H) / e(pk_i, w) (E_i == 1 iff share i is valid):
//     every share valid  =>  e(sum_G r_i d_i, H) * e(-sum_G r_i pk_i, w) == prod E_i^r_i == 1
// and, for r_i drawn uniformly from a set of 2^k scalars AFTER the shares are fixed (a ChaCha20
// stream under a fresh 256-bit host key per call; k = 128 by default, 64 optional), an invalid
// share makes the equation fail except with probability <= 2^-k per check (every point is in the
// prime-order subgroup: decode checks it, so E_i has order 1 or r).
//
// Single-error location.  Next to the plain sum the item pass also forms the position-weighted
// sum (weights p_i distinct in [0, |G|): p_i = bitrev_k(i) for share i of a group of 2^k, which
// the reduction tree forms with one doubling per level, rlc_common.h), so each group yields
//     T = prod E_i^r_i      and      T_w = prod E_i^(p_i r_i).
// If exactly one share b is wrong, T_w == T^(p_b): the search over p = 0..|G|-1 finds it with
// |G|-1 GT multiplications instead of per-share pairings, and the rest of the group is valid.
// With two or more wrong shares, T_w == T^p holds for some p only if prod_i E_i^(r_i (p_i - p))
// == 1 with a nonzero exponent on a wrong share, i.e. with probability <= 2^-k per p (the same
// argument as the plain check), <= |G| 2^-k per located group; such groups are split.
//
// This file holds the per-item pass (k_rlc_items: decode, r_i, the tile and sub-tile sums)
// and the final decision (k_rlc_finalize); the pairing-product checks of those sums run on
// the cooperative GT arithmetic in hbtc_check.hip:
//     k_chk_plain / k_chk_pair   plain (and weighted) checks of every 64-share tile; a failing
//                   tile with one wrong share is located right there, the others are listed
//     k_chk_split   listed tiles split in halves, quarters, eighths (left child checked, right
//                   child derived), single wrong shares located at every level
//     k_chk_leaves  the exact per-share check for eighths with >= 2 wrong shares
// Work per share in the honest case: decode + r_i d_i (the x-adic joint double-and-add, curve.h
// xadic_mul_uniform) + r_i pk_i (mixed additions from the key set's fixed-base table) + a share
// of the wave's reduction tree; the pairing work is per group.
#include "rlc_common.h"

#ifndef HBTC_PART
#define HBTC_PART 0
#endif
#define HBTC_IN_PART(n) (HBTC_PART == 0 || HBTC_PART == (n))

namespace hbtc {

#if HBTC_IN_PART(6)
// ------------------------------------------------------------------------------ per item
// One wave per tile: decode every share (the subgroup test yields [|x|] d on the way), draw the
// x-adic scalar r_i = d0 + d1 x + d2 mu + d3 mu x (four ChaCha20 digits of key.bits / 4 bits,
// mu = -x^2 the eigenvalue of phi: 2^key.bits distinct residues mod r, rlc_common.h), compute
// r_i d_i by one joint double-and-add over the digits' bits (curve.h xadic_mul_uniform) and
// r_i pk_i from the fixed-base table, then the plain and weighted group sums.  Items that cannot be checked (decode error, unknown sender) get their final status
// here and contribute the identity; a ciphertext whose own H / w failed to decode is resolved
// by k_rlc_finalize.  Needs nothing from the per-ciphertext preparation, so it runs
// concurrently with k_g2_prepare on another stream.
#ifndef HBTC_ITEMS_PRIO
#define HBTC_ITEMS_PRIO 0  // wave priority of the item pass (experiments: 3 = above the check levels)
#endif
#ifndef HBTC_SAC8_LDS
#define HBTC_SAC8_LDS 1  // three of the eight entries in LDS (the reduction's arrays, unused then)
#endif
#ifndef HBTC_ITEMS_WAVES
// minimum waves per SIMD the register allocation must allow (round 5, C3 shares/s: one wave with
// the whole 8-entry table in registers + AGPRs 11.7 M, two waves with the table partly spilled
// 13.4 M, profiles/r05/run1/)
#define HBTC_ITEMS_WAVES 2
#endif
// The item pass as two kernels: the decode half at three waves per SIMD (332 B/lane), the scalar
// half at two (its x-adic table) -- C3 13.6 -> 14.1 M shares/s against the single two-wave kernel
// (profiles/r05/run12/)
#ifndef HBTC_RLC_SPLIT
#define HBTC_RLC_SPLIT 1
#endif
#ifndef HBTC_RLC_DEC_WAVES
#define HBTC_RLC_DEC_WAVES 3
#endif
#if HBTC_RLC_SPLIT
// The decode half (HBTC_RLC_SPLIT): zcash G1 decode with the endomorphism subgroup test, whose
// first half [|x|] d is kept (t1) for the x-adic table; DECODE_ERR into status, everything else
// RLC_PENDING for k_rlc_items.
__global__ void __launch_bounds__(64, HBTC_RLC_DEC_WAVES) k_rlc_decode(
    const Tile* __restrict__ tiles, const uint32_t* __restrict__ idx, const uint8_t* __restrict__ shares,
    const int32_t* __restrict__ pk_status, uint32_t n_pk, G1A* __restrict__ dec, G1J* __restrict__ t1s,
    int32_t* __restrict__ status) {
  const Tile tile = tiles[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  if (lane >= tile.count) return;
  const size_t item = (size_t)tile.first + lane;
  const uint32_t id = idx[item];
  int32_t st = HBTC_RLC_PENDING;
  if (id < n_pk && pk_status[id] == HBTC_ACCEPT) {
    uint32_t w[12];
    rlc_load_words(w, shares, item, 12);
    G1A d;
    if (!g1_decompress(d, w, false)) {
      st = HBTC_DECODE_ERR;
    } else if (!d.inf) {
      // the subgroup test (curve.h g1_in_subgroup_t1) with its operands parked in the outputs:
      // d and t1 = [|x|] d go to memory as soon as they exist and d is read back for the final
      // comparison, so the second multiplication runs with only t1 live beside its accumulator
      // (332 -> 192 B/lane of scratch at three waves per SIMD)
      dec[item] = d;
      G1J t1, t2;
      jac_mul_u64(t1, d, BLS_X_ABS);
      t1s[item] = t1;
      jac_mul_u64_jac(t2, t1, BLS_X_ABS);  // [x^2] d
      __asm__ volatile("" ::: "memory");   // d is re-read, not kept in registers
      const G1A dd = dec[item];
      Fq bx, ny, beta;
      fq_set(beta, G1_BETA);
      fq_mul(bx, dd.x, beta);
      fq_neg(ny, dd.y);  // phi(d) == -[x^2] d  <=>  (beta x, -y) == [x^2] d
      if (jac_is_inf(t2) || !jac_eq_aff(t2, bx, ny)) st = HBTC_DECODE_ERR;
    } else {
      G1J t1;
      jac_set_inf(t1);
      dec[item] = d;
      t1s[item] = t1;
    }
  }
  status[item] = st;
}
#endif

__global__ void __launch_bounds__(64, HBTC_ITEMS_WAVES) k_rlc_items(
    const Tile* __restrict__ tiles, const uint32_t* __restrict__ idx,
    const uint8_t* __restrict__ shares, const G1A* __restrict__ pk,
    const int32_t* __restrict__ pk_status, const PtXY* __restrict__ pk_tab, uint32_t n_pk,
    RlcKey key, Suspects sus, TileSums* __restrict__ sums, G1A* __restrict__ dec,
    int32_t* __restrict__ status, const G1J* __restrict__ t1s) {
#if HBTC_ITEMS_PRIO > 0
  __builtin_amdgcn_s_setprio(HBTC_ITEMS_PRIO);
#endif
  // the reduction's two arrays, and before them the x-adic table's three LDS entries (18 KB:
  // 3 x 24 words x 64 lanes, curve.h xadic_mul_sac8<LDS3>): one wave per block, so the table
  // reads are over before the reduction writes
  __shared__ G1J red[128];
  G1J* redA = red;
  G1J* redB = red + 64;
  const Tile tile = tiles[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  const size_t item = (size_t)tile.first + lane;
  G1J S, P;
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
      G1A d;
      G1J t1;  // [|x|] d from the subgroup test: [x] d = -t1, the x-adic table's second entry
#if HBTC_RLC_SPLIT
      const bool dec_ok = status[item] != HBTC_DECODE_ERR;  // k_rlc_decode ran first
      if (dec_ok) {
        d = dec[item];
        t1 = t1s[item];
      }
#else
      uint32_t w[12];
      rlc_load_words(w, shares, item, 12);
      const bool dec_ok = g1_decompress_t1(d, t1, w);
#endif
      if (!dec_ok) {
        st = HBTC_DECODE_ERR;
      } else {
#if !HBTC_RLC_SPLIT
        dec[item] = d;  // for the exact leaf checks and the combine (no second decode)
#endif
        if (is_suspect(sus, id)) {
          st = HBTC_RLC_LEAF;  // straight to an exact check, outside the group sums
        } else {
          const XDigits xd = rlc_digits(key, item);
          if (!d.inf) {
            jac_neg(t1, t1);
            Fq beta;
            fq_set(beta, G1_BETA);
#if HBTC_XADIC8
#if HBTC_ITEMS_WAVES >= 2 && HBTC_SAC8_LDS
            xadic_mul_sac8<Fq, true>(S, d, t1, beta, xd.d[0], xd.d[1], xd.d[2], xd.d[3], xd.nbits,
                                     reinterpret_cast<uint32_t*>(red), lane);
#else
            xadic_mul_sac8(S, d, t1, beta, xd.d[0], xd.d[1], xd.d[2], xd.d[3], xd.nbits);
#endif
#else
            G1A xp, pxp;
            xadic_table(xp, pxp, d, t1);
            xadic_mul_uniform(S, d, xp, pxp, beta, xd.d[0], xd.d[1], xd.d[2], xd.d[3], xd.nbits);
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
  TileSums* ts = sums + blockIdx.x;
  rlc_reduce_sp(redA, redB, S, P, lane, ts->S, ts->SW, ts->P, ts->PW, ts->SH, ts->SHW, ts->PH,
                ts->PHW, ts->SQ, ts->SQW, ts->PQ, ts->PQW);
}
#endif  // part 6

#if HBTC_IN_PART(6)
// Every item still pending passed some group check: ACCEPT.  Items of a ciphertext whose own
// H / w failed to decode: INSTANCE_ERR.  With sender tracking on, the REJECTs of every sender
// are counted (k_track_update turns the counts into tracking stamps).
__global__ void __launch_bounds__(64) k_rlc_finalize(const Tile* __restrict__ tiles,
                                                     const int32_t* __restrict__ h_status,
                                                     const int32_t* __restrict__ w_status,
                                                     int32_t* __restrict__ status,
                                                     const uint32_t* __restrict__ idx, uint32_t n_pk,
                                                     uint32_t* __restrict__ rejects) {
  const Tile tile = tiles[blockIdx.x];
  if (threadIdx.x >= tile.count) return;
  const uint32_t i = tile.first + threadIdx.x;
  if (h_status[tile.inst] != HBTC_ACCEPT || w_status[tile.inst] != HBTC_ACCEPT) {
    status[i] = HBTC_INSTANCE_ERR;
  } else {
    const int32_t st = status[i];
    if (st == HBTC_RLC_PENDING) {
      status[i] = HBTC_ACCEPT;
    } else if (st == HBTC_REJECT && rejects) {
      const uint32_t id = idx[i];
      if (id < n_pk) atomicAdd(rejects + id, 1u);
    }
  }
}

// status `from` -> `to` (the pair checks run through the SignatureShare path: a Q that fails to
// decode is the item's own DECODE_ERR there, not an instance error)
__global__ void __launch_bounds__(256) k_status_remap(uint32_t n, int32_t* __restrict__ status,
                                                      int32_t from, int32_t to) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && status[i] == from) status[i] = to;
}

// A sender whose REJECTs in this call reach `thresh` (1/8 of the call's average shares per
// sender: a liar, not a sender hit by a stray corrupted share) is stamped with the call number;
// the counts are cleared for the next call.
__global__ void __launch_bounds__(256) k_track_update(uint32_t n_pk, uint32_t* __restrict__ rejects,
                                                      uint32_t* __restrict__ last_bad, uint32_t now,
                                                      uint32_t thresh) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_pk) return;
  const uint32_t r = rejects[i];
  if (r == 0) return;
  if (r >= thresh) last_bad[i] = now;
  rejects[i] = 0;
}
#endif  // part 6

// ------------------------------------------------------------------------------ launchers
static inline uint32_t rlc_blocks(uint64_t n, uint32_t bs) { return (uint32_t)((n + bs - 1) / bs); }

#if HBTC_IN_PART(6)
bool rlc_items_split() { return HBTC_RLC_SPLIT != 0; }
hipError_t launch_rlc_items(hipStream_t s, uint32_t n_tiles, const Tile* tiles, const uint32_t* idx,
                            const uint8_t* shares, const G1A* pk, const int32_t* pk_status,
                            const PtXY* pk_tab, uint32_t n_pk, RlcKey key, Suspects sus,
                            TileSums* sums, G1A* dec, int32_t* status, G1J* t1s,
                            hipEvent_t after_decode) {
  if (n_tiles == 0) return hipSuccess;
#if HBTC_RLC_SPLIT
  hipLaunchKernelGGL(k_rlc_decode, dim3(n_tiles), dim3(64), 0, s, tiles, idx, shares, pk_status, n_pk,
                     dec, t1s, status);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (after_decode && (e = hipEventRecord(after_decode, s)) != hipSuccess) return e;
#endif
  hipLaunchKernelGGL(k_rlc_items, dim3(n_tiles), dim3(64), 0, s, tiles, idx, shares, pk, pk_status,
                     pk_tab, n_pk, key, sus, sums, dec, status, t1s);
  return hipGetLastError();
}
hipError_t launch_rlc_finalize(hipStream_t s, uint32_t n_tiles, const Tile* tiles,
                               const int32_t* h_status, const int32_t* w_status, int32_t* status,
                               const uint32_t* idx, uint32_t n_pk, uint32_t* rejects,
                               uint32_t* last_bad, uint32_t now, uint32_t thresh) {
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rlc_finalize, dim3(n_tiles), dim3(64), 0, s, tiles, h_status, w_status,
                     status, idx, n_pk, last_bad ? rejects : nullptr);
  if (last_bad)
    hipLaunchKernelGGL(k_track_update, dim3(rlc_blocks(n_pk, 256)), dim3(256), 0, s, n_pk, rejects,
                       last_bad, now, thresh);
  return hipGetLastError();
}
hipError_t launch_status_remap(hipStream_t s, uint32_t n, int32_t* status, int32_t from, int32_t to) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_status_remap, dim3(rlc_blocks(n, 256)), dim3(256), 0, s, n, status, from, to);
  return hipGetLastError();
}
#endif  // part 6

}  // namespace hbtc
