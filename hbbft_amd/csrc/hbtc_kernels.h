// Launch interface between the C-ABI host code (hbtc_api.hip) and the gfx950 kernels
// (hbtc_kernels.hip).  Every launcher enqueues on `s` and returns hipGetLastError().
#pragma once
#include <hip/hip_runtime.h>

#include "hbtc.h"
#include "pairing.h"

namespace hbtc {

// Up to 64 consecutive items of ONE instance: one wave (workgroup) per tile, so the
// instance's line tables are read with wave-uniform loads.
struct Tile {
  uint32_t inst, first, count, pad;
};
constexpr uint32_t TILE_ITEMS = 64;

// ---- RLC batch verification (hbtc_rlc.hip)
constexpr int32_t HBTC_RLC_PENDING = -1;  // internal: decided by a group check or a leaf check
constexpr int32_t HBTC_RLC_LEAF = -2;     // internal: a tracked sender's share, listed for a leaf check
// Sender tracking (hbtc.h hbtc_set_sender_tracking): a sender with many shares REJECTed (>= 1/8
// of the call's average shares per sender) in one of the last SUSPECT_WINDOW calls on a key set
// is tracked; its shares skip the group sums and go
// straight to the exact leaf checks, so f Byzantine senders who lie in every epoch no longer
// make every tile and sub-tile of the honest shares fail.  Decisions are unchanged (every share
// still gets an exact verdict); only the work differs.
constexpr uint32_t SUSPECT_WINDOW = 16;
struct Suspects {
  const uint32_t* last_bad;  // per sender: the call number of its last REJECT (0 = none); null = off
  uint32_t now;              // this call's number (>= 1)
  uint32_t* leaf_count;      // the leaf list the item pass appends tracked shares to
  uint32_t* leaves;
  uint32_t all;              // every share to the leaf list (a small call's exact checks)
};
__device__ __forceinline__ bool is_suspect(const Suspects& s, uint32_t id) {
  if (s.all) return true;
  if (!s.last_bad) return false;
  const uint32_t b = s.last_bad[id];
  return b != 0 && s.now - b <= SUSPECT_WINDOW;
}
struct RlcKey {
  uint32_t k[8];  // ChaCha20 key, fresh from the host's random source for every call
  uint32_t bits;  // 128 (default): four 32-bit x-adic digits (rlc_common.h); 64: 16-bit digits
};
// Partial sums of one tile: [0..7] the 8-share sub-tiles, [8] the whole tile.  The weighted
// sums carry the position of every share inside its group (0..7 in a sub-tile, 0..63 in the
// tile): they locate a single wrong share without per-share pairings (hbtc_rlc.hip).
struct TileSums {
  G1J S[9];   // sum r_i d_i
  G1J P[9];   // sum r_i pk_i
  G1J SW[9];  // sum pos_i r_i d_i
  G1J PW[9];  // sum pos_i r_i pk_i
  // the two 32-share halves (weights = position inside the half): the level between a failing
  // tile and its sub-tiles in the plain-first schedule (hbtc_check.hip)
  G1J SH[2], SHW[2], PH[2], PHW[2];
  // the LEFT 16-share quarter of each half (quarters 0 and 2): the split levels check a listed
  // node's left child and derive the right one (hbtc_check.hip k_chk_split)
  G1J SQ[2], SQW[2], PQ[2], PQW[2];
};

// Partial sums of one tile of SignatureShares (hbtc_sig.hip): S = sum r_i sigma_i in G2 and
// P = sum r_i pk_i in G1, plain and position-weighted, [0..7] sub-tiles and [8] the tile.
struct SigTileSums {
  G2J S[9];
  G2J SW[9];
  G1J P[9];
  G1J PW[9];
};
// Projective line table of a G2 point (pairing.h g2_proj_lines): 3 Fq2 per Miller step.
constexpr uint32_t PLINES_FQ2 = 3 * MILLER_STEPS;

// Fixed-base table of every public-key share (built once per key set, resident in HBM):
// tab[(i * PK_TAB_WIN + w) * 256 + v] = v * 2^(8w) * pk_i for w < 4 and v * 2^(8(w-4)) * [x] pk_i
// for w >= 4 (affine, v >= 1), so the x-adic RLC scalar's r_i pk_i (rlc_common.h rlc_pk_mul_x)
// is 4 nbits / 8 mixed additions and no doublings (16 for 128-bit scalars, 8 for 64-bit).
constexpr int PK_TAB_WIN = 8;
// windows the scalar halves of an RLC call use
__host__ __device__ constexpr int rlc_windows(uint32_t bits) { return bits == 128 ? 8 : 4; }
struct PtXY {
  Fq x, y;
};

hipError_t launch_pk_table(hipStream_t s, const G1A* pk, const int32_t* pk_status, uint32_t n,
                           PtXY* tab, Fq* ws);
// split item pass (k_rlc_decode + k_rlc_items): t1s is n_items G1J of workspace ([|x|] d)
bool rlc_items_split();
hipError_t launch_rlc_items(hipStream_t s, uint32_t n_tiles, const Tile* tiles, const uint32_t* idx,
                            const uint8_t* shares, const G1A* pk, const int32_t* pk_status,
                            const PtXY* pk_tab, uint32_t n_pk, RlcKey key, Suspects sus,
                            TileSums* sums, G1A* dec, int32_t* status, G1J* t1s,
                            hipEvent_t after_decode = nullptr);
// Final decisions; with last_bad != null, counts every sender's REJECTs in `rejects` and stamps
// last_bad[i] = now for the senders with >= thresh of them (clearing the counts).
hipError_t launch_status_remap(hipStream_t s, uint32_t n, int32_t* status, int32_t from, int32_t to);
hipError_t launch_rlc_finalize(hipStream_t s, uint32_t n_tiles, const Tile* tiles,
                               const int32_t* h_status, const int32_t* w_status, int32_t* status,
                               const uint32_t* idx, uint32_t n_pk, uint32_t* rejects,
                               uint32_t* last_bad, uint32_t now, uint32_t thresh);
// the pairing-product checks (hbtc_check.hip, cooperative GT arithmetic of gt6.h)
// Group checks, plain first (hbtc_check.hip): level 0 = tiles (n_direct groups), level 1 =
// the 8 sub-tiles of the *n_listed tiles of sub_list.  The plain pass stores a failing group's
// T (6 Fq2 at Tbuf[6 g]) and lists g; the weighted pass locates a single wrong share, else
// lists the tile (level 0, out_list = sub_list) or the group's pending shares (level 1,
// out_list = leaves as (item, instance) pairs).
hipError_t launch_chk_plain(hipStream_t s, int level, uint32_t max_groups, uint32_t n_direct,
                            const uint32_t* n_listed, const uint32_t* sub_list,
                            const uint32_t* list2, const Tile* tiles, const TileSums* sums,
                            const G2A* h_aff, const Line* h_lines, const G2A* w_aff,
                            const Line* w_lines, const int32_t* h_status, const int32_t* w_status,
                            Fq2* Tbuf, uint32_t* fail_count, uint32_t* fail_list);
hipError_t launch_chk_halves(hipStream_t s, uint32_t max_tiles, const uint32_t* n_listed,
                             const uint32_t* tile_list, const Tile* tiles, const TileSums* sums,
                             const G2A* h_aff, const Line* h_lines, const G2A* w_aff,
                             const Line* w_lines, const Fq2* Ttile, Fq2* Thalf,
                             uint32_t* fail_count, uint32_t* fail_list);
// The list a split level appends to (hbtc_check.hip k_chk_split): node codes (tile << 3 | node
// index at the node's size), the node's GT values T and U (6 Fq2 each per entry) and its weight
// form ab = log2(alpha) | beta << 8.  list == nullptr: no split listing (the older levels).
struct SplitOut {
  uint32_t* count;
  uint32_t* list;
  Fq2* T;
  Fq2* U;
  uint32_t* ab;
};
hipError_t launch_chk_weighted(hipStream_t s, int level, uint32_t max_groups,
                               const uint32_t* fail_count, const uint32_t* fail_list,
                               const uint32_t* sub_list, const uint32_t* list2, const Tile* tiles,
                               const TileSums* sums, const G2A* h_aff, const Line* h_lines,
                               const G2A* w_aff, const Line* w_lines, const int32_t* h_status,
                               const int32_t* w_status, const Fq2* Tbuf, int32_t* status,
                               uint32_t* out_count, uint32_t* out_list, SplitOut split);
hipError_t launch_chk_pair(hipStream_t s, int level, bool to_leaves, uint32_t max_groups,
                           uint32_t n_direct, const uint32_t* n_listed, const uint32_t* sub_list,
                           const Tile* tiles, const TileSums* sums, const G2A* h_aff,
                           const Line* h_lines, const G2A* w_aff, const Line* w_lines,
                           const int32_t* h_status, const int32_t* w_status, int32_t* status,
                           uint32_t* out_count, uint32_t* out_list, SplitOut split);
// Split level `level` (1..3) over the *n_in listed nodes: checks each node's left child, derives
// the right one, locates single wrong shares in both, lists unresolved children into `split`
// (level 3: their pending shares to the leaf list).
// rep = 3: the latency form (18-lane groups, one unit per wave: gt6.h Pos.rep) for levels too
// small to fill the chip; rep = 1: the throughput form.
hipError_t launch_chk_split(hipStream_t s, int level, int rep, uint32_t max_nodes,
                            const uint32_t* n_in, const uint32_t* in_list, const Fq2* in_T,
                            const Fq2* in_U, const uint32_t* in_ab, const Tile* tiles,
                            const TileSums* sums, const G2A* h_aff, const Line* h_lines,
                            const G2A* w_aff, const Line* w_lines, int32_t* status,
                            uint32_t* leaf_count, uint32_t* leaves, SplitOut split);
// Leaf checks: the latency form takes a list of at most rep3_limit leaves, the throughput form
// a longer one (both launched; the count is on the device).  rep3_limit = 0: throughput only.
hipError_t launch_chk_leaves_rep3(hipStream_t s, uint32_t max_leaves, uint32_t rep3_limit,
                                  const uint32_t* leaf_count, const uint32_t* leaves,
                                  const uint32_t* idx, const G1A* dec, const G1A* pk,
                                  const G2A* h_aff, const Line* h_lines, const G2A* w_aff,
                                  const Line* w_lines, int32_t* status);
hipError_t launch_chk_leaves(hipStream_t s, uint32_t max_leaves, const uint32_t* leaf_count,
                             const uint32_t* leaves, const uint32_t* idx, const G1A* dec,
                             const G1A* pk, const G2A* h_aff, const Line* h_lines,
                             const G2A* w_aff, const Line* w_lines, int32_t* status,
                             uint32_t rep3_limit = 0);

// ---- RLC batch verification of SignatureShares (hbtc_sig.hip, checks in hbtc_check.hip)
hipError_t launch_sig_items(hipStream_t s, uint32_t n_tiles, const Tile* tiles, const uint32_t* idx,
                            const uint8_t* sigs, const G1A* pk, const int32_t* pk_status,
                            const PtXY* pk_tab, uint32_t n_pk, RlcKey key, Suspects sus,
                            SigTileSums* sums, G2A* dec, int32_t* status);
// Projective line tables of the G2 sums the next check level needs: mode 0 every tile
// (2 per tile: plain, weighted), mode 1 the 8 sub-tiles of the listed tiles (16 per listed
// tile), mode 2 the listed leaf shares (decoded sigma).  inf[g] = 1: the sum is infinity.
// (mode 2 handles leaves [base, base + max_groups) of the list: chunks bound the tables)
// The exact small-call path of SignatureShares (and pair checks) in one launch (hbtc_sig.hip
// k_sig_exact): decode, leaf listing of every decodable share of a known sender, its projective
// line table at its leaf position, the psi subgroup test at the end of the line walk.  Tables
// must hold n items.  hipErrorNotSupported when built without the lane-pair kernels.
bool sig_exact_built();
hipError_t launch_sig_exact(hipStream_t s, uint32_t n, const uint32_t* idx, const uint8_t* sigs,
                            const int32_t* pk_status, uint32_t n_pk, const Tile* tiles, uint32_t n_tiles,
                            uint32_t* leaf_count, uint32_t* leaves, G2A* dec, Fq2* tables, uint32_t* inf,
                            int32_t* status);
hipError_t launch_plines(hipStream_t s, int mode, uint32_t max_groups, uint32_t base,
                         const uint32_t* count, const uint32_t* list, const Tile* tiles,
                         const SigTileSums* sums, const G2A* dec, Fq2* tables, uint32_t* inf);
hipError_t launch_sigchk_tiles(hipStream_t s, uint32_t n_tiles, const Tile* tiles,
                               const SigTileSums* sums, const Fq2* tables, const uint32_t* inf,
                               const G2A* h_aff, const Line* h_lines, const int32_t* h_status,
                               int32_t* status, uint32_t* sub_count, uint32_t* sub_list,
                               bool to_leaves);
hipError_t launch_sigchk_subs(hipStream_t s, uint32_t max_tiles, const uint32_t* sub_count,
                              const uint32_t* sub_list, const Tile* tiles,
                              const SigTileSums* sums, const Fq2* tables, const uint32_t* inf,
                              const G2A* h_aff, const Line* h_lines, int32_t* status,
                              uint32_t* leaf_count, uint32_t* leaves);
hipError_t launch_sigchk_leaves(hipStream_t s, uint32_t base, uint32_t chunk,
                                const uint32_t* leaf_count, const uint32_t* leaves,
                                const uint32_t* idx, const G1A* pk, const Fq2* tables,
                                const uint32_t* inf, const G2A* h_aff, const Line* h_lines,
                                int32_t* status, uint32_t rep3_limit = 0);
// the latency form (rep 3) of the SignatureShare tile checks and of a short leaf list
hipError_t launch_sigchk_tiles_rep3(hipStream_t s, uint32_t n_tiles, const Tile* tiles,
                                    const SigTileSums* sums, const Fq2* tables, const uint32_t* inf,
                                    const G2A* h_aff, const Line* h_lines, const int32_t* h_status,
                                    int32_t* status, uint32_t* sub_count, uint32_t* sub_list,
                                    bool to_leaves);
hipError_t launch_sigchk_leaves_rep3(hipStream_t s, uint32_t chunk, uint32_t rep3_limit,
                                     const uint32_t* leaf_count, const uint32_t* leaves,
                                     const uint32_t* idx, const G1A* pk, const Fq2* tables,
                                     const uint32_t* inf, const G2A* h_aff, const Line* h_lines,
                                     int32_t* status);

hipError_t launch_g1_decode(hipStream_t s, const uint8_t* in, uint32_t n, G1A* out,
                            int32_t* status);
// Decode + affine-normalised line tables of n0 + n1 G2 arguments (two input arrays, outputs
// contiguous); ws holds 3 * MILLER_STEPS Fq2 per argument.
// Copy prepared G2 tables entry by entry between slot arrays (ss / ds null: identity).
hipError_t launch_g2_tab_copy(hipStream_t s, uint32_t n, const uint32_t* ss, const uint32_t* ds, const G2A* saff,
                              const int32_t* sst, const Line* sl, G2A* daff, int32_t* dst, Line* dl);
hipError_t launch_g2_prepare(hipStream_t s, const uint8_t* in0, uint32_t n0, const uint8_t* in1,
                             uint32_t n1, G2A* aff, Line* lines, Fq2* ws, int32_t* status);
// ---- pair batches e(A_i, Q_i) == e(G1, W_i) by RLC (hbtc_pb.hip, checks in hbtc_check.hip)
// items: decode A (null: the G1 generator), Q (q_trusted: no subgroup check), W; r_i A_i (affine)
// -> rA, decoded Q -> Qdec, the plain sums of r_i W_i per 64-item tile and 8-item sub-tile (S[]
// of SigTileSums), statuses PENDING / DECODE_ERR
hipError_t launch_pb_gather(hipStream_t s, uint32_t n, const uint32_t* list, const uint8_t* a,
                            const uint8_t* q, const uint8_t* w, uint8_t* ga, uint8_t* gq, uint8_t* gw);
hipError_t launch_pb_scatter(hipStream_t s, uint32_t n, const uint32_t* list, const int32_t* gst,
                             int32_t* st);
hipError_t launch_pb_items(hipStream_t s, uint32_t n, const uint8_t* a_c48, const uint8_t* q_c96,
                           bool q_trusted, const uint8_t* w_c96, RlcKey key, G1A* rA, G2A* Qdec,
                           G2A* Wdec, SigTileSums* sums, int32_t* status, G1A* adec = nullptr);
// r_i W_i of the PENDING items and the tile / sub-tile sums S, on lane pairs (hbtc_sig.hip; the
// second launch of launch_pb_items)
hipError_t launch_pb_wsum(hipStream_t s, uint32_t n, RlcKey key, const G2A* wdec, const int32_t* status,
                          SigTileSums* sums);
// g_i = [k0 + k1 x^2] A_i (compressed) for the ACCEPTed items, zero bytes for the others
hipError_t launch_pb_mul_glv(hipStream_t s, uint32_t n, const G1A* adec, const int32_t* status,
                             const uint32_t* k0, const uint32_t* k1, uint8_t* out_c48);
// projective line tables (PLINES_FQ2 per item) of the pending items' Q
hipError_t launch_pb_lines(hipStream_t s, uint32_t n, const G2A* Qdec, const int32_t* status,
                           Fq2* tables);
// partial Miller products of the 8-item sub-tiles (6 Fq2 per sub-tile into fbuf)
hipError_t launch_pb_ml(hipStream_t s, uint32_t n_items, const G1A* rA, const Fq2* qtab,
                        const int32_t* status, Fq2* fbuf);
// group checks from the partials: level 0 every tile (n_direct), level 1 the 8 sub-tiles of the
// *n_listed tiles of list; failing tiles -> out_list (level 0), failing sub-tiles' pending items
// -> out_list (level 1)
hipError_t launch_pb_fe(hipStream_t s, int level, uint32_t max_groups, uint32_t n_items,
                        uint32_t n_direct, const uint32_t* n_listed, const uint32_t* list,
                        const Fq2* fbuf, const Fq2* wtab, const uint32_t* winf, int32_t* status,
                        uint32_t* out_count, uint32_t* out_list);
// k_i P_i; base_stride / scalar_stride 0 = one base / scalar for every item
hipError_t launch_point_mul(hipStream_t s, int group, uint32_t n, const uint8_t* base,
                            uint32_t base_stride, const uint8_t* scalars, uint32_t scalar_stride,
                            uint8_t* out, int32_t* status);

// ---- batched Pippenger MSM + Lagrange combine (hbtc_msm.hip)
// n_msm MSMs of n terms each; signed c-bit digits over W = ceil(256 / c) windows, 2^(c-1)
// buckets per window in segments of 8 (c >= 4).
struct MsmPlan {
  uint32_t n_msm, n, c, W;
};
hipError_t launch_select(hipStream_t s, uint32_t n_inst, const uint32_t* offsets, uint32_t t,
                         const int32_t* status, const uint32_t* idx, uint32_t* sel_pos,
                         uint32_t* sel_idx, uint32_t* sel_cnt);
// Lagrange through factorial tables (hbtc_msm.hip k_lagrange_fact): fact / inv_fact of 0..n
// (Montgomery), the selection counts, and a per-instance flag the fallback kernels skip
struct LagrangeFact {
  const Fr* fact;
  const Fr* inv_fact;
  uint32_t n;
  const uint32_t* sel_cnt;
  uint32_t* done;
};
hipError_t launch_fact_tables(hipStream_t s, uint32_t n, Fr* part, Fr* fact, Fr* inv_fact);
// lambda: n_inst * t canonical coefficients; ws: n_inst * t Fr of workspace; lf: null = the O(t)
// per term kernels for every instance
hipError_t launch_lagrange_sel(hipStream_t s, uint32_t n_inst, uint32_t t, const uint32_t* sel_idx,
                               Fr* lambda, Fr* ws, uint32_t* dup, const LagrangeFact* lf = nullptr);
hipError_t launch_msm_digits(hipStream_t s, const MsmPlan& p, const uint32_t* scalars,
                             int16_t* digits, uint32_t* list, uint32_t* roff);
hipError_t launch_msm_gather_g1(hipStream_t s, uint32_t n_inst, uint32_t t, const uint32_t* sel_pos,
                                const uint32_t* sel_cnt, const G1A* dec, G1A* pts);
hipError_t launch_msm_gather_g2(hipStream_t s, uint32_t n_inst, uint32_t t, const uint32_t* sel_pos,
                                const uint32_t* sel_cnt, const G2A* dec, G2A* pts);
// G2 combine terms (lambda [n_msm][n] canonical, pts [n_msm][n]) -> 4n GLS terms per msm with
// 64-bit scalars (sc4: 8 words each) and the points P, [u]P, [u^2]P, [u^3]P (hbtc_msm.hip)
hipError_t launch_msm_gls_g2(hipStream_t s, uint32_t n_msm, uint32_t n, const uint32_t* lambda,
                             const G2A* pts, uint32_t* sc4, G2A* pts4);
// G1 combine terms -> 2n GLV terms per msm with 128-bit scalars: P, [u^2]P = -φ(P)
hipError_t launch_msm_glv_g1(hipStream_t s, uint32_t n_msm, uint32_t n, const uint32_t* lambda,
                             const G1A* pts, uint32_t* sc2, G1A* pts2);
hipError_t launch_msm_decode_g1(hipStream_t s, uint32_t n_msm, uint32_t n, uint32_t stride,
                                const uint8_t* pts_c, const uint32_t* sel_pos,
                                const uint32_t* sel_cnt, const int32_t* item_status,
                                const G1A* dec, G1A* pts, uint32_t* bad);
hipError_t launch_msm_reduce_g1(hipStream_t s, const MsmPlan& p, const G1A* pts,
                                const uint32_t* pts_map, const uint32_t* list, const uint32_t* roff, G1J* part, G1J* wsum,
                                const uint32_t* sel_cnt, uint32_t t, const uint32_t* bad,
                                const uint32_t* dup, int32_t* status, uint8_t* out);
hipError_t launch_msm_decode_g2(hipStream_t s, uint32_t n_msm, uint32_t n, uint32_t stride,
                                const uint8_t* pts_c, const uint32_t* sel_pos,
                                const uint32_t* sel_cnt, const int32_t* item_status,
                                const G2A* dec, G2A* pts, uint32_t* bad);
hipError_t launch_msm_reduce_g2(hipStream_t s, const MsmPlan& p, const G2A* pts,
                                const uint32_t* pts_map, const uint32_t* list, const uint32_t* roff, G2J* part, G2J* wsum,
                                const uint32_t* sel_cnt, uint32_t t, const uint32_t* bad,
                                const uint32_t* dup, int32_t* status, uint8_t* out,
                                uint8_t* parity);

// ---- small combines, t <= COMB_SMALL_T shares per instance, one workgroup each (hbtc_comb.hip)
constexpr uint32_t COMB_SMALL_T = 64;
constexpr uint32_t COMB_SMALL_BS = 128;  // two lanes per selected share
struct CombSmallArgs {
  uint32_t t;
  const uint32_t* offsets;     // CSR instances over the items
  const int32_t* item_status;  // null: the first t items; else the first t ACCEPTed ones
  const uint32_t* idx;         // node index per item (x = idx + 1)
  const uint8_t* pts;          // compressed items (48 / 96 B)
  const void* dec;             // decoded items (Aff<F>*, used for ACCEPTed items) or null; by_node: per node
  uint32_t by_node;            // points are dec[idx[item]] (a key set's resident pk), never decoded
  uint32_t n_nodes;            // by_node: entries of dec (an idx past it counts as a decode error)
  int32_t* inst_status;        // per output slot (instance k, subset j: k * n_sub + j)
  uint8_t* out;                // compressed sums per slot (unused with cmp)
  uint8_t* parity;             // G2 Signature::parity per slot, or null
  const void* cmp;             // Aff<F>*: compare the sum with it (status ACCEPT / REJECT) instead of encoding
  const uint32_t* only;        // per instance: run only where only[k] != 0 (null: all)
  const PtXY* xtab;            // by_node, G1: the key set's fixed-base table, whose entry
                               // (node * PK_TAB_WIN + 4) * 256 + 1 is [x] pk (so [u] pk = -it is
                               // free instead of 64 doublings); null: computed
  uint32_t nocheck;            // decode without the subgroup test: speculative subsets, whose
                               // sums are kept only when every item passed the verification's
                               // full decode (k_coin_commit)
};
// group 1: G1 (DecryptionShares, key-set pk), 2: G2 (SignatureShares).  n_sub > 1: speculative
// subsets, block (k, j) leaves out instance k's j-th item
hipError_t launch_comb_small(hipStream_t s, int group, uint32_t n_inst, uint32_t n_sub,
                             const CombSmallArgs& a);
hipError_t launch_coin_commit(hipStream_t s, uint32_t n_inst, uint32_t t, const uint32_t* offsets,
                              const int32_t* item_status, uint32_t n_sub, const int32_t* spec_cst,
                              const uint8_t* spec_sig, const uint8_t* spec_par,
                              const int32_t* spec_master, int32_t* cst, uint8_t* sig, uint8_t* par,
                              int32_t* master, uint32_t* redo);

// ---- SyncKeyGen (hbtc_skg.hip)
hipError_t launch_skg_sym_scalars(hipStream_t s, uint32_t n_parts, uint32_t M, const Fr* U,
                                  uint32_t u_stride, const Fr* V, uint32_t v_stride,
                                  const uint32_t* ij, const Fr* tail, Fr* out);
hipError_t launch_skg_ack_rows(hipStream_t s, uint32_t n_acks, uint32_t t1, const Fr* rows,
                               const uint32_t* ack_part, const uint32_t* ack_sender,
                               const Fr* vals, int32_t* status);


// ---- Reliable Broadcast (hbtc_bcast.hip)
hipError_t launch_gf_apply(hipStream_t s, uint32_t n_jobs, const uint32_t* jobs, uint8_t* shards,
                           uint64_t stride, uint32_t len, uint32_t n_out, const uint32_t* out_rows,
                           uint32_t n_in, const uint32_t* in_rows, const uint32_t* tabs);
hipError_t launch_merkle_tree(hipStream_t s, uint32_t n_inst, uint32_t n, uint32_t leaf_len,
                              const uint8_t* leaves, uint64_t stride, uint32_t n_dig, uint8_t* out);
hipError_t launch_merkle_validate(hipStream_t s, uint32_t n, uint32_t n_nodes, const uint64_t* voff,
                                  const uint8_t* values, const uint32_t* idx, const uint32_t* doff,
                                  const uint8_t* digests, const uint8_t* roots, int32_t* status);

}  // namespace hbtc
