// C ABI of the batched threshold-crypto verifier (include/hbtc.h): context, resident key
// tables, workspaces, batch shaping (tiles) and kernel timing.  Device work lives in
// hbtc_kernels.hip.  Every entry point validates its arguments and fails loudly (negative
// return + hbtc_last_error) — there is no CPU fallback anywhere in the product path.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "hbtc_kernels.h"

using namespace hbtc;

#include <functional>

namespace hbtc {
// hbtc_hash.hip: host hash_g2 pieces + the GPU cofactor clearing
void hash_g2_c96(const uint8_t* msg, size_t len, uint8_t* out96);
void g1_g2_message(const uint8_t* g1_c48, const uint8_t* msg, size_t len, std::vector<uint8_t>& m);
void hash_g2_candidate(const uint8_t* msg, size_t len, G2A& p);
void hash_g1_g2_c96(const uint8_t* g1_c48, const uint8_t* msg, size_t len, uint8_t* out96);
hipError_t launch_hash_cand(hipStream_t s, uint32_t n, const uint8_t* g1_c48, const uint8_t* msgs,
                            const uint32_t* offsets, G2A* cand);
hipError_t launch_chacha04_words(hipStream_t s, const uint32_t* seed8, uint32_t n, uint32_t* out);
hipError_t launch_unframe(hipStream_t s, uint32_t n, uint32_t size, const uint8_t* framed, uint8_t* items);
hipError_t launch_stage_copy(hipStream_t s, const void* src, void* dst, size_t bytes);
hipError_t launch_zero_u32(hipStream_t s, uint32_t* p, size_t n);
void hash_bytes(const uint8_t* g1_c48, size_t len, uint8_t* out);
void parallel_items(uint32_t n, const std::function<void(uint32_t)>& f);
bool hash_offsets_ok(uint32_t n, const uint32_t* offsets);
hipError_t launch_g2_clear_cofactor(hipStream_t s, uint32_t n, const G2A* in, uint8_t* out_c96,
                                    int32_t* st);
}  // namespace hbtc

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

struct Keyset {
  G1A* pk = nullptr;
  int32_t* st = nullptr;
  PtXY* tab = nullptr;  // fixed-base tables (n * PK_TAB_WIN * 256 points, ~196 KB per share)
  uint32_t* last_bad = nullptr;  // sender tracking: the call that last flagged each sender
  uint32_t* rejects = nullptr;   // per-sender REJECT counts of the running call
  uint32_t calls = 0;            // RLC verification calls on this key set
  uint32_t n = 0;
  G1A* master = nullptr;         // hbtc_keyset_set_master: the decoded master public key
};

constexpr uint32_t FACT_N = 65535;  // factorial tables of the Lagrange coefficients (node indices < FACT_N)

struct Span {
  std::string family;
  hipEvent_t a, b;
};

// Pinned host staging buffer for small host-shaped tables (tiles, offsets); `ev` marks the
// completion of the last copy out of it, so it is reused without synchronising a stream.
constexpr unsigned STAGE_SLOTS = 4;

struct Stage {
  void* h = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  bool used = false;
};

}  // namespace

// One verification lane: its stream (item pass, checks, then the combine of the same epoch), the
// shared preparation stream, their events, and the device ranges its last verification read and
// wrote (the hazards a call on another lane checks).
struct Lane {
  hipStream_t stream = nullptr, s_prep = nullptr;
  hipEvent_t ev_main = nullptr, ev_prep = nullptr, done = nullptr;
  hipEvent_t items_done = nullptr;  // recorded after the lane's last item pass
  bool items_rec = false;
  hipEvent_t dec_done = nullptr;  // recorded after the decode half of the lane's last G1 item pass
  bool dec_rec = false;
  int dec_flip = 0;  // alternates the lane's decoded-item buffers (a combine may still read one)
  std::vector<std::pair<uintptr_t, uintptr_t>> rd, wr;
  bool busy = false;
};

struct hbtc_ctx {
  int device = 0;
  // Verification calls rotate over NL lanes (hbbft processes the current epoch and up to
  // max_future_epochs = 3 more, src/honey_badger/builder.rs:37, honey_badger.rs:122), so epoch
  // k+1's item pass fills the SIMDs that epoch k's check levels and combine leave idle, and a
  // small epoch's chain of check latencies overlaps three others; `stream` / `s_prep` /
  // `s_comb` / `ev_*` / `ws_suffix` are the lane of the most recent verification (its combine
  // runs on the same stream, after it).  Measured (C3 / 125-ciphertext slice / C2, ms per epoch):
  // 2 lanes + a combine stream 107 / 24.4 / 45.3, 3 lanes 100.3 / 22.5 / 36.0, 4 lanes
  // 97.5 / 20.7 / 35.8, 4 lanes with the preparation on the lane stream 98.0 / 22.2 / 38.9.
  // Round 5 (C3 / 125 / 250-ciphertext slices): 4 lanes 71.5 / 14.1 / 24.3, 6 lanes
  // 71.0 / 12.7 / 23.1, 8 lanes 71.2 / 13.3 / 23.0 (profiles/r05/run15/) -- the slices gain only
  // from more epochs in flight than hbbft ever has (current + max_future_epochs = 3), so 4.
#ifndef HBTC_LANES
#define HBTC_LANES 4
#endif
  static constexpr int NL = HBTC_LANES;
  Lane lanes[NL];
  int lane = 0;
  int last_items_lane = -1;  // the lane of the most recent item pass (items_gate)
  bool pin_lane = false;  // host entry points: stay on the lane their uploads went to
  // item passes of the lanes run one after the other (HBTC_ITEMS_SERIAL, default 1): epoch
  // k+1's item pass then overlaps epoch k's check levels instead of sharing the chip with epoch
  // k's item pass; 2 also staggers the small passes, each decode after the previous one
  int items_serial = 1;
  int n_cu = 256;               // compute units of the device (check schedule, check_mode)
  int check_mode_forced = -1;  // HBTC_CHECK_MODE
  bool g2_gls = true;          // G2 combines through the ψ split (HBTC_G2_GLS=0: 255-bit terms)
  bool g1_glv = true;          // G1 combines through the φ split (HBTC_G1_GLV=0: 255-bit terms)
  // combines of t <= COMB_SMALL_T shares in one launch (hbtc_comb.hip; HBTC_COMB_SMALL=0: the
  // Pippenger chain for every t)
  bool comb_small = true;
  // hbtc_coin_decide's speculative combines (HBTC_COIN_SPEC=0: combine after the checks only)
  bool coin_spec = true;
  // hbtc_prepare_g2: per-instance G2 tables built ahead of the shares, resident, keyed by the
  // point's 96 bytes (a slot: decoded point, status, 68 affine lines)
  struct Prep {
    std::unordered_map<std::string, uint32_t> slot;
    std::vector<uint32_t> free;
    uint32_t cap = 0, top = 0;
    G2A* aff = nullptr;
    int32_t* st = nullptr;
    Line* lines = nullptr;
  } prep;
  // the host copies of the per-instance G2 arguments of the call in progress (set by the entry
  // points that take host bytes, for the prepared-table lookup of prepare_g2)
  struct HostG2 {
    const uint8_t *d0 = nullptr, *h0 = nullptr, *d1 = nullptr, *h1 = nullptr;
  } host_g2;
  // the exact small-call path of SignatureShares / pair checks as one fused launch (k_sig_exact;
  // HBTC_SIG_FUSED=0: decode, listing and line tables as three launches)
  bool sig_fused = true;
  // factorial tables of the Lagrange coefficients (k_lagrange_fact): 0..FACT_N, built at the first
  // Pippenger combine (HBTC_LAGRANGE_FACT=0: the O(t) per term kernels)
  bool lagrange_fact = true;
  Fr *fact = nullptr, *inv_fact = nullptr;
  std::string ws_suffix;
  hipStream_t stream = nullptr;  // main: items, checks, leaves
  hipStream_t s_prep = nullptr;  // per-instance G2 preparation, overlapped with the item pass
  hipStream_t s_comb = nullptr;  // combines: the current lane's stream (after its verification)
  hipEvent_t ev_main = nullptr, ev_prep = nullptr, ev_comb = nullptr;
  hipEvent_t ev_ext = nullptr, ev_ext2 = nullptr, ev_ext3 = nullptr;  // external-stream ordering
  // speculative coin combines (hbtc_coin_decide), created on first use, high priority
  hipStream_t s_spec = nullptr, s_spec2 = nullptr;  // G2 combines / G1 master checks
  hipEvent_t ev_spec_in = nullptr, ev_spec_out = nullptr, ev_spec_out2 = nullptr;
  std::map<std::string, Stage> stages;
  std::map<std::string, unsigned> stage_next;
  std::mutex mu;
  std::string err;
  std::map<uint32_t, Keyset> keysets;
  uint32_t next_keyset = 1;
  std::map<std::string, DevBuf> bufs;
  // Workspace buffers (device, and pinned host stages) outgrown while queued work may still use
  // them.  Each retirement batch carries a fence: one event recorded on every stream that could
  // read the old buffers.  A batch is freed once its fence has completed (checked at the next
  // growth, without waiting) or at the next sync; hipFree / hipHostFree in the middle of a
  // pipelined sequence would otherwise wait for the whole device on every growth.
  struct Retired {
    std::vector<void*> dev, host;
    std::vector<hipEvent_t> fence;
  };
  std::vector<Retired> graveyard;
  std::vector<void*> retiring_dev, retiring_host;  // collected by the growth in progress
  int verify_mode = HBTC_MODE_RLC;
  bool track_senders = true;
  uint32_t rlc_bits = 128;  // hbtc_set_rlc_bits (default: the curve's ~2^-128 level)
  bool probe_cold = true;  // probe pass on a cold key set (HBTC_PROBE=0: off)
  // failing tiles go through the split levels (check the left child, derive the right one;
  // k_chk_split) instead of halves / sub-tiles (HBTC_SPLIT=0: the round-3 levels)
  bool split_levels = true;
  // items per pair-batch chunk (pb_verify_dev; HBTC_PB_CHUNK overrides, a multiple of 64): the
  // chunk's per-item line tables (19.6 KB per item, ~5.1 GB at 2^18) stay cached in the
  // workspace until hbtc_trim_workspace
  uint32_t pb_chunk = 1u << 18;
  // layout of the small check levels (split levels, leaves) of calls on the paired schedules:
  // 3 = the latency form (gt6.h Pos.rep), 1 = the throughput form; HBTC_GT_REP overrides
  int small_rep = 3;
  // RLC-mode share calls with fewer items than this skip the group sums: the item pass only
  // decodes and lists every share for the exact cooperative leaf checks (hbtc_set_exact_below;
  // HBTC_EXACT_BELOW)
  uint32_t exact_below = 256;
  uint64_t probes = 0;     // probe passes run
  const uint32_t* last_leaf_count = nullptr;  // device counter of the last RLC call
  // Device ranges that combines still read, each with the event recorded after that combine:
  // work on another lane that writes an overlapping range waits on it first (combines run
  // concurrently with the NEXT verifications; hbtc.h: *_dev calls are ordered).
  struct PendingRead {
    uintptr_t lo, hi;
    hipEvent_t ev;
  };
  std::vector<PendingRead> comb_reads;
  // the decoded shares of the last RLC DecryptionShare verification (reused by a combine of
  // the same item arrays: no second decode / subgroup check)
  struct LastDec {
    const int32_t* status = nullptr;
    const uint8_t* shares = nullptr;
    uint32_t n_items = 0;
    const G1A* dec = nullptr;   // DecryptionShares (G1)
    const G2A* dec2 = nullptr;  // SignatureShares (G2)
  } last_dec;
  // Reed-Solomon plans (hbtc_rs_*): device row lists and nibble tables per (k, p, pattern)
  struct GfPlan {
    uint32_t *out_rows = nullptr, *in_rows = nullptr, *tabs = nullptr;
    uint32_t n_out = 0, n_in = 0;
  };
  std::map<std::string, GfPlan> gf_plans;
  // Asynchronous host-buffer epochs (hbtc_*_epoch_submit / hbtc_wait): at most one ticket per
  // lane in flight, its inputs and outputs in pinned staging owned by that lane.
  struct Ticket {
    uint64_t id = 0;
    bool active = false;
    hipEvent_t ev = nullptr;
    void* h_in = nullptr;
    size_t in_cap = 0;
    void* h_out = nullptr;
    size_t out_cap = 0;
    int32_t* status = nullptr;
    uint8_t* out = nullptr;
    uint8_t* parity = nullptr;
    int32_t* inst_status = nullptr;
    size_t n_items = 0, n_inst = 0, pt = 0;
    bool combined = false;
  };
  Ticket tickets[NL];
  uint64_t next_ticket = 1;
  std::random_device rd;
  bool timing = false;
  std::vector<Span> spans;
  std::map<std::string, std::pair<double, uint64_t>> totals;
};

namespace {

#define HB_CHECK(c, expr)                                                                   \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) {                                                                 \
      (c)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                         \
      return HBTC_ERR_DEVICE;                                                               \
    }                                                                                       \
  } while (0)

#define HB_TRY(expr)            \
  do {                          \
    int rc_ = (expr);           \
    if (rc_ != HBTC_OK) return rc_; \
  } while (0)

int fail(hbtc_ctx* c, int code, const std::string& msg) {
  c->err = msg;
  return code;
}

// The workspace names of one buffer on every lane: the current suffix is the lane's tag ("" or
// "#l") followed by what a pass appends (".probe").
std::string lane_tag(int l) { return l ? "#" + std::to_string(l) : std::string(); }
std::vector<std::string> lane_keys(const hbtc_ctx* c, const std::string& name) {
  const std::string tag = lane_tag(c->lane);
  const std::string extra =
      c->ws_suffix.compare(0, tag.size(), tag) == 0 ? c->ws_suffix.substr(tag.size()) : c->ws_suffix;
  std::vector<std::string> keys;
  for (int l = 0; l < hbtc_ctx::NL; ++l) keys.push_back(name + lane_tag(l) + extra);
  return keys;
}

// Close the batch of buffers retired by the growth in progress: a fence on every lane stream,
// the preparation stream and the speculation stream.
int retire_fence(hbtc_ctx* c) {
  if (c->retiring_dev.empty() && c->retiring_host.empty()) return HBTC_OK;
  hbtc_ctx::Retired r;
  r.dev.swap(c->retiring_dev);
  r.host.swap(c->retiring_host);
  std::vector<hipStream_t> streams;
  for (const Lane& l : c->lanes) {
    streams.push_back(l.stream);
    streams.push_back(l.s_prep);
  }
  if (c->s_spec) streams.push_back(c->s_spec);
  if (c->s_spec2) streams.push_back(c->s_spec2);
  hipError_t e = hipSuccess;
  for (hipStream_t st : streams) {
    hipEvent_t ev = nullptr;
    if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) break;
    r.fence.push_back(ev);
    if ((e = hipEventRecord(ev, st)) != hipSuccess) break;
  }
  c->graveyard.push_back(std::move(r));  // kept even on error: freed at sync / destroy
  HB_CHECK(c, e);
  return HBTC_OK;
}

// Free the retired batches whose fence has completed (wait = true: every batch, after waiting for
// its fence).  The list is taken out first, so a failing free cannot lead to a second one.
int reap_retired(hbtc_ctx* c, bool wait) {
  if (c->graveyard.empty()) return HBTC_OK;
  std::vector<hbtc_ctx::Retired> all;
  all.swap(c->graveyard);
  hipError_t first = hipSuccess;
  for (hbtc_ctx::Retired& r : all) {
    bool done = true;
    for (hipEvent_t ev : r.fence) {
      const hipError_t q = wait ? hipEventSynchronize(ev) : hipEventQuery(ev);
      if (q == hipErrorNotReady) {
        done = false;
        break;
      }
      if (q != hipSuccess && first == hipSuccess) first = q;
    }
    if (!done) {
      c->graveyard.push_back(std::move(r));
      continue;
    }
    for (void* p : r.dev) {
      const hipError_t e = hipFree(p);
      if (e != hipSuccess && first == hipSuccess) first = e;
    }
    for (void* p : r.host) {
      const hipError_t e = hipHostFree(p);
      if (e != hipSuccess && first == hipSuccess) first = e;
    }
    for (hipEvent_t ev : r.fence) (void)hipEventDestroy(ev);
  }
  HB_CHECK(c, first);
  return HBTC_OK;
}

// Grow-only named device workspace, one per lane.  A buffer that grows (a small call followed
// by a large one) grows on EVERY lane at once, and the old ones are retired until the next sync,
// not freed: hipFree waits for the whole device, and lanes whose first call of the new size came
// later used to grow mid-pipeline (c1's blocking calls, then C2's pipelined ones in one process:
// 17-22 ms per C2 step for the first steps against 13.2).
int ws(hbtc_ctx* c, const char* name, size_t bytes, void** out) {
  const std::string key = c->ws_suffix.empty() ? std::string(name) : std::string(name) + c->ws_suffix;
  DevBuf& b = c->bufs[key];
  if (bytes == 0) bytes = 16;
  if (b.cap < bytes) {
    HB_TRY(reap_retired(c, false));
    const size_t want = bytes + bytes / 4;
    // buffers past 256 MB (the pair batches' per-chunk line tables: 5 GB) grow on their own
    // lane only: the calls that need them are long, and four copies would hold 20 GB
    const bool all_lanes = want <= ((size_t)256 << 20);
    for (const std::string& k : lane_keys(c, name)) {
      if (!all_lanes && k != key) continue;
      DevBuf& x = c->bufs[k];
      if (x.cap >= bytes && k != key) continue;
      if (x.p) c->retiring_dev.push_back(x.p);
      x.p = nullptr;
      x.cap = 0;
      hipError_t e = hipMalloc(&x.p, want);
      if (e != hipSuccess) {
        (void)retire_fence(c);
        return fail(c, HBTC_ERR_OOM, std::string("hipMalloc ") + name);
      }
      x.cap = want;
    }
    HB_TRY(retire_fence(c));
  }
  *out = b.p;
  return HBTC_OK;
}

template <class T>
int wst(hbtc_ctx* c, const char* name, size_t count, T** out) {
  void* p;
  HB_TRY(ws(c, name, count * sizeof(T), &p));
  *out = static_cast<T*>(p);
  return HBTC_OK;
}

int upload(hbtc_ctx* c, const char* name, const void* src, size_t bytes, void** out) {
  HB_TRY(ws(c, name, bytes, out));
  if (bytes) HB_CHECK(c, hipMemcpyAsync(*out, src, bytes, hipMemcpyHostToDevice, c->stream));
  return HBTC_OK;
}

int download(hbtc_ctx* c, void* dst, const void* src, size_t bytes) {
  if (bytes) HB_CHECK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
  return HBTC_OK;
}

int sync(hbtc_ctx* c) {
  for (Lane& l : c->lanes) {
    HB_CHECK(c, hipStreamSynchronize(l.stream));
    HB_CHECK(c, hipStreamSynchronize(l.s_prep));
  }
  if (c->s_spec) HB_CHECK(c, hipStreamSynchronize(c->s_spec));
  if (c->s_spec2) HB_CHECK(c, hipStreamSynchronize(c->s_spec2));
  return reap_retired(c, true);
}

void select_lane(hbtc_ctx* c, int l) {
  c->lane = l;
  c->stream = c->lanes[l].stream;
  c->s_prep = c->lanes[l].s_prep;
  c->ev_main = c->lanes[l].ev_main;
  c->ev_prep = c->lanes[l].ev_prep;
  c->s_comb = c->lanes[l].stream;
  c->ws_suffix = l ? "#" + std::to_string(l) : "";
}

bool ranges_overlap(const std::vector<std::pair<uintptr_t, uintptr_t>>& a,
                    const std::vector<std::pair<uintptr_t, uintptr_t>>& b) {
  for (const auto& x : a)
    for (const auto& y : b)
      if (x.first < y.second && y.first < x.second) return true;
  return false;
}

// Wait on `me` for every other lane's last verification whose device ranges conflict with
// (rd, wr) (write/write, read/write either way).
int wait_conflicts(hbtc_ctx* c, int me_l, const std::vector<std::pair<uintptr_t, uintptr_t>>& rd,
                   const std::vector<std::pair<uintptr_t, uintptr_t>>& wr) {
  for (int o = 0; o < hbtc_ctx::NL; ++o) {
    const Lane& other = c->lanes[o];
    if (o == me_l || !other.busy) continue;
    if (ranges_overlap(wr, other.wr) || ranges_overlap(rd, other.wr) || ranges_overlap(wr, other.rd))
      HB_CHECK(c, hipStreamWaitEvent(c->lanes[me_l].stream, other.done, 0));
  }
  return HBTC_OK;
}

// Start a verification on the next lane: it waits for another lane's last verification only
// when their device ranges conflict.
int begin_verify(hbtc_ctx* c, std::vector<std::pair<uintptr_t, uintptr_t>> rd,
                 std::vector<std::pair<uintptr_t, uintptr_t>> wr) {
  const int l = c->pin_lane ? c->lane : (c->lane + 1) % hbtc_ctx::NL;
  select_lane(c, l);
  Lane& me = c->lanes[l];
  HB_TRY(wait_conflicts(c, l, rd, wr));
  me.rd = std::move(rd);
  me.wr = std::move(wr);
  return HBTC_OK;
}

// Another asynchronous operation on the current lane (e.g. unframing): it waits for other lanes
// on conflicting ranges, and its ranges join the lane's, so a later verification on another lane
// orders itself after it when it reads what this writes.
int lane_async(hbtc_ctx* c, std::initializer_list<std::pair<uintptr_t, uintptr_t>> rd,
               std::initializer_list<std::pair<uintptr_t, uintptr_t>> wr) {
  Lane& me = c->lanes[c->lane];
  const std::vector<std::pair<uintptr_t, uintptr_t>> r(rd), w(wr);
  HB_TRY(wait_conflicts(c, c->lane, r, w));
  me.rd.insert(me.rd.end(), r.begin(), r.end());
  me.wr.insert(me.wr.end(), w.begin(), w.end());
  return HBTC_OK;
}

int end_verify(hbtc_ctx* c) {
  Lane& me = c->lanes[c->lane];
  HB_CHECK(c, hipEventRecord(me.done, me.stream));
  me.busy = true;
  return HBTC_OK;
}

// An item pass of n_tiles waves about to start on the current lane waits for the most recent
// item pass (on another lane): large item passes form one chain, so each runs alone on the chip
// beside the other lanes' check levels.  A pass that fits the chip in one round (at most two
// waves per SIMD: 8 n_cu) is not chained -- the 125-ciphertext slice (2,000 tiles) runs 16.3
// instead of 17.4 ms per epoch unchained, the 250 one (4,000) 29.3-29.9 chained against 30.6-31.4,
// C3 (16,000) 84.2-84.5 against 85.1 (profiles/r04/run22/, run23/).  HBTC_ITEMS_SERIAL=2 also
// staggers the small passes (each decode after the previous lane's decode, to break the lanes'
// lockstep in the slice's trace): 125-ciphertext slice 14.0-14.2 against 13.6-13.8 ms, 250 and
// C3 unchanged (profiles/r06/run22/), so not the default.
int items_gate(hbtc_ctx* c, uint32_t n_tiles) {
  const int o = c->last_items_lane;
  if (!c->items_serial || o < 0 || o == c->lane) return HBTC_OK;
  if (n_tiles > 8u * (uint32_t)c->n_cu)
    HB_CHECK(c, hipStreamWaitEvent(c->stream, c->lanes[o].items_done, 0));
  else if (c->items_serial == 2 && c->lanes[o].dec_rec)  // a small pass: after the previous decode
    HB_CHECK(c, hipStreamWaitEvent(c->stream, c->lanes[o].dec_done, 0));
  return HBTC_OK;
}
int items_mark(hbtc_ctx* c) {
  Lane& me = c->lanes[c->lane];
  HB_CHECK(c, hipEventRecord(me.items_done, me.stream));
  me.items_rec = true;
  c->last_items_lane = c->lane;
  return HBTC_OK;
}

struct PinLane {
  hbtc_ctx* c;
  explicit PinLane(hbtc_ctx* cc) : c(cc) { c->pin_lane = true; }
  ~PinLane() { c->pin_lane = false; }
};

std::pair<uintptr_t, uintptr_t> rng(const void* p, size_t bytes) {
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
  return {lo, lo + bytes};
}

// `waiter` runs everything enqueued after this behind all work already on `on`.
int stream_after(hbtc_ctx* c, hipStream_t waiter, hipStream_t on, hipEvent_t ev) {
  HB_CHECK(c, hipEventRecord(ev, on));
  HB_CHECK(c, hipStreamWaitEvent(waiter, ev, 0));
  return HBTC_OK;
}

// Main-stream work about to write [p, p + bytes): wait for every pending combine that reads
// an overlapping range; forget combines that have completed.
int guard_write(hbtc_ctx* c, const void* p, size_t bytes) {
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p), hi = lo + bytes;
  auto& v = c->comb_reads;
  for (size_t i = 0; i < v.size();) {
    if (hipEventQuery(v[i].ev) == hipSuccess) {
      (void)hipEventDestroy(v[i].ev);
      v[i] = v.back();
      v.pop_back();
      continue;
    }
    if (v[i].lo < hi && lo < v[i].hi) HB_CHECK(c, hipStreamWaitEvent(c->stream, v[i].ev, 0));
    ++i;
  }
  return HBTC_OK;
}

// A combine just enqueued on s_comb reads these ranges until it completes.
int note_comb_reads(hbtc_ctx* c, std::initializer_list<std::pair<const void*, size_t>> ranges) {
  hipEvent_t ev;
  HB_CHECK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HB_CHECK(c, hipEventRecord(ev, c->s_comb));
  bool first = true;
  for (const auto& r : ranges) {
    if (!r.first || !r.second) continue;
    hipEvent_t e = ev;
    if (!first) {  // one event per entry: entries are destroyed independently
      HB_CHECK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      HB_CHECK(c, hipEventRecord(e, c->s_comb));
    }
    first = false;
    const uintptr_t lo = reinterpret_cast<uintptr_t>(r.first);
    c->comb_reads.push_back({lo, lo + r.second, e});
  }
  if (first) (void)hipEventDestroy(ev);
  return HBTC_OK;
}

// Record a kernel family's launch between two events on the stream it runs on.
template <class F>
int timed_on(hbtc_ctx* c, hipStream_t st, const char* family, F&& launch) {
  Span sp;
  if (c->timing) {
    HB_CHECK(c, hipEventCreate(&sp.a));
    HB_CHECK(c, hipEventCreate(&sp.b));
    HB_CHECK(c, hipEventRecord(sp.a, st));
  }
  hipError_t e = launch();
  if (e != hipSuccess) return fail(c, HBTC_ERR_DEVICE, std::string(family) + " launch: " + hipGetErrorString(e));
  if (c->timing) {
    HB_CHECK(c, hipEventRecord(sp.b, st));
    sp.family = family;
    c->spans.push_back(sp);
  }
  return HBTC_OK;
}
template <class F>
int timed(hbtc_ctx* c, const char* family, F&& launch) {
  return timed_on(c, c->stream, family, launch);
}

// Host table -> device workspace `name` through its pinned stage, ordered on `st`.
int stage_upload(hbtc_ctx* c, const char* name, const void* src, size_t bytes, hipStream_t st,
                 void** d_out) {
  // a ring of pinned host buffers per name: the host waits only for the copy out of the slot
  // it reuses, STAGE_SLOTS calls back, not for the previous call's (which may sit behind a
  // whole verification on its stream) -- the host stays ahead of the device
  const std::string base = c->ws_suffix.empty() ? std::string(name) : std::string(name) + c->ws_suffix;
  const unsigned slot = c->stage_next[base]++ % STAGE_SLOTS;
  Stage& sg = c->stages[base + "@" + std::to_string(slot)];
  if (sg.used) HB_CHECK(c, hipEventSynchronize(sg.ev));  // the copy out of this slot is done
  if (sg.cap < bytes || !sg.h) {
    // every slot of every lane grows at once, the old buffers retired, not freed: hipHostFree
    // waits for the device (slots outgrown one by one by a larger call than the ones before
    // stalled every lane in flight: C2 after a few small calls)
    const size_t want = bytes + bytes / 4 + 256;
    for (const std::string& k : lane_keys(c, name))
      for (unsigned j = 0; j < STAGE_SLOTS; ++j) {
        Stage& x = c->stages[k + "@" + std::to_string(j)];
        if (x.h && x.cap >= bytes && &x != &sg) continue;
        if (x.h) c->retiring_host.push_back(x.h);
        x.h = nullptr;
        x.cap = 0;
        const hipError_t e = hipHostMalloc(&x.h, want, hipHostMallocMapped | hipHostMallocPortable);
        if (e != hipSuccess) {
          (void)retire_fence(c);
          HB_CHECK(c, e);
        }
        x.cap = want;
      }
    HB_TRY(retire_fence(c));
  }
  if (!sg.ev) HB_CHECK(c, hipEventCreateWithFlags(&sg.ev, hipEventDisableTiming));
  if (bytes) memcpy(sg.h, src, bytes);
  HB_TRY(ws(c, name, bytes, d_out));
  if (bytes) {
    void* src = nullptr;
    HB_CHECK(c, hipHostGetDevicePointer(&src, sg.h, 0));
    HB_CHECK(c, launch_stage_copy(st, src, *d_out, bytes));
  }
  HB_CHECK(c, hipEventRecord(sg.ev, st));
  sg.used = true;
  return HBTC_OK;
}

int collect_spans(hbtc_ctx* c) {
  for (Span& sp : c->spans) {
    HB_CHECK(c, hipEventSynchronize(sp.b));
    float ms = 0.f;
    HB_CHECK(c, hipEventElapsedTime(&ms, sp.a, sp.b));
    auto& t = c->totals[sp.family];
    t.first += ms;
    t.second += 1;
    (void)hipEventDestroy(sp.a);
    (void)hipEventDestroy(sp.b);
  }
  c->spans.clear();
  return HBTC_OK;
}

int check_offsets(hbtc_ctx* c, uint32_t n_inst, const uint32_t* offsets, uint32_t* n_items) {
  if (!offsets) return fail(c, HBTC_ERR_ARG, "offsets is NULL");
  if (offsets[0] != 0) return fail(c, HBTC_ERR_ARG, "offsets[0] must be 0");
  for (uint32_t k = 0; k < n_inst; ++k)
    if (offsets[k + 1] < offsets[k]) return fail(c, HBTC_ERR_ARG, "offsets must be non-decreasing");
  *n_items = offsets[n_inst];
  return HBTC_OK;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Split every instance into tiles of <= 64 items and upload the table (and, when asked, the
// first tile of every instance) through pinned stages on the main stream.
int make_tiles(hbtc_ctx* c, uint32_t n_inst, const uint32_t* offsets, Tile** d_tiles,
               uint32_t* n_tiles, uint32_t** d_inst_tiles = nullptr) {
  std::vector<Tile> tiles;
  std::vector<uint32_t> inst_tiles(n_inst + 1);
  for (uint32_t k = 0; k < n_inst; ++k) {
    inst_tiles[k] = (uint32_t)tiles.size();
    for (uint32_t s = offsets[k]; s < offsets[k + 1]; s += TILE_ITEMS) {
      const uint32_t cnt = offsets[k + 1] - s < TILE_ITEMS ? offsets[k + 1] - s : TILE_ITEMS;
      tiles.push_back(Tile{k, s, cnt, 0});
    }
  }
  inst_tiles[n_inst] = (uint32_t)tiles.size();
  void* p;
  HB_TRY(stage_upload(c, "tiles", tiles.data(), tiles.size() * sizeof(Tile), c->stream, &p));
  *d_tiles = static_cast<Tile*>(p);
  *n_tiles = (uint32_t)tiles.size();
  if (d_inst_tiles) {
    HB_TRY(stage_upload(c, "inst_tiles", inst_tiles.data(), inst_tiles.size() * 4, c->stream, &p));
    *d_inst_tiles = static_cast<uint32_t*>(p);
  }
  return HBTC_OK;
}

int get_keyset(hbtc_ctx* c, uint32_t id, Keyset** ks) {
  auto it = c->keysets.find(id);
  if (it == c->keysets.end()) return fail(c, HBTC_ERR_NO_KEYSET, "unknown keyset id");
  *ks = &it->second;
  return HBTC_OK;
}

// Decode + line tables for the per-instance G2 arguments: d0 (n items) and, when d1 is given,
// d1 (n more) in one launch pair; outputs for d1 start at index n.
// The host bytes of a call's per-instance G2 arguments, for prepare_g2's lookup of prepared
// tables, for the duration of one entry point.
struct HostG2Args {
  hbtc_ctx* c;
  HostG2Args(hbtc_ctx* cx, const void* d0, const uint8_t* h0, const void* d1 = nullptr, const uint8_t* h1 = nullptr)
      : c(cx) {
    c->host_g2 = {static_cast<const uint8_t*>(d0), h0, static_cast<const uint8_t*>(d1), h1};
  }
  ~HostG2Args() { c->host_g2 = {}; }
};

int prepare_g2(hbtc_ctx* c, const uint8_t* d0, const uint8_t* d1, uint32_t n, G2A** aff,
               int32_t** st, Line** lines, hipStream_t on = nullptr) {
  hipStream_t strm = on ? on : c->stream;
  const uint32_t m = d1 ? 2 * n : n;
  Fq2* wsp;
  HB_TRY(wst(c, "g2.aff", m, aff));
  HB_TRY(wst(c, "g2.st", m, st));
  HB_TRY(wst(c, "g2.lines", (size_t)m * MILLER_STEPS, lines));
  // every argument prepared (hbtc_prepare_g2): gather the resident tables instead of building them
  const auto& hg = c->host_g2;
  if (!c->prep.slot.empty() && hg.d0 == d0 && hg.h0 && hg.d1 == d1 && (!d1 || hg.h1)) {
    std::vector<uint32_t> slots(m);
    bool all = true;
    for (uint32_t i = 0; i < m && all; ++i) {
      const uint8_t* key = i < n ? hg.h0 + (size_t)96 * i : hg.h1 + (size_t)96 * (i - n);
      auto it = c->prep.slot.find(std::string(reinterpret_cast<const char*>(key), 96));
      if (it == c->prep.slot.end()) all = false; else slots[i] = it->second;
    }
    if (all) {
      void* p;
      HB_TRY(stage_upload(c, "g2.slots", slots.data(), (size_t)4 * m, strm, &p));
      const uint32_t* d_slots = static_cast<const uint32_t*>(p);
      G2A* a = *aff;
      int32_t* s = *st;
      Line* l = *lines;
      return timed_on(c, strm, "prepare_cached", [&] {
        return launch_g2_tab_copy(strm, m, d_slots, nullptr, c->prep.aff, c->prep.st, c->prep.lines, a, s, l);
      });
    }
  }
  HB_TRY(wst(c, "g2.ws", (size_t)m * 3 * MILLER_STEPS, &wsp));
  G2A* a = *aff;
  int32_t* s = *st;
  Line* l = *lines;
  return timed_on(c, strm, "prepare", [&] {
    return launch_g2_prepare(strm, d0, n, d1, d1 ? n : 0, a, l, wsp, s);
  });
}

// Sender tracking view of one RLC call on key set ks (hbtc_kernels.h Suspects).
Suspects suspects_of(hbtc_ctx* c, Keyset* ks, uint32_t* leaf_count, uint32_t* leaves) {
  Suspects s{nullptr, 0, leaf_count, leaves, 0};
  if (c->track_senders) {
    s.last_bad = ks->last_bad;
    s.now = ++ks->calls;
  }
  return s;
}

// REJECTs that flag a sender in one call: 1/8 of the call's average shares per sender (>= 1).
uint32_t track_threshold(const Keyset* ks, uint32_t n_items) {
  const uint64_t t = (uint64_t)n_items / (8ull * ks->n);
  return t ? (uint32_t)t : 1u;
}

// REJECTs that flag a sender in a probe pass: half of the probe's average shares per sender (>= 2).
// A probe is small, so the call threshold (1/8 of the average) would flag honest senders hit by one
// stray corrupted share -- their shares would then take the exact checks for 16 calls.
uint32_t probe_threshold(const Keyset* ks, uint32_t n_items) {
  const uint64_t t = (uint64_t)n_items / (2ull * ks->n);
  return t > 2 ? (uint32_t)t : 2u;
}

// Group-check schedule of one RLC call.  The plain-first form (5 levels: plain and weighted
// checks of tiles, then of sub-tiles, then leaves) does the least work and is right when the
// call fills the chip; a call with few tiles (a rank's slice under strong scaling, a small
// epoch) is bound by the chain of check latencies instead, so it pairs the plain and weighted
// checks of a group in one launch: tiles -> sub-tiles -> leaves (3 levels; C3 slices of 125
// ciphertexts: 25.8 ms per epoch against 32.4 plain-first), or tiles -> leaves (2 levels) for
// calls so small that their ~8.6 leaf checks per tile (1 % wrong shares) cost less than a level.  hbtc_set_check_schedule (or the environment's
// HBTC_CHECK_MODE = plain | pair3 | pair2) forces one.
enum { CHK_PLAIN_FIRST = HBTC_CHECK_PLAIN_FIRST, CHK_PAIR_SUBS = HBTC_CHECK_PAIR_SUBS,
       CHK_PAIR_LEAVES = HBTC_CHECK_PAIR_LEAVES };
int check_mode(hbtc_ctx* c, uint32_t n_tiles) {
  if (c->check_mode_forced >= 0) return c->check_mode_forced;
  const uint32_t simds = 4u * (uint32_t)c->n_cu;
  if (n_tiles <= simds / 2u) return CHK_PAIR_LEAVES;
  if (n_tiles <= 2u * simds) return CHK_PAIR_SUBS;
  return CHK_PLAIN_FIRST;
}

// ---------------------------------------------------------------- device-pointer cores
// The per-ciphertext G2 preparation of a DecryptionShare call (decoded H / w, statuses, lines).
struct G2Prep {
  const G2A* h_aff;
  const int32_t* h_st;
  const Line* h_lines;
  const G2A* w_aff;
  const int32_t* w_st;
  const Line* w_lines;
};
uint32_t probe_size(const hbtc_ctx* c, const Keyset* ks, uint32_t n_ct);
int rlc_dec_pass(hbtc_ctx* c, Keyset* ks, uint32_t n_ct, const uint32_t* offsets,
                 const uint32_t* d_idx, const uint8_t* d_share, int32_t* d_status, const G2Prep& pp,
                 bool exact = false);

int dec_shares_dev(hbtc_ctx* c, uint32_t keyset_id, uint32_t n_ct, const uint8_t* d_H,
                   const uint8_t* d_w, const uint32_t* offsets, const uint32_t* d_idx,
                   const uint8_t* d_share, int32_t* d_status) {
  Keyset* ks;
  HB_TRY(get_keyset(c, keyset_id, &ks));
  uint32_t n_items;
  HB_TRY(check_offsets(c, n_ct, offsets, &n_items));
  if (n_items == 0) return HBTC_OK;
  if (!aligned16(d_H) || !aligned16(d_w) || !aligned16(d_share))
    return fail(c, HBTC_ERR_ARG, "item arrays must be 16-byte aligned");
  HB_TRY(begin_verify(c, {rng(d_H, 96 * (size_t)n_ct), rng(d_w, 96 * (size_t)n_ct),
                          rng(d_idx, 4 * (size_t)n_items), rng(d_share, 48 * (size_t)n_items)},
                      {rng(d_status, 4 * (size_t)n_items)}));
  G2A *h_aff, *w_aff;
  int32_t *h_st, *w_st;
  Line *h_lines, *w_lines;
  Tile* tiles;
  uint32_t n_tiles;
  // RLC batch verification with hierarchical fallback (hbtc_rlc.hip).  The per-ciphertext G2
  // preparation runs on s_prep concurrently with the item pass; the checks wait for both.
  HB_TRY(stream_after(c, c->s_prep, c->stream, c->ev_main));
  HB_TRY(prepare_g2(c, d_H, d_w, n_ct, &h_aff, &h_st, &h_lines, c->s_prep));
  w_aff = h_aff + n_ct;
  w_st = h_st + n_ct;
  w_lines = h_lines + (size_t)n_ct * MILLER_STEPS;
  const G2Prep prep{h_aff, h_st, h_lines, w_aff, w_st, w_lines};
  // Cold key set (no RLC call on it yet, sender tracking on): a probe pass over the first
  // ciphertexts finds the senders who lie on all of them before the call proper, so f Byzantine
  // senders do not send most of the first epoch's shares to the exact checks.
  // per-share mode, or a small call: no group sums, every share gets the exact cooperative leaf
  // check (the per-share mode's count of pairing checks, on the leaf kernels' layout)
  const bool exact = c->verify_mode == HBTC_MODE_PER_SHARE || n_items < c->exact_below;
  const uint32_t n_probe = exact ? 0 : probe_size(c, ks, n_ct);
  if (n_probe) {
    HB_TRY(rlc_dec_pass(c, ks, n_probe, offsets, d_idx, d_share, nullptr, prep));
    ++c->probes;
  }
  HB_TRY(rlc_dec_pass(c, ks, n_ct, offsets, d_idx, d_share, d_status, prep, exact));
  return end_verify(c);
}

// Instances of a call's probe pass: n_ct / 16 (at most 64) on a cold key set, else 0.
uint32_t probe_size(const hbtc_ctx* c, const Keyset* ks, uint32_t n_ct) {
  if (!c->track_senders || !c->probe_cold || ks->calls != 0 || n_ct < 32) return 0;
  return std::min<uint32_t>(64u, n_ct / 16u);
}

// One RLC pass over instances [0, n_ct) of a call whose G2 preparation is `pp`: tiles, item pass,
// group-check levels, leaves, final statuses into d_status.  d_status == nullptr: the probe pass
// (statuses into scratch, its own workspace: only its sender-tracking counts matter).  exact: a
// small call -- the item pass decodes and lists every share, no group levels, no tracking.
int rlc_dec_pass(hbtc_ctx* c, Keyset* ks, uint32_t n_ct, const uint32_t* offsets,
                 const uint32_t* d_idx, const uint8_t* d_share, int32_t* d_status, const G2Prep& pp,
                 bool exact) {
  const bool probe = d_status == nullptr;
  const uint32_t n_items = offsets[n_ct];
  const std::string suffix0 = c->ws_suffix;
  struct Restore {
    hbtc_ctx* c;
    std::string s;
    ~Restore() { c->ws_suffix = s; }
  } restore{c, suffix0};
  if (probe) {
    c->ws_suffix = suffix0 + ".probe";
    HB_TRY(wst(c, "rlc.status", n_items, &d_status));
  }
  const G2A *h_aff = pp.h_aff, *w_aff = pp.w_aff;
  const int32_t *h_st = pp.h_st, *w_st = pp.w_st;
  const Line *h_lines = pp.h_lines, *w_lines = pp.w_lines;
  Tile* tiles;
  uint32_t n_tiles;
  HB_TRY(make_tiles(c, n_ct, offsets, &tiles, &n_tiles));
  RlcKey key;
  for (int i = 0; i < 8; ++i) key.k[i] = c->rd();
  key.bits = c->rlc_bits;
  TileSums* sums;
  G1A* dec;
  uint32_t *counters, *sub_list, *leaves, *tw_list, *sw_list, *hw_list, *hl_list;
  Fq2 *t_tiles, *t_subs, *t_halves;
  HB_TRY(wst(c, "rlc.sums", n_tiles, &sums));
  // two alternating buffers: a combine of the previous call may still read the other one
  if (probe) {
    HB_TRY(wst(c, "rlc.dec0", n_items, &dec));
  } else {
    c->lanes[c->lane].dec_flip ^= 1;
    HB_TRY(wst(c, c->lanes[c->lane].dec_flip ? "rlc.dec1" : "rlc.dec0", n_items, &dec));
    HB_TRY(guard_write(c, d_status, (size_t)n_items * 4));
    HB_TRY(guard_write(c, dec, (size_t)n_items * sizeof(G1A)));
    c->last_dec = {d_status, d_share, n_items, dec, nullptr};
  }
  // counters: [0] leaves, [1] listed tiles (half / sub-tile pass), [2] failing tiles, [3] failing
  // subs, [4] failing halves, [5] listed halves, [6..8] the split levels' lists
  HB_TRY(wst(c, "rlc.counters", 9, &counters));
  HB_TRY(wst(c, "rlc.sub_list", n_tiles, &sub_list));
  HB_TRY(wst(c, "rlc.tw_list", n_tiles, &tw_list));
  HB_TRY(wst(c, "rlc.sw_list", (size_t)8 * n_tiles, &sw_list));
  HB_TRY(wst(c, "rlc.t_tiles", (size_t)6 * n_tiles, &t_tiles));
  HB_TRY(wst(c, "rlc.t_subs", (size_t)48 * n_tiles, &t_subs));
  HB_TRY(wst(c, "rlc.t_halves", (size_t)12 * n_tiles, &t_halves));
  HB_TRY(wst(c, "rlc.hw_list", (size_t)2 * n_tiles, &hw_list));
  HB_TRY(wst(c, "rlc.hl_list", (size_t)2 * n_tiles, &hl_list));
  HB_TRY(wst(c, "rlc.leaves", (size_t)2 * n_items, &leaves));
  uint32_t* leaf_count = counters;
  uint32_t* sub_count = counters + 1;
  uint32_t* tw_count = counters + 2;
  uint32_t* sw_count = counters + 3;
  uint32_t* hw_count = counters + 4;
  uint32_t* hl_count = counters + 5;
  HB_CHECK(c, launch_zero_u32(c->stream, counters, 9));
  // the split levels' lists: level l lists up to n_tiles 2^(l-1) nodes with their T, U (6 Fq2 each)
  const int chk_mode = check_mode(c, n_tiles);
  // the split levels pay on the plain-first schedule (C3: 86.2 -> 84.7 ms per epoch); on the
  // paired ones the sub-tile level is one launch where splitting is three dependent ones (the
  // 125-ciphertext slice: 17.1 ms per epoch without, 18.5 with; profiles/r04/run4/)
  const bool split = !exact && c->split_levels && chk_mode == CHK_PLAIN_FIRST;
  SplitOut sp[3] = {};
  if (split) {
    for (int l = 0; l < 3; ++l) {
      const size_t cap = (size_t)n_tiles << l;
      const std::string nm = "rlc.split" + std::to_string(l);
      sp[l].count = counters + 6 + l;
      HB_TRY(wst(c, (nm + ".list").c_str(), cap, &sp[l].list));
      HB_TRY(wst(c, (nm + ".ab").c_str(), cap, &sp[l].ab));
      HB_TRY(wst(c, (nm + ".T").c_str(), 6 * cap, &sp[l].T));
      HB_TRY(wst(c, (nm + ".U").c_str(), 6 * cap, &sp[l].U));
    }
  }
  const SplitOut no_split{};
  const Suspects sus =
      exact ? Suspects{nullptr, 0, leaf_count, leaves, 1} : suspects_of(c, ks, leaf_count, leaves);
  HB_TRY(items_gate(c, n_tiles));
  G1J* t1s = nullptr;
  if (rlc_items_split()) HB_TRY(wst(c, "rlc.t1", n_items, &t1s));
  HB_TRY(timed(c, "rlc_items", [&] {
    return launch_rlc_items(c->stream, n_tiles, tiles, d_idx, d_share, ks->pk, ks->st, ks->tab,
                            ks->n, key, sus, sums, dec, d_status, t1s, c->lanes[c->lane].dec_done);
  }));
  c->lanes[c->lane].dec_rec = rlc_items_split();
  HB_TRY(items_mark(c));
  HB_TRY(stream_after(c, c->stream, c->s_prep, c->ev_prep));
  if (exact) {
    // no group levels: every decoded share is on the leaf list
  } else if (chk_mode != CHK_PLAIN_FIRST) {
    // latency form: paired levels (hbtc_check.hip k_chk_pair)
    const bool two = chk_mode == CHK_PAIR_LEAVES;
    HB_TRY(timed(c, "chk_tiles", [&] {
      return launch_chk_pair(c->stream, 0, two, n_tiles, n_tiles, nullptr, nullptr, tiles, sums,
                             h_aff, h_lines, w_aff, w_lines, h_st, w_st, d_status,
                             two ? leaf_count : sub_count, two ? leaves : sub_list,
                             split ? sp[0] : no_split);
    }));
    if (!two && !split)
      HB_TRY(timed(c, "chk_subs", [&] {
        return launch_chk_pair(c->stream, 1, true, 8 * n_tiles, 0, sub_count, sub_list, tiles, sums,
                               h_aff, h_lines, w_aff, w_lines, h_st, w_st, d_status, leaf_count,
                               leaves, no_split);
      }));
  } else {  // throughput form: plain first (k_chk_plain / k_chk_halves / k_chk_weighted)
    HB_TRY(timed(c, "chk_tiles", [&] {
      return launch_chk_plain(c->stream, 0, n_tiles, n_tiles, nullptr, nullptr, nullptr, tiles, sums,
                              h_aff, h_lines, w_aff, w_lines, h_st, w_st, t_tiles, tw_count, tw_list);
    }));
    HB_TRY(timed(c, "chk_tiles_w", [&] {
      return launch_chk_weighted(c->stream, 0, n_tiles, tw_count, tw_list, nullptr, nullptr, tiles,
                                 sums, h_aff, h_lines, w_aff, w_lines, h_st, w_st, t_tiles, d_status,
                                 sub_count, sub_list, split ? sp[0] : no_split);
    }));
  }
  // small calls (the paired schedules): their later levels hold a few hundred checks at most,
  // a chain of check latencies, so they run in the latency form
  const int rep = chk_mode == CHK_PLAIN_FIRST && !exact ? 1 : c->small_rep;
  if (exact) {
  } else if (split) {
    // split levels: listed tiles -> halves -> quarters -> eighths (unresolved eighths: leaves)
    static const char* const fam[3] = {"chk_split1", "chk_split2", "chk_split3"};
    for (int l = 1; l <= 3; ++l) {
      const SplitOut& in = sp[l - 1];
      HB_TRY(timed(c, fam[l - 1], [&] {
        return launch_chk_split(c->stream, l, rep, n_tiles << (l - 1), in.count, in.list, in.T, in.U,
                                in.ab, tiles, sums, h_aff, h_lines, w_aff, w_lines, d_status,
                                leaf_count, leaves, l < 3 ? sp[l] : no_split);
      }));
    }
  } else if (chk_mode == CHK_PLAIN_FIRST) {
    HB_TRY(timed(c, "chk_halves", [&] {
      return launch_chk_halves(c->stream, n_tiles, sub_count, sub_list, tiles, sums, h_aff, h_lines,
                               w_aff, w_lines, t_tiles, t_halves, hw_count, hw_list);
    }));
    HB_TRY(timed(c, "chk_halves_w", [&] {
      return launch_chk_weighted(c->stream, 2, 2 * n_tiles, hw_count, hw_list, sub_list, nullptr,
                                 tiles, sums, h_aff, h_lines, w_aff, w_lines, h_st, w_st, t_halves,
                                 d_status, hl_count, hl_list, no_split);
    }));
    HB_TRY(timed(c, "chk_subs", [&] {
      return launch_chk_plain(c->stream, 3, 8 * n_tiles, 0, hl_count, sub_list, hl_list, tiles, sums,
                              h_aff, h_lines, w_aff, w_lines, h_st, w_st, t_subs, sw_count, sw_list);
    }));
    HB_TRY(timed(c, "chk_subs_w", [&] {
      return launch_chk_weighted(c->stream, 3, 8 * n_tiles, sw_count, sw_list, sub_list, hl_list,
                                 tiles, sums, h_aff, h_lines, w_aff, w_lines, h_st, w_st, t_subs,
                                 d_status, leaf_count, leaves, no_split);
    }));
  }
  HB_TRY(timed(c, "chk_leaves", [&] {
    // the latency form for lists of at most two leaves per SIMD (one wave each), the throughput
    // form for longer ones (tracked senders put one share per liar per ciphertext on the list)
    const uint32_t lim = rep == 3 ? 8u * (uint32_t)c->n_cu : 0u;
    const hipError_t e = launch_chk_leaves_rep3(c->stream, n_items, lim, leaf_count, leaves, d_idx, dec,
                                                ks->pk, h_aff, h_lines, w_aff, w_lines, d_status);
    if (e != hipSuccess) return e;
    return launch_chk_leaves(c->stream, n_items, leaf_count, leaves, d_idx, dec, ks->pk, h_aff,
                             h_lines, w_aff, w_lines, d_status, lim);
  }));
  if (!probe) c->last_leaf_count = leaf_count;
  return timed(c, "rlc_finalize", [&] {
    return launch_rlc_finalize(c->stream, n_tiles, tiles, h_st, w_st, d_status, d_idx, ks->n,
                               ks->rejects + (size_t)c->lane * ks->n,
                               const_cast<uint32_t*>(sus.last_bad), sus.now,
                               probe ? probe_threshold(ks, n_items) : track_threshold(ks, n_items));
  });
}

int sig_shares_dev(hbtc_ctx* c, uint32_t keyset_id, uint32_t n_inst, const uint8_t* d_H,
                   const uint32_t* offsets, const uint32_t* d_idx, const uint8_t* d_sig,
                   int32_t* d_status) {
  Keyset* ks;
  HB_TRY(get_keyset(c, keyset_id, &ks));
  uint32_t n_items;
  HB_TRY(check_offsets(c, n_inst, offsets, &n_items));
  if (n_items == 0) return HBTC_OK;
  if (!aligned16(d_H) || !aligned16(d_sig))
    return fail(c, HBTC_ERR_ARG, "item arrays must be 16-byte aligned");
  HB_TRY(begin_verify(c, {rng(d_H, 96 * (size_t)n_inst), rng(d_idx, 4 * (size_t)n_items),
                          rng(d_sig, 96 * (size_t)n_items)},
                      {rng(d_status, 4 * (size_t)n_items)}));
  HB_TRY(guard_write(c, d_status, (size_t)n_items * 4));
  if (c->last_dec.status == d_status) c->last_dec = {};
  G2A* h_aff;
  int32_t* h_st;
  Line* h_lines;
  Tile* tiles;
  uint32_t n_tiles;
  // RLC batch verification (hbtc_sig.hip): H's line tables on s_prep beside the item pass; the
  // G2 sums' projective line tables before each check level.
  HB_TRY(stream_after(c, c->s_prep, c->stream, c->ev_main));
  HB_TRY(prepare_g2(c, d_H, nullptr, n_inst, &h_aff, &h_st, &h_lines, c->s_prep));
  HB_TRY(make_tiles(c, n_inst, offsets, &tiles, &n_tiles));
  RlcKey key;
  for (int i = 0; i < 8; ++i) key.k[i] = c->rd();
  key.bits = c->rlc_bits;
  constexpr uint32_t LEAF_CHUNK = 1u << 15;
  const size_t n_tables = std::max<size_t>((size_t)16 * n_tiles, LEAF_CHUNK);
  SigTileSums* sums;
  G2A* dec;
  Fq2* tables;
  uint32_t *inf, *counters, *sub_list, *leaves;
  HB_TRY(wst(c, "sig.sums", n_tiles, &sums));
  c->lanes[c->lane].dec_flip ^= 1;
  HB_TRY(wst(c, c->lanes[c->lane].dec_flip ? "sig.dec1" : "sig.dec0", n_items, &dec));
  HB_TRY(guard_write(c, dec, (size_t)n_items * sizeof(G2A)));
  c->last_dec = {d_status, d_sig, n_items, nullptr, dec};
  HB_TRY(wst(c, "sig.tables", n_tables * PLINES_FQ2, &tables));
  HB_TRY(wst(c, "sig.inf", n_tables, &inf));
  HB_TRY(wst(c, "sig.counters", 2, &counters));
  HB_TRY(wst(c, "sig.sub_list", n_tiles, &sub_list));
  HB_TRY(wst(c, "sig.leaves", (size_t)2 * n_items, &leaves));
  uint32_t* leaf_count = counters;
  uint32_t* sub_count = counters + 1;
  HB_CHECK(c, launch_zero_u32(c->stream, counters, 2));
  // per-share mode, or a small call: the item pass decodes and lists every share for the exact
  // leaf checks
  const bool exact = c->verify_mode == HBTC_MODE_PER_SHARE || n_items < c->exact_below;
  const Suspects sus =
      exact ? Suspects{nullptr, 0, leaf_count, leaves, 1} : suspects_of(c, ks, leaf_count, leaves);
  // the exact path in one launch when every share's line table fits the buffer (k_sig_exact:
  // decode, listing, line tables with the subgroup test at the end of their walk)
  const bool fused = exact && c->sig_fused && n_items <= n_tables;
  HB_TRY(items_gate(c, n_tiles));
  HB_TRY(timed(c, "sig_items", [&] {
    if (fused)
      return launch_sig_exact(c->stream, n_items, d_idx, d_sig, ks->st, ks->n, tiles, n_tiles, leaf_count,
                              leaves, dec, tables, inf, d_status);
    return launch_sig_items(c->stream, n_tiles, tiles, d_idx, d_sig, ks->pk, ks->st, ks->tab, ks->n,
                            key, sus, sums, dec, d_status);
  }));
  HB_TRY(items_mark(c));
  if (!exact)
    HB_TRY(timed(c, "sig_lines", [&] {
      return launch_plines(c->stream, 0, 2 * n_tiles, 0, nullptr, nullptr, tiles, sums, dec, tables,
                           inf);
    }));
  HB_TRY(stream_after(c, c->stream, c->s_prep, c->ev_prep));
  // paired checks either way (plain and weighted value of a group per unit); a small call goes
  // from the tiles straight to the leaves (check_mode)
  const bool to_leaves = check_mode(c, n_tiles) == CHK_PAIR_LEAVES;
  // the small calls' levels (tiles -> leaves: fewer tiles than half the SIMDs) are chains of check
  // latencies: the latency form (gt6.h Pos.rep = 3), unless HBTC_GT_REP=1
  const bool rep3 = (to_leaves || exact) && c->small_rep == 3;
  if (!exact) {
    HB_TRY(timed(c, "chk_tiles", [&] {
      if (rep3)
        return launch_sigchk_tiles_rep3(c->stream, n_tiles, tiles, sums, tables, inf, h_aff,
                                        h_lines, h_st, d_status, leaf_count, leaves, true);
      return launch_sigchk_tiles(c->stream, n_tiles, tiles, sums, tables, inf, h_aff, h_lines, h_st,
                                 d_status, to_leaves ? leaf_count : sub_count,
                                 to_leaves ? leaves : sub_list, to_leaves);
    }));
  }
  if (!to_leaves && !exact) {
    HB_TRY(timed(c, "sig_lines", [&] {
      return launch_plines(c->stream, 1, 16 * n_tiles, 0, sub_count, sub_list, tiles, sums, dec,
                           tables, inf);
    }));
    HB_TRY(timed(c, "chk_subs", [&] {
      return launch_sigchk_subs(c->stream, n_tiles, sub_count, sub_list, tiles, sums, tables, inf,
                                h_aff, h_lines, d_status, leaf_count, leaves);
    }));
  }
  // leaves in chunks: launches past the device-side count exit at once.  A chunk as large as the
  // table buffer already is (16 tables per tile for the sub-tile level), so a large call issues a
  // few launch pairs rather than n_items / LEAF_CHUNK (C4: 4 instead of 20 -- the empty ones wait
  // for free CU slots behind the other lanes' item passes)
  const uint32_t leaf_chunk = (uint32_t)n_tables;
  for (uint32_t base = 0; base < n_items; base += leaf_chunk) {
    const uint32_t chunk = std::min(leaf_chunk, n_items - base);
    if (!fused)
      HB_TRY(timed(c, "sig_lines", [&] {
        return launch_plines(c->stream, 2, chunk, base, leaf_count, leaves, tiles, sums, dec, tables,
                             inf);
      }));
    HB_TRY(timed(c, "chk_leaves", [&] {
      // a short list (<= 2 leaves per SIMD, all in the first chunk) in the latency form
      const uint32_t lim = (rep3 && base == 0) ? std::min(chunk, 8u * (uint32_t)c->n_cu) : 0u;
      const hipError_t e = launch_sigchk_leaves_rep3(c->stream, chunk, lim, leaf_count, leaves, d_idx,
                                                     ks->pk, tables, inf, h_aff, h_lines, d_status);
      if (e != hipSuccess) return e;
      return launch_sigchk_leaves(c->stream, base, chunk, leaf_count, leaves, d_idx, ks->pk, tables,
                                  inf, h_aff, h_lines, d_status, lim);
    }));
  }
  c->last_leaf_count = leaf_count;
  HB_TRY(timed(c, "rlc_finalize", [&] {
    return launch_rlc_finalize(c->stream, n_tiles, tiles, h_st, h_st, d_status, d_idx, ks->n,
                               ks->rejects + (size_t)c->lane * ks->n,
                               const_cast<uint32_t*>(sus.last_bad), sus.now,
                               track_threshold(ks, n_items));
  }));
  return end_verify(c);
}

// Window width of a batch of n-term MSMs of scalars < 2^bits: minimise W * (mixed adds + bucket
// adds) in Fqm (mixed add 11, full add 16, segment scaling ~15 per bit per 8 buckets), W =
// ceil((bits + 1) / c) windows (the signed recoding's last carry needs the extra bit).
uint32_t msm_window(uint32_t n, uint32_t bits = 255) {
  uint32_t best = 4;
  double best_cost = 1e300;
  for (uint32_t c = 4; c <= 13; ++c) {
    const double B = double(1u << (c - 1)), W = double((bits + c) / c);
    const double cost = W * (11.0 * n + 16.0 * B + (B / 8) * 15.0 * c) + W * c * 7.0;
    if (cost < best_cost) {
      best_cost = cost;
      best = c;
    }
  }
  return best;
}

// Window width by the LONGEST per-lane chain instead (in Fqm): a segment thread of
// k_msm_buckets walks 8n/B list terms (mixed adds), 8 rank sums and a small multiple; k_msm_wsum
// adds S = B/8 segments; k_msm_final runs (bits + 1) doublings and W adds.  For batches too small
// to fill the GPU the combine's time is this chain, not the total work.
uint32_t msm_window_latency(uint32_t n, uint32_t bits) {
  uint32_t best = 4;
  double best_cost = 1e300;
  for (uint32_t c = 4; c <= 13; ++c) {
    const double B = double(1u << (c - 1)), S = B / 8, W = double((bits + c) / c);
    const double cost = 11.0 * n / S + 16.0 * 8 + 23.0 * (c - 1) + 16.0 * S + 7.0 * (bits + 1) + 16.0 * W;
    if (cost < best_cost) {
      best_cost = cost;
      best = c;
    }
  }
  return best;
}

MsmPlan msm_plan(uint32_t n_msm, uint32_t n, uint32_t bits = 255) {
  MsmPlan p;
  p.n_msm = n_msm;
  p.n = n;
  p.c = msm_window(n, bits);
  if (bits <= 128) {  // the φ / ψ-split combines: short scalars, often latency-bound batches
    const uint64_t lanes = (uint64_t)n_msm * ((bits + p.c) / p.c) * std::max(1u, (1u << (p.c - 1)) / 8);
    if (lanes < 65536) p.c = msm_window_latency(n, bits);
  }
  p.W = (bits + p.c) / p.c;
  return p;
}

// Digits, bucket lists and the bucket reduction of a planned batch (points already decoded into
// `pts`), ordered on `st`.  `tag` prefixes the workspace names.
template <class F>
int msm_run(hbtc_ctx* c, hipStream_t st, const MsmPlan& p, const uint32_t* d_scalars,
            const Aff<F>* d_pts, const uint32_t* sel_cnt, uint32_t t, const uint32_t* d_bad,
            const uint32_t* d_dup, int32_t* d_status, uint8_t* d_out, uint8_t* d_parity,
            const uint32_t* d_pts_map = nullptr) {
  const uint64_t terms = (uint64_t)p.n_msm * p.n;
  const uint64_t mw = (uint64_t)p.n_msm * p.W;
  const uint32_t B = 1u << (p.c - 1), S = B / 8;
  int16_t* d_digits;
  uint32_t *d_list, *d_roff;
  Jac<F>*d_part, *d_wsum;
  HB_TRY(wst(c, "msm.digits", terms * p.W, &d_digits));
  HB_TRY(wst(c, "msm.list", terms * p.W, &d_list));
  HB_TRY(wst(c, "msm.roff", mw * (B + 1), &d_roff));
  HB_TRY(ws(c, "msm.part", mw * S * sizeof(Jac<F>), (void**)&d_part));
  HB_TRY(ws(c, "msm.wsum", mw * sizeof(Jac<F>), (void**)&d_wsum));
  HB_TRY(timed_on(c, st, "comb_digits", [&] {
    return launch_msm_digits(st, p, d_scalars, d_digits, d_list, d_roff);
  }));
  return timed_on(c, st, "combine", [&] {
    if constexpr (sizeof(F) == sizeof(Fq))
      return launch_msm_reduce_g1(st, p, d_pts, d_pts_map, d_list, d_roff, d_part, d_wsum, sel_cnt, t, d_bad,
                                  d_dup, d_status, d_out);
    else
      return launch_msm_reduce_g2(st, p, d_pts, d_pts_map, d_list, d_roff, d_part, d_wsum, sel_cnt, t, d_bad,
                                  d_dup, d_status, d_out, d_parity);
  });
}

// Lagrange combine on s_comb: ordered after everything already on the main stream (its inputs),
// overlapped with whatever the main stream does next.  The first t items of every instance are
// combined; with d_item_status, the first t items whose status is ACCEPT (hbbft combines only
// verified shares: coin.rs:185-191 iterates `received_shares`, td.rs:184 `shares`, both holding
// verified shares only).
int combine_dev(hbtc_ctx* c, int group, uint32_t n_inst, const uint32_t* offsets,
                const uint32_t* d_idx, const uint8_t* d_pts, uint32_t t, uint8_t* d_out,
                uint8_t* d_parity, int32_t* d_inst_status, const int32_t* d_item_status = nullptr) {
  uint32_t n_items;
  HB_TRY(check_offsets(c, n_inst, offsets, &n_items));
  if (n_inst == 0) return HBTC_OK;
  if (t == 0) return fail(c, HBTC_ERR_ARG, "t must be >= 1");
  if (!aligned16(d_pts) || !aligned16(d_out))
    return fail(c, HBTC_ERR_ARG, "point arrays must be 16-byte aligned");
  hipStream_t sc = c->s_comb;
  {  // on the current lane, after the verification that produced the statuses (or whatever
     // wrote the inputs), and behind any other lane that writes one of them
    const std::vector<std::pair<uintptr_t, uintptr_t>> reads = {
        rng(d_idx, (size_t)n_items * 4), rng(d_pts, (size_t)n_items * (group == 1 ? 48 : 96)),
        rng(d_item_status, d_item_status ? (size_t)n_items * 4 : 0)};
    for (int o = 0; o < hbtc_ctx::NL; ++o) {
      Lane& other = c->lanes[o];
      if (o != c->lane && other.busy && ranges_overlap(reads, other.wr))
        HB_TRY(stream_after(c, sc, other.stream, other.ev_main));
    }
  }
  void* p;
  HB_TRY(stage_upload(c, "comb.offsets", offsets, ((size_t)n_inst + 1) * 4, sc, &p));
  uint32_t* d_off = static_cast<uint32_t*>(p);
  const size_t pbytes = group == 1 ? 48 : 96;
  if (c->comb_small && t <= COMB_SMALL_T) {
    // one launch per batch (hbtc_comb.hip): selection, Lagrange, per-share double-and-add and the
    // tree sum in one workgroup per instance, on the decoded shares of the verification when this
    // combine follows it over the same arrays
    const auto& ld = c->last_dec;
    const bool same = d_item_status && ld.status == d_item_status && ld.shares == d_pts &&
                      ld.n_items == n_items;
    const void* dec = same ? (group == 1 ? (const void*)ld.dec : (const void*)ld.dec2) : nullptr;
    CombSmallArgs a{};
    a.t = t;
    a.offsets = d_off;
    a.item_status = d_item_status;
    a.idx = d_idx;
    a.pts = d_pts;
    a.dec = dec;
    a.inst_status = d_inst_status;
    a.out = d_out;
    a.parity = group == 2 ? d_parity : nullptr;
    HB_TRY(timed_on(c, sc, "combine", [&] { return launch_comb_small(sc, group, n_inst, 1, a); }));
    return note_comb_reads(c, {{d_idx, (size_t)n_items * 4}, {d_pts, n_items * pbytes},
                               {d_item_status, d_item_status ? (size_t)n_items * 4 : 0},
                               {dec, dec ? n_items * (group == 1 ? sizeof(G1A) : sizeof(G2A)) : 0}});
  }
  const uint64_t terms = (uint64_t)n_inst * t;
  uint32_t *d_sel_pos, *d_sel_idx, *d_sel_cnt, *d_dup, *d_bad;
  Fr *d_lambda, *d_lws;
  HB_TRY(wst(c, "comb.lws", terms, &d_lws));
  HB_TRY(wst(c, "comb.sel_pos", terms, &d_sel_pos));
  HB_TRY(wst(c, "comb.sel_idx", terms, &d_sel_idx));
  HB_TRY(wst(c, "comb.sel_cnt", n_inst, &d_sel_cnt));
  HB_TRY(wst(c, "comb.dup", n_inst, &d_dup));
  HB_TRY(wst(c, "comb.bad", n_inst, &d_bad));
  HB_TRY(wst(c, "comb.lambda", terms, &d_lambda));
  HB_CHECK(c, launch_zero_u32(sc, d_dup, n_inst));
  HB_CHECK(c, launch_zero_u32(sc, d_bad, n_inst));
  LagrangeFact lf{};
  if (c->lagrange_fact && !c->fact) {
    // once per context: 0! .. FACT_N! and their inverses, then every stream may read them.  One
    // allocation holds both tables and the build's partial products (nothing is freed in the
    // middle of the pipeline: hipFree synchronises the device), and the tables are published
    // only once built; if any step fails the context keeps the O(t) coefficients instead
    // (a half-built table would give wrong coefficients under an ACCEPT status).
    const size_t n = FACT_N + 1;
    Fr* tab = nullptr;
    hipError_t e = hipMalloc(&tab, sizeof(Fr) * (2 * n + FACT_N / 256 + 1));
    if (e == hipSuccess) e = launch_fact_tables(sc, FACT_N, tab + 2 * n, tab, tab + n);
    if (e == hipSuccess) e = hipStreamSynchronize(sc);
    if (e == hipSuccess) {
      c->fact = tab;
      c->inv_fact = tab + n;
    } else {
      if (tab) (void)hipFree(tab);
      c->lagrange_fact = false;
      HB_CHECK(c, e);
    }
  }
  if (c->lagrange_fact) {
    uint32_t* d_done;
    HB_TRY(wst(c, "comb.fact_done", n_inst, &d_done));
    lf = LagrangeFact{c->fact, c->inv_fact, FACT_N, d_sel_cnt, d_done};
  }
  HB_TRY(timed_on(c, sc, "lagrange", [&] {
    hipError_t e = launch_select(sc, n_inst, d_off, t, d_item_status, d_idx, d_sel_pos, d_sel_idx,
                                 d_sel_cnt);
    if (e != hipSuccess) return e;
    return launch_lagrange_sel(sc, n_inst, t, d_sel_idx, d_lambda, d_lws, d_dup,
                               c->lagrange_fact ? &lf : nullptr);
  }));
  const MsmPlan plan = msm_plan(n_inst, t);
  const size_t pb = group == 1 ? 48 : 96;
  if (group == 1) {
    // the decoded shares of the verification that produced d_item_status, when it is the last
    // RLC DecryptionShare call over these very arrays
    const auto& ld = c->last_dec;
    const G1A* dec = (d_item_status && ld.status == d_item_status && ld.shares == d_pts &&
                      ld.n_items == n_items)
                         ? ld.dec
                         : nullptr;
    G1A* d_aff;
    HB_TRY(wst(c, "comb.g1", terms, &d_aff));
    HB_TRY(timed_on(c, sc, "comb_decode", [&] {
      if (dec)  // every selected item is ACCEPTed and was decoded by the verification
        return launch_msm_gather_g1(sc, n_inst, t, d_sel_pos, d_sel_cnt, dec, d_aff);
      return launch_msm_decode_g1(sc, n_inst, t, t, d_pts, d_sel_pos, d_sel_cnt, d_item_status,
                                  nullptr, d_aff, d_bad);
    }));
    if (c->g1_glv) {
      // φ = [-x^2] on G1: two 128-bit terms per share (k_msm_glv_g1), a Horner chain of ~128
      // doublings instead of ~255
      G1A* d_aff2;
      uint32_t* d_sc2;
      HB_TRY(wst(c, "comb.g1x2", 2 * terms, &d_aff2));
      HB_TRY(wst(c, "comb.lws2", 2 * terms * 8, &d_sc2));
      HB_TRY(timed_on(c, sc, "comb_digits", [&] {
        return launch_msm_glv_g1(sc, n_inst, t, (const uint32_t*)d_lambda, d_aff, d_sc2, d_aff2);
      }));
      const MsmPlan plan2 = msm_plan(n_inst, 2 * t, 128);
      HB_TRY(msm_run<Fq>(c, sc, plan2, d_sc2, d_aff2, d_sel_cnt, t, d_bad, d_dup, d_inst_status, d_out,
                         nullptr));
    } else {
      HB_TRY(msm_run<Fq>(c, sc, plan, (const uint32_t*)d_lambda, d_aff, d_sel_cnt, t, d_bad, d_dup,
                         d_inst_status, d_out, nullptr));
    }
    return note_comb_reads(c, {{d_idx, (size_t)n_items * 4}, {d_pts, n_items * pb},
                               {d_item_status, d_item_status ? (size_t)n_items * 4 : 0},
                               {dec, dec ? n_items * sizeof(G1A) : 0}});
  }
  const auto& ld = c->last_dec;
  const G2A* dec2 = (d_item_status && ld.status == d_item_status && ld.shares == d_pts &&
                     ld.n_items == n_items)
                        ? ld.dec2
                        : nullptr;
  G2A* d_aff;
  HB_TRY(wst(c, "comb.g2", terms, &d_aff));
  HB_TRY(timed_on(c, sc, "comb_decode", [&] {
    if (dec2) return launch_msm_gather_g2(sc, n_inst, t, d_sel_pos, d_sel_cnt, dec2, d_aff);
    return launch_msm_decode_g2(sc, n_inst, t, t, d_pts, d_sel_pos, d_sel_cnt, d_item_status,
                                nullptr, d_aff, d_bad);
  }));
  if (c->g2_gls) {
    // ψ = [x] on G2: four 64-bit terms per share (k_msm_gls_g2), so the Horner chain of the
    // final pass is ~64 doublings instead of ~255 (the G2 combine is the lane's latency tail)
    G2A* d_aff4;
    uint32_t* d_sc4;
    HB_TRY(wst(c, "comb.g2x4", 4 * terms, &d_aff4));
    HB_TRY(wst(c, "comb.lws4", 4 * terms * 8, &d_sc4));
    HB_TRY(timed_on(c, sc, "comb_digits", [&] {
      return launch_msm_gls_g2(sc, n_inst, t, (const uint32_t*)d_lambda, d_aff, d_sc4, d_aff4);
    }));
    const MsmPlan plan4 = msm_plan(n_inst, 4 * t, 64);
    HB_TRY(msm_run<Fq2>(c, sc, plan4, d_sc4, d_aff4, d_sel_cnt, t, d_bad, d_dup, d_inst_status,
                        d_out, d_parity));
  } else {
    HB_TRY(msm_run<Fq2>(c, sc, plan, (const uint32_t*)d_lambda, d_aff, d_sel_cnt, t, d_bad, d_dup,
                        d_inst_status, d_out, d_parity));
  }
  return note_comb_reads(c, {{d_idx, (size_t)n_items * 4}, {d_pts, n_items * pb},
                             {d_item_status, d_item_status ? (size_t)n_items * 4 : 0},
                             {dec2, dec2 ? n_items * sizeof(G2A) : 0}});
}

int point_mul_host(hbtc_ctx* c, int group, uint32_t n, const uint8_t* base,
                   uint32_t base_stride, const uint8_t* scalars, uint8_t* out, int32_t* status) {
  const size_t pb = group == 1 ? 48 : 96;
  if (base_stride > 1) return fail(c, HBTC_ERR_ARG, "base_stride must be 0 or 1");
  if (n == 0) return HBTC_OK;
  void *d_base, *d_k, *d_out, *d_st;
  HB_TRY(upload(c, "in0", base, pb * (base_stride ? n : 1), &d_base));
  HB_TRY(upload(c, "in1", scalars, (size_t)32 * n, &d_k));
  HB_TRY(ws(c, "out0", pb * n, &d_out));
  HB_TRY(ws(c, "out1", (size_t)4 * n, &d_st));
  HB_TRY(timed(c, "mul", [&] {
    return launch_point_mul(c->stream, group, n, (const uint8_t*)d_base, base_stride,
                            (const uint8_t*)d_k, 1, (uint8_t*)d_out, (int32_t*)d_st);
  }));
  HB_TRY(download(c, out, d_out, pb * n));
  HB_TRY(download(c, status, d_st, (size_t)4 * n));
  return sync(c);
}

// ---------------------------------------------------------------- asynchronous host epochs
size_t round256(size_t x) { return (x + 255) & ~(size_t)255; }

int pinned_grow(hbtc_ctx* c, void** h, size_t* cap, size_t bytes) {
  if (*cap >= bytes && *h) return HBTC_OK;
  HB_TRY(reap_retired(c, false));
  if (*h) c->retiring_host.push_back(*h);  // retired behind a fence (see retire_fence)
  *h = nullptr;
  *cap = 0;
  const size_t want = bytes + bytes / 4 + 256;
  const hipError_t e = hipHostMalloc(h, want, hipHostMallocDefault);
  HB_TRY(retire_fence(c));
  HB_CHECK(c, e);
  *cap = want;
  return HBTC_OK;
}

// The ticket's results are on the host: copy them out of the pinned staging into the caller's
// buffers.
int finish_ticket(hbtc_ctx* c, hbtc_ctx::Ticket& T) {
  if (!T.active) return HBTC_OK;
  HB_CHECK(c, hipEventSynchronize(T.ev));
  const uint8_t* o = static_cast<const uint8_t*>(T.h_out);
  size_t off = 0;
  memcpy(T.status, o, 4 * T.n_items);
  off = round256(4 * T.n_items);
  if (T.combined) {
    memcpy(T.out, o + off, T.pt * T.n_inst);
    off += round256(T.pt * T.n_inst);
    if (T.parity) memcpy(T.parity, o + off, T.n_inst);
    off += round256(T.n_inst);
    memcpy(T.inst_status, o + off, 4 * T.n_inst);
  }
  T.active = false;
  return HBTC_OK;
}

// One epoch from host buffers without blocking: inputs into the next lane's pinned staging,
// H2D, verification, the combine of the first t verified shares of every instance (t > 0) and
// D2H of the results, all on that lane's stream (group 1: DecryptionShares, 2: SignatureShares).
int epoch_submit(hbtc_ctx* c, int group, uint32_t keyset_id, uint32_t n_inst, const uint8_t* H,
                 const uint8_t* w, const uint32_t* offsets, const uint32_t* idx, const uint8_t* items,
                 uint32_t t, int32_t* status, uint8_t* out, uint8_t* parity, int32_t* inst_status,
                 uint64_t* ticket) {
  uint32_t n;
  HB_TRY(check_offsets(c, n_inst, offsets, &n));
  const size_t pt = group == 1 ? 48 : 96;
  const int l = (c->lane + 1) % hbtc_ctx::NL;
  hbtc_ctx::Ticket& T = c->tickets[l];
  HB_TRY(finish_ticket(c, T));  // the lane's previous epoch (its staging is reused)
  if (!T.ev) HB_CHECK(c, hipEventCreateWithFlags(&T.ev, hipEventDisableTiming));
  select_lane(c, l);
  const size_t sH = 96 * (size_t)n_inst, sW = group == 1 ? sH : 0, sI = 4 * (size_t)n, sP = pt * n;
  const size_t oW = round256(sH), oI = oW + round256(sW), oP = oI + round256(sI);
  HB_TRY(pinned_grow(c, &T.h_in, &T.in_cap, oP + sP));
  uint8_t* hi = static_cast<uint8_t*>(T.h_in);
  if (sH) memcpy(hi, H, sH);
  if (sW) memcpy(hi + oW, w, sW);
  if (sI) memcpy(hi + oI, idx, sI);
  if (sP) memcpy(hi + oP, items, sP);
  void *d_H, *d_w = nullptr, *d_idx, *d_items, *d_st, *d_out = nullptr, *d_par = nullptr, *d_cst = nullptr;
  HB_TRY(ws(c, "ep.H", sH, &d_H));
  if (sW) HB_TRY(ws(c, "ep.w", sW, &d_w));
  HB_TRY(ws(c, "ep.idx", sI, &d_idx));
  HB_TRY(ws(c, "ep.items", sP, &d_items));
  HB_TRY(ws(c, "ep.status", 4 * (size_t)n, &d_st));
  HB_TRY(guard_write(c, d_H, sH));
  HB_TRY(guard_write(c, d_idx, sI));
  HB_TRY(guard_write(c, d_items, sP));
  if (sH) HB_CHECK(c, hipMemcpyAsync(d_H, hi, sH, hipMemcpyHostToDevice, c->stream));
  if (sW) HB_CHECK(c, hipMemcpyAsync(d_w, hi + oW, sW, hipMemcpyHostToDevice, c->stream));
  if (sI) HB_CHECK(c, hipMemcpyAsync(d_idx, hi + oI, sI, hipMemcpyHostToDevice, c->stream));
  if (sP) HB_CHECK(c, hipMemcpyAsync(d_items, hi + oP, sP, hipMemcpyHostToDevice, c->stream));
  const bool comb = t > 0 && n_inst > 0;
  {
    PinLane pin(c);  // the uploads above went to lane l: verification and combine stay there
    HostG2Args hg(c, d_H, sH ? hi : nullptr, d_w, sW ? hi + oW : nullptr);
    if (group == 1)
      HB_TRY(dec_shares_dev(c, keyset_id, n_inst, (const uint8_t*)d_H, (const uint8_t*)d_w, offsets,
                            (const uint32_t*)d_idx, (const uint8_t*)d_items, (int32_t*)d_st));
    else
      HB_TRY(sig_shares_dev(c, keyset_id, n_inst, (const uint8_t*)d_H, offsets, (const uint32_t*)d_idx,
                            (const uint8_t*)d_items, (int32_t*)d_st));
    if (comb) {
      HB_TRY(ws(c, "ep.out", pt * n_inst, &d_out));
      if (group == 2) HB_TRY(ws(c, "ep.par", n_inst, &d_par));
      HB_TRY(ws(c, "ep.cst", 4 * (size_t)n_inst, &d_cst));
      HB_TRY(combine_dev(c, group, n_inst, offsets, (const uint32_t*)d_idx, (const uint8_t*)d_items, t,
                         (uint8_t*)d_out, (uint8_t*)d_par, (int32_t*)d_cst, (const int32_t*)d_st));
      HB_TRY(stream_after(c, c->stream, c->s_comb, c->ev_comb));
    }
  }
  const size_t q1 = round256(4 * (size_t)n), q2 = q1 + round256(pt * n_inst), q3 = q2 + round256(n_inst);
  HB_TRY(pinned_grow(c, &T.h_out, &T.out_cap, q3 + 4 * (size_t)n_inst + 16));
  uint8_t* ho = static_cast<uint8_t*>(T.h_out);
  if (n) HB_CHECK(c, hipMemcpyAsync(ho, d_st, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
  if (comb) {
    HB_CHECK(c, hipMemcpyAsync(ho + q1, d_out, pt * n_inst, hipMemcpyDeviceToHost, c->stream));
    if (d_par) HB_CHECK(c, hipMemcpyAsync(ho + q2, d_par, n_inst, hipMemcpyDeviceToHost, c->stream));
    HB_CHECK(c, hipMemcpyAsync(ho + q3, d_cst, 4 * (size_t)n_inst, hipMemcpyDeviceToHost, c->stream));
  }
  HB_CHECK(c, hipEventRecord(T.ev, c->stream));
  T.status = status;
  T.out = out;
  T.parity = group == 2 ? parity : nullptr;
  T.inst_status = inst_status;
  T.n_items = n;
  T.n_inst = n_inst;
  T.pt = pt;
  T.combined = comb;
  T.active = true;
  T.id = c->next_ticket++;
  *ticket = T.id;
  return HBTC_OK;
}

struct Guard {
  hbtc_ctx* c;
  std::lock_guard<std::mutex> lk;
  explicit Guard(hbtc_ctx* ctx) : c(ctx), lk(ctx->mu) { (void)hipSetDevice(ctx->device); }
};

}  // namespace

// ============================================================================ C ABI
extern "C" {

int hbtc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* hbtc_version(void) { return "hbtc 0.1 gfx950 (HIP, VALU 32-bit-limb Montgomery)"; }

int hbtc_ctx_create(int device, hbtc_ctx** out) {
  if (!out) return HBTC_ERR_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return HBTC_ERR_DEVICE;
  if (hipSetDevice(device) != hipSuccess) return HBTC_ERR_DEVICE;
  hbtc_ctx* c = new hbtc_ctx();
  c->device = device;
  if (const char* e = getenv("HBTC_ITEMS_SERIAL")) c->items_serial = atoi(e);
  if (const char* e = getenv("HBTC_G2_GLS")) c->g2_gls = atoi(e) != 0;
  if (const char* e = getenv("HBTC_G1_GLV")) c->g1_glv = atoi(e) != 0;
  if (const char* e = getenv("HBTC_COMB_SMALL")) c->comb_small = atoi(e) != 0;
  if (const char* e = getenv("HBTC_COIN_SPEC")) c->coin_spec = atoi(e) != 0;
  c->sig_fused = sig_exact_built();
  if (const char* e = getenv("HBTC_SIG_FUSED")) c->sig_fused = c->sig_fused && atoi(e) != 0;
  if (const char* e = getenv("HBTC_TRACK")) c->track_senders = atoi(e) != 0;
  if (const char* e = getenv("HBTC_LAGRANGE_FACT")) c->lagrange_fact = atoi(e) != 0;
  if (const char* e = getenv("HBTC_PROBE")) c->probe_cold = atoi(e) != 0;
  if (const char* e = getenv("HBTC_SPLIT")) c->split_levels = atoi(e) != 0;
  if (const char* e = getenv("HBTC_GT_REP")) c->small_rep = atoi(e) == 1 ? 1 : 3;
  if (const char* e = getenv("HBTC_EXACT_BELOW")) c->exact_below = (uint32_t)atol(e);
  if (const char* e = getenv("HBTC_RLC_BITS")) {  // A/B runs: 64 or 128, like hbtc_set_rlc_bits
    const int b = atoi(e);
    if (b == 64 || b == 128) c->rlc_bits = (uint32_t)b;
  }
  if (const char* e = getenv("HBTC_PB_CHUNK")) {
    const long v = atol(e);
    if (v >= 64 && v % 64 == 0 && v <= (1l << 20)) c->pb_chunk = (uint32_t)v;
  }
  if (const char* e = getenv("HBTC_CHECK_MODE")) {
    const std::string m(e);
    c->check_mode_forced = m == "plain" ? 0 : m == "pair3" ? 1 : m == "pair2" ? 2 : -1;
  }
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
      c->n_cu = prop.multiProcessorCount;
  }
  // NL lane streams and the preparation stream (GPU_MAX_HW_QUEUES = 4: with 4 lanes two streams
  // share a hardware queue, which costs concurrency, never correctness: every wait is on an
  // event recorded by work submitted earlier).  The G2 preparation stream is shared by the lanes
  // (its work is short and ordered anyway); a lane's combines run on the lane's own stream.
  // a failing HIP call is reported on stderr with its name and error (no context exists yet to
  // hold the message); the objects created so far are released by hbtc_ctx_destroy
  auto created = [&](hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    fprintf(stderr, "hbtc_ctx_create(device %d): %s failed: %s (%d)\n", device, what,
            hipGetErrorString(e), (int)e);
    return false;
  };
  for (Lane& l : c->lanes)
    if (!created(hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking), "hipStreamCreateWithFlags") ||
        !created(hipEventCreateWithFlags(&l.ev_main, hipEventDisableTiming), "hipEventCreateWithFlags") ||
        !created(hipEventCreateWithFlags(&l.ev_prep, hipEventDisableTiming), "hipEventCreateWithFlags") ||
        !created(hipEventCreateWithFlags(&l.done, hipEventDisableTiming), "hipEventCreateWithFlags") ||
        !created(hipEventCreateWithFlags(&l.items_done, hipEventDisableTiming), "hipEventCreateWithFlags") ||
        !created(hipEventCreateWithFlags(&l.dec_done, hipEventDisableTiming), "hipEventCreateWithFlags")) {
      hbtc_ctx_destroy(c);
      return HBTC_ERR_DEVICE;
    }
  // the preparation is a short latency-bound chain (few waves) that the checks wait for: its
  // stream has the highest priority, so its workgroups are dispatched ahead of the item pass's
  int prio_least = 0, prio_greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess) prio_greatest = 0;
  if (!created(hipStreamCreateWithPriority(&c->lanes[0].s_prep, hipStreamNonBlocking, prio_greatest),
               "hipStreamCreateWithPriority")) {
    hbtc_ctx_destroy(c);
    return HBTC_ERR_DEVICE;
  }
  for (Lane& l : c->lanes) l.s_prep = c->lanes[0].s_prep;
  select_lane(c, 0);
  if (!created(hipEventCreateWithFlags(&c->ev_comb, hipEventDisableTiming), "hipEventCreateWithFlags") ||
      !created(hipEventCreateWithFlags(&c->ev_ext, hipEventDisableTiming), "hipEventCreateWithFlags") ||
      !created(hipEventCreateWithFlags(&c->ev_ext2, hipEventDisableTiming), "hipEventCreateWithFlags") ||
      !created(hipEventCreateWithFlags(&c->ev_ext3, hipEventDisableTiming), "hipEventCreateWithFlags")) {
    hbtc_ctx_destroy(c);
    return HBTC_ERR_DEVICE;
  }
  *out = c;
  return HBTC_OK;
}

void hbtc_ctx_destroy(hbtc_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  for (auto& kv : c->bufs)
    if (kv.second.p) (void)hipFree(kv.second.p);
  (void)retire_fence(c);
  (void)reap_retired(c, true);
  if (c->fact) (void)hipFree(c->fact);  // inv_fact lives in the same allocation
  if (c->prep.aff) (void)hipFree(c->prep.aff);
  if (c->prep.st) (void)hipFree(c->prep.st);
  if (c->prep.lines) (void)hipFree(c->prep.lines);
  for (auto& kv : c->keysets) {
    (void)hipFree(kv.second.pk);
    (void)hipFree(kv.second.st);
    (void)hipFree(kv.second.tab);
    (void)hipFree(kv.second.last_bad);
    (void)hipFree(kv.second.rejects);
    (void)hipFree(kv.second.master);
  }
  for (Span& sp : c->spans) {
    (void)hipEventDestroy(sp.a);
    (void)hipEventDestroy(sp.b);
  }
  for (auto& r : c->comb_reads) (void)hipEventDestroy(r.ev);
  for (auto& kv : c->gf_plans) {
    (void)hipFree(kv.second.out_rows);
    (void)hipFree(kv.second.in_rows);
    (void)hipFree(kv.second.tabs);
  }
  for (auto& tk : c->tickets) {
    if (tk.active && tk.ev) (void)hipEventSynchronize(tk.ev);
    if (tk.ev) (void)hipEventDestroy(tk.ev);
    if (tk.h_in) (void)hipHostFree(tk.h_in);
    if (tk.h_out) (void)hipHostFree(tk.h_out);
  }
  for (auto& kv : c->stages) {
    if (kv.second.h) (void)hipHostFree(kv.second.h);
    if (kv.second.ev) (void)hipEventDestroy(kv.second.ev);
  }
  // (a context whose creation failed part-way has some of these still null)
  auto ev_free = [](hipEvent_t e) {
    if (e) (void)hipEventDestroy(e);
  };
  for (Lane& l : c->lanes) {
    ev_free(l.ev_main);
    ev_free(l.ev_prep);
    ev_free(l.done);
    ev_free(l.items_done);
    ev_free(l.dec_done);
    if (l.stream) (void)hipStreamDestroy(l.stream);
  }
  if (c->lanes[0].s_prep) (void)hipStreamDestroy(c->lanes[0].s_prep);
  ev_free(c->ev_comb);
  ev_free(c->ev_ext);
  ev_free(c->ev_ext2);
  ev_free(c->ev_ext3);
  ev_free(c->ev_spec_in);
  ev_free(c->ev_spec_out);
  ev_free(c->ev_spec_out2);
  if (c->s_spec) (void)hipStreamDestroy(c->s_spec);
  if (c->s_spec2) (void)hipStreamDestroy(c->s_spec2);
  delete c;
}

const char* hbtc_last_error(hbtc_ctx* c) { return c ? c->err.c_str() : "null context"; }

int hbtc_keyset_load(hbtc_ctx* c, const uint8_t* pk_c48, uint32_t n, uint32_t* keyset_id,
                     uint32_t* n_bad) {
  if (!c || !pk_c48 || !keyset_id || n == 0) return HBTC_ERR_ARG;
  Guard g(c);
  Keyset ks;
  ks.n = n;
  HB_CHECK(c, hipMalloc(&ks.pk, sizeof(G1A) * n));
  HB_CHECK(c, hipMalloc(&ks.st, sizeof(int32_t) * n));
  void* d_in;
  HB_TRY(upload(c, "in0", pk_c48, (size_t)48 * n, &d_in));
  HB_TRY(timed(c, "prepare", [&] {
    return launch_g1_decode(c->stream, (const uint8_t*)d_in, n, ks.pk, ks.st);
  }));
  HB_CHECK(c, hipMalloc(&ks.tab, sizeof(PtXY) * (size_t)n * PK_TAB_WIN * 256));
  HB_CHECK(c, hipMalloc(&ks.last_bad, sizeof(uint32_t) * n));
  HB_CHECK(c, launch_zero_u32(c->stream, ks.last_bad, n));
  HB_CHECK(c, hipMalloc(&ks.rejects, hbtc_ctx::NL * sizeof(uint32_t) * n));  // one count array per lane
  HB_CHECK(c, launch_zero_u32(c->stream, ks.rejects, hbtc_ctx::NL * (size_t)n));
  Fq* tab_ws;
  HB_TRY(wst(c, "pktab.ws", (size_t)n * PK_TAB_WIN * 512, &tab_ws));
  HB_TRY(timed(c, "prepare", [&] {
    return launch_pk_table(c->stream, ks.pk, ks.st, n, ks.tab, tab_ws);
  }));
  std::vector<int32_t> st(n);
  HB_TRY(download(c, st.data(), ks.st, sizeof(int32_t) * n));
  HB_TRY(sync(c));
  uint32_t bad = 0;
  for (uint32_t i = 0; i < n; ++i) bad += st[i] != HBTC_ACCEPT;
  if (n_bad) *n_bad = bad;
  const uint32_t id = c->next_keyset++;
  c->keysets[id] = ks;
  *keyset_id = id;
  return HBTC_OK;
}

int hbtc_keyset_free(hbtc_ctx* c, uint32_t keyset_id) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  auto it = c->keysets.find(keyset_id);
  if (it == c->keysets.end()) return fail(c, HBTC_ERR_NO_KEYSET, "unknown keyset id");
  HB_TRY(sync(c));
  (void)hipFree(it->second.pk);
  (void)hipFree(it->second.st);
  (void)hipFree(it->second.tab);
  (void)hipFree(it->second.last_bad);
  (void)hipFree(it->second.rejects);
  (void)hipFree(it->second.master);
  c->keysets.erase(it);
  return HBTC_OK;
}

int hbtc_verify_sig_shares(hbtc_ctx* c, uint32_t keyset_id, uint32_t n_inst, const uint8_t* H,
                           const uint32_t* offsets, const uint32_t* idx, const uint8_t* sig,
                           int32_t* status) {
  if (!c || (n_inst && (!H || !offsets))) return HBTC_ERR_ARG;
  Guard g(c);
  uint32_t n;
  HB_TRY(check_offsets(c, n_inst, offsets, &n));
  if (n && (!idx || !sig || !status)) return fail(c, HBTC_ERR_ARG, "NULL item array");
  void *d_H, *d_idx, *d_sig, *d_st;
  HB_TRY(upload(c, "in0", H, (size_t)96 * n_inst, &d_H));
  HB_TRY(upload(c, "in1", idx, (size_t)4 * n, &d_idx));
  HB_TRY(upload(c, "in2", sig, (size_t)96 * n, &d_sig));
  HB_TRY(ws(c, "out0", (size_t)4 * n, &d_st));
  PinLane pin(c);  // the uploads above went to the current lane
  HostG2Args hg(c, d_H, H);
  HB_TRY(sig_shares_dev(c, keyset_id, n_inst, (const uint8_t*)d_H, offsets,
                        (const uint32_t*)d_idx, (const uint8_t*)d_sig, (int32_t*)d_st));
  HB_TRY(download(c, status, d_st, (size_t)4 * n));
  return sync(c);
}

// hbtc.h hbtc_prepare_g2: the new points' tables built by the usual preparation (k_g2_steps +
// k_g2_norm) into a scratch batch, then copied into their resident slots.
int hbtc_prepare_g2(hbtc_ctx* c, uint32_t n, const uint8_t* pts, int32_t* out_status) {
  if (!c || (n && !pts)) return HBTC_ERR_ARG;
  Guard g(c);
  if (n == 0) return HBTC_OK;
  HB_TRY(sync(c));  // no call in flight reads a slot this one fills
  auto& P = c->prep;
  std::vector<uint32_t> fresh;  // positions of points not prepared yet (first occurrence)
  {
    std::unordered_map<std::string, uint32_t> seen;
    for (uint32_t i = 0; i < n; ++i) {
      std::string key(reinterpret_cast<const char*>(pts + (size_t)96 * i), 96);
      if (P.slot.count(key) || seen.count(key)) continue;
      seen.emplace(std::move(key), i);
      fresh.push_back(i);
    }
  }
  const uint32_t m = (uint32_t)fresh.size();
  if (m) {
    const uint32_t reuse = std::min<uint32_t>(m, (uint32_t)P.free.size());
    const uint32_t need = P.top + (m - reuse);
    if (need > P.cap) {  // grow: new arrays, the resident slots copied over
      const uint32_t cap = std::max<uint32_t>(std::max<uint32_t>(2 * P.cap, need), 64);
      G2A* aff = nullptr;
      int32_t* st = nullptr;
      Line* lines = nullptr;
      hipError_t e = hipMalloc(&aff, sizeof(G2A) * cap);
      if (e == hipSuccess) e = hipMalloc(&st, sizeof(int32_t) * cap);
      if (e == hipSuccess) e = hipMalloc(&lines, sizeof(Line) * (size_t)cap * MILLER_STEPS);
      if (e == hipSuccess && P.top) e = launch_g2_tab_copy(c->stream, P.top, nullptr, nullptr, P.aff, P.st, P.lines,
                                                          aff, st, lines);
      if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
      if (e != hipSuccess) {
        if (aff) (void)hipFree(aff);
        if (st) (void)hipFree(st);
        if (lines) (void)hipFree(lines);
        HB_CHECK(c, e);
      }
      if (P.aff) (void)hipFree(P.aff);
      if (P.st) (void)hipFree(P.st);
      if (P.lines) (void)hipFree(P.lines);
      P.aff = aff;
      P.st = st;
      P.lines = lines;
      P.cap = cap;
    }
    std::vector<uint32_t> slots(m);
    std::vector<uint8_t> in((size_t)96 * m);
    for (uint32_t j = 0; j < m; ++j) {
      if (!P.free.empty()) {
        slots[j] = P.free.back();
        P.free.pop_back();
      } else {
        slots[j] = P.top++;
      }
      memcpy(in.data() + (size_t)96 * j, pts + (size_t)96 * fresh[j], 96);
    }
    void *d_in, *d_slots;
    G2A* taff;
    int32_t* tst;
    Line* tl;
    Fq2* tws;
    HB_TRY(upload(c, "prep.in", in.data(), in.size(), &d_in));
    HB_TRY(upload(c, "prep.slots", slots.data(), (size_t)4 * m, &d_slots));
    HB_TRY(wst(c, "prep.aff", m, &taff));
    HB_TRY(wst(c, "prep.st", m, &tst));
    HB_TRY(wst(c, "prep.lines", (size_t)m * MILLER_STEPS, &tl));
    HB_TRY(wst(c, "prep.ws", (size_t)m * 3 * MILLER_STEPS, &tws));
    HB_TRY(timed(c, "prepare", [&] {
      return launch_g2_prepare(c->stream, (const uint8_t*)d_in, m, nullptr, 0, taff, tl, tws, tst);
    }));
    HB_CHECK(c, launch_g2_tab_copy(c->stream, m, nullptr, (const uint32_t*)d_slots, taff, tst, tl, P.aff, P.st,
                                   P.lines));
    HB_TRY(sync(c));
    for (uint32_t j = 0; j < m; ++j)
      P.slot.emplace(std::string(reinterpret_cast<const char*>(pts + (size_t)96 * fresh[j]), 96), slots[j]);
  }
  if (out_status) {
    std::vector<int32_t> st(P.top);
    HB_CHECK(c, hipMemcpy(st.data(), P.st, sizeof(int32_t) * P.top, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i)
      out_status[i] = st[P.slot.at(std::string(reinterpret_cast<const char*>(pts + (size_t)96 * i), 96))];
  }
  return HBTC_OK;
}

int hbtc_unprepare_g2(hbtc_ctx* c, uint32_t n, const uint8_t* pts) {
  if (!c || (n && !pts)) return HBTC_ERR_ARG;
  Guard g(c);
  HB_TRY(sync(c));  // calls in flight may still read the slots
  for (uint32_t i = 0; i < n; ++i) {
    auto it = c->prep.slot.find(std::string(reinterpret_cast<const char*>(pts + (size_t)96 * i), 96));
    if (it == c->prep.slot.end()) continue;
    c->prep.free.push_back(it->second);
    c->prep.slot.erase(it);
  }
  return HBTC_OK;
}

int hbtc_prepared_g2_count(hbtc_ctx* c, uint32_t* count) {
  if (!c || !count) return HBTC_ERR_ARG;
  Guard g(c);
  *count = (uint32_t)c->prep.slot.size();
  return HBTC_OK;
}

int hbtc_keyset_set_master(hbtc_ctx* c, uint32_t keyset_id, const uint8_t* mpk) {
  if (!c || !mpk) return HBTC_ERR_ARG;
  Guard g(c);
  Keyset* ks;
  HB_TRY(get_keyset(c, keyset_id, &ks));
  HB_TRY(sync(c));
  if (ks->master) {
    (void)hipFree(ks->master);
    ks->master = nullptr;
  }
  G1A* d_m;
  HB_CHECK(c, hipMalloc(&d_m, sizeof(G1A)));
  int32_t st = -1;
  // every step after the allocation frees d_m on failure (the error paths leaked it)
  const int rc = [&]() -> int {
    int32_t* d_st;
    void* d_in;
    HB_TRY(upload(c, "in0", mpk, 48, &d_in));
    HB_TRY(wst(c, "out0", 1, &d_st));
    HB_CHECK(c, launch_g1_decode(c->stream, (const uint8_t*)d_in, 1, d_m, d_st));
    HB_TRY(download(c, &st, d_st, 4));
    return sync(c);
  }();
  if (rc != HBTC_OK || st != HBTC_ACCEPT) {
    (void)hipFree(d_m);
    return rc != HBTC_OK ? rc : fail(c, HBTC_ERR_ARG, "master public key fails to decode");
  }
  ks->master = d_m;
  return HBTC_OK;
}

// hbtc.h hbtc_coin_decide: the share checks on the lane stream (sig_shares_dev), the speculative
// leave-one-out combines and master checks on s_spec beside them, then the commit and the
// status-driven combine + master check of the instances the speculation missed.
int hbtc_coin_decide(hbtc_ctx* c, uint32_t keyset_id, uint32_t n_inst, const uint8_t* H,
                     const uint32_t* offsets, const uint32_t* idx, const uint8_t* sig, uint32_t t,
                     int32_t* status, uint8_t* sig_out, uint8_t* parity, int32_t* coin_status) {
  if (!c || (n_inst && (!H || !offsets || !sig_out || !parity || !coin_status))) return HBTC_ERR_ARG;
  Guard g(c);
  Keyset* ks;
  HB_TRY(get_keyset(c, keyset_id, &ks));
  if (!ks->master) return fail(c, HBTC_ERR_ARG, "key set has no master key (hbtc_keyset_set_master)");
  if (t == 0 || t > COMB_SMALL_T) return fail(c, HBTC_ERR_ARG, "t must be in 1..64");
  uint32_t n;
  HB_TRY(check_offsets(c, n_inst, offsets, &n));
  if (n_inst == 0) return HBTC_OK;
  if (n && (!idx || !sig || !status)) return fail(c, HBTC_ERR_ARG, "NULL item array");
  const size_t n1 = std::max<uint32_t>(n, 1);
  void *d_H, *d_idx, *d_sig, *d_st;
  HB_TRY(upload(c, "in0", H, (size_t)96 * n_inst, &d_H));
  HB_TRY(upload(c, "in1", idx, (size_t)4 * n, &d_idx));
  HB_TRY(upload(c, "in2", sig, (size_t)96 * n, &d_sig));
  HB_TRY(ws(c, "out0", (size_t)4 * n1, &d_st));
  PinLane pin(c);  // the uploads above went to the current lane
  void* p;
  HB_TRY(stage_upload(c, "coin.offsets", offsets, ((size_t)n_inst + 1) * 4, c->stream, &p));
  const uint32_t* d_off = static_cast<const uint32_t*>(p);
  int32_t *d_cst, *d_master;
  uint8_t *d_sig_out, *d_par;
  uint32_t* d_redo;
  HB_TRY(wst(c, "coin.cst", n_inst, &d_cst));
  HB_TRY(wst(c, "coin.master", n_inst, &d_master));
  HB_TRY(wst(c, "coin.sig", (size_t)96 * n_inst, &d_sig_out));
  HB_TRY(wst(c, "coin.par", n_inst, &d_par));
  HB_TRY(wst(c, "coin.redo", n_inst, &d_redo));
  // speculation: the leave-one-out subsets of the first t + 1 items, beside the share checks
  const uint32_t n_sub = t + 1;
  const bool spec = c->coin_spec && (uint64_t)n_inst * n_sub <= 256;
  int32_t *s_cst = nullptr, *s_master = nullptr;
  uint8_t *s_sig = nullptr, *s_par = nullptr;
  if (spec) {
    if (!c->s_spec) {
      int lo = 0, hi = 0;
      if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
      HB_CHECK(c, hipStreamCreateWithPriority(&c->s_spec, hipStreamNonBlocking, hi));
      HB_CHECK(c, hipStreamCreateWithPriority(&c->s_spec2, hipStreamNonBlocking, hi));
      HB_CHECK(c, hipEventCreateWithFlags(&c->ev_spec_in, hipEventDisableTiming));
      HB_CHECK(c, hipEventCreateWithFlags(&c->ev_spec_out, hipEventDisableTiming));
      HB_CHECK(c, hipEventCreateWithFlags(&c->ev_spec_out2, hipEventDisableTiming));
    }
    const size_t slots = (size_t)n_inst * n_sub;
    HB_TRY(wst(c, "coin.s_cst", slots, &s_cst));
    HB_TRY(wst(c, "coin.s_master", slots, &s_master));
    HB_TRY(wst(c, "coin.s_sig", slots * 96, &s_sig));
    HB_TRY(wst(c, "coin.s_par", slots, &s_par));
    HB_CHECK(c, hipEventRecord(c->ev_spec_in, c->stream));  // after the uploads
    HB_CHECK(c, hipStreamWaitEvent(c->s_spec, c->ev_spec_in, 0));
    CombSmallArgs a{};
    a.t = t;
    a.offsets = d_off;
    a.idx = (const uint32_t*)d_idx;
    a.pts = (const uint8_t*)d_sig;
    a.inst_status = s_cst;
    a.out = s_sig;
    a.parity = s_par;
    a.nocheck = 1;  // a subset is committed only when all its items passed the full decode
    CombSmallArgs m{};
    m.t = t;
    m.offsets = d_off;
    m.idx = (const uint32_t*)d_idx;
    m.dec = ks->pk;
    m.by_node = 1;
    m.n_nodes = ks->n;
    m.inst_status = s_master;
    m.cmp = ks->master;
    m.xtab = ks->tab;
    // the G2 combines and the G1 master checks of the subsets are independent: two streams
    HB_CHECK(c, hipStreamWaitEvent(c->s_spec2, c->ev_spec_in, 0));
    HB_TRY(timed_on(c, c->s_spec, "coin_spec", [&] { return launch_comb_small(c->s_spec, 2, n_inst, n_sub, a); }));
    HB_TRY(timed_on(c, c->s_spec2, "coin_spec_master", [&] {
      return launch_comb_small(c->s_spec2, 1, n_inst, n_sub, m);
    }));
    HB_CHECK(c, hipEventRecord(c->ev_spec_out2, c->s_spec2));
    HB_CHECK(c, hipStreamWaitEvent(c->s_spec, c->ev_spec_out2, 0));
    HB_CHECK(c, hipEventRecord(c->ev_spec_out, c->s_spec));
  }
  {
    HostG2Args hg(c, d_H, H);
    HB_TRY(sig_shares_dev(c, keyset_id, n_inst, (const uint8_t*)d_H, offsets, (const uint32_t*)d_idx,
                          (const uint8_t*)d_sig, (int32_t*)d_st));
  }
  const int32_t* d_item = (const int32_t*)d_st;
  if (spec) {
    HB_CHECK(c, hipStreamWaitEvent(c->stream, c->ev_spec_out, 0));
    HB_TRY(timed(c, "coin_commit", [&] {
      return launch_coin_commit(c->stream, n_inst, t, d_off, d_item, n_sub, s_cst, s_sig, s_par,
                                s_master, d_cst, d_sig_out, d_par, d_master, d_redo);
    }));
  }
  {  // the status-driven combine and master check (only the instances the speculation missed)
    const auto& ld = c->last_dec;
    const bool same = ld.status == d_item && ld.shares == (const uint8_t*)d_sig && ld.n_items == n;
    CombSmallArgs a{};
    a.t = t;
    a.offsets = d_off;
    a.item_status = d_item;
    a.idx = (const uint32_t*)d_idx;
    a.pts = (const uint8_t*)d_sig;
    a.dec = same ? (const void*)ld.dec2 : nullptr;
    a.inst_status = d_cst;
    a.out = d_sig_out;
    a.parity = d_par;
    a.only = spec ? d_redo : nullptr;
    CombSmallArgs m{};
    m.t = t;
    m.offsets = d_off;
    m.item_status = d_item;
    m.idx = (const uint32_t*)d_idx;
    m.dec = ks->pk;
    m.by_node = 1;
    m.n_nodes = ks->n;
    m.inst_status = d_master;
    m.cmp = ks->master;
    m.xtab = ks->tab;
    m.only = spec ? d_redo : nullptr;
    HB_TRY(timed(c, "combine", [&] {
      hipError_t e = launch_comb_small(c->stream, 2, n_inst, 1, a);
      if (e != hipSuccess) return e;
      return launch_comb_small(c->stream, 1, n_inst, 1, m);
    }));
  }
  std::vector<int32_t> cst(n_inst), mst(n_inst);
  HB_TRY(download(c, status, d_st, (size_t)4 * n));
  HB_TRY(download(c, sig_out, d_sig_out, (size_t)96 * n_inst));
  HB_TRY(download(c, parity, d_par, n_inst));
  HB_TRY(download(c, cst.data(), d_cst, (size_t)4 * n_inst));
  HB_TRY(download(c, mst.data(), d_master, (size_t)4 * n_inst));
  HB_TRY(sync(c));
  for (uint32_t k = 0; k < n_inst; ++k) coin_status[k] = cst[k] != HBTC_ACCEPT ? cst[k] : mst[k];
  return HBTC_OK;
}

// A few pair checks e(A_i, Q_i) == e(G1, W_i) (fewer than c->exact_below items): they have the
// SignatureShare check's form (pk := A, H := Q, sigma := W), so they take its exact small-call
// path with one instance per item -- A decoded (into d_adec when given), Q's line tables on
// s_prep, the item pass decoding W with every item on the leaf list, W's projective lines, the
// cooperative leaf checks.  Four dependent launches for c1's master signature instead of the
// pair batch's item pass, line tables, Miller partials and final exponentiation.  Statuses as
// the pair check's: an A, Q or W that fails to decode is the item's DECODE_ERR.
int pb_small_exact_chunk(hbtc_ctx* c, uint32_t n, const uint8_t* d_a, const uint8_t* d_q,
                         const uint8_t* d_w, int32_t* d_status, G1A* d_adec) {
  std::vector<uint32_t> offsets(n + 1), idx(n);
  for (uint32_t i = 0; i <= n; ++i) offsets[i] = i;
  for (uint32_t i = 0; i < n; ++i) idx[i] = i;
  G1A* A = d_adec;
  int32_t* a_st;
  if (!A) HB_TRY(wst(c, "pbx.a", n, &A));
  HB_TRY(wst(c, "pbx.ast", n, &a_st));
  void* p;
  HB_TRY(stage_upload(c, "pbx.idx", idx.data(), (size_t)4 * n, c->stream, &p));
  const uint32_t* d_idx = static_cast<const uint32_t*>(p);
  HB_TRY(stream_after(c, c->s_prep, c->stream, c->ev_main));
  G2A* h_aff;
  int32_t* h_st;
  Line* h_lines;
  HB_TRY(prepare_g2(c, d_q, nullptr, n, &h_aff, &h_st, &h_lines, c->s_prep));
  Tile* tiles;
  uint32_t n_tiles;
  HB_TRY(make_tiles(c, n, offsets.data(), &tiles, &n_tiles));
  SigTileSums* sums;
  G2A* dec;
  Fq2* tables;
  uint32_t *inf, *counters, *leaves;
  HB_TRY(wst(c, "pbx.sums", n_tiles, &sums));
  HB_TRY(wst(c, "pbx.dec", n, &dec));
  HB_TRY(wst(c, "pbx.tables", (size_t)n * PLINES_FQ2, &tables));
  HB_TRY(wst(c, "pbx.inf", n, &inf));
  HB_TRY(wst(c, "pbx.counters", 2, &counters));
  HB_TRY(wst(c, "pbx.leaves", (size_t)2 * n, &leaves));
  HB_CHECK(c, launch_zero_u32(c->stream, counters, 2));
  HB_TRY(timed(c, "pb_decode", [&] { return launch_g1_decode(c->stream, d_a, n, A, a_st); }));
  RlcKey key{};  // no group sums (Suspects.all): the scalars and the pk table are never read
  key.bits = c->rlc_bits;
  const Suspects sus{nullptr, 0, counters, leaves, 1};
  HB_TRY(timed(c, "sig_items", [&] {
    if (c->sig_fused)  // W decoded, listed and its line table built in one launch (k_sig_exact)
      return launch_sig_exact(c->stream, n, d_idx, d_w, a_st, n, tiles, n_tiles, counters, leaves, dec,
                              tables, inf, d_status);
    return launch_sig_items(c->stream, n_tiles, tiles, d_idx, d_w, A, a_st, nullptr, n, key, sus, sums,
                            dec, d_status);
  }));
  HB_TRY(stream_after(c, c->stream, c->s_prep, c->ev_prep));
  if (!c->sig_fused)
    HB_TRY(timed(c, "sig_lines", [&] {
      return launch_plines(c->stream, 2, n, 0, counters, leaves, tiles, sums, dec, tables, inf);
    }));
  HB_TRY(timed(c, "chk_leaves", [&] {
    const uint32_t lim = c->small_rep == 3 ? std::min(n, 8u * (uint32_t)c->n_cu) : 0u;
    const hipError_t e = launch_sigchk_leaves_rep3(c->stream, n, lim, counters, leaves, d_idx, A,
                                                   tables, inf, h_aff, h_lines, d_status);
    if (e != hipSuccess) return e;
    return launch_sigchk_leaves(c->stream, 0, n, counters, leaves, d_idx, A, tables, inf, h_aff,
                                h_lines, d_status, lim);
  }));
  return timed(c, "rlc_finalize", [&] {
    const hipError_t e = launch_rlc_finalize(c->stream, n_tiles, tiles, h_st, h_st, d_status, d_idx,
                                             n, nullptr, nullptr, 0, 1);
    if (e != hipSuccess) return e;
    return launch_status_remap(c->stream, n, d_status, HBTC_INSTANCE_ERR, HBTC_DECODE_ERR);
  });
}

// pb_small_exact over any n: chunks of PBX_CHUNK items (19.6 KB of line tables per item).
constexpr uint32_t PBX_CHUNK = 1u << 15;
int pb_small_exact(hbtc_ctx* c, uint32_t n, const uint8_t* d_a, const uint8_t* d_q,
                   const uint8_t* d_w, int32_t* d_status, G1A* d_adec) {
  if (!d_a) return fail(c, HBTC_ERR_ARG, "pair checks need their G1 arguments");
  for (uint32_t base = 0; base < n; base += PBX_CHUNK) {
    const uint32_t m = std::min(PBX_CHUNK, n - base);
    HB_TRY(pb_small_exact_chunk(c, m, d_a + (size_t)48 * base, d_q + (size_t)96 * base,
                                d_w + (size_t)96 * base, d_status + base, d_adec ? d_adec + base : nullptr));
  }
  return HBTC_OK;
}

// The exact checks of the items a pair batch's failing sub-tiles listed (`count` on the device):
// gathered into a compact batch, checked by pb_small_exact, statuses scattered back.  The count
// is read back first (a failing sub-tile is rare; pair batches run inside blocking host calls).
int pb_exact_list(hbtc_ctx* c, uint32_t m, const uint8_t* a, const uint8_t* q, const uint8_t* w,
                  int32_t* st, const uint32_t* d_count, const uint32_t* d_list) {
  uint32_t cnt = 0;
  HB_TRY(download(c, &cnt, d_count, 4));
  HB_CHECK(c, hipStreamSynchronize(c->stream));
  if (cnt == 0) return HBTC_OK;
  if (cnt > m) return fail(c, HBTC_ERR_DEVICE, "pair batch: leaf count past the chunk");
  uint8_t *ga, *gq, *gw;
  int32_t* gst;
  HB_TRY(wst(c, "pbl.a", (size_t)48 * cnt, &ga));
  HB_TRY(wst(c, "pbl.q", (size_t)96 * cnt, &gq));
  HB_TRY(wst(c, "pbl.w", (size_t)96 * cnt, &gw));
  HB_TRY(wst(c, "pbl.st", cnt, &gst));
  HB_CHECK(c, launch_pb_gather(c->stream, cnt, d_list, a, q, w, ga, gq, gw));
  HB_TRY(pb_small_exact(c, cnt, ga, gq, gw, gst, nullptr));
  HB_CHECK(c, launch_pb_scatter(c->stream, cnt, d_list, gst, st));
  return HBTC_OK;
}

// e(A_i, Q_i) == e(G1, W_i) for n items in device memory (A required: every caller passes its
// G1 arguments, and the exact fallbacks gather them; Q trusted: our own hash output, decoded
// without the subgroup check; statuses ACCEPT / REJECT /
// DECODE_ERR).  RLC mode: the pair-batch path of hbtc_pb.hip in chunks of
// c->pb_chunk items (the per-item line tables are 19.6 KB each): item pass, Q line tables,
// partial Miller products per 8-item sub-tile, the 64-item tile checks, the 8-item sub-tiles of
// failing tiles, the exact cooperative checks of the items of failing sub-tiles (pb_exact_list); a
// fresh RLC key per chunk.  Per-share mode and small calls: the exact checks for every item.
int pb_verify_dev(hbtc_ctx* c, uint32_t n, const uint8_t* d_a, const uint8_t* d_q, bool q_trusted,
                  const uint8_t* d_w, int32_t* d_status, G1A* d_adec = nullptr) {
  if (n && !d_a) return fail(c, HBTC_ERR_ARG, "pair checks need their G1 arguments");
  if (c->verify_mode == HBTC_MODE_PER_SHARE || n < c->exact_below)
    return pb_small_exact(c, n, d_a, d_q, d_w, d_status, d_adec);
  const uint32_t PB_CHUNK = c->pb_chunk;
  for (uint32_t base = 0; base < n; base += PB_CHUNK) {
    const uint32_t m = std::min(PB_CHUNK, n - base);
    const uint32_t T = (m + 63) / 64;
    G1A* rA;
    G2A *qdec, *wdec;
    SigTileSums* sums;
    Fq2 *qtab, *wtab, *fbuf;
    uint32_t *winf, *counters, *tlist, *leaves;
    HB_TRY(wst(c, "pb.ra", m, &rA));
    HB_TRY(wst(c, "pb.qdec", m, &qdec));
    HB_TRY(wst(c, "pb.wdec", m, &wdec));
    HB_TRY(wst(c, "pb.sums", T, &sums));
    HB_TRY(wst(c, "pb.qtab", (size_t)m * PLINES_FQ2, &qtab));
    HB_TRY(wst(c, "pb.wtab", (size_t)8 * T * PLINES_FQ2, &wtab));
    HB_TRY(wst(c, "pb.winf", (size_t)8 * T, &winf));
    HB_TRY(wst(c, "pb.fbuf", (size_t)8 * T * 6, &fbuf));
    HB_TRY(wst(c, "pb.counters", 2, &counters));
    HB_TRY(wst(c, "pb.tlist", T, &tlist));
    HB_TRY(wst(c, "pb.leaves", m, &leaves));
    const uint8_t* a = d_a + (size_t)48 * base;
    const uint8_t* q = d_q + (size_t)96 * base;
    const uint8_t* w = d_w + (size_t)96 * base;
    int32_t* st = d_status + base;
    RlcKey key;
    for (int i = 0; i < 8; ++i) key.k[i] = c->rd();
    key.bits = c->rlc_bits;
    HB_CHECK(c, launch_zero_u32(c->stream, counters, 2));
    HB_TRY(timed(c, "pb_items", [&] {
      return launch_pb_items(c->stream, m, a, q, q_trusted, w, key, rA, qdec, wdec, sums, st,
                             d_adec ? d_adec + base : nullptr);
    }));
    HB_TRY(timed(c, "pb_lines", [&] { return launch_pb_lines(c->stream, m, qdec, st, qtab); }));
    HB_TRY(timed(c, "pb_ml", [&] { return launch_pb_ml(c->stream, m, rA, qtab, st, fbuf); }));
    HB_TRY(timed(c, "pb_checks", [&] {
      const hipError_t e = launch_plines(c->stream, 3, T, 0, nullptr, nullptr, nullptr, sums, nullptr,
                                         wtab, winf);
      if (e != hipSuccess) return e;
      return launch_pb_fe(c->stream, 0, T, m, T, nullptr, nullptr, fbuf, wtab, winf, st, counters,
                          tlist);
    }));
    HB_TRY(timed(c, "pb_checks", [&] {
      const hipError_t e = launch_plines(c->stream, 4, 8 * T, 0, counters, tlist, nullptr, sums,
                                         nullptr, wtab, winf);
      if (e != hipSuccess) return e;
      return launch_pb_fe(c->stream, 1, 8 * T, m, 0, counters, tlist, fbuf, wtab, winf, st,
                          counters + 1, leaves);
    }));
    HB_TRY(pb_exact_list(c, m, a, q, w, st, counters + 1, leaves));
  }
  return HBTC_OK;
}

int hbtc_verify_sigs(hbtc_ctx* c, uint32_t n, const uint8_t* pk, const uint8_t* H,
                     const uint8_t* sig, int32_t* status) {
  if (!c || (n && (!pk || !H || !sig || !status))) return HBTC_ERR_ARG;
  Guard g(c);
  if (n == 0) return HBTC_OK;
  void *d_pk, *d_H, *d_sig, *d_st;
  HB_TRY(upload(c, "in0", pk, (size_t)48 * n, &d_pk));
  HB_TRY(upload(c, "in1", H, (size_t)96 * n, &d_H));
  HB_TRY(upload(c, "in2", sig, (size_t)96 * n, &d_sig));
  HB_TRY(ws(c, "out0", (size_t)4 * n, &d_st));
  // e(pk, H) == e(G1, sig)
  HB_TRY(pb_verify_dev(c, n, (const uint8_t*)d_pk, (const uint8_t*)d_H, false, (const uint8_t*)d_sig,
                       (int32_t*)d_st));
  HB_TRY(download(c, status, d_st, (size_t)4 * n));
  return sync(c);
}

int hbtc_verify_ciphertexts(hbtc_ctx* c, uint32_t n, const uint8_t* u, const uint8_t* H,
                            const uint8_t* w, int32_t* status) {
  if (!c || (n && (!u || !H || !w || !status))) return HBTC_ERR_ARG;
  Guard g(c);
  if (n == 0) return HBTC_OK;
  void *d_u, *d_H, *d_w, *d_st;
  HB_TRY(upload(c, "in0", u, (size_t)48 * n, &d_u));
  HB_TRY(upload(c, "in1", H, (size_t)96 * n, &d_H));
  HB_TRY(upload(c, "in2", w, (size_t)96 * n, &d_w));
  HB_TRY(ws(c, "out0", (size_t)4 * n, &d_st));
  // e(G1, w) == e(u, H), checked as e(u, H) == e(G1, w)
  HB_TRY(pb_verify_dev(c, n, (const uint8_t*)d_u, (const uint8_t*)d_H, false, (const uint8_t*)d_w,
                       (int32_t*)d_st));
  HB_TRY(download(c, status, d_st, (size_t)4 * n));
  return sync(c);
}

int hbtc_combine_sigs(hbtc_ctx* c, uint32_t n_inst, const uint32_t* offsets, const uint32_t* idx,
                      const uint8_t* sig, uint32_t t, uint8_t* out_sig, uint8_t* out_parity,
                      int32_t* inst_status) {
  if (!c || (n_inst && (!offsets || !out_sig || !out_parity || !inst_status))) return HBTC_ERR_ARG;
  Guard g(c);
  if (n_inst == 0) return HBTC_OK;
  uint32_t n;
  HB_TRY(check_offsets(c, n_inst, offsets, &n));
  void *d_idx, *d_sig, *d_out, *d_par, *d_st;
  HB_TRY(upload(c, "in0", idx, (size_t)4 * n, &d_idx));
  HB_TRY(upload(c, "in1", sig, (size_t)96 * n, &d_sig));
  HB_TRY(ws(c, "out0", (size_t)96 * n_inst, &d_out));
  HB_TRY(ws(c, "out1", (size_t)n_inst, &d_par));
  HB_TRY(ws(c, "out2", (size_t)4 * n_inst, &d_st));
  HB_TRY(combine_dev(c, 2, n_inst, offsets, (const uint32_t*)d_idx, (const uint8_t*)d_sig, t,
                     (uint8_t*)d_out, (uint8_t*)d_par, (int32_t*)d_st));
  HB_TRY(stream_after(c, c->stream, c->s_comb, c->ev_comb));
  HB_TRY(download(c, out_sig, d_out, (size_t)96 * n_inst));
  HB_TRY(download(c, out_parity, d_par, (size_t)n_inst));
  HB_TRY(download(c, inst_status, d_st, (size_t)4 * n_inst));
  return sync(c);
}

int hbtc_verify_dec_shares(hbtc_ctx* c, uint32_t keyset_id, uint32_t n_ct, const uint8_t* H,
                           const uint8_t* w, const uint32_t* offsets, const uint32_t* idx,
                           const uint8_t* share, int32_t* status) {
  if (!c || (n_ct && (!H || !w || !offsets))) return HBTC_ERR_ARG;
  Guard g(c);
  uint32_t n;
  HB_TRY(check_offsets(c, n_ct, offsets, &n));
  if (n && (!idx || !share || !status)) return fail(c, HBTC_ERR_ARG, "NULL item array");
  void *d_H, *d_w, *d_idx, *d_sh, *d_st;
  HB_TRY(upload(c, "in0", H, (size_t)96 * n_ct, &d_H));
  HB_TRY(upload(c, "in1", w, (size_t)96 * n_ct, &d_w));
  HB_TRY(upload(c, "in2", idx, (size_t)4 * n, &d_idx));
  HB_TRY(upload(c, "in3", share, (size_t)48 * n, &d_sh));
  HB_TRY(ws(c, "out0", (size_t)4 * n, &d_st));
  PinLane pin(c);  // the uploads above went to the current lane
  HostG2Args hg(c, d_H, H, d_w, w);
  HB_TRY(dec_shares_dev(c, keyset_id, n_ct, (const uint8_t*)d_H, (const uint8_t*)d_w, offsets,
                        (const uint32_t*)d_idx, (const uint8_t*)d_sh, (int32_t*)d_st));
  HB_TRY(download(c, status, d_st, (size_t)4 * n));
  return sync(c);
}

int hbtc_combine_dec(hbtc_ctx* c, uint32_t n_ct, const uint32_t* offsets, const uint32_t* idx,
                     const uint8_t* share, uint32_t t, uint8_t* out_g, int32_t* inst_status) {
  if (!c || (n_ct && (!offsets || !out_g || !inst_status))) return HBTC_ERR_ARG;
  Guard g(c);
  if (n_ct == 0) return HBTC_OK;
  uint32_t n;
  HB_TRY(check_offsets(c, n_ct, offsets, &n));
  void *d_idx, *d_sh, *d_out, *d_st;
  HB_TRY(upload(c, "in0", idx, (size_t)4 * n, &d_idx));
  HB_TRY(upload(c, "in1", share, (size_t)48 * n, &d_sh));
  HB_TRY(ws(c, "out0", (size_t)48 * n_ct, &d_out));
  HB_TRY(ws(c, "out2", (size_t)4 * n_ct, &d_st));
  HB_TRY(combine_dev(c, 1, n_ct, offsets, (const uint32_t*)d_idx, (const uint8_t*)d_sh, t,
                     (uint8_t*)d_out, nullptr, (int32_t*)d_st));
  HB_TRY(stream_after(c, c->stream, c->s_comb, c->ev_comb));
  HB_TRY(download(c, out_g, d_out, (size_t)48 * n_ct));
  HB_TRY(download(c, inst_status, d_st, (size_t)4 * n_ct));
  return sync(c);
}

int hbtc_g1_mul(hbtc_ctx* c, uint32_t n, const uint8_t* base, uint32_t base_stride,
                const uint8_t* scalars, uint8_t* out, int32_t* status) {
  if (!c || (n && (!base || !scalars || !out || !status))) return HBTC_ERR_ARG;
  Guard g(c);
  return point_mul_host(c, 1, n, base, base_stride, scalars, out, status);
}

int hbtc_g2_mul(hbtc_ctx* c, uint32_t n, const uint8_t* base, uint32_t base_stride,
                const uint8_t* scalars, uint8_t* out, int32_t* status) {
  if (!c || (n && (!base || !scalars || !out || !status))) return HBTC_ERR_ARG;
  Guard g(c);
  return point_mul_host(c, 2, n, base, base_stride, scalars, out, status);
}

// ---- device-resident variants
int hbtc_dev_alloc(hbtc_ctx* c, size_t bytes, void** d_ptr) {
  if (!c || !d_ptr) return HBTC_ERR_ARG;
  Guard g(c);
  HB_CHECK(c, hipMalloc(d_ptr, bytes ? bytes : 16));
  return HBTC_OK;
}

int hbtc_dev_free(hbtc_ctx* c, void* d_ptr) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  HB_TRY(sync(c));
  HB_CHECK(c, hipFree(d_ptr));
  return HBTC_OK;
}

int hbtc_dev_upload(hbtc_ctx* c, void* d_dst, const void* h_src, size_t bytes) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  HB_TRY(guard_write(c, d_dst, bytes));  // a combine still reading the old contents
  for (int o = 0; o < hbtc_ctx::NL; ++o)  // or a verification on another lane
    if (o != c->lane && c->lanes[o].busy) HB_CHECK(c, hipStreamWaitEvent(c->stream, c->lanes[o].done, 0));
  HB_CHECK(c, hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, c->stream));
  HB_CHECK(c, hipStreamSynchronize(c->stream));
  return HBTC_OK;
}

int hbtc_dev_download(hbtc_ctx* c, void* h_dst, const void* d_src, size_t bytes) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  HB_TRY(sync(c));  // results of any stream (verification, combines) are complete
  HB_CHECK(c, hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, c->stream));
  return sync(c);
}

int hbtc_sync(hbtc_ctx* c) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  return sync(c);
}

int hbtc_stream_wait_ctx(hbtc_ctx* c, void* stream) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  hipStream_t ext = static_cast<hipStream_t>(stream);
  for (Lane& l : c->lanes) {  // the lane events are re-recorded: waits capture them at once
    HB_TRY(stream_after(c, ext, l.stream, c->ev_ext));
    HB_TRY(stream_after(c, ext, l.s_prep, c->ev_ext2));
  }
  return HBTC_OK;
}

int hbtc_ctx_wait_stream(hbtc_ctx* c, void* stream) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  HB_CHECK(c, hipEventRecord(c->ev_ext, static_cast<hipStream_t>(stream)));
  for (Lane& l : c->lanes) {
    HB_CHECK(c, hipStreamWaitEvent(l.stream, c->ev_ext, 0));
    HB_CHECK(c, hipStreamWaitEvent(l.s_prep, c->ev_ext, 0));
  }
  return HBTC_OK;
}

int hbtc_unframe_points_dev(hbtc_ctx* c, uint32_t n, uint32_t point_size, const uint8_t* d_framed,
                            uint8_t* d_items) {
  if (!c || (point_size != 48 && point_size != 96) || (n && (!d_framed || !d_items))) return HBTC_ERR_ARG;
  Guard g(c);
  if ((reinterpret_cast<uintptr_t>(d_framed) & 3u) || !aligned16(d_items))
    return fail(c, HBTC_ERR_ARG, "framed input must be 4-byte, items 16-byte aligned");
  HB_TRY(guard_write(c, d_items, (size_t)n * point_size));
  HB_TRY(lane_async(c, {rng(d_framed, (size_t)n * (point_size + 8))}, {rng(d_items, (size_t)n * point_size)}));
  HB_TRY(timed(c, "unframe", [&] { return launch_unframe(c->stream, n, point_size, d_framed, d_items); }));
  return end_verify(c);
}

int hbtc_dec_epoch_submit(hbtc_ctx* c, uint32_t keyset_id, uint32_t n_ct, const uint8_t* H_c96,
                          const uint8_t* w_c96, const uint32_t* offsets, const uint32_t* idx,
                          const uint8_t* share_c48, uint32_t t, int32_t* status, uint8_t* out_g_c48,
                          int32_t* inst_status, uint64_t* ticket) {
  if (!c || !ticket || (n_ct && (!H_c96 || !w_c96 || !offsets))) return HBTC_ERR_ARG;
  Guard g(c);
  uint32_t n;
  HB_TRY(check_offsets(c, n_ct, offsets, &n));
  if (n && (!idx || !share_c48 || !status)) return fail(c, HBTC_ERR_ARG, "NULL item array");
  if (t && n_ct && (!out_g_c48 || !inst_status)) return fail(c, HBTC_ERR_ARG, "NULL combine output");
  return epoch_submit(c, 1, keyset_id, n_ct, H_c96, w_c96, offsets, idx, share_c48, t, status, out_g_c48,
                      nullptr, inst_status, ticket);
}

int hbtc_sig_epoch_submit(hbtc_ctx* c, uint32_t keyset_id, uint32_t n_inst, const uint8_t* H_c96,
                          const uint32_t* offsets, const uint32_t* idx, const uint8_t* sig_c96,
                          uint32_t t, int32_t* status, uint8_t* out_sig_c96, uint8_t* out_parity,
                          int32_t* inst_status, uint64_t* ticket) {
  if (!c || !ticket || (n_inst && (!H_c96 || !offsets))) return HBTC_ERR_ARG;
  Guard g(c);
  uint32_t n;
  HB_TRY(check_offsets(c, n_inst, offsets, &n));
  if (n && (!idx || !sig_c96 || !status)) return fail(c, HBTC_ERR_ARG, "NULL item array");
  if (t && n_inst && (!out_sig_c96 || !out_parity || !inst_status))
    return fail(c, HBTC_ERR_ARG, "NULL combine output");
  return epoch_submit(c, 2, keyset_id, n_inst, H_c96, nullptr, offsets, idx, sig_c96, t, status, out_sig_c96,
                      out_parity, inst_status, ticket);
}

int hbtc_wait(hbtc_ctx* c, uint64_t ticket) {
  if (!c || ticket == 0) return HBTC_ERR_ARG;
  Guard g(c);
  for (auto& T : c->tickets)
    if (T.active && T.id == ticket) return finish_ticket(c, T);
  return ticket < c->next_ticket ? HBTC_OK : fail(c, HBTC_ERR_ARG, "unknown ticket");
}

int hbtc_verify_dec_shares_dev(hbtc_ctx* c, uint32_t keyset_id, uint32_t n_ct,
                               const uint8_t* d_H, const uint8_t* d_w, const uint32_t* offsets,
                               const uint32_t* d_idx, const uint8_t* d_share, int32_t* d_status) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  return dec_shares_dev(c, keyset_id, n_ct, d_H, d_w, offsets, d_idx, d_share, d_status);
}

int hbtc_verify_sig_shares_dev(hbtc_ctx* c, uint32_t keyset_id, uint32_t n_inst,
                               const uint8_t* d_H, const uint32_t* offsets,
                               const uint32_t* d_idx, const uint8_t* d_sig, int32_t* d_status) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  return sig_shares_dev(c, keyset_id, n_inst, d_H, offsets, d_idx, d_sig, d_status);
}

int hbtc_combine_dec_dev(hbtc_ctx* c, uint32_t n_ct, const uint32_t* offsets,
                         const uint32_t* d_idx, const uint8_t* d_share, uint32_t t,
                         uint8_t* d_out_g, int32_t* d_inst_status) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  return combine_dev(c, 1, n_ct, offsets, d_idx, d_share, t, d_out_g, nullptr, d_inst_status);
}

int hbtc_combine_sigs_dev(hbtc_ctx* c, uint32_t n_inst, const uint32_t* offsets,
                          const uint32_t* d_idx, const uint8_t* d_sig, uint32_t t,
                          uint8_t* d_out_sig, uint8_t* d_out_parity, int32_t* d_inst_status) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  return combine_dev(c, 2, n_inst, offsets, d_idx, d_sig, t, d_out_sig, d_out_parity,
                     d_inst_status);
}

int hbtc_combine_dec_verified_dev(hbtc_ctx* c, uint32_t n_ct, const uint32_t* offsets,
                                  const uint32_t* d_idx, const uint8_t* d_share,
                                  const int32_t* d_status, uint32_t t, uint8_t* d_out_g,
                                  int32_t* d_inst_status) {
  if (!c || !d_status) return HBTC_ERR_ARG;
  Guard g(c);
  return combine_dev(c, 1, n_ct, offsets, d_idx, d_share, t, d_out_g, nullptr, d_inst_status,
                     d_status);
}

int hbtc_combine_sigs_verified_dev(hbtc_ctx* c, uint32_t n_inst, const uint32_t* offsets,
                                   const uint32_t* d_idx, const uint8_t* d_sig,
                                   const int32_t* d_status, uint32_t t, uint8_t* d_out_sig,
                                   uint8_t* d_out_parity, int32_t* d_inst_status) {
  if (!c || !d_status) return HBTC_ERR_ARG;
  Guard g(c);
  return combine_dev(c, 2, n_inst, offsets, d_idx, d_sig, t, d_out_sig, d_out_parity,
                     d_inst_status, d_status);
}

namespace {
// k mod r for a 256-bit little-endian scalar (k < 2^256 < 3r: at most two subtractions)
void scalar_mod_r(uint32_t* out, const uint8_t* in) {
  static const uint32_t R[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
  uint32_t k[8];
  memcpy(k, in, 32);
  for (int rep = 0; rep < 2; ++rep) {
    bool ge = true;
    for (int i = 7; i >= 0; --i)
      if (k[i] != R[i]) {
        ge = k[i] > R[i];
        break;
      }
    if (!ge) break;
    uint64_t borrow = 0;
    for (int i = 0; i < 8; ++i) {
      const uint64_t d = (uint64_t)k[i] - R[i] - borrow;
      k[i] = (uint32_t)d;
      borrow = (d >> 63) & 1u;
    }
  }
  memcpy(out, k, 32);
}

// n_msm MSMs of n terms on s_comb from device buffers: term i of MSM m is compressed item
// m * stride + i (terms i >= stride: the generator), canonical scalars [m][n].  Writes the
// compressed results and ACCEPT / DECODE_ERR per MSM.
int msm_dev(hbtc_ctx* c, int group, uint32_t n_msm, uint32_t n, uint32_t stride,
            const uint8_t* d_pts, const uint32_t* d_sc, uint8_t* d_out, int32_t* d_st) {
  hipStream_t sc = c->s_comb;
  const uint64_t terms = (uint64_t)n_msm * n;
  std::vector<uint32_t> cnt(n_msm, n);
  void* d_cnt;
  HB_TRY(stage_upload(c, "msm.cnt", cnt.data(), (size_t)n_msm * 4, sc, &d_cnt));
  uint32_t* d_bad;
  HB_TRY(wst(c, "msm.bad", n_msm, &d_bad));
  HB_CHECK(c, launch_zero_u32(sc, d_bad, n_msm));
  const MsmPlan p = msm_plan(n_msm, n);
  if (group == 1) {
    G1A* d_aff;
    HB_TRY(wst(c, "msm.g1", terms, &d_aff));
    HB_TRY(timed_on(c, sc, "comb_decode", [&] {
      return launch_msm_decode_g1(sc, n_msm, n, stride, d_pts, nullptr, (const uint32_t*)d_cnt,
                                  nullptr, nullptr, d_aff, d_bad);
    }));
    return msm_run<Fq>(c, sc, p, d_sc, d_aff, (const uint32_t*)d_cnt, n, d_bad, nullptr, d_st,
                       d_out, nullptr);
  }
  G2A* d_aff;
  HB_TRY(wst(c, "msm.g2", terms, &d_aff));
  HB_TRY(timed_on(c, sc, "comb_decode", [&] {
    return launch_msm_decode_g2(sc, n_msm, n, stride, d_pts, nullptr, (const uint32_t*)d_cnt,
                                nullptr, nullptr, d_aff, d_bad);
  }));
  return msm_run<Fq2>(c, sc, p, d_sc, d_aff, (const uint32_t*)d_cnt, n, d_bad, nullptr, d_st,
                      d_out, nullptr);
}

// MSMs per chunk so that the digit / list workspaces stay near 2^27 entries.
uint32_t msm_chunk(uint32_t n_msm, uint32_t n) {
  const MsmPlan full = msm_plan(n_msm, n);
  const uint64_t cap_terms = (1ull << 27) / full.W;
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n_msm, cap_terms / n));
}

// Batched MSMs from host buffers, chunked over MSMs.
int msm_host(hbtc_ctx* c, int group, uint32_t n_msm, uint32_t n, const uint8_t* pts,
             const uint8_t* scalars, uint8_t* out, int32_t* status) {
  if (n_msm == 0) return HBTC_OK;
  if (n == 0) return fail(c, HBTC_ERR_ARG, "n must be >= 1");
  const size_t pb = group == 1 ? 48 : 96;
  const uint32_t chunk = msm_chunk(n_msm, n);
  hipStream_t sc = c->s_comb;
  HB_TRY(sync(c));
  std::vector<uint32_t> red((size_t)chunk * n * 8);
  for (uint32_t m0 = 0; m0 < n_msm; m0 += chunk) {
    const uint32_t mc = std::min(chunk, n_msm - m0);
    const uint64_t terms = (uint64_t)mc * n;
    for (uint64_t i = 0; i < terms; ++i)
      scalar_mod_r(&red[i * 8], scalars + ((uint64_t)m0 * n + i) * 32);
    void *d_pts, *d_sc, *d_out, *d_st;
    HB_TRY(ws(c, "msm.in_pts", terms * pb, &d_pts));
    HB_TRY(ws(c, "msm.in_sc", terms * 32, &d_sc));
    HB_TRY(ws(c, "msm.out", (size_t)mc * pb, &d_out));
    HB_TRY(ws(c, "msm.st", (size_t)mc * 4, &d_st));
    HB_CHECK(c, hipMemcpyAsync(d_pts, pts + (uint64_t)m0 * n * pb, terms * pb,
                               hipMemcpyHostToDevice, sc));
    HB_CHECK(c, hipMemcpyAsync(d_sc, red.data(), terms * 32, hipMemcpyHostToDevice, sc));
    HB_TRY(msm_dev(c, group, mc, n, n, (const uint8_t*)d_pts, (const uint32_t*)d_sc,
                   (uint8_t*)d_out, (int32_t*)d_st));
    HB_CHECK(c, hipMemcpyAsync(out + (uint64_t)m0 * pb, d_out, (size_t)mc * pb,
                               hipMemcpyDeviceToHost, sc));
    HB_CHECK(c, hipMemcpyAsync(status + m0, d_st, (size_t)mc * 4, hipMemcpyDeviceToHost, sc));
    HB_CHECK(c, hipStreamSynchronize(sc));
  }
  return HBTC_OK;
}

// ---- SyncKeyGen (hbtc_skg.hip): Fr helpers on the host (the same field.h code)
void fr_set_zero(Fr& r) {
  for (int i = 0; i < 8; ++i) r.v[i] = 0;
}
bool fr_load_canonical(Fr& r, const uint8_t* le32) {
  memcpy(r.v, le32, 32);
  return limbs_lt_const<8>(r, FR_R);
}
Fr fr_mont_of(const Fr& canon) {
  Fr m;
  fr_to_mont(m, canon);
  return m;
}
Fr fr_random(hbtc_ctx* c) {
  uint8_t b[32];
  for (int i = 0; i < 8; ++i) {
    const uint32_t w = c->rd();
    memcpy(b + 4 * i, &w, 4);
  }
  Fr k;
  scalar_mod_r(k.v, b);
  return k;
}
Fr fr_neg_canon(const Fr& mont) {  // -(a) as a canonical scalar, a in Montgomery form
  Fr z, n, cn;
  fr_set_zero(z);
  fr_sub(n, z, mont);
  fr_from_mont(cn, n);
  return cn;
}
static std::vector<uint32_t> skg_ij_table(uint32_t t1) {  // coeff_pos order: pos = j(j+1)/2 + i, i <= j
  std::vector<uint32_t> ij;
  ij.reserve((size_t)t1 * (t1 + 1) / 2);
  for (uint32_t j = 0; j < t1; ++j)
    for (uint32_t i = 0; i <= j; ++i) ij.push_back(i | (j << 16));
  return ij;
}
bool is_g1_infinity_c48(const uint8_t* p) {
  if (p[0] != 0xc0) return false;
  for (int i = 1; i < 48; ++i)
    if (p[i]) return false;
  return true;
}

// "MSM == O" checks of n_chk equations over BivarCommitments: equation e uses commitment
// blk[e] (device compressed commitments [part][M]), scalars s_ij from U (shared) and V_e
// (Montgomery, stride v_stride), and the generator term tail_e (canonical).
// result[e] = ACCEPT / REJECT / DECODE_ERR.
int skg_checks(hbtc_ctx* c, uint32_t t1, const uint8_t* d_commit, uint32_t n_chk,
               const uint32_t* blk, const Fr* U, const Fr* V, uint32_t v_stride, const Fr* tail,
               int32_t* result) {
  if (n_chk == 0) return HBTC_OK;
  const uint32_t M = t1 * (t1 + 1) / 2, n = M + 1;
  hipStream_t sc = c->s_comb;
  const std::vector<uint32_t> ij = skg_ij_table(t1);
  void *d_ij, *d_U;
  HB_TRY(stage_upload(c, "skg.ij", ij.data(), ij.size() * 4, sc, &d_ij));
  HB_TRY(stage_upload(c, "skg.U", U, (size_t)t1 * sizeof(Fr), sc, &d_U));
  const uint32_t chunk = msm_chunk(n_chk, n);
  std::vector<uint8_t> out((size_t)chunk * 48);
  std::vector<int32_t> st(chunk);
  for (uint32_t e0 = 0; e0 < n_chk; e0 += chunk) {
    const uint32_t ec = std::min(chunk, n_chk - e0);
    void *d_V, *d_tail, *d_sc, *d_out, *d_st, *d_pts;
    HB_TRY(stage_upload(c, "skg.V", V + (size_t)e0 * v_stride,
                        (size_t)((ec - 1) * v_stride + t1) * sizeof(Fr), sc, &d_V));
    HB_TRY(stage_upload(c, "skg.tail", tail + e0, (size_t)ec * sizeof(Fr), sc, &d_tail));
    HB_TRY(ws(c, "skg.sc", (size_t)ec * n * sizeof(Fr), &d_sc));
    HB_TRY(ws(c, "skg.out", (size_t)ec * 48, &d_out));
    HB_TRY(ws(c, "skg.st", (size_t)ec * 4, &d_st));
    HB_TRY(timed_on(c, sc, "skg_scalars", [&] {
      return launch_skg_sym_scalars(sc, ec, M, (const Fr*)d_U, 0, (const Fr*)d_V, v_stride,
                                    (const uint32_t*)d_ij, (const Fr*)d_tail, (Fr*)d_sc);
    }));
    // the commitments of this chunk in equation order (device-to-device; contiguous blocks of
    // one copy each when the equations are the Parts themselves)
    const uint8_t* pts = d_commit + (size_t)blk[e0] * M * 48;
    bool contiguous = true;
    for (uint32_t e = 1; e < ec && contiguous; ++e) contiguous = blk[e0 + e] == blk[e0] + e;
    if (!contiguous) {
      HB_TRY(ws(c, "skg.pts", (size_t)ec * M * 48, &d_pts));
      for (uint32_t e = 0; e < ec; ++e)
        HB_CHECK(c, hipMemcpyAsync((uint8_t*)d_pts + (size_t)e * M * 48,
                                   d_commit + (size_t)blk[e0 + e] * M * 48, (size_t)M * 48,
                                   hipMemcpyDeviceToDevice, sc));
      pts = (const uint8_t*)d_pts;
    }
    HB_TRY(msm_dev(c, 1, ec, n, M, pts, (const uint32_t*)d_sc, (uint8_t*)d_out, (int32_t*)d_st));
    HB_CHECK(c, hipMemcpyAsync(out.data(), d_out, (size_t)ec * 48, hipMemcpyDeviceToHost, sc));
    HB_CHECK(c, hipMemcpyAsync(st.data(), d_st, (size_t)ec * 4, hipMemcpyDeviceToHost, sc));
    HB_CHECK(c, hipStreamSynchronize(sc));
    for (uint32_t e = 0; e < ec; ++e)
      result[e0 + e] = st[e] == HBTC_DECODE_ERR           ? HBTC_DECODE_ERR
                       : is_g1_infinity_c48(&out[48 * e]) ? HBTC_ACCEPT
                                                          : HBTC_REJECT;
  }
  return HBTC_OK;
}
}  // namespace

int hbtc_skg_check_parts(hbtc_ctx* c, uint32_t n_parts, uint32_t t, uint32_t our_idx,
                         const uint8_t* commit_c48, const uint8_t* rows_le32,
                         int32_t* part_status) {
  if (!c || (n_parts && (!commit_c48 || !rows_le32 || !part_status))) return HBTC_ERR_ARG;
  if (t >= 0xffffu) return HBTC_ERR_ARG;
  Guard g(c);
  if (n_parts == 0) return HBTC_OK;
  HB_TRY(sync(c));
  const uint32_t t1 = t + 1, M = t1 * (t1 + 1) / 2;
  // rho_i (fresh per call) and x^j with x = our_idx + 1, both Montgomery
  std::vector<Fr> U(t1), V(t1);
  Fr x, xp;
  fr_from_u64(x, (uint64_t)our_idx + 1);
  fr_from_u64(xp, 1);
  for (uint32_t j = 0; j < t1; ++j) {
    U[j] = fr_mont_of(fr_random(c));
    V[j] = xp;
    fr_mul(xp, xp, x);
  }
  // tail_p = -(sum_i rho_i a_{p,i}); a row coefficient >= r fails bincode's Fr decoding
  // (InvalidPartMessage, sync_key_gen.rs:359-364)
  std::vector<Fr> tail(n_parts);
  std::vector<uint8_t> row_bad(n_parts, 0);
  for (uint32_t p = 0; p < n_parts; ++p) {
    Fr acc;
    fr_set_zero(acc);
    for (uint32_t i = 0; i < t1; ++i) {
      Fr a;
      if (!fr_load_canonical(a, rows_le32 + ((size_t)p * t1 + i) * 32)) {
        row_bad[p] = 1;
        break;
      }
      Fr prod;
      fr_mul(prod, U[i], fr_mont_of(a));
      fr_add(acc, acc, prod);
    }
    tail[p] = fr_neg_canon(acc);
  }
  void* d_commit;
  HB_TRY(ws(c, "skg.commit", (size_t)n_parts * M * 48, &d_commit));
  HB_CHECK(c, hipMemcpyAsync(d_commit, commit_c48, (size_t)n_parts * M * 48,
                             hipMemcpyHostToDevice, c->s_comb));
  std::vector<uint32_t> blk(n_parts);
  for (uint32_t p = 0; p < n_parts; ++p) blk[p] = p;
  HB_TRY(skg_checks(c, t1, (const uint8_t*)d_commit, n_parts, blk.data(), U.data(), V.data(), 0,
                    tail.data(), part_status));
  for (uint32_t p = 0; p < n_parts; ++p)
    if (row_bad[p] && part_status[p] != HBTC_DECODE_ERR) part_status[p] = HBTC_REJECT;
  return HBTC_OK;
}

int hbtc_skg_check_acks(hbtc_ctx* c, uint32_t n_parts, uint32_t t, uint32_t our_idx,
                        const uint8_t* commit_c48, const uint8_t* rows_le32,
                        const uint8_t* row_ok, uint32_t n_acks, const uint32_t* ack_part,
                        const uint32_t* ack_sender, const uint8_t* vals_le32,
                        int32_t* ack_status) {
  if (!c || (n_acks && (!commit_c48 || !row_ok || !ack_part || !ack_sender || !vals_le32 ||
                        !ack_status)))
    return HBTC_ERR_ARG;
  if (t >= 0xffffu) return HBTC_ERR_ARG;
  Guard g(c);
  if (n_acks == 0) return HBTC_OK;
  const uint32_t t1 = t + 1, M = t1 * (t1 + 1) / 2;
  std::vector<Fr> vals(n_acks);
  std::vector<uint8_t> val_bad(n_acks, 0);
  for (uint32_t a = 0; a < n_acks; ++a) {
    if (ack_part[a] >= n_parts) return fail(c, HBTC_ERR_ARG, "ack_part out of range");
    if (!fr_load_canonical(vals[a], vals_le32 + (size_t)a * 32)) val_bad[a] = 1;
  }
  HB_TRY(sync(c));
  hipStream_t sc = c->s_comb;
  // (1) Acks of Parts whose row this node verified: val == row(sender + 1)
  bool any_row = false;
  for (uint32_t p = 0; p < n_parts && !any_row; ++p) any_row = row_ok[p] != 0;
  if (any_row) {
    if (!rows_le32) return fail(c, HBTC_ERR_ARG, "rows_le32 is NULL");
    std::vector<Fr> rows((size_t)n_parts * t1);
    for (size_t k = 0; k < rows.size(); ++k) {
      Fr a;
      memcpy(a.v, rows_le32 + k * 32, 32);
      rows[k] = fr_mont_of(a);
    }
    void *d_rows, *d_part, *d_snd, *d_vals, *d_st;
    HB_TRY(upload(c, "skg.rows", rows.data(), rows.size() * sizeof(Fr), &d_rows));
    HB_TRY(upload(c, "skg.ack_part", ack_part, (size_t)n_acks * 4, &d_part));
    HB_TRY(upload(c, "skg.ack_snd", ack_sender, (size_t)n_acks * 4, &d_snd));
    HB_TRY(upload(c, "skg.vals", vals.data(), (size_t)n_acks * sizeof(Fr), &d_vals));
    HB_TRY(ws(c, "skg.ack_st", (size_t)n_acks * 4, &d_st));
    HB_TRY(timed(c, "skg_ack_rows", [&] {
      return launch_skg_ack_rows(c->stream, n_acks, t1, (const Fr*)d_rows,
                                 (const uint32_t*)d_part, (const uint32_t*)d_snd,
                                 (const Fr*)d_vals, (int32_t*)d_st);
    }));
    HB_TRY(download(c, ack_status, d_st, (size_t)n_acks * 4));
    HB_TRY(sync(c));
  }
  // (2) Parts without a verified row: one random linear combination of their Acks each,
  // sum_a rho_a evaluate(x, y_a) == [sum_a rho_a val_a] G1
  std::vector<std::vector<uint32_t>> by_part(n_parts);
  for (uint32_t a = 0; a < n_acks; ++a)
    if (!row_ok[ack_part[a]] && !val_bad[a]) by_part[ack_part[a]].push_back(a);
  std::vector<uint32_t> parts;
  for (uint32_t p = 0; p < n_parts; ++p)
    if (!by_part[p].empty()) parts.push_back(p);
  if (!parts.empty()) {
    std::vector<Fr> U(t1);
    Fr x, xp;
    fr_from_u64(x, (uint64_t)our_idx + 1);
    fr_from_u64(xp, 1);
    for (uint32_t j = 0; j < t1; ++j) {
      U[j] = xp;
      fr_mul(xp, xp, x);
    }
    void* d_commit;
    HB_TRY(ws(c, "skg.commit", (size_t)n_parts * M * 48, &d_commit));
    HB_CHECK(c, hipMemcpyAsync(d_commit, commit_c48, (size_t)n_parts * M * 48,
                               hipMemcpyHostToDevice, sc));
    auto powers = [&](uint32_t sender, Fr* out) {  // (sender + 1)^j, Montgomery
      Fr y, yp;
      fr_from_u64(y, (uint64_t)sender + 1);
      fr_from_u64(yp, 1);
      for (uint32_t j = 0; j < t1; ++j) {
        out[j] = yp;
        fr_mul(yp, yp, y);
      }
    };
    std::vector<Fr> V(parts.size() * t1), tail(parts.size()), yp(t1);
    for (size_t q = 0; q < parts.size(); ++q) {
      Fr* Y = &V[q * t1];
      for (uint32_t j = 0; j < t1; ++j) fr_set_zero(Y[j]);
      Fr acc;
      fr_set_zero(acc);
      for (uint32_t a : by_part[parts[q]]) {
        const Fr rho = fr_mont_of(fr_random(c));
        powers(ack_sender[a], yp.data());
        for (uint32_t j = 0; j < t1; ++j) {
          Fr tm;
          fr_mul(tm, rho, yp[j]);
          fr_add(Y[j], Y[j], tm);
        }
        Fr tv;
        fr_mul(tv, rho, fr_mont_of(vals[a]));
        fr_add(acc, acc, tv);
      }
      tail[q] = fr_neg_canon(acc);
    }
    std::vector<int32_t> res(parts.size());
    HB_TRY(skg_checks(c, t1, (const uint8_t*)d_commit, (uint32_t)parts.size(), parts.data(),
                      U.data(), V.data(), t1, tail.data(), res.data()));
    // (3) a failing combination: every Ack of that Part checked exactly
    std::vector<uint32_t> exact, eblk;
    for (size_t q = 0; q < parts.size(); ++q) {
      for (uint32_t a : by_part[parts[q]]) {
        if (res[q] == HBTC_ACCEPT) {
          ack_status[a] = HBTC_ACCEPT;
        } else if (res[q] == HBTC_DECODE_ERR) {
          ack_status[a] = HBTC_DECODE_ERR;  // the Part's commitment itself does not decode
        } else {
          exact.push_back(a);
          eblk.push_back(parts[q]);
        }
      }
    }
    if (!exact.empty()) {
      std::vector<Fr> V2(exact.size() * t1), tail2(exact.size());
      for (size_t e = 0; e < exact.size(); ++e) {
        powers(ack_sender[exact[e]], &V2[e * t1]);
        tail2[e] = fr_neg_canon(fr_mont_of(vals[exact[e]]));
      }
      std::vector<int32_t> res2(exact.size());
      HB_TRY(skg_checks(c, t1, (const uint8_t*)d_commit, (uint32_t)exact.size(), eblk.data(),
                        U.data(), V2.data(), t1, tail2.data(), res2.data()));
      for (size_t e = 0; e < exact.size(); ++e)
        ack_status[exact[e]] = res2[e] == HBTC_ACCEPT ? HBTC_ACCEPT : HBTC_REJECT;
    }
  }
  for (uint32_t a = 0; a < n_acks; ++a)
    if (val_bad[a]) ack_status[a] = HBTC_DECODE_ERR;
  return HBTC_OK;
}

int hbtc_commitment_evaluate(hbtc_ctx* c, uint32_t n_coeff, const uint8_t* commit_c48,
                             uint32_t n_x, const uint32_t* xs, uint8_t* out_c48, int32_t* status) {
  if (!c || (n_x && (!commit_c48 || !xs || !out_c48 || !status)) || (n_x && n_coeff == 0))
    return HBTC_ERR_ARG;
  Guard g(c);
  if (n_x == 0) return HBTC_OK;
  // one MSM per point x: sum_j x^j C_j (the coefficients repeated per MSM)
  const uint32_t chunk = std::max<uint32_t>(1, std::min<uint32_t>(n_x, (uint32_t)((64ull << 20) / (48ull * n_coeff + 32ull * n_coeff))));
  std::vector<uint8_t> pts((size_t)chunk * n_coeff * 48), sc((size_t)chunk * n_coeff * 32);
  for (uint32_t x0 = 0; x0 < n_x; x0 += chunk) {
    const uint32_t m = std::min(chunk, n_x - x0);
    for (uint32_t k = 0; k < m; ++k) {
      memcpy(&pts[(size_t)k * n_coeff * 48], commit_c48, (size_t)n_coeff * 48);
      Fr x, p, cn;
      fr_from_u64(x, xs[x0 + k]);
      fr_from_u64(p, 1);
      for (uint32_t j = 0; j < n_coeff; ++j) {
        fr_from_mont(cn, p);
        memcpy(&sc[((size_t)k * n_coeff + j) * 32], cn.v, 32);
        fr_mul(p, p, x);
      }
    }
    HB_TRY(msm_host(c, 1, m, n_coeff, pts.data(), sc.data(), out_c48 + (size_t)x0 * 48, status + x0));
  }
  return HBTC_OK;
}

int hbtc_g1_msm(hbtc_ctx* c, uint32_t n_msm, uint32_t n, const uint8_t* pts_c48,
                const uint8_t* scalars_le32, uint8_t* out_c48, int32_t* status) {
  if (!c || (n_msm && (!pts_c48 || !scalars_le32 || !out_c48 || !status))) return HBTC_ERR_ARG;
  Guard g(c);
  return msm_host(c, 1, n_msm, n, pts_c48, scalars_le32, out_c48, status);
}

int hbtc_g2_msm(hbtc_ctx* c, uint32_t n_msm, uint32_t n, const uint8_t* pts_c96,
                const uint8_t* scalars_le32, uint8_t* out_c96, int32_t* status) {
  if (!c || (n_msm && (!pts_c96 || !scalars_le32 || !out_c96 || !status))) return HBTC_ERR_ARG;
  Guard g(c);
  return msm_host(c, 2, n_msm, n, pts_c96, scalars_le32, out_c96, status);
}

int hbtc_set_check_schedule(hbtc_ctx* c, int schedule) {
  if (!c || schedule < HBTC_CHECK_AUTO || schedule > HBTC_CHECK_PAIR_LEAVES) return HBTC_ERR_ARG;
  Guard g(c);
  c->check_mode_forced = schedule;
  return HBTC_OK;
}

int hbtc_set_sender_tracking(hbtc_ctx* c, int enable) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  c->track_senders = enable != 0;
  return HBTC_OK;
}

int hbtc_set_exact_below(hbtc_ctx* c, uint32_t n_items) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  c->exact_below = n_items;
  return HBTC_OK;
}

int hbtc_set_rlc_bits(hbtc_ctx* c, uint32_t bits) {
  if (!c || (bits != 64 && bits != 128)) return HBTC_ERR_ARG;
  Guard g(c);
  c->rlc_bits = bits;
  return HBTC_OK;
}

int hbtc_trim_workspace(hbtc_ctx* c) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  HB_TRY(sync(c));
  for (auto& kv : c->bufs)
    if (kv.second.p) (void)hipFree(kv.second.p);
  c->bufs.clear();
  c->last_dec = {};
  c->last_leaf_count = nullptr;
  return HBTC_OK;
}

int hbtc_get_rlc_bits(hbtc_ctx* c, uint32_t* bits) {
  if (!c || !bits) return HBTC_ERR_ARG;
  Guard g(c);
  *bits = c->rlc_bits;
  return HBTC_OK;
}

int hbtc_check_schedule_for(hbtc_ctx* c, uint32_t n_tiles, int* schedule) {
  if (!c || !schedule) return HBTC_ERR_ARG;
  Guard g(c);
  *schedule = check_mode(c, n_tiles);
  return HBTC_OK;
}

int hbtc_set_verify_mode(hbtc_ctx* c, int mode) {
  if (!c || (mode != HBTC_MODE_PER_SHARE && mode != HBTC_MODE_RLC)) return HBTC_ERR_ARG;
  Guard g(c);
  c->verify_mode = mode;
  return HBTC_OK;
}

int hbtc_rlc_last_leaves(hbtc_ctx* c, uint32_t* leaves) {
  if (!c || !leaves) return HBTC_ERR_ARG;
  Guard g(c);
  *leaves = 0;
  if (!c->last_leaf_count) return HBTC_OK;
  HB_CHECK(c, hipMemcpyAsync(leaves, c->last_leaf_count, 4, hipMemcpyDeviceToHost, c->stream));
  return sync(c);
}

int hbtc_timing_enable(hbtc_ctx* c, int enable) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  c->timing = enable != 0;
  return HBTC_OK;
}

int hbtc_timing_read(hbtc_ctx* c, const char* family, double* total_ms, uint64_t* launches) {
  if (!c || !family) return HBTC_ERR_ARG;
  Guard g(c);
  HB_TRY(collect_spans(c));
  auto it = c->totals.find(family);
  if (total_ms) *total_ms = it == c->totals.end() ? 0.0 : it->second.first;
  if (launches) *launches = it == c->totals.end() ? 0 : it->second.second;
  return HBTC_OK;
}

int hbtc_timing_reset(hbtc_ctx* c) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  HB_TRY(collect_spans(c));
  c->totals.clear();
  return HBTC_OK;
}

// ---- hashes with the cofactor clearing on the GPU (the host draws the candidates)
// hash_g2(msg_i) (g1 == null) or hash_g1_g2(g1_i, msg_i) for a batch, entirely on the GPU: the
// candidate draw (k_hash_cand: sha3, rand 0.4 ChaCha, G2::rand's loop) and [h2] P; a candidate
// whose [h2] P is O (probability ~2^-250) continues G2::rand's loop on the host (exact).
static int hash_batch_gpu(hbtc_ctx* c, uint32_t n, const uint8_t* g1_c48, const uint8_t* msgs,
                          const uint32_t* offsets, uint8_t* out_c96, uint8_t** d_out_keep = nullptr) {
  HB_TRY(sync(c));
  void *d_msgs, *d_off, *d_g1 = nullptr;
  G2A* d_cand;
  uint8_t* d_out;
  int32_t* d_st;
  HB_TRY(upload(c, "hash.msgs", msgs, offsets[n] ? offsets[n] : 1, &d_msgs));
  HB_TRY(upload(c, "hash.off", offsets, (size_t)4 * (n + 1), &d_off));
  if (g1_c48) HB_TRY(upload(c, "hash.g1", g1_c48, (size_t)48 * n, &d_g1));
  HB_TRY(wst(c, "hash.cand", n, &d_cand));
  HB_TRY(wst(c, "hash.out", (size_t)n * 96, &d_out));
  HB_TRY(wst(c, "hash.st", n, &d_st));
  HB_TRY(timed(c, "hash", [&] {
    return launch_hash_cand(c->stream, n, (const uint8_t*)d_g1, (const uint8_t*)d_msgs,
                            (const uint32_t*)d_off, d_cand);
  }));
  HB_TRY(timed(c, "hash", [&] { return launch_g2_clear_cofactor(c->stream, n, d_cand, d_out, d_st); }));
  std::vector<int32_t> st(n);
  HB_CHECK(c, hipMemcpyAsync(out_c96, d_out, (size_t)n * 96, hipMemcpyDeviceToHost, c->stream));
  HB_CHECK(c, hipMemcpyAsync(st.data(), d_st, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
  HB_TRY(sync(c));
  for (uint32_t i = 0; i < n; ++i)  // [h2] P = O: G2::rand draws again (host, exact)
    if (st[i]) {
      if (g1_c48)
        hash_g1_g2_c96(g1_c48 + 48 * (size_t)i, msgs + offsets[i], offsets[i + 1] - offsets[i],
                       out_c96 + 96 * (size_t)i);
      else
        hash_g2_c96(msgs + offsets[i], offsets[i + 1] - offsets[i], out_c96 + 96 * (size_t)i);
    }
  if (d_out_keep) *d_out_keep = d_out;
  return HBTC_OK;
}

int hbtc_hash_g2_batch_gpu(hbtc_ctx* c, uint32_t n, const uint8_t* msgs, const uint32_t* offsets,
                           uint8_t* out_c96) {
  if (!c) return HBTC_ERR_ARG;
  if (n == 0) return HBTC_OK;
  if (!offsets || !out_c96 || (!msgs && offsets[n]) || !hash_offsets_ok(n, offsets))
    return HBTC_ERR_ARG;
  Guard g(c);
  return hash_batch_gpu(c, n, nullptr, msgs, offsets, out_c96);
}

int hbtc_chacha04_words_gpu(hbtc_ctx* c, const uint32_t* seed8, uint32_t n, uint32_t* out) {
  if (!c || !seed8 || (!out && n)) return HBTC_ERR_ARG;
  if (n == 0) return HBTC_OK;
  Guard g(c);
  uint32_t* d_out;
  HB_TRY(wst(c, "out0", n, &d_out));
  HB_TRY(timed(c, "hash", [&] { return launch_chacha04_words(c->stream, seed8, n, d_out); }));
  HB_CHECK(c, hipMemcpyAsync(out, d_out, (size_t)4 * n, hipMemcpyDeviceToHost, c->stream));
  return sync(c);
}

int hbtc_hash_g1_g2_batch_gpu(hbtc_ctx* c, uint32_t n, const uint8_t* g1_c48, const uint8_t* msgs,
                              const uint32_t* offsets, uint8_t* out_c96) {
  if (!c) return HBTC_ERR_ARG;
  if (n == 0) return HBTC_OK;
  if (!g1_c48 || !offsets || !out_c96 || (!msgs && offsets[n]) || !hash_offsets_ok(n, offsets))
    return HBTC_ERR_ARG;
  Guard g(c);
  return hash_batch_gpu(c, n, g1_c48, msgs, offsets, out_c96);
}

// k (canonical, < r, 8 little-endian limbs) = k1 x^2 + k0 with k0 < x^2 and k1 < 2^128 (k < r <
// x^4): binary long division by x^2 = 0xac45a4010001a4020000000100000000.
static void split_by_x2(const uint32_t* k, uint32_t* k0, uint32_t* k1) {
  static const uint32_t X2[4] = {0x00000000u, 0x00000001u, 0x0001a402u, 0xac45a401u};
  uint32_t rem[5] = {0, 0, 0, 0, 0};
  uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int bit = 255; bit >= 0; --bit) {
    for (int j = 4; j > 0; --j) rem[j] = (rem[j] << 1) | (rem[j - 1] >> 31);  // rem = 2 rem + bit
    rem[0] = (rem[0] << 1) | ((k[bit >> 5] >> (bit & 31)) & 1u);
    bool ge = rem[4] != 0;
    if (!ge) {
      ge = true;
      for (int j = 3; j >= 0; --j)
        if (rem[j] != X2[j]) {
          ge = rem[j] > X2[j];
          break;
        }
    }
    if (ge) {
      uint64_t borrow = 0;
      for (int j = 0; j < 5; ++j) {
        const uint64_t d = (uint64_t)rem[j] - (j < 4 ? X2[j] : 0u) - borrow;
        rem[j] = (uint32_t)d;
        borrow = (d >> 63) & 1u;
      }
      q[bit >> 5] |= 1u << (bit & 31);
    }
  }
  for (int j = 0; j < 4; ++j) {
    k0[j] = rem[j];
    k1[j] = q[j];
  }
}

int hbtc_decrypt(hbtc_ctx* c, uint32_t n, const uint8_t* sk_le32, const uint8_t* u_c48,
                 const uint8_t* w_c96, const uint8_t* msgs, const uint32_t* offsets, uint8_t* out,
                 int32_t* status) {
  if (!c) return HBTC_ERR_ARG;
  if (n == 0) return HBTC_OK;
  if (!sk_le32 || !u_c48 || !w_c96 || !offsets || !status || (offsets[n] && (!msgs || !out)) ||
      !hash_offsets_ok(n, offsets))
    return HBTC_ERR_ARG;
  Guard g(c);
  // 1. H_i = hash_g1_g2(u_i, v_i) on the GPU
  std::vector<uint8_t> H((size_t)n * 96);
  HB_TRY(hash_batch_gpu(c, n, u_c48, msgs, offsets, H.data()));
  // 2. Ciphertext::verify: e(G1, w) == e(u, H);  3. g = sk * u
  Fr k;
  scalar_mod_r(k.v, sk_le32);
  void *d_u, *d_H, *d_w, *d_st, *d_k, *d_g, *d_gst;
  HB_TRY(upload(c, "in0", u_c48, (size_t)48 * n, &d_u));
  HB_TRY(upload(c, "in1", H.data(), (size_t)96 * n, &d_H));
  HB_TRY(upload(c, "in2", w_c96, (size_t)96 * n, &d_w));
  HB_TRY(upload(c, "in3", k.v, 32, &d_k));
  HB_TRY(ws(c, "out0", (size_t)4 * n, &d_st));
  HB_TRY(ws(c, "out1", (size_t)48 * n, &d_g));
  HB_TRY(ws(c, "out2", (size_t)4 * n, &d_gst));
  // H is this call's own hash output (cofactor cleared: in the subgroup by construction)
  const bool rlc = c->verify_mode == HBTC_MODE_RLC;
  G1A* d_adec = nullptr;
  if (rlc) HB_TRY(wst(c, "dec.adec", n, &d_adec));
  HB_TRY(pb_verify_dev(c, n, (const uint8_t*)d_u, (const uint8_t*)d_H, true, (const uint8_t*)d_w,
                       (int32_t*)d_st, d_adec));
  if (rlc) {
    // g = sk u on the u decoded by the pair batch, for the ciphertexts that verify:
    // sk = k0 + k1 x^2 (k0 < x^2), [sk] u = [k0] u + [k1] (beta x, -y)
    uint32_t k0[4], k1[4];
    split_by_x2(k.v, k0, k1);
    HB_TRY(timed(c, "mul", [&] {
      return launch_pb_mul_glv(c->stream, n, d_adec, (const int32_t*)d_st, k0, k1, (uint8_t*)d_g);
    }));
    HB_CHECK(c, hipMemsetAsync(d_gst, 0, (size_t)4 * n, c->stream));  // statuses are in d_st
  } else {
    HB_TRY(timed(c, "mul", [&] {
      return launch_point_mul(c->stream, 1, n, (const uint8_t*)d_u, 1, (const uint8_t*)d_k, 0,
                              (uint8_t*)d_g, (int32_t*)d_gst);
    }));
  }
  std::vector<uint8_t> gb((size_t)n * 48);
  std::vector<int32_t> gst(n);
  HB_TRY(download(c, status, d_st, (size_t)4 * n));
  HB_TRY(download(c, gb.data(), d_g, (size_t)48 * n));
  HB_TRY(download(c, gst.data(), d_gst, (size_t)4 * n));
  HB_TRY(sync(c));
  // 4. plaintext = v XOR hash_bytes(g, |v|) for the ciphertexts that verify
  parallel_items(n, [&](uint32_t i) {
    if (status[i] == HBTC_ACCEPT && gst[i] != HBTC_ACCEPT) status[i] = HBTC_DECODE_ERR;
    const size_t len = offsets[i + 1] - offsets[i];
    uint8_t* o = out + offsets[i];
    if (status[i] != HBTC_ACCEPT) {
      if (len) memset(o, 0, len);
      return;
    }
    hash_bytes(gb.data() + 48 * (size_t)i, len, o);
    for (size_t j2 = 0; j2 < len; ++j2) o[j2] ^= msgs[offsets[i] + j2];
  });
  return HBTC_OK;
}

}  // extern "C"

// ============================================================================ Reliable Broadcast
// reed-solomon-erasure 3.1 (hbbft's Coding, /root/reference/src/broadcast/broadcast.rs:395-459):
// GF(2^8) mod x^8 + x^4 + x^3 + x^2 + 1 (0x11D), generator 2; build_matrix(k, n) =
// vandermonde(n, k) * inverse(top k x k) (systematic); encode = the parity rows times the data;
// reconstruct_shards = the inverse of the rows of the first k present shards for the missing
// data, then the parity rows for the missing parity.  The matrices are built and inverted here
// (once per shape / presence pattern, cached); the byte work runs in k_gf_apply.
namespace {
struct Gf {
  uint8_t exp[512], log[256];
  Gf() {
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
      exp[i] = exp[i + 255] = (uint8_t)x;
      log[x] = (uint8_t)i;
      x <<= 1;
      if (x & 0x100) x ^= 0x11D;
    }
    exp[510] = exp[511] = exp[0];
    log[0] = 0;
  }
  uint8_t mul(uint8_t a, uint8_t b) const { return a && b ? exp[log[a] + log[b]] : 0; }
  uint8_t inv(uint8_t a) const { return exp[(255 - log[a]) % 255]; }
  uint8_t pow(uint8_t a, unsigned n) const {  // galois_8::exp
    if (n == 0) return 1;
    if (a == 0) return 0;
    return exp[(log[a] * (size_t)n) % 255];
  }
};
const Gf& gf() {
  static const Gf g;
  return g;
}
typedef std::vector<std::vector<uint8_t>> GfMat;

bool gf_invert(GfMat m, GfMat& inv) {
  const size_t n = m.size();
  const Gf& g = gf();
  inv.assign(n, std::vector<uint8_t>(n, 0));
  for (size_t i = 0; i < n; ++i) inv[i][i] = 1;
  for (size_t c = 0; c < n; ++c) {
    size_t p = c;
    while (p < n && !m[p][c]) ++p;
    if (p == n) return false;
    std::swap(m[c], m[p]);
    std::swap(inv[c], inv[p]);
    const uint8_t f = g.inv(m[c][c]);
    for (size_t j = 0; j < n; ++j) {
      m[c][j] = g.mul(f, m[c][j]);
      inv[c][j] = g.mul(f, inv[c][j]);
    }
    for (size_t r = 0; r < n; ++r) {
      const uint8_t e = m[r][c];
      if (r == c || !e) continue;
      for (size_t j = 0; j < n; ++j) {
        m[r][j] ^= g.mul(e, m[c][j]);
        inv[r][j] ^= g.mul(e, inv[c][j]);
      }
    }
  }
  return true;
}

// build_matrix(k, k + p), rows [0, k + p)
const GfMat& rs_matrix(uint32_t k, uint32_t p) {
  static std::mutex mu;
  static std::map<std::pair<uint32_t, uint32_t>, GfMat> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({k, p});
  if (it != cache.end()) return it->second;
  const Gf& g = gf();
  const uint32_t n = k + p;
  GfMat v(n, std::vector<uint8_t>(k));
  for (uint32_t r = 0; r < n; ++r)
    for (uint32_t c = 0; c < k; ++c) v[r][c] = g.pow((uint8_t)r, c);
  GfMat top(v.begin(), v.begin() + k), ti;
  gf_invert(top, ti);  // a Vandermonde matrix of distinct points: always invertible
  GfMat m(n, std::vector<uint8_t>(k, 0));
  for (uint32_t r = 0; r < n; ++r)
    for (uint32_t j = 0; j < k; ++j) {
      uint8_t acc = 0;
      for (uint32_t q = 0; q < k; ++q) acc ^= g.mul(v[r][q], ti[q][j]);
      m[r][j] = acc;
    }
  return cache.emplace(std::make_pair(k, p), std::move(m)).first->second;
}

// nibble tables of coefficient c (k_gf_apply): c * x and c * 16x for x < 16, 4 bytes per dword
void nib_tables(uint8_t c, uint32_t* t) {
  const Gf& g = gf();
  for (int w = 0; w < 8; ++w) {
    uint32_t v = 0;
    for (int b = 0; b < 4; ++b) {
      const unsigned x = (unsigned)(4 * (w & 3) + b);
      v |= (uint32_t)g.mul(c, (uint8_t)(w < 4 ? x : x << 4)) << (8 * b);
    }
    t[w] = v;
  }
}

int gf_plan(hbtc_ctx* c, const std::string& key, const std::vector<uint32_t>& out_rows,
            const std::vector<uint32_t>& in_rows, const GfMat& coef, const hbtc_ctx::GfPlan** out) {
  auto it = c->gf_plans.find(key);
  if (it == c->gf_plans.end()) {
    if (c->gf_plans.size() >= 256) {  // presence patterns are few per era; bound the cache anyway
      // a gf_apply launched on ANY lane may still read these tables (rs_*_dev calls rotate
      // lanes): drain every lane before freeing
      HB_TRY(sync(c));
      for (auto& kv : c->gf_plans) {
        (void)hipFree(kv.second.out_rows);
        (void)hipFree(kv.second.in_rows);
        (void)hipFree(kv.second.tabs);
      }
      c->gf_plans.clear();
    }
    hbtc_ctx::GfPlan pl;
    pl.n_out = (uint32_t)out_rows.size();
    pl.n_in = (uint32_t)in_rows.size();
    std::vector<uint32_t> tabs((size_t)pl.n_out * pl.n_in * 8);
    for (uint32_t r = 0; r < pl.n_out; ++r)
      for (uint32_t j = 0; j < pl.n_in; ++j) nib_tables(coef[r][j], &tabs[((size_t)r * pl.n_in + j) * 8]);
    HB_CHECK(c, hipMalloc(&pl.out_rows, 4 * std::max<size_t>(1, pl.n_out)));
    HB_CHECK(c, hipMalloc(&pl.in_rows, 4 * std::max<size_t>(1, pl.n_in)));
    HB_CHECK(c, hipMalloc(&pl.tabs, 4 * std::max<size_t>(1, tabs.size())));
    HB_CHECK(c, hipMemcpy(pl.out_rows, out_rows.data(), 4 * out_rows.size(), hipMemcpyHostToDevice));
    HB_CHECK(c, hipMemcpy(pl.in_rows, in_rows.data(), 4 * in_rows.size(), hipMemcpyHostToDevice));
    HB_CHECK(c, hipMemcpy(pl.tabs, tabs.data(), 4 * tabs.size(), hipMemcpyHostToDevice));
    it = c->gf_plans.emplace(key, pl).first;
  }
  *out = &it->second;
  return HBTC_OK;
}

int rs_check(hbtc_ctx* c, uint32_t k, uint32_t p, uint32_t len) {
  // ReedSolomon::new: TooFewDataShards / TooFewParityShards / TooManyShards (> 256)
  if (k == 0 || p == 0 || k + p > 256) return fail(c, HBTC_ERR_ARG, "shard counts (ReedSolomon::new)");
  if (len == 0) return fail(c, HBTC_ERR_ARG, "empty shards");
  return HBTC_OK;
}

int rs_encode_dev(hbtc_ctx* c, uint32_t k, uint32_t p, uint32_t len, uint32_t n_inst, uint8_t* d) {
  HB_TRY(rs_check(c, k, p, len));
  if (n_inst == 0) return HBTC_OK;
  const size_t bytes = (size_t)n_inst * (k + p) * len;
  HB_TRY(begin_verify(c, {rng(d, bytes)}, {rng(d, bytes)}));
  const std::string key = "enc/" + std::to_string(k) + "/" + std::to_string(p);
  const hbtc_ctx::GfPlan* pl;
  if (!c->gf_plans.count(key)) {
    const GfMat& m = rs_matrix(k, p);
    std::vector<uint32_t> outs(p), ins(k);
    for (uint32_t i = 0; i < p; ++i) outs[i] = k + i;
    for (uint32_t i = 0; i < k; ++i) ins[i] = i;
    HB_TRY(gf_plan(c, key, outs, ins, GfMat(m.begin() + k, m.end()), &pl));
  } else {
    pl = &c->gf_plans[key];
  }
  HB_TRY(timed(c, "rs", [&] {
    return launch_gf_apply(c->stream, n_inst, nullptr, d, (uint64_t)(k + p) * len, len, pl->n_out,
                           pl->out_rows, pl->n_in, pl->in_rows, pl->tabs);
  }));
  return end_verify(c);
}

int rs_reconstruct_dev(hbtc_ctx* c, uint32_t k, uint32_t p, uint32_t len, uint32_t n_inst, uint8_t* d,
                       const uint8_t* present, int32_t* status) {
  HB_TRY(rs_check(c, k, p, len));
  if (n_inst == 0) return HBTC_OK;
  if (!present || !status) return fail(c, HBTC_ERR_ARG, "present / status");
  const uint32_t n = k + p;
  const size_t bytes = (size_t)n_inst * n * len;
  HB_TRY(begin_verify(c, {rng(d, bytes)}, {rng(d, bytes)}));
  // group the instances by presence pattern
  std::map<std::string, std::vector<uint32_t>> groups;
  for (uint32_t i = 0; i < n_inst; ++i) {
    std::string pat(n, '0');
    uint32_t cnt = 0;
    for (uint32_t j = 0; j < n; ++j)
      if (present[(size_t)i * n + j]) {
        pat[j] = '1';
        ++cnt;
      }
    if (cnt < k) {
      status[i] = HBTC_NOT_ENOUGH_SHARES;  // TooFewShardsPresent
      continue;
    }
    status[i] = HBTC_ACCEPT;
    if (cnt < n) groups[pat].push_back(i);
  }
  const GfMat& m = rs_matrix(k, p);
  for (auto& kv : groups) {
    const std::string& pat = kv.first;
    std::vector<uint32_t> use, miss_d, miss_p, all_d(k);
    for (uint32_t j = 0; j < n; ++j) {
      if (pat[j] == '1' && use.size() < k) use.push_back(j);
      if (pat[j] == '0') (j < k ? miss_d : miss_p).push_back(j);
    }
    for (uint32_t j = 0; j < k; ++j) all_d[j] = j;
    uint32_t* d_jobs;
    HB_TRY(stage_upload(c, "rs.jobs", kv.second.data(), 4 * kv.second.size(), c->stream,
                        reinterpret_cast<void**>(&d_jobs)));
    const uint64_t stride = (uint64_t)n * len;
    const uint32_t nj = (uint32_t)kv.second.size();
    if (!miss_d.empty()) {
      const std::string key = "dec/" + std::to_string(k) + "/" + pat;
      const hbtc_ctx::GfPlan* pl;
      if (!c->gf_plans.count(key)) {
        GfMat sub, inv;
        for (uint32_t j : use) sub.push_back(m[j]);
        if (!gf_invert(sub, inv)) return fail(c, HBTC_ERR_DEVICE, "singular decode matrix");
        GfMat rows;
        for (uint32_t j : miss_d) rows.push_back(inv[j]);
        HB_TRY(gf_plan(c, key, miss_d, use, rows, &pl));
      } else {
        pl = &c->gf_plans[key];
      }
      HB_TRY(timed(c, "rs", [&] {
        return launch_gf_apply(c->stream, nj, d_jobs, d, stride, len, pl->n_out, pl->out_rows,
                               pl->n_in, pl->in_rows, pl->tabs);
      }));
    }
    if (!miss_p.empty()) {
      std::string mp(p, '0');
      for (uint32_t j : miss_p) mp[j - k] = '1';
      const std::string key = "par/" + std::to_string(k) + "/" + mp;
      const hbtc_ctx::GfPlan* pl;
      if (!c->gf_plans.count(key)) {
        GfMat rows;
        for (uint32_t j : miss_p) rows.push_back(m[j]);
        HB_TRY(gf_plan(c, key, miss_p, all_d, rows, &pl));
      } else {
        pl = &c->gf_plans[key];
      }
      HB_TRY(timed(c, "rs", [&] {
        return launch_gf_apply(c->stream, nj, d_jobs, d, stride, len, pl->n_out, pl->out_rows,
                               pl->n_in, pl->in_rows, pl->tabs);
      }));
    }
  }
  return end_verify(c);
}

uint32_t merkle_digests(uint32_t n) {
  uint32_t t = n;
  while (n > 1) {
    n = (n + 1) / 2;
    t += n;
  }
  return t;
}

int merkle_trees_dev(hbtc_ctx* c, uint32_t n, uint32_t len, uint32_t n_inst, const uint8_t* d_leaves,
                     uint8_t* d_out) {
  if (n_inst == 0 || n == 0) return HBTC_OK;
  if (reinterpret_cast<uintptr_t>(d_out) & 7u) return fail(c, HBTC_ERR_ARG, "digests must be 8-byte aligned");
  const uint32_t nd = merkle_digests(n);
  HB_TRY(begin_verify(c, {rng(d_leaves, (size_t)n_inst * n * len)}, {rng(d_out, (size_t)n_inst * nd * 32)}));
  HB_TRY(timed(c, "merkle", [&] {
    return launch_merkle_tree(c->stream, n_inst, n, len, d_leaves, (uint64_t)n * len, nd, d_out);
  }));
  return end_verify(c);
}

int merkle_validate_dev(hbtc_ctx* c, uint32_t n, uint32_t n_nodes, const uint64_t* d_voff,
                        const uint8_t* d_values, const uint32_t* d_idx, const uint32_t* d_doff,
                        const uint8_t* d_dig, const uint8_t* d_roots, int32_t* d_status) {
  if (n == 0) return HBTC_OK;
  if ((reinterpret_cast<uintptr_t>(d_dig) & 7u) || (reinterpret_cast<uintptr_t>(d_roots) & 7u))
    return fail(c, HBTC_ERR_ARG, "digests / roots must be 8-byte aligned");
  HB_TRY(begin_verify(c, {rng(d_voff, 8 * ((size_t)n + 1)), rng(d_idx, 4 * (size_t)n),
                          rng(d_doff, 4 * ((size_t)n + 1)), rng(d_roots, 32 * (size_t)n)},
                      {rng(d_status, 4 * (size_t)n)}));
  HB_TRY(timed(c, "merkle_validate", [&] {
    return launch_merkle_validate(c->stream, n, n_nodes, d_voff, d_values, d_idx, d_doff, d_dig, d_roots,
                                  d_status);
  }));
  return end_verify(c);
}
}  // namespace

extern "C" {

uint32_t hbtc_merkle_digest_count(uint32_t n_leaves) { return n_leaves ? merkle_digests(n_leaves) : 0; }

int hbtc_rs_encode_dev(hbtc_ctx* c, uint32_t k, uint32_t p, uint32_t shard_len, uint32_t n_inst,
                       uint8_t* d_shards) {
  if (!c || (n_inst && !d_shards)) return HBTC_ERR_ARG;
  Guard g(c);
  return rs_encode_dev(c, k, p, shard_len, n_inst, d_shards);
}

int hbtc_rs_reconstruct_dev(hbtc_ctx* c, uint32_t k, uint32_t p, uint32_t shard_len, uint32_t n_inst,
                            uint8_t* d_shards, const uint8_t* present, int32_t* status) {
  if (!c || (n_inst && !d_shards)) return HBTC_ERR_ARG;
  Guard g(c);
  return rs_reconstruct_dev(c, k, p, shard_len, n_inst, d_shards, present, status);
}

int hbtc_merkle_trees_dev(hbtc_ctx* c, uint32_t n_leaves, uint32_t leaf_len, uint32_t n_inst,
                          const uint8_t* d_leaves, uint8_t* d_digests) {
  if (!c || (n_inst && n_leaves && (!d_leaves || !d_digests))) return HBTC_ERR_ARG;
  Guard g(c);
  return merkle_trees_dev(c, n_leaves, leaf_len, n_inst, d_leaves, d_digests);
}

int hbtc_merkle_validate_dev(hbtc_ctx* c, uint32_t n, uint32_t n_nodes, const uint64_t* d_value_off,
                             const uint8_t* d_values, const uint32_t* d_index,
                             const uint32_t* d_digest_off, const uint8_t* d_digests,
                             const uint8_t* d_roots, int32_t* d_status) {
  if (!c) return HBTC_ERR_ARG;
  Guard g(c);
  return merkle_validate_dev(c, n, n_nodes, d_value_off, d_values, d_index, d_digest_off, d_digests,
                             d_roots, d_status);
}

// host-buffer forms: upload, the device core, download, wait
int hbtc_rs_encode(hbtc_ctx* c, uint32_t k, uint32_t p, uint32_t shard_len, uint32_t n_inst,
                   uint8_t* shards) {
  if (!c || (n_inst && !shards)) return HBTC_ERR_ARG;
  Guard g(c);
  HB_TRY(rs_check(c, k, p, shard_len));
  const size_t bytes = (size_t)n_inst * (k + p) * shard_len;
  if (!bytes) return HBTC_OK;
  HB_TRY(sync(c));
  PinLane pin(c);  // the uploads below and the core run on one lane
  void* d;
  HB_TRY(upload(c, "rs.host", shards, bytes, &d));
  HB_TRY(rs_encode_dev(c, k, p, shard_len, n_inst, (uint8_t*)d));
  HB_TRY(download(c, shards, d, bytes));
  return sync(c);
}

int hbtc_rs_reconstruct(hbtc_ctx* c, uint32_t k, uint32_t p, uint32_t shard_len, uint32_t n_inst,
                        uint8_t* shards, const uint8_t* present, int32_t* status) {
  if (!c || (n_inst && (!shards || !present || !status))) return HBTC_ERR_ARG;
  Guard g(c);
  HB_TRY(rs_check(c, k, p, shard_len));
  const size_t bytes = (size_t)n_inst * (k + p) * shard_len;
  if (!bytes) return HBTC_OK;
  HB_TRY(sync(c));
  PinLane pin(c);  // the uploads below and the core run on one lane
  void* d;
  HB_TRY(upload(c, "rs.host", shards, bytes, &d));
  HB_TRY(rs_reconstruct_dev(c, k, p, shard_len, n_inst, (uint8_t*)d, present, status));
  HB_TRY(download(c, shards, d, bytes));
  return sync(c);
}

int hbtc_merkle_trees(hbtc_ctx* c, uint32_t n_leaves, uint32_t leaf_len, uint32_t n_inst,
                      const uint8_t* leaves, uint8_t* digests) {
  if (!c || (n_inst && n_leaves && (!leaves || !digests))) return HBTC_ERR_ARG;
  Guard g(c);
  if (!n_inst || !n_leaves) return HBTC_OK;
  HB_TRY(sync(c));
  PinLane pin(c);  // the uploads below and the core run on one lane
  void *dl, *dd;
  const size_t out_bytes = (size_t)n_inst * merkle_digests(n_leaves) * 32;
  HB_TRY(upload(c, "mk.leaves", leaves, (size_t)n_inst * n_leaves * leaf_len, &dl));
  HB_TRY(ws(c, "mk.out", out_bytes, &dd));
  HB_TRY(merkle_trees_dev(c, n_leaves, leaf_len, n_inst, (const uint8_t*)dl, (uint8_t*)dd));
  HB_TRY(download(c, digests, dd, out_bytes));
  return sync(c);
}

int hbtc_merkle_validate(hbtc_ctx* c, uint32_t n, uint32_t n_nodes, const uint64_t* value_off,
                         const uint8_t* values, const uint32_t* index, const uint32_t* digest_off,
                         const uint8_t* digests, const uint8_t* roots, int32_t* status) {
  if (!c || (n && (!value_off || !index || !digest_off || !roots || !status))) return HBTC_ERR_ARG;
  Guard g(c);
  if (!n) return HBTC_OK;
  HB_TRY(sync(c));
  PinLane pin(c);  // the uploads below and the core run on one lane
  void *dv, *dvo, *di, *ddo, *dd, *dr, *ds;
  HB_TRY(upload(c, "mv.values", values, value_off[n], &dv));
  HB_TRY(upload(c, "mv.voff", value_off, 8 * ((size_t)n + 1), &dvo));
  HB_TRY(upload(c, "mv.idx", index, 4 * (size_t)n, &di));
  HB_TRY(upload(c, "mv.doff", digest_off, 4 * ((size_t)n + 1), &ddo));
  HB_TRY(upload(c, "mv.dig", digests, 32 * (size_t)digest_off[n], &dd));
  HB_TRY(upload(c, "mv.roots", roots, 32 * (size_t)n, &dr));
  HB_TRY(ws(c, "mv.status", 4 * (size_t)n, &ds));
  HB_TRY(merkle_validate_dev(c, n, n_nodes, (const uint64_t*)dvo, (const uint8_t*)dv, (const uint32_t*)di,
                             (const uint32_t*)ddo, (const uint8_t*)dd, (const uint8_t*)dr, (int32_t*)ds));
  HB_TRY(download(c, status, ds, 4 * (size_t)n));
  return sync(c);
}

}  // extern "C"
