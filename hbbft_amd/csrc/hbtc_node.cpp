// Multi-device node context: one hbbft node driving several GPUs of one host (include/hbtc.h,
// hbtc_node_*).  hbbft runs one process per node (/root/reference/src/messaging.rs:188) and a
// node has one epoch's crypto at a time in the common case (max_future_epochs = 3,
// src/honey_badger/builder.rs:37), so a node's epoch is split across its GPUs (strong
// scaling) rather than handing each GPU a separate epoch:
//
//   verification  the item range [0, n) is cut into equal contiguous slices, one per device;
//                 an instance crossing a cut becomes one sub-instance per side with the same H
//                 (and w).  The RLC groups are 64-share tiles inside an instance, so a split
//                 instance needs no exchange between devices: each verdict is final where it
//                 is computed, and the devices write disjoint slices of the caller's status.
//   combines      whole instances, balanced by share count (a Lagrange combine is one MSM).
//
// Every device runs its slice through its own context (own streams, own key-set copy) on its
// own host thread; the gather is the disjoint write-back of each slice.  Only the public C ABI
// of the per-device contexts is used here.
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hbtc.h"

struct hbtc_node {
  std::vector<hbtc_ctx*> ctx;
  std::vector<std::vector<uint32_t>> keysets;  // node keyset id - 1 -> per-device id
  std::mutex mu;
  std::string err;
};

namespace {

int node_fail(hbtc_node* nd, int code, const std::string& msg) {
  nd->err = msg;
  return code;
}

// Run fn(d) for every device on its own thread; the first failure is reported.
template <class F>
int run_devices(hbtc_node* nd, F&& fn) {
  const size_t n = nd->ctx.size();
  std::vector<int> rc(n, HBTC_OK);
  std::vector<std::thread> th;
  th.reserve(n);
  for (size_t d = 0; d < n; ++d) th.emplace_back([&, d] { rc[d] = fn(d); });
  for (auto& t : th) t.join();
  for (size_t d = 0; d < n; ++d)
    if (rc[d] != HBTC_OK)
      return node_fail(nd, rc[d], "device " + std::to_string(d) + ": " + hbtc_last_error(nd->ctx[d]));
  return HBTC_OK;
}

bool offsets_ok(uint32_t n_inst, const uint32_t* offsets) {
  if (!offsets || offsets[0] != 0) return false;
  for (uint32_t k = 0; k < n_inst; ++k)
    if (offsets[k + 1] < offsets[k]) return false;
  return true;
}

// One device's slice of a verification batch: items [lo, hi), its sub-instances.
struct Slice {
  uint32_t lo = 0, hi = 0;
  std::vector<uint32_t> parent;   // instance of each sub-instance
  std::vector<uint32_t> offsets;  // relative to lo
};

std::vector<Slice> item_slices(uint32_t n_dev, uint32_t n_inst, const uint32_t* offsets) {
  const uint64_t total = offsets[n_inst];
  std::vector<Slice> s(n_dev);
  uint32_t k = 0;
  for (uint32_t d = 0; d < n_dev; ++d) {
    Slice& sl = s[d];
    sl.lo = (uint32_t)(total * d / n_dev);
    sl.hi = (uint32_t)(total * (d + 1) / n_dev);
    sl.offsets.push_back(0);
    while (k < n_inst && offsets[k + 1] <= sl.lo) ++k;  // instances ending before the slice
    for (uint32_t j = k; j < n_inst && offsets[j] < sl.hi; ++j) {
      const uint32_t a = std::max(offsets[j], sl.lo), b = std::min(offsets[j + 1], sl.hi);
      if (a >= b) continue;
      sl.parent.push_back(j);
      sl.offsets.push_back(b - sl.lo);
    }
  }
  return s;
}

// Whole instances per device, balanced by share count: device d takes [first[d], first[d+1]).
std::vector<uint32_t> instance_cuts(uint32_t n_dev, uint32_t n_inst, const uint32_t* offsets) {
  const uint64_t total = offsets[n_inst];
  std::vector<uint32_t> first(n_dev + 1, n_inst);
  first[0] = 0;
  uint32_t k = 0;
  for (uint32_t d = 1; d < n_dev; ++d) {
    const uint64_t target = total * d / n_dev;
    while (k < n_inst && offsets[k] < target) ++k;
    first[d] = std::max(first[d - 1], k);
  }
  if (total == 0)  // instances without items: spread by count
    for (uint32_t d = 0; d <= n_dev; ++d) first[d] = (uint32_t)((uint64_t)n_inst * d / n_dev);
  return first;
}

std::vector<uint8_t> gather_rows(const uint8_t* base, size_t row, const std::vector<uint32_t>& which) {
  std::vector<uint8_t> out(which.size() * row + 16);
  for (size_t i = 0; i < which.size(); ++i) memcpy(&out[i * row], base + which[i] * row, row);
  return out;
}

int keyset_of(hbtc_node* nd, uint32_t id, size_t d, uint32_t* out) {
  if (id == 0 || id > nd->keysets.size() || nd->keysets[id - 1].empty())
    return node_fail(nd, HBTC_ERR_NO_KEYSET, "unknown node keyset id");
  *out = nd->keysets[id - 1][d];
  return HBTC_OK;
}

// Combines: whole instances per device; rebased offsets, disjoint output rows.
template <class F>
int node_combine(hbtc_node* nd, uint32_t n_inst, const uint32_t* offsets, F&& call) {
  if (!offsets_ok(n_inst, offsets)) return node_fail(nd, HBTC_ERR_ARG, "bad offsets");
  const auto first = instance_cuts((uint32_t)nd->ctx.size(), n_inst, offsets);
  return run_devices(nd, [&](size_t d) {
    const uint32_t a = first[d], b = first[d + 1];
    if (a == b) return HBTC_OK;
    std::vector<uint32_t> off(b - a + 1);
    for (uint32_t k = a; k <= b; ++k) off[k - a] = offsets[k] - offsets[a];
    return call(d, a, b - a, off.data(), offsets[a]);
  });
}

}  // namespace

extern "C" {

int hbtc_shard_items(uint32_t n_dev, uint32_t dev, uint32_t n_inst, const uint32_t* offsets,
                     uint32_t* lo, uint32_t* hi, uint32_t* n_sub, uint32_t* parent,
                     uint32_t* sub_offsets) {
  if (n_dev == 0 || dev >= n_dev || !offsets_ok(n_inst, offsets) || !lo || !hi || !n_sub)
    return HBTC_ERR_ARG;
  const Slice sl = std::move(item_slices(n_dev, n_inst, offsets)[dev]);
  *lo = sl.lo;
  *hi = sl.hi;
  *n_sub = (uint32_t)sl.parent.size();
  if (parent) std::copy(sl.parent.begin(), sl.parent.end(), parent);
  if (sub_offsets) std::copy(sl.offsets.begin(), sl.offsets.end(), sub_offsets);
  return HBTC_OK;
}

int hbtc_shard_instances(uint32_t n_dev, uint32_t n_inst, const uint32_t* offsets, uint32_t* first) {
  if (n_dev == 0 || !first || !offsets_ok(n_inst, offsets)) return HBTC_ERR_ARG;
  const auto f = instance_cuts(n_dev, n_inst, offsets);
  std::copy(f.begin(), f.end(), first);
  return HBTC_OK;
}

int hbtc_node_create(int n_devices, const int* devices, hbtc_node** out) {
  if (!out || n_devices <= 0) return HBTC_ERR_ARG;
  *out = nullptr;
  hbtc_node* nd = new hbtc_node();
  for (int d = 0; d < n_devices; ++d) {
    hbtc_ctx* c = nullptr;
    const int rc = hbtc_ctx_create(devices ? devices[d] : d, &c);
    if (rc != HBTC_OK) {
      for (hbtc_ctx* x : nd->ctx) hbtc_ctx_destroy(x);
      delete nd;
      return rc;
    }
    nd->ctx.push_back(c);
  }
  *out = nd;
  return HBTC_OK;
}

void hbtc_node_destroy(hbtc_node* nd) {
  if (!nd) return;
  for (hbtc_ctx* c : nd->ctx) hbtc_ctx_destroy(c);
  delete nd;
}

const char* hbtc_node_last_error(hbtc_node* nd) { return nd ? nd->err.c_str() : "null node"; }

int hbtc_node_devices(hbtc_node* nd) { return nd ? (int)nd->ctx.size() : 0; }

hbtc_ctx* hbtc_node_context(hbtc_node* nd, int d) {
  return nd && d >= 0 && d < (int)nd->ctx.size() ? nd->ctx[d] : nullptr;
}

int hbtc_node_set_verify_mode(hbtc_node* nd, int mode) {
  if (!nd) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  return run_devices(nd, [&](size_t d) { return hbtc_set_verify_mode(nd->ctx[d], mode); });
}

int hbtc_node_set_rlc_bits(hbtc_node* nd, uint32_t bits) {
  if (!nd) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  return run_devices(nd, [&](size_t d) { return hbtc_set_rlc_bits(nd->ctx[d], bits); });
}

int hbtc_node_keyset_load(hbtc_node* nd, const uint8_t* pk_c48, uint32_t n, uint32_t* keyset_id,
                          uint32_t* n_bad) {
  if (!nd || !pk_c48 || !keyset_id || n == 0) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  std::vector<uint32_t> ids(nd->ctx.size()), bad(nd->ctx.size());
  const int rc = run_devices(nd, [&](size_t d) {
    return hbtc_keyset_load(nd->ctx[d], pk_c48, n, &ids[d], &bad[d]);
  });
  if (rc != HBTC_OK) return rc;
  nd->keysets.push_back(ids);
  *keyset_id = (uint32_t)nd->keysets.size();
  if (n_bad) *n_bad = bad[0];
  return HBTC_OK;
}

int hbtc_node_keyset_free(hbtc_node* nd, uint32_t keyset_id) {
  if (!nd) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  uint32_t dummy;
  const int rc0 = keyset_of(nd, keyset_id, 0, &dummy);
  if (rc0 != HBTC_OK) return rc0;
  std::vector<uint32_t>& ids = nd->keysets[keyset_id - 1];
  const int rc = run_devices(nd, [&](size_t d) { return hbtc_keyset_free(nd->ctx[d], ids[d]); });
  ids.clear();
  return rc;
}

int hbtc_node_verify_dec_shares(hbtc_node* nd, uint32_t keyset_id, uint32_t n_ct,
                                const uint8_t* H_c96, const uint8_t* w_c96,
                                const uint32_t* offsets, const uint32_t* idx,
                                const uint8_t* share_c48, int32_t* status) {
  if (!nd || (n_ct && (!H_c96 || !w_c96))) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  if (!offsets_ok(n_ct, offsets)) return node_fail(nd, HBTC_ERR_ARG, "bad offsets");
  if (offsets[n_ct] && (!idx || !share_c48 || !status)) return node_fail(nd, HBTC_ERR_ARG, "NULL item array");
  const auto slices = item_slices((uint32_t)nd->ctx.size(), n_ct, offsets);
  return run_devices(nd, [&](size_t d) {
    const Slice& sl = slices[d];
    if (sl.hi == sl.lo) return HBTC_OK;
    uint32_t ks;
    if (keyset_of(nd, keyset_id, d, &ks) != HBTC_OK) return HBTC_ERR_NO_KEYSET;
    const auto H = gather_rows(H_c96, 96, sl.parent), w = gather_rows(w_c96, 96, sl.parent);
    return hbtc_verify_dec_shares(nd->ctx[d], ks, (uint32_t)sl.parent.size(), H.data(), w.data(),
                                  sl.offsets.data(), idx + sl.lo, share_c48 + (size_t)sl.lo * 48,
                                  status + sl.lo);
  });
}

int hbtc_node_verify_sig_shares(hbtc_node* nd, uint32_t keyset_id, uint32_t n_inst,
                                const uint8_t* H_c96, const uint32_t* offsets,
                                const uint32_t* idx, const uint8_t* sig_c96, int32_t* status) {
  if (!nd || (n_inst && !H_c96)) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  if (!offsets_ok(n_inst, offsets)) return node_fail(nd, HBTC_ERR_ARG, "bad offsets");
  if (offsets[n_inst] && (!idx || !sig_c96 || !status)) return node_fail(nd, HBTC_ERR_ARG, "NULL item array");
  const auto slices = item_slices((uint32_t)nd->ctx.size(), n_inst, offsets);
  return run_devices(nd, [&](size_t d) {
    const Slice& sl = slices[d];
    if (sl.hi == sl.lo) return HBTC_OK;
    uint32_t ks;
    if (keyset_of(nd, keyset_id, d, &ks) != HBTC_OK) return HBTC_ERR_NO_KEYSET;
    const auto H = gather_rows(H_c96, 96, sl.parent);
    return hbtc_verify_sig_shares(nd->ctx[d], ks, (uint32_t)sl.parent.size(), H.data(),
                                  sl.offsets.data(), idx + sl.lo, sig_c96 + (size_t)sl.lo * 96,
                                  status + sl.lo);
  });
}

int hbtc_node_combine_dec(hbtc_node* nd, uint32_t n_ct, const uint32_t* offsets,
                          const uint32_t* idx, const uint8_t* share_c48, uint32_t t,
                          uint8_t* out_g_c48, int32_t* inst_status) {
  if (!nd) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  return node_combine(nd, n_ct, offsets, [&](size_t d, uint32_t k0, uint32_t nk, const uint32_t* off,
                                             uint32_t i0) {
    return hbtc_combine_dec(nd->ctx[d], nk, off, idx + i0, share_c48 + (size_t)i0 * 48, t,
                            out_g_c48 + (size_t)k0 * 48, inst_status + k0);
  });
}

int hbtc_node_combine_sigs(hbtc_node* nd, uint32_t n_inst, const uint32_t* offsets,
                           const uint32_t* idx, const uint8_t* sig_c96, uint32_t t,
                           uint8_t* out_sig_c96, uint8_t* out_parity, int32_t* inst_status) {
  if (!nd) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  return node_combine(nd, n_inst, offsets, [&](size_t d, uint32_t k0, uint32_t nk,
                                               const uint32_t* off, uint32_t i0) {
    return hbtc_combine_sigs(nd->ctx[d], nk, off, idx + i0, sig_c96 + (size_t)i0 * 96, t,
                             out_sig_c96 + (size_t)k0 * 96, out_parity + k0, inst_status + k0);
  });
}

}  // extern "C"

// ---- device-resident parts (asynchronous per device) ---------------------------------------
namespace {
template <class F>
int node_parts(hbtc_node* nd, const hbtc_node_part* parts, F&& call) {
  if (!nd || !parts) return HBTC_ERR_ARG;
  for (size_t d = 0; d < nd->ctx.size(); ++d)
    if (parts[d].n_inst && !offsets_ok(parts[d].n_inst, parts[d].offsets))
      return node_fail(nd, HBTC_ERR_ARG, "part " + std::to_string(d) + ": bad offsets");
  return run_devices(nd, [&](size_t d) { return parts[d].n_inst ? call(d, parts[d]) : HBTC_OK; });
}
}  // namespace

extern "C" {

int hbtc_node_verify_sig_shares_dev(hbtc_node* nd, uint32_t keyset_id, const hbtc_node_part* parts) {
  if (!nd) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  return node_parts(nd, parts, [&](size_t d, const hbtc_node_part& p) {
    uint32_t ks;
    if (keyset_of(nd, keyset_id, d, &ks) != HBTC_OK) return HBTC_ERR_NO_KEYSET;
    return hbtc_verify_sig_shares_dev(nd->ctx[d], ks, p.n_inst, p.d_H_c96, p.offsets, p.d_idx,
                                      p.d_items, p.d_status);
  });
}

int hbtc_node_verify_dec_shares_dev(hbtc_node* nd, uint32_t keyset_id, const hbtc_node_part* parts) {
  if (!nd) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  return node_parts(nd, parts, [&](size_t d, const hbtc_node_part& p) {
    uint32_t ks;
    if (keyset_of(nd, keyset_id, d, &ks) != HBTC_OK) return HBTC_ERR_NO_KEYSET;
    return hbtc_verify_dec_shares_dev(nd->ctx[d], ks, p.n_inst, p.d_H_c96, p.d_w_c96, p.offsets,
                                      p.d_idx, p.d_items, p.d_status);
  });
}

int hbtc_node_combine_sigs_verified_dev(hbtc_node* nd, const hbtc_node_part* parts, uint32_t t) {
  if (!nd) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  return node_parts(nd, parts, [&](size_t d, const hbtc_node_part& p) {
    return hbtc_combine_sigs_verified_dev(nd->ctx[d], p.n_inst, p.offsets, p.d_idx, p.d_items,
                                          p.d_status, t, p.d_out, p.d_out_parity, p.d_inst_status);
  });
}

int hbtc_node_combine_dec_verified_dev(hbtc_node* nd, const hbtc_node_part* parts, uint32_t t) {
  if (!nd) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  return node_parts(nd, parts, [&](size_t d, const hbtc_node_part& p) {
    return hbtc_combine_dec_verified_dev(nd->ctx[d], p.n_inst, p.offsets, p.d_idx, p.d_items,
                                         p.d_status, t, p.d_out, p.d_inst_status);
  });
}

int hbtc_node_sync(hbtc_node* nd) {
  if (!nd) return HBTC_ERR_ARG;
  std::lock_guard<std::mutex> lk(nd->mu);
  return run_devices(nd, [&](size_t d) { return hbtc_sync(nd->ctx[d]); });
}

}  // extern "C"
