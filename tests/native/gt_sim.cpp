// Host simulator for the wavefront-cooperative GT arithmetic (hbbft_amd/csrc/gt6.h): each
// lane of a (partial) wave is a host thread; the lanes meet at every cross-lane exchange, so
// the SAME source the gfx950 check kernels run is tested on the CPU against the serial tower
// arithmetic of pairing.h.  Test infrastructure only: built into tests/native's host library,
// never into the product.
#include <array>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "gt6.h"

using namespace hbtc;

namespace {

struct Sim {
  uint32_t n = 0;
  std::mutex mu;
  std::condition_variable cv;
  uint32_t arrived = 0;
  uint64_t gen = 0;
  std::vector<std::array<uint32_t, 12>> slots;
  std::vector<int> flags;
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

Sim* g_sim = nullptr;
thread_local uint32_t tl_lane = 0;

void run_lanes(uint32_t n, const std::function<void(uint32_t)>& fn) {
  Sim s;
  s.n = n;
  s.slots.resize(n);
  s.flags.resize(n);
  g_sim = &s;
  std::vector<std::thread> th;
  for (uint32_t l = 0; l < n; ++l)
    th.emplace_back([&, l] {
      tl_lane = l;
      fn(l);
    });
  for (auto& t : th) t.join();
  g_sim = nullptr;
}

void load_words(uint32_t* w, const uint8_t* b, int nwords) {
  for (int i = 0; i < nwords; ++i)
    w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
           ((uint32_t)b[4 * i + 3] << 24);
}
void store_words(uint8_t* b, const uint32_t* w, int nwords) {
  for (int i = 0; i < nwords; ++i)
    for (int j = 0; j < 4; ++j) b[4 * i + j] = (uint8_t)(w[i] >> (8 * j));
}
// big-endian canonical 48 bytes <-> Montgomery Fq
void fq_load_be(Fq& a, const uint8_t* in) {
  uint32_t w[12];
  load_words(w, in, 12);
  Fq c;
  fq_from_be_words(c, w);
  fq_to_mont(a, c);
}
void fq_store_be(uint8_t* out, const Fq& a) {
  Fq c;
  fq_from_mont(c, a);
  uint32_t w[12];
  fq_to_be_words(w, c);
  store_words(out, w, 12);
}
// tower Fq12 <-> 576 bytes (c0.c0.c0, c0.c0.c1, c0.c1.c0, ... c1.c2.c1: the hosttest layout)
Fq2* tower_slot(Fq12& f, int i) {
  Fq6* s = i < 3 ? &f.c0 : &f.c1;
  const int j = i % 3;
  return j == 0 ? &s->c0 : (j == 1 ? &s->c1 : &s->c2);
}
void fq12_load(Fq12& f, const uint8_t* in) {
  for (int i = 0; i < 6; ++i) {
    fq_load_be(tower_slot(f, i)->c0, in + 96 * i);
    fq_load_be(tower_slot(f, i)->c1, in + 96 * i + 48);
  }
}
void fq12_store(uint8_t* out, Fq12& f) {
  for (int i = 0; i < 6; ++i) {
    fq_store_be(out + 96 * i, tower_slot(f, i)->c0);
    fq_store_be(out + 96 * i + 48, tower_slot(f, i)->c1);
  }
}
// flat coefficient k <-> tower slot: f_0 = c0.c0, f_1 = c1.c0, f_2 = c0.c1, f_3 = c1.c1,
// f_4 = c0.c2, f_5 = c1.c2  (tower slot index i: c0.c{0,1,2} = 0,1,2, c1.c{0,1,2} = 3,4,5)
int flat_to_tower(uint32_t k) { return (k & 1u ? 3 : 0) + (int)(k >> 1); }

struct HostLines {
  const Line* l;
  void load(Line& out, int j) const { out = l[j]; }
};

bool decode_g1(G1A& p, const uint8_t* in) {
  uint32_t w[12];
  load_words(w, in, 12);
  return g1_decompress(p, w);
}
bool decode_g2(G2A& p, const uint8_t* in) {
  uint32_t w[24];
  load_words(w, in, 24);
  return g2_decompress(p, w);
}

}  // namespace

namespace hbtc {
namespace gt {
uint32_t lane_id() { return tl_lane; }
void fetch_words(uint32_t* r, const uint32_t* x, int n, uint32_t src) {
  Sim& s = *g_sim;
  memcpy(s.slots[tl_lane].data(), x, 4 * n);
  s.barrier();
  memcpy(r, s.slots[src % s.n].data(), 4 * n);
  s.barrier();
}
uint32_t shfl(uint32_t v, uint32_t src) {
  uint32_t r;
  fetch_words(&r, &v, 1, src);
  return r;
}
bool wave_any(bool p) {
  Sim& s = *g_sim;
  s.flags[tl_lane] = p ? 1 : 0;
  s.barrier();
  bool any = false;
  for (uint32_t l = 0; l < s.n; ++l) any |= s.flags[l] != 0;
  s.barrier();
  return any;
}
}  // namespace gt
}  // namespace hbtc

extern "C" {

// One GT operation on 6 simulated lanes against its tower form:
//   0 mul  1 sqr  2 cyclotomic sqr  3/4/5 frobenius^1/2/3  6 conj  7 final exp  8 easy part
//   9 exp_by_x.  out576 = the flat result in tower layout; returns 0.
int ht_gt_op(int op, const uint8_t* a576, const uint8_t* b576, uint8_t* out576) {
  Fq12 A, B, R;
  fq12_load(A, a576);
  fq12_load(B, b576);
  run_lanes(6, [&](uint32_t l) {
    const gt::Pos ps = gt::pos();
    Fq2 a = *tower_slot(A, flat_to_tower(l)), b = *tower_slot(B, flat_to_tower(l)), r;
    switch (op) {
      case 0: gt::mul(r, a, b, ps); break;
      case 1: gt::sqr(r, a, ps); break;
      case 2: r = a; gt::cyc_sqr(r, ps); break;
      case 3: case 4: case 5: r = a; gt::frob(r, op - 2, ps); break;
      case 6: r = a; gt::conj(r, ps); break;
      case 7: gt::final_exp(r, a, ps); break;
      case 8: gt::easy_part(r, a, ps); break;
      default: gt::exp_by_x(r, a, ps); break;
    }
    *tower_slot(R, flat_to_tower(l)) = r;  // distinct slots per lane
  });
  fq12_store(out576, R);
  return 0;
}

// The same operations in the replicated layout (gt6.h Pos.rep = 3: 18 lanes, coefficient k on
// lanes 3k..3k+2, every Fq2 product split over them).  Returns 0 if all three sub-lanes of every
// coefficient agree (out576 = sub-lane 0's values), 1 otherwise.
int ht_gt_op_rep(int op, uint32_t rep, const uint8_t* a576, const uint8_t* b576, uint8_t* out576) {
  Fq12 A, B, R;
  fq12_load(A, a576);
  fq12_load(B, b576);
  std::vector<Fq2> res(6 * rep);
  run_lanes(6 * rep, [&](uint32_t l) {
    const gt::Pos ps = gt::pos(rep);
    Fq2 a = *tower_slot(A, flat_to_tower(ps.k)), b = *tower_slot(B, flat_to_tower(ps.k)), r;
    switch (op) {
      case 0: gt::mul(r, a, b, ps); break;
      case 1: gt::sqr(r, a, ps); break;
      case 2: r = a; gt::cyc_sqr(r, ps); break;
      case 3: case 4: case 5: r = a; gt::frob(r, op - 2, ps); break;
      case 6: r = a; gt::conj(r, ps); break;
      case 7: gt::final_exp(r, a, ps); break;
      case 8: gt::easy_part(r, a, ps); break;
      default: gt::exp_by_x(r, a, ps); break;
    }
    res[l] = r;  // distinct slots per lane
  });
  int bad = 0;
  for (uint32_t k = 0; k < 6; ++k) {
    *tower_slot(R, flat_to_tower(k)) = res[rep * k];
    for (uint32_t j = 1; j < rep; ++j) bad |= !fq2_eq(res[rep * k], res[rep * k + j]);
  }
  fq12_store(out576, R);
  return bad;
}

// Binary-GCD Fq inversion (gt6.h) on n values, one simulated lane each: Montgomery in / out,
// values as 48-byte big-endian canonical integers (converted to / from Montgomery here).
int ht_fq_inv_binary(uint32_t n, const uint8_t* in48, uint8_t* out48) {
  std::vector<Fq> a(n), r(n);
  for (uint32_t i = 0; i < n; ++i) fq_load_be(a[i], in48 + 48 * i);
  run_lanes(n, [&](uint32_t l) { fq_inv_binary(r[l], a[l]); });
  for (uint32_t i = 0; i < n; ++i) fq_store_be(out48 + 48 * i, r[i]);
  return 0;
}

// The serial tower version of the same operations (pairing.h / field.h).
int ht_tower_op(int op, const uint8_t* a576, const uint8_t* b576, uint8_t* out576) {
  Fq12 A, B, R;
  fq12_load(A, a576);
  fq12_load(B, b576);
  switch (op) {
    case 0: fq12_mul(R, A, B); break;
    case 1: fq12_sqr(R, A); break;
    case 2: fq12_cyclotomic_sqr(R, A); break;
    case 3: case 4: case 5: fq12_frob(R, A, op - 2); break;
    case 6: fq12_conj(R, A); break;
    case 7: final_exponentiation(R, A); break;
    case 8: {
      Fq12 t0, t1;
      fq12_inv(t0, A);
      fq12_conj(t1, A);
      fq12_mul(R, t1, t0);
      break;
    }
    default: fq12_exp_by_x(R, A); break;
  }
  fq12_store(out576, R);
  return 0;
}

// Pairing-product check e(P1, Q1) e(-P2, Q2) on 12 simulated lanes: group 0 takes the pairs
// in order, group 1 swapped; P1 / P2 are given Jacobian scalings z1, z2 (canonical, 48 B BE;
// z = 1 keeps the serial loop's exact Miller value).  Outputs group 0's Miller value and final
// value (tower layout).  Returns bit 0: group values equal, bit 1: group 0 result is one,
// bit 2: group 1 result is one; -1 on a decode error.
int ht_gt_check_rep(uint32_t rep, const uint8_t* p1, const uint8_t* q1, const uint8_t* p2,
                    const uint8_t* q2, const uint8_t* z1, const uint8_t* z2, uint8_t* out_f576,
                    uint8_t* out_e576);
int ht_gt_check(const uint8_t* p1, const uint8_t* q1, const uint8_t* p2, const uint8_t* q2,
                const uint8_t* z1, const uint8_t* z2, uint8_t* out_f576, uint8_t* out_e576) {
  return ht_gt_check_rep(1, p1, q1, p2, q2, z1, z2, out_f576, out_e576);
}
// ... on 12 rep simulated lanes (rep = 3: the replicated latency form, two groups of 18)
int ht_gt_check_rep(uint32_t rep, const uint8_t* p1, const uint8_t* q1, const uint8_t* p2,
                    const uint8_t* q2, const uint8_t* z1, const uint8_t* z2, uint8_t* out_f576,
                    uint8_t* out_e576) {
  G1A P1, P2;
  G2A Q1, Q2;
  if (!decode_g1(P1, p1) || !decode_g1(P2, p2) || !decode_g2(Q1, q1) || !decode_g2(Q2, q2))
    return -1;
  static Line l1[MILLER_STEPS], l2[MILLER_STEPS];
  if (!Q1.inf) g2_precompute_lines(l1, Q1);
  if (!Q2.inf) g2_precompute_lines(l2, Q2);
  auto jac = [](G1J& J, const G1A& A, const uint8_t* zb) {
    jac_from_aff(J, A);
    if (A.inf) return;
    Fq z, z2, z3;
    fq_load_be(z, zb);
    fq_sqr(z2, z);
    fq_mul(z3, z2, z);
    fq_mul(J.x, A.x, z2);
    fq_mul(J.y, A.y, z3);
    J.z = z;
  };
  G1J J1, J2;
  jac(J1, P1, z1);
  jac(J2, P2, z2);
  fq_neg(J2.y, J2.y);  // -P2
  const bool use1 = !P1.inf && !Q1.inf, use2 = !P2.inf && !Q2.inf;
  Fq12 F, E, E1;
  bool one0 = false, one1 = false, same = true;
  std::mutex mu;
  const uint32_t gs = 6 * rep;
  run_lanes(2 * gs, [&](uint32_t l) {
    const gt::Pos ps = gt::pos(rep);
    gt::MillerArg a{l1, nullptr, J1, use1}, b{l2, nullptr, J2, use2};
    Fq2 f, e;
    if (l < gs)
      gt::miller2(f, a, b, ps);
    else
      gt::miller2(f, b, a, ps);
    gt::final_exp(e, f, ps);
    const bool one = gt::is_one(e, ps);
    // compare the two groups' final values coefficient by coefficient
    Fq2 other;
    gt::fetch2(other, e, l < gs ? l + gs : l - gs);
    const bool eq = gt::group_all(fq2_eq(e, other), ps);
    std::lock_guard<std::mutex> lk(mu);
    if (ps.sub != 0) {
      same &= eq;
      return;
    }
    if (l < gs) {
      *tower_slot(F, flat_to_tower(ps.k)) = f;
      *tower_slot(E, flat_to_tower(ps.k)) = e;
      one0 = one;
    } else {
      *tower_slot(E1, flat_to_tower(ps.k)) = e;
      one1 = one;
    }
    same &= eq;
  });
  fq12_store(out_f576, F);
  fq12_store(out_e576, E);
  return (same ? 1 : 0) | (one0 ? 2 : 0) | (one1 ? 4 : 0);
}

// Signature-share form of the check on 6 simulated lanes: e(P1, Q1) e(-G1, Q2) with Q1's
// affine-normalised lines (P1 Jacobian-scaled by z1) and Q2's PROJECTIVE lines evaluated at
// the fixed affine -G1 (gt6.h miller2_t<true>).  Outputs the final value (tower layout);
// returns 1 if it is one, 0 if not, -1 on a decode error.
int ht_gt_check_proj(const uint8_t* p1, const uint8_t* q1, const uint8_t* q2, const uint8_t* z1,
                     uint8_t* out_e576) {
  G1A P1;
  G2A Q1, Q2;
  if (!decode_g1(P1, p1) || !decode_g2(Q1, q1) || !decode_g2(Q2, q2)) return -1;
  static Line l1[MILLER_STEPS];
  static Fq2 pl[3 * MILLER_STEPS];
  if (!Q1.inf) g2_precompute_lines(l1, Q1);
  if (!Q2.inf) g2_proj_lines(pl, Q2);
  G1J J1, NG;
  jac_from_aff(J1, P1);
  if (!P1.inf) {
    Fq z, zz2, zz3;
    fq_load_be(z, z1);
    fq_sqr(zz2, z);
    fq_mul(zz3, zz2, z);
    fq_mul(J1.x, P1.x, zz2);
    fq_mul(J1.y, P1.y, zz3);
    J1.z = z;
  }
  fq_set(NG.x, G1_GEN_X);
  fq_set(NG.y, G1_GEN_Y);
  fq_neg(NG.y, NG.y);
  fq_one(NG.z);
  Fq12 E;
  bool one = false;
  std::mutex mu;
  run_lanes(6, [&](uint32_t l) {
    const gt::Pos ps = gt::pos();
    gt::MillerArg a{l1, nullptr, J1, !P1.inf && !Q1.inf}, b{nullptr, pl, NG, !Q2.inf};
    Fq2 f, e;
    gt::miller2_t<true>(f, a, b, ps);
    gt::final_exp(e, f, ps);
    const bool o = gt::is_one(e, ps);
    std::lock_guard<std::mutex> lk(mu);
    *tower_slot(E, flat_to_tower(ps.k)) = e;
    one = o;
  });
  fq12_store(out_e576, E);
  return one ? 1 : 0;
}

// The serial reference: miller_loop_2 with the same line tables, then the final exponentiation.
int ht_serial_check(const uint8_t* p1, const uint8_t* q1, const uint8_t* p2, const uint8_t* q2,
                    uint8_t* out_f576, uint8_t* out_e576) {
  G1A P1, P2;
  G2A Q1, Q2;
  if (!decode_g1(P1, p1) || !decode_g1(P2, p2) || !decode_g2(Q1, q1) || !decode_g2(Q2, q2))
    return -1;
  static Line l1[MILLER_STEPS], l2[MILLER_STEPS];
  if (!Q1.inf) g2_precompute_lines(l1, Q1);
  if (!Q2.inf) g2_precompute_lines(l2, Q2);
  G1A nP2;
  aff_neg(nP2, P2);
  Fq12 f, e;
  miller_loop_2(f, HostLines{l1}, P1, !P1.inf && !Q1.inf, HostLines{l2}, nP2, !P2.inf && !Q2.inf);
  final_exponentiation(e, f);
  fq12_store(out_f576, f);
  fq12_store(out_e576, e);
  return fq12_is_one(e) ? 1 : 0;
}

}  // extern "C"
