// Debug harness (r06): the psi subgroup test of one G2 encoding, one-lane vs lane-pair form.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "pair.h"
using namespace hbtc;
__global__ void k_test(const uint32_t* w24, int* out) {
  const uint32_t lane = threadIdx.x;
  uint32_t w[24];
  for (int i = 0; i < 24; ++i) w[i] = w24[i];
  G2A sg;
  const bool dec = g2_decompress(sg, w, false);
  const bool one = dec && g2_in_subgroup(sg);
  G2Ap Q;
  g2p_from_full(Q, sg);
  Fq2 tables[3 * MILLER_STEPS];
  G2Jp T;
  g2p_walk_lines(tables, T, Q);
  const bool pair = g2p_psi_test(T, Q);
  // the one-lane [|x|] Q by the same walk
  G2J t1;
  jac_mul_u64(t1, sg, BLS_X_ABS);
  // compare pair T (assembled) with t1
  Fq ox, oy, oz;
  fq_xchg(ox, T.x.v);
  fq_xchg(oy, T.y.v);
  fq_xchg(oz, T.z.v);
  G2J tp;
  tp.x.c0 = (lane & 1) ? ox : T.x.v; tp.x.c1 = (lane & 1) ? T.x.v : ox;
  tp.y.c0 = (lane & 1) ? oy : T.y.v; tp.y.c1 = (lane & 1) ? T.y.v : oy;
  tp.z.c0 = (lane & 1) ? oz : T.z.v; tp.z.c1 = (lane & 1) ? T.z.v : oz;
  const bool same = jac_eq(tp, t1);
  Fq2 px, py, npy;
  g2_psi(px, py, sg);
  fq2_neg(npy, py);
  const bool one_eq = jac_eq_aff(t1, px, npy);
  const bool pair_eq_full = jac_eq_aff(tp, px, npy);
  if (lane < 2) {
    out[lane * 8 + 0] = dec; out[lane * 8 + 1] = one; out[lane * 8 + 2] = pair;
    out[lane * 8 + 3] = same; out[lane * 8 + 4] = one_eq; out[lane * 8 + 5] = pair_eq_full;
    out[lane * 8 + 6] = jac_is_inf(t1); out[lane * 8 + 7] = 0;
  }
}
int main(int argc, char** argv) {
  const char* hex = argv[1];
  uint8_t b[96];
  for (int i = 0; i < 96; ++i) sscanf(hex + 2 * i, "%2hhx", &b[i]);
  uint32_t w[24];
  memcpy(w, b, 96);
  uint32_t* dw; int* dout;
  hipMalloc(&dw, 96); hipMalloc(&dout, 64);
  hipMemcpy(dw, w, 96, hipMemcpyHostToDevice);
  hipMemset(dout, 0xff, 64);
  hipLaunchKernelGGL(k_test, dim3(1), dim3(64), 0, 0, dw, dout);
  int out[16];
  hipMemcpy(out, dout, 64, hipMemcpyDeviceToHost);
  for (int l = 0; l < 2; ++l)
    printf("lane %d: decoded %d one-lane-subgroup %d pair-psi-test %d pairT==oneT %d one_eq %d pairT_eq %d t1inf %d\n", l, out[l*8],
           out[l*8+1], out[l*8+2], out[l*8+3], out[l*8+4], out[l*8+5], out[l*8+6]);
  return 0;
}
