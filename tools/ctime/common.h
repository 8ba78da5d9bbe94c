// Compile-time / resource probes for pieces of the kernel arithmetic (not product code).
#include "pairing.h"
using namespace hbtc;
struct TL {
  const Line* __restrict__ l;
  __device__ __forceinline__ void load(Line& o, int j) const { o = l[j]; }
};
#if defined(T_DEC)
__global__ void __launch_bounds__(64) k(const uint32_t* w_in, G1A* out, int* st) {
  uint32_t w[12];
  for (int i = 0; i < 12; ++i) w[i] = w_in[threadIdx.x * 12 + i];
  G1A p;
  bool ok = g1_decompress(p, w);
  out[threadIdx.x] = p;
  st[threadIdx.x] = ok;
}
#elif defined(T_FE)
__global__ void __launch_bounds__(64) k(const Fq12* in, int* st) {
  Fq12 f = in[threadIdx.x], e;
  final_exponentiation(e, f);
  st[threadIdx.x] = fq12_is_one(e);
}
#elif defined(T_ML)
__global__ void __launch_bounds__(64) k(const Line* l1, const Line* l2, const G1A* P, Fq12* out) {
  Fq12 f;
  G1A a = P[threadIdx.x], b = P[threadIdx.x + 64];
  miller_loop_2(f, TL{l1}, a, true, TL{l2}, b, true);
  out[threadIdx.x] = f;
}
#elif defined(T_FMUL)
__global__ void __launch_bounds__(64) k(const Fq12* in, Fq12* out) {
  Fq12 f = in[threadIdx.x], g = in[threadIdx.x + 64];
  fq12_mul(f, f, g);
  out[threadIdx.x] = f;
}
#elif defined(T_QMUL)
__global__ void __launch_bounds__(64) k(const Fq* in, Fq* out) {
  Fq f = in[threadIdx.x], g = in[threadIdx.x + 64];
  for (int i = 0; i < 100; ++i) fq_mul(f, f, g);
  out[threadIdx.x] = f;
}
#endif
