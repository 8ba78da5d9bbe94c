// Microbenchmarks of the Fq arithmetic core on gfx950 (tools only, not product code): decides
// the Montgomery-multiplication shape (rolled / unrolled / interleaved) and measures the Miller
// loop and final exponentiation in isolation.  Prints one line per variant:
//   name  ms  Fqm/s (lane-level)  Fqm/s / (29.51e12 / 288)  [fraction of the mad_u64 roofline]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "pairing.h"

using namespace hbtc;

#define CHK(x)                                                                        \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);   \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

constexpr int ITERS = 256;

// 3-way interleaved CIOS: three independent products in one rolled loop (ILP 3).
__device__ __forceinline__ void mont_mul_x3(Fq& r0, const Fq& a0, const Fq& b0, Fq& r1, const Fq& a1,
                                            const Fq& b1, Fq& r2, const Fq& a2, const Fq& b2) {
  uint32_t t0[14], t1[14], t2[14];
#pragma unroll
  for (int j = 0; j < 14; ++j) t0[j] = t1[j] = t2[j] = 0;
  Fq x0 = b0, x1 = b1, x2 = b2;
#pragma unroll 1
  for (int i = 0; i < 12; ++i) {
    const uint32_t c0i = x0.v[0], c1i = x1.v[0], c2i = x2.v[0];
#pragma unroll
    for (int j = 0; j < 11; ++j) {
      x0.v[j] = x0.v[j + 1];
      x1.v[j] = x1.v[j + 1];
      x2.v[j] = x2.v[j + 1];
    }
    uint64_t s0[12], s1[12], s2[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      s0[j] = (uint64_t)a0.v[j] * c0i + t0[j];
      s1[j] = (uint64_t)a1.v[j] * c1i + t1[j];
      s2[j] = (uint64_t)a2.v[j] * c2i + t2[j];
    }
    uint32_t k0 = 0, k1 = 0, k2 = 0;
    t0[0] = (uint32_t)s0[0];
    t1[0] = (uint32_t)s1[0];
    t2[0] = (uint32_t)s2[0];
#pragma unroll
    for (int j = 1; j < 12; ++j) {
      t0[j] = addc32((uint32_t)s0[j], (uint32_t)(s0[j - 1] >> 32), k0, &k0);
      t1[j] = addc32((uint32_t)s1[j], (uint32_t)(s1[j - 1] >> 32), k1, &k1);
      t2[j] = addc32((uint32_t)s2[j], (uint32_t)(s2[j - 1] >> 32), k2, &k2);
    }
    t0[12] = addc32(t0[12], (uint32_t)(s0[11] >> 32), k0, &k0);
    t1[12] = addc32(t1[12], (uint32_t)(s1[11] >> 32), k1, &k1);
    t2[12] = addc32(t2[12], (uint32_t)(s2[11] >> 32), k2, &k2);
    t0[13] = k0;
    t1[13] = k1;
    t2[13] = k2;
    const uint32_t q0 = t0[0] * FQ_NP, q1 = t1[0] * FQ_NP, q2 = t2[0] * FQ_NP;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      s0[j] = (uint64_t)q0 * FQ_P[j] + t0[j];
      s1[j] = (uint64_t)q1 * FQ_P[j] + t1[j];
      s2[j] = (uint64_t)q2 * FQ_P[j] + t2[j];
    }
    k0 = k1 = k2 = 0;
#pragma unroll
    for (int j = 1; j < 12; ++j) {
      t0[j - 1] = addc32((uint32_t)s0[j], (uint32_t)(s0[j - 1] >> 32), k0, &k0);
      t1[j - 1] = addc32((uint32_t)s1[j], (uint32_t)(s1[j - 1] >> 32), k1, &k1);
      t2[j - 1] = addc32((uint32_t)s2[j], (uint32_t)(s2[j - 1] >> 32), k2, &k2);
    }
    t0[11] = addc32(t0[12], (uint32_t)(s0[11] >> 32), k0, &k0);
    t1[11] = addc32(t1[12], (uint32_t)(s1[11] >> 32), k1, &k1);
    t2[11] = addc32(t2[12], (uint32_t)(s2[11] >> 32), k2, &k2);
    t0[12] = t0[13] + k0;
    t1[12] = t1[13] + k1;
    t2[12] = t2[13] + k2;
  }
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    r0.v[j] = t0[j];
    r1.v[j] = t1[j];
    r2.v[j] = t2[j];
  }
}

template <int UNROLL, int CHAINS>
__global__ void __launch_bounds__(256) k_fqmul(const Fq* in, Fq* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  Fq g = in[i & 1023];
  Fq x[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) x[c] = in[(i + c + 1) & 1023];
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) mont_mul<12, UNROLL>(x[c], x[c], g, FQ_P, FQ_NP);
  }
  Fq acc = x[0];
#pragma unroll
  for (int c = 1; c < CHAINS; ++c) fq_add(acc, acc, x[c]);
  out[i] = acc;
}

__global__ void __launch_bounds__(256) k_fqmul_x3(const Fq* in, Fq* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  Fq g = in[i & 1023];
  Fq x0 = in[(i + 1) & 1023], x1 = in[(i + 2) & 1023], x2 = in[(i + 3) & 1023];
  for (int it = 0; it < ITERS; ++it) mont_mul_x3(x0, x0, g, x1, x1, g, x2, x2, g);
  fq_add(x0, x0, x1);
  fq_add(x0, x0, x2);
  out[i] = x0;
}

struct TL {
  const Line* __restrict__ l;
  __device__ __forceinline__ void load(Line& o, int j) const { o = l[j]; }
};

__global__ void __launch_bounds__(64) k_miller(const Line* lines, const G1A* P, Fq12* out) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  Fq12 f;
  G1A a = P[i & 1023], b = P[(i + 7) & 1023];
  miller_loop_2(f, TL{lines}, a, true, TL{lines + MILLER_STEPS}, b, true);
  out[i] = f;
}

__global__ void __launch_bounds__(64) k_finalexp(const Fq12* in, Fq12* out) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  Fq12 f = in[i & 1023], e;
  final_exponentiation(e, f);
  out[i] = e;
}

__global__ void __launch_bounds__(64) k_g1dec(const uint32_t* w_in, G1A* out) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  uint32_t w[12];
  for (int k = 0; k < 12; ++k) w[k] = w_in[(i & 1023) * 12 + k];
  G1A p;
  bool ok = g1_decompress(p, w);
  p.inf |= ok ? 0 : 2;
  out[i] = p;
}

template <class K>
float timeit(K launch, int reps) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  launch();
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) launch();
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const double peak_fqm = 29.51e12 / 288.0;
  void *d_in, *d_out, *d_lines, *d_pts, *d_f;
  const int nthreads = 256 * 1024;  // 4 waves per SIMD worth of lanes
  CHK(hipMalloc(&d_in, sizeof(Fq) * 1024));
  CHK(hipMalloc(&d_out, sizeof(Fq12) * 16384 * 64));  // largest grid below: 1M lanes
  CHK(hipMalloc(&d_lines, sizeof(Line) * 2 * MILLER_STEPS));
  CHK(hipMalloc(&d_pts, sizeof(G1A) * 1024));
  CHK(hipMalloc(&d_f, sizeof(Fq12) * 1024));
  // deterministic junk inputs in [0, p): small values are fine for timing
  {
    Fq* h = (Fq*)malloc(sizeof(Fq) * 1024);
    for (int i = 0; i < 1024; ++i)
      for (int j = 0; j < 12; ++j) h[i].v[j] = (j == 11) ? 0x1000u + i : 0x9e3779b9u * (i + 3 * j + 1);
    CHK(hipMemcpy(d_in, h, sizeof(Fq) * 1024, hipMemcpyHostToDevice));
    Line* hl = (Line*)malloc(sizeof(Line) * 2 * MILLER_STEPS);
    for (int i = 0; i < 2 * MILLER_STEPS; ++i) {
      hl[i].a.c0 = h[i];
      hl[i].a.c1 = h[i + 1];
      hl[i].b.c0 = h[i + 2];
      hl[i].b.c1 = h[i + 3];
    }
    CHK(hipMemcpy(d_lines, hl, sizeof(Line) * 2 * MILLER_STEPS, hipMemcpyHostToDevice));
    G1A* hp = (G1A*)malloc(sizeof(G1A) * 1024);
    for (int i = 0; i < 1024; ++i) {
      hp[i].x = h[i];
      hp[i].y = h[(i + 5) & 1023];
      hp[i].inf = 0;
    }
    CHK(hipMemcpy(d_pts, hp, sizeof(G1A) * 1024, hipMemcpyHostToDevice));
    Fq12* hf = (Fq12*)malloc(sizeof(Fq12) * 1024);
    for (int i = 0; i < 1024; ++i) {
      Fq* q = (Fq*)&hf[i];
      for (int k = 0; k < 12; ++k) q[k] = h[(i + k) & 1023];
    }
    CHK(hipMemcpy(d_f, hf, sizeof(Fq12) * 1024, hipMemcpyHostToDevice));
  }
  auto report = [&](const char* name, float ms, double fqm) {
    const double rate = fqm / (ms * 1e-3);
    printf("%-34s %9.3f ms  %9.3e Fqm/s  %.3f of mad roofline\n", name, ms, rate, rate / peak_fqm);
  };
  for (int waves_per_simd : {1, 2, 4, 8}) {
    const int blocks = 1024 * waves_per_simd / 4;  // 256-thread blocks = 4 waves
    const double fqm1 = (double)blocks * 256 * ITERS;
    char nm[64];
    snprintf(nm, sizeof nm, "fq_mul rolled ILP1  w/simd=%d", waves_per_simd);
    report(nm, timeit([&] { hipLaunchKernelGGL((k_fqmul<1, 1>), dim3(blocks), dim3(256), 0, 0, (const Fq*)d_in, (Fq*)d_out); }, 3), fqm1);
    snprintf(nm, sizeof nm, "fq_mul rolled ILP3  w/simd=%d", waves_per_simd);
    report(nm, timeit([&] { hipLaunchKernelGGL((k_fqmul<1, 3>), dim3(blocks), dim3(256), 0, 0, (const Fq*)d_in, (Fq*)d_out); }, 3), 3 * fqm1);
    snprintf(nm, sizeof nm, "fq_mul unrolled ILP1 w/simd=%d", waves_per_simd);
    report(nm, timeit([&] { hipLaunchKernelGGL((k_fqmul<12, 1>), dim3(blocks), dim3(256), 0, 0, (const Fq*)d_in, (Fq*)d_out); }, 3), fqm1);
    snprintf(nm, sizeof nm, "fq_mul unrolled ILP3 w/simd=%d", waves_per_simd);
    report(nm, timeit([&] { hipLaunchKernelGGL((k_fqmul<12, 3>), dim3(blocks), dim3(256), 0, 0, (const Fq*)d_in, (Fq*)d_out); }, 3), 3 * fqm1);
    snprintf(nm, sizeof nm, "fq_mul x3-interleaved w/simd=%d", waves_per_simd);
    report(nm, timeit([&] { hipLaunchKernelGGL(k_fqmul_x3, dim3(blocks), dim3(256), 0, 0, (const Fq*)d_in, (Fq*)d_out); }, 3), 3 * fqm1);
  }
  const int nb = 16384;  // 1M lanes, like one C3 epoch
  report("miller_loop_2 (1M lanes)", timeit([&] { hipLaunchKernelGGL(k_miller, dim3(nb), dim3(64), 0, 0, (const Line*)d_lines, (const G1A*)d_pts, (Fq12*)d_out); }, 1), 7808.0 * nb * 64);
  report("final_exponentiation (1M lanes)", timeit([&] { hipLaunchKernelGGL(k_finalexp, dim3(nb), dim3(64), 0, 0, (const Fq12*)d_f, (Fq12*)d_out); }, 1), 8297.0 * nb * 64);
  report("g1_decompress (1M lanes)", timeit([&] { hipLaunchKernelGGL(k_g1dec, dim3(nb), dim3(64), 0, 0, (const uint32_t*)d_in, (G1A*)d_out); }, 1), 1654.0 * nb * 64);
  return 0;
}
