// Fq Montgomery-multiplication shape microbenchmark for gfx950 (tool, not product code).
// Variants: rolled CIOS (round-1 default), fully unrolled CIOS, and product-scanning (FIPS)
// with the 64-bit multiply-add's carry-out feeding a 32-bit column-overflow counter
// (grouped inline-asm MACs).  Prints time, Fqm/s and the fraction of the measured
// v_mad_u64_u32 roofline (29.51e12 / 288 Fqm/s), plus a cross-check of the three results.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "field.h"
#include "fq_fips.h"
#include "fq_fips_asm.h"
using namespace hbtc;
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
constexpr int ITERS = 512;

// V 0-2: products (rolled / unrolled CIOS, C++-glued FIPS); 3: one-block asm FIPS product;
// 4: squaring through the FIPS product; 5: one-block asm FIPS squaring (b ignored); 6 / 7: the
// product / squaring as the shared subroutine of fq_fips_sr.h (build with -DHBTC_FQMUL_SR)
template <int V>
__device__ __forceinline__ void mulv(Fq& r, const Fq& a, const Fq& b) {
  if constexpr (V == 0) mont_mul<12, 1>(r, a, b, FQ_P, FQ_NP);
  else if constexpr (V == 1) mont_mul<12, 12>(r, a, b, FQ_P, FQ_NP);
  else if constexpr (V == 2) mont_mul_fips(r.v, a.v, b.v, FQ_P, FQ_NP);
  else if constexpr (V == 4) mont_mul_fips(r.v, a.v, a.v, FQ_P, FQ_NP);
#if defined(__HIP_DEVICE_COMPILE__)
  else if constexpr (V == 3) fips::mont_mul_asm(r.v, a.v, b.v);
  else if constexpr (V == 5) fips::mont_sqr_asm(r.v, a.v);
  else if constexpr (V == 6) fips::mont_mul_sr(r.v, a.v, b.v);  // subroutine (fq_fips_sr.h)
  else fips::mont_sqr_sr(r.v, a.v);
#endif
}

template <int V, int ILP, int WAVES>
__global__ void __launch_bounds__(256, WAVES) k_mul(const Fq* in, Fq* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  Fq x[ILP];
  const Fq y = in[(i + 1) & 1023];
#pragma unroll
  for (int j = 0; j < ILP; ++j) x[j] = in[(i + 7 * j) & 1023];
#pragma unroll 1
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int j = 0; j < ILP; ++j) mulv<V>(x[j], x[j], y);
#pragma unroll
  for (int j = 1; j < ILP; ++j)
#pragma unroll
    for (int l = 0; l < 12; ++l) x[0].v[l] ^= x[j].v[l];
  out[i] = x[0];
}

template <int V>
__global__ void k_check(const Fq* in, Fq* out) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  Fq r;
  mulv<V>(r, in[i], in[(i * 7 + 3) & 1023]);
  Fq c;
  fq_canon(c, r);
  out[i] = c;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs=%d\n", prop.gcnArchName, prop.multiProcessorCount);
  std::vector<Fq> h(1024);
  uint64_t s = 0x1234567;
  for (auto& f : h) {
    for (int l = 0; l < 12; ++l) { s = s * 6364136223846793005ull + 1442695040888963407ull; f.v[l] = (uint32_t)(s >> 32); }
    f.v[11] &= 0x0fffffffu;  // < 2^380 < 2p
  }
  Fq *d_in, *d_out;
  const int nthreads = 256 * 2048;
  CHK(hipMalloc(&d_in, sizeof(Fq) * 1024));
  CHK(hipMalloc(&d_out, sizeof(Fq) * nthreads));
  CHK(hipMemcpy(d_in, h.data(), sizeof(Fq) * 1024, hipMemcpyHostToDevice));
  // cross-check
  std::vector<Fq> rv[8];
  auto chk = [&](auto kern, int v) {
    rv[v].resize(1024);
    hipLaunchKernelGGL(kern, dim3(16), dim3(64), 0, 0, d_in, d_out);
    CHK(hipMemcpy(rv[v].data(), d_out, sizeof(Fq) * 1024, hipMemcpyDeviceToHost));
  };
  chk(k_check<0>, 0);
  chk(k_check<1>, 1);
  chk(k_check<2>, 2);
  chk(k_check<3>, 3);
  chk(k_check<4>, 4);
  chk(k_check<5>, 5);
  chk(k_check<6>, 6);
  chk(k_check<7>, 7);
  int bad = 0, bad_sq = 0;
  for (int i = 0; i < 1024; ++i) {
    Fq hr, hs;
    mont_mul<12, 1>(hr, h[i], h[(i * 7 + 3) & 1023], FQ_P, FQ_NP);
    fq_canon(hr, hr);
    mont_mul<12, 1>(hs, h[i], h[i], FQ_P, FQ_NP);
    fq_canon(hs, hs);
    for (int l = 0; l < 12; ++l) {
      for (int v : {0, 1, 2, 3, 6}) bad += rv[v][i].v[l] != hr.v[l];
      for (int v : {4, 5, 7}) bad_sq += rv[v][i].v[l] != hs.v[l];
    }
  }
  printf("cross-check vs host CIOS: products %s (%d limb mismatches), squarings %s (%d)\n",
         bad ? "FAIL" : "ok", bad, bad_sq ? "FAIL" : "ok", bad_sq);
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const double peak = 29.51e12 / 288.0;
  auto run = [&](const char* name, auto kern, int blocks, int ilp) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d_in, d_out);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d_in, d_out);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    const double fqm = (double)blocks * 256 * ITERS * ilp;
    printf("%-40s blocks=%5d %8.3f ms %9.3e Fqm/s %.3f of mad roofline  %.1f ns/Fqm/wave\n", name, blocks, ms,
           fqm / (ms * 1e-3), fqm / (ms * 1e-3) / peak, ms * 1e6 / (ITERS * ilp));
  };
  // blocks of 256 threads = 4 waves; 256 CUs x W blocks -> W waves per SIMD
#define RUNV(V, NAME)                                                                   \
  run(NAME " ILP1 1w/SIMD", k_mul<V, 1, 1>, 256, 1);                                   \
  run(NAME " ILP2 1w/SIMD", k_mul<V, 2, 1>, 256, 2);                                   \
  run(NAME " ILP1 2w/SIMD", k_mul<V, 1, 2>, 512, 1);                                   \
  run(NAME " ILP1 4w/SIMD", k_mul<V, 1, 4>, 1024, 1);                                  \
  run(NAME " ILP2 4w/SIMD", k_mul<V, 2, 4>, 1024, 2);                                  \
  run(NAME " ILP1 8w/SIMD", k_mul<V, 1, 8>, 2048, 1);
  RUNV(2, "FIPS asm (C++ glued)")
  RUNV(3, "FIPS one-block asm")
  RUNV(4, "sqr via FIPS product")
  RUNV(5, "sqr one-block asm")
  RUNV(6, "FIPS subroutine (s_swappc)")
  RUNV(7, "sqr subroutine (s_swappc)")
  return 0;
}
