// Integer-multiply throughput microbenchmark for gfx950 (MI355X).
// Decides the Fq limb scheme (SURVEY.md §7 "Hard parts"): measures per-instruction
// throughput of the candidate 32x32 / 24x24 multiply forms and the carry adds.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

constexpr int NACC = 8;
constexpr int INNER = 64;

__global__ void __launch_bounds__(256) k_mad_u64(uint64_t* out, uint32_t seed, int iters) {
  uint32_t a = threadIdx.x * 2654435761u + seed, b = seed ^ 0x9e3779b9u;
  uint64_t acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = a + j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < INNER; ++u)
#pragma unroll
      for (int j = 0; j < NACC; ++j) {
        uint64_t sc;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[j]), "=s"(sc) : "v"(a), "v"(b));
      }
  }
  uint64_t s = 0; for (int j = 0; j < NACC; ++j) s ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

#define K_U32(NAME, INSN)                                                              \
  __global__ void __launch_bounds__(256) NAME(uint64_t* out, uint32_t seed, int iters) { \
    uint32_t a = threadIdx.x * 2654435761u + seed, b = seed ^ 0x9e3779b9u;            \
    uint32_t acc[NACC];                                                               \
    for (int j = 0; j < NACC; ++j) acc[j] = a + j;                                    \
    for (int i = 0; i < iters; ++i) {                                                 \
      _Pragma("unroll") for (int u = 0; u < INNER; ++u)                               \
      _Pragma("unroll") for (int j = 0; j < NACC; ++j)                                \
        asm volatile(INSN " %0, %0, %1" : "+v"(acc[j]) : "v"(b));                     \
    }                                                                                 \
    uint64_t s = 0; for (int j = 0; j < NACC; ++j) s ^= acc[j];                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                   \
  }

K_U32(k_mul_lo, "v_mul_lo_u32")
K_U32(k_mul_hi, "v_mul_hi_u32")
K_U32(k_mul_u24, "v_mul_u32_u24")
K_U32(k_mul_hi_u24, "v_mul_hi_u32_u24")
K_U32(k_add_u32, "v_add_u32")

__global__ void __launch_bounds__(256) k_mad_u24(uint64_t* out, uint32_t seed, int iters) {
  uint32_t a = threadIdx.x * 2654435761u + seed, b = seed ^ 0x9e3779b9u;
  uint32_t acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = a + j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < INNER; ++u)
#pragma unroll
      for (int j = 0; j < NACC; ++j)
        asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[j]) : "v"(a), "v"(b));
  }
  uint64_t s = 0; for (int j = 0; j < NACC; ++j) s ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// add-with-carry chain: v_add_co_u32 + v_addc_co_u32 pairs (what a 64-bit add costs)
__global__ void __launch_bounds__(256) k_addc(uint64_t* out, uint32_t seed, int iters) {
  uint32_t a = threadIdx.x * 2654435761u + seed, b = seed ^ 0x9e3779b9u;
  uint64_t acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = a + j;
  uint64_t bb = ((uint64_t)b << 32) | a;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < INNER; ++u)
#pragma unroll
      for (int j = 0; j < NACC; ++j) {
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[j]) : "v"(bb));
      }
  }
  uint64_t s = 0; for (int j = 0; j < NACC; ++j) s ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_fma_f64(uint64_t* out, uint32_t seed, int iters) {
  double a = 1.0000001 + threadIdx.x * 1e-9, b = 0.9999999;
  double acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = a + j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < INNER; ++u)
#pragma unroll
      for (int j = 0; j < NACC; ++j)
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[j]) : "v"(a), "v"(b));
  }
  double s = 0; for (int j = 0; j < NACC; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void __launch_bounds__(256) k_fma_f32(uint64_t* out, uint32_t seed, int iters) {
  float a = 1.0000001f + threadIdx.x * 1e-9f, b = 0.9999999f;
  float acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = a + j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < INNER; ++u)
#pragma unroll
      for (int j = 0; j < NACC; ++j)
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[j]) : "v"(a), "v"(b));
  }
  float s = 0; for (int j = 0; j < NACC; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

typedef void (*kfn)(uint64_t*, uint32_t, int);

int main() {
  hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs=%d clock=%d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  const int blocks = prop.multiProcessorCount * 8, threads = 256, iters = 200;
  uint64_t* d; CHK(hipMalloc(&d, sizeof(uint64_t) * blocks * threads));
  struct { const char* name; kfn f; } ks[] = {
    {"v_mad_u64_u32", k_mad_u64}, {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi},
    {"v_mul_u32_u24", k_mul_u24}, {"v_mul_hi_u32_u24", k_mul_hi_u24}, {"v_mad_u32_u24", k_mad_u24},
    {"v_add_u32", k_add_u32}, {"v_lshl_add_u64", k_addc}, {"v_fma_f64", k_fma_f64}, {"v_fma_f32", k_fma_f32}};
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 7u, iters);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 7u + r, iters);
    CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    double ops = 5.0 * blocks * threads * (double)iters * INNER * NACC;
    printf("%-18s %8.3f ms  %8.2f Tops/s (lane-ops)\n", k.name, ms, ops / (ms * 1e-3) / 1e12);
  }
  return 0;
}
