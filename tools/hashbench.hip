// tools/hashbench.hip — VALU cost of the reference's bucket hash (hash_functions.h:8-16) on gfx950,
// in wave-cycles per hash, for the formulations the split and walk kernels could use
// (the one-pass split was VALU-bound on hashing).
//   0: murmurhash64 as written (the compiler's 64-bit multiplies: v_mad_u64_u32 + 2 v_mul_lo_u32)
//   1: the cross terms of each 64-bit product from 16-bit halves with 24-bit multiplies
//   2: one 32x32 v_mul_lo_u32 chain (reference point)
//   3: one v_mad_u64_u32 chain (reference point)
// Every thread hashes ITERS dependent values, 16 waves per CU on every CU; the kernel time is
// converted to cycles at the in-kernel clock (s_memtime / s_memrealtime at 100 MHz).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hashbench tools/hashbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr uint64_t kC = 0xd6e8feb86659fd93ULL;

__device__ __forceinline__ uint64_t mur(uint64_t x) {
  x ^= x >> 32;
  x *= kC;
  x ^= x >> 32;
  x *= kC;
  x ^= x >> 32;
  return x;
}

// v_mul_u32_u24 (the compiler folds the 16-bit-half algebra back into v_mul_lo_u32 otherwise)
__device__ __forceinline__ uint32_t mul24(uint32_t a, uint32_t b) {
  uint32_t r;
  asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// low 32 bits of a * b from 16-bit halves (full-rate 24-bit multiplies)
__device__ __forceinline__ uint32_t mul_lo_u24(uint32_t a, uint32_t b) {
  const uint32_t a0 = a & 0xFFFFu, a1 = a >> 16, b0 = b & 0xFFFFu, b1 = b >> 16;
  const uint32_t mid = mul24(a0, b1) + mul24(a1, b0);
  return mul24(a0, b0) + (mid << 16);
}

__device__ __forceinline__ uint64_t mul64_u24(uint64_t x, uint64_t c) {
  const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32), cl = (uint32_t)c, ch = (uint32_t)(c >> 32);
  const uint64_t ll = (uint64_t)xl * cl;  // v_mad_u64_u32
  return ll + ((uint64_t)(mul_lo_u24(xl, ch) + mul_lo_u24(xh, cl)) << 32);
}

__device__ __forceinline__ uint64_t mur_u24(uint64_t x) {
  x ^= x >> 32;
  x = mul64_u24(x, kC);
  x ^= x >> 32;
  x = mul64_u24(x, kC);
  x ^= x >> 32;
  return x;
}

template <int V, int ITERS>
__global__ __launch_bounds__(1024) void hash_loop(uint64_t seed, unsigned long long *sink, unsigned long long *clk) {
  uint64_t a = seed + blockIdx.x * 1024ull + threadIdx.x, b = a * 3 + 1, c = a * 7 + 5, d = a * 11 + 9;
  uint32_t u = (uint32_t)a, w = (uint32_t)b, y = (uint32_t)c, z = (uint32_t)d;
  uint64_t t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int i = 0; i < ITERS; ++i) {  // four independent chains per thread
    if (V == 0) {
      a = mur(a); b = mur(b); c = mur(c); d = mur(d);
    } else if (V == 1) {
      a = mur_u24(a); b = mur_u24(b); c = mur_u24(c); d = mur_u24(d);
    } else if (V == 2) {
      u = u * 0x6659fd93u + 1; w = w * 0x6659fd93u + 1; y = y * 0x6659fd93u + 1; z = z * 0x6659fd93u + 1;
    } else {
      a = (uint64_t)(uint32_t)a * 0x6659fd93u + (a >> 32); b = (uint64_t)(uint32_t)b * 0x6659fd93u + (b >> 32);
      c = (uint64_t)(uint32_t)c * 0x6659fd93u + (c >> 32); d = (uint64_t)(uint32_t)d * 0x6659fd93u + (d >> 32);
    }
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  const unsigned long long v = V >= 2 && V < 3 ? (unsigned long long)(u ^ w ^ y ^ z) : (a ^ b ^ c ^ d);
  if (v == 0x123456789ull) atomicAdd(sink, 1ull);  // keeps the chains live
}

__global__ void check_u24(unsigned long long *bad) {
  uint64_t x = 0x9E3779B97F4A7C15ull * (blockIdx.x * 256ull + threadIdx.x + 1);
  for (int i = 0; i < 64; ++i, x = x * 6364136223846793005ull + 1442695040888963407ull)
    if (mur(x) != mur_u24(x)) atomicAdd(bad, 1ull);
}

template <int V>
void run(const char *name, int cus) {
  constexpr int kIters = 4096;
  unsigned long long *sink, *clk;
  CK(hipMalloc(&sink, 8));
  CK(hipMalloc(&clk, 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((hash_loop<V, kIters>), dim3(cus), dim3(1024), 0, 0, 1ull, sink, clk);  // warm
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL((hash_loop<V, kIters>), dim3(cus), dim3(1024), 0, 0, 7ull, sink, clk);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[2];
  CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
  const double ghz = h[1] ? (double)h[0] / (double)h[1] * 0.1 : 2.4;
  // 16 waves per CU over 4 SIMDs: wave-cycles per op = SIMD cycles / (waves per SIMD * ops per wave)
  const double ops = 4.0 * kIters;  // ops per thread
  const double simd_cycles = ms * 1e-3 * ghz * 1e9;
  printf("%-34s %8.3f ms  clock %.2f GHz  %.1f SIMD-cycles per wave-op  (%.2f G ops/s)\n", name, ms, ghz,
         simd_cycles / (4.0 * ops), (double)cus * 1024 * ops / (ms * 1e-3) / 1e9);
  CK(hipFree(sink));
  CK(hipFree(clk));
}

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  unsigned long long *bad, hb = 0;
  CK(hipMalloc(&bad, 8));
  CK(hipMemset(bad, 0, 8));
  hipLaunchKernelGGL(check_u24, dim3(4096), dim3(256), 0, 0, bad);
  CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  printf("24-bit form mismatches over 2^26 inputs: %llu\n", hb);
  run<0>("murmurhash64 (compiler mul64)", cus);
  run<1>("murmurhash64 (24-bit cross terms)", cus);
  run<2>("v_mul_lo_u32 + add chain", cus);
  run<3>("v_mad_u64_u32 chain", cus);
  return 0;
}
