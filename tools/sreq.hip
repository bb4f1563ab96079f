// sreq.hip — measurement tool (not product): is the scalar data path a second source of L2 read
// requests beside the vector L1 (whose ~90 reads in flight per CU bound probe_walk2)?
// Random 32-byte windows from an L2-resident 4 MiB region (the walk's table window), every XCD
// reading the same region.  Modes (rate = windows / s over the whole chip):
//   vec    each lane pair loads a random window (two 16-byte halves: one L2 request), 8 in flight
//   sca    each wave loads whole random windows with s_load_dwordx8 (uniform address), 4 in flight
//   mix    every wave does both per iteration: 8 vector loads per lane + S scalar windows
// Loads only (the scalar path is never written through).
//   sreq [vec|sca|mix] [S]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef unsigned int u32x8 __attribute__((ext_vector_type(8)));

constexpr uint32_t kWinBits = 17;  // 2^17 windows of 32 B = 4 MiB

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Four scalar window loads AND their wait in one asm statement: the compiler must never see a
// destination register before its load has landed (an in-flight s_load whose destination the
// compiler reused for the next address faulted the first version of this tool).
__device__ __forceinline__ void sload8x4(const void *a, const void *b, const void *c, const void *d, u32x8 &ra,
                                         u32x8 &rb, u32x8 &rc, u32x8 &rd) {
  asm volatile(
      "s_load_dwordx8 %0, %4, 0x0\n\t"
      "s_load_dwordx8 %1, %5, 0x0\n\t"
      "s_load_dwordx8 %2, %6, 0x0\n\t"
      "s_load_dwordx8 %3, %7, 0x0\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&s"(ra), "=&s"(rb), "=&s"(rc), "=&s"(rd)
      : "s"(a), "s"(b), "s"(c), "s"(d)
      : "memory");
}

template <int MODE>  // 0 vec, 1 sca, 2 mix
__global__ __launch_bounds__(256) void reads(const uint4 *win, uint32_t iters, uint32_t S, uint32_t *sink) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  uint32_t acc = 0, sacc = 0;
  for (uint32_t i = 0; i < iters; ++i) {
    if (MODE != 1) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      u32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t w = mix32((wid * iters + i) * 512u + u * 64u + (lane >> 1)) & ((1u << kWinBits) - 1u);
        v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(win) + 2 * w + (lane & 1u));
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].w;
    }
    if (MODE != 0) {
      const uint32_t n = MODE == 1 ? 8u : S;
      for (uint32_t u0 = 0; u0 < n; u0 += 8) {
        const char *a[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const uint32_t w = mix32((wid * iters + i) * 4096u + (u0 + u) * 131u + 7u) & ((1u << kWinBits) - 1u);
          a[u] = (const char *)win + (size_t)__builtin_amdgcn_readfirstlane((int)w) * 32;
        }
        u32x8 r[8];
        sload8x4(a[0], a[1], a[2], a[3], r[0], r[1], r[2], r[3]);
        sload8x4(a[4], a[5], a[6], a[7], r[4], r[5], r[6], r[7]);
#pragma unroll
        for (int u = 0; u < 8; ++u) sacc ^= r[u][0] ^ r[u][7];
      }
    }
  }
  if ((acc ^ sacc) == 0x12345678u) sink[blockIdx.x] = acc ^ sacc;
}

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "vec";
  const uint32_t S = argc > 2 ? (uint32_t)atoi(argv[2]) : 8;
  const int m = !strcmp(mode, "vec") ? 0 : !strcmp(mode, "sca") ? 1 : 2;
  uint4 *win;
  uint32_t *sink;
  CK(hipMalloc(&win, (size_t)32 << kWinBits));
  CK(hipMemset(win, 1, (size_t)32 << kWinBits));
  CK(hipMalloc(&sink, 1 << 20));
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned grid = cus * 8;  // 8 workgroups of 4 waves per CU: 32 waves
  const uint32_t iters = 200;
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    if (m == 0) hipLaunchKernelGGL(reads<0>, dim3(grid), dim3(256), 0, 0, win, iters, S, sink);
    if (m == 1) hipLaunchKernelGGL(reads<1>, dim3(grid), dim3(256), 0, 0, win, iters, S, sink);
    if (m == 2) hipLaunchKernelGGL(reads<2>, dim3(grid), dim3(256), 0, 0, win, iters, S, sink);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep) best = ms < best ? ms : best;
  }
  const double waves = (double)grid * 4;
  const double vwin = m == 1 ? 0 : waves * iters * 8 * 32;  // 8 loads x 32 lane pairs per wave-iteration
  const double swin = m == 0 ? 0 : waves * iters * (m == 1 ? 8 : S);
  printf("%-4s S %2u  %.3f ms  vector %.1f G windows/s  scalar %.1f G windows/s  total %.1f G/s\n", mode, S, best,
         vwin / (best * 1e-3) / 1e9, swin / (best * 1e-3) / 1e9, (vwin + swin) / (best * 1e-3) / 1e9);
  return 0;
}
