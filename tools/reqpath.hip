// tools/reqpath.hip — which paths raise a CU's rate of random 32-byte reads from an L2-resident
// window (the probe walk's access, DESIGN.md §3.2: bound by ~75 vector-L1 misses in flight per CU)?
//   vec   : lane pairs, 16 B each (probe_walk's form), R windows in flight per pair
//   lds   : the same windows by LDS-DMA (global_load_lds_dwordx4, per-lane source address)
//   scal  : wave-uniform windows by scalar loads (s_load_dwordx8 through the scalar cache)
//   mix   : vec + scal in one wave's loop
// Each XCD reads its own region (blockIdx % 8), so a 2-4 MiB region is L2-resident.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/reqpath tools/reqpath.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__device__ __forceinline__ uint32_t lcg(uint32_t s) { return s * 1664525u + 1013904223u; }
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  return x ^ (x >> 16);
}

typedef __attribute__((address_space(4))) const uint64_t cu64_t;
struct __attribute__((aligned(32))) Win { uint64_t s[4]; };

// region_mask: windows (of 4 slots) per region - 1; VEC windows per lane pair and SC scalar windows
// per wave in flight each step.
template <int VEC, int SC, bool LDSDMA, int LN = 2, int VL = 0>
__global__ __launch_bounds__(256) void reqpath(const int64_t *table, uint32_t region_log2, uint32_t region_mask,
                                               int iters, unsigned long long *sink) {
  __shared__ __attribute__((aligned(16))) int64_t s_win[VEC > 0 ? 4 * 64 * VEC : 1];
  const uint32_t xcd = blockIdx.x & 7u;
  const int64_t *base = table + (region_log2 >= 27 ? 0ull : ((uint64_t)xcd << region_log2));
  const uint32_t lane = threadIdx.x & 63u, sub = lane & (LN - 1), wave = threadIdx.x >> 6;
  uint32_t st = mix32(blockIdx.x * 256u + threadIdx.x / LN + 7u);
  uint32_t ss = __builtin_amdgcn_readfirstlane(mix32(blockIdx.x * 4u + wave + 99u));
  int64_t acc = 0;
  uint64_t sacc = 0;
  for (int it = 0; it < iters; ++it) {
    if constexpr (VEC > 0) {
      if constexpr (LDSDMA) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          st = lcg(st);
          const uint32_t w = (st >> 8) & region_mask & ~(uint32_t)(LN / 2 - 1);
          const int64_t *src = base + (uint64_t)w * 4 + 2 * sub;
          __builtin_amdgcn_global_load_lds((const void *)src, (__attribute__((address_space(3))) void *)&s_win[(wave * VEC + k) * 128],
                                           16, 0, 0);
        }
        longlong2 v[VL > 0 ? VL : 1];
#pragma unroll
        for (int k = 0; k < VL; ++k) {
          st = lcg(st);
          const uint32_t w = (st >> 8) & region_mask;
          v[k] = *reinterpret_cast<const longlong2 *>(base + (uint64_t)w * 4 + 2 * (lane & 1u));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < VL; ++k) acc ^= v[k].x ^ v[k].y;
        acc ^= s_win[(wave * VEC) * 128 + 2 * lane];
      } else {
        longlong2 v[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          st = lcg(st);
          const uint32_t w = (st >> 8) & region_mask;
          v[k] = *reinterpret_cast<const longlong2 *>(base + (uint64_t)w * 4 + 2 * sub);
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) acc ^= v[k].x ^ v[k].y;
      }
    }
    if constexpr (SC > 0) {
      Win v[SC];
#pragma unroll
      for (int k = 0; k < SC; ++k) {
        ss = lcg(ss);
        const uint32_t w = (ss >> 8) & region_mask;
        cu64_t *p = (cu64_t *)(uintptr_t)(base + (uint64_t)w * 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[k].s[q] = p[q];
      }
#pragma unroll
      for (int k = 0; k < SC; ++k) sacc ^= v[k].s[0] ^ v[k].s[1] ^ v[k].s[2] ^ v[k].s[3];
    }
  }
  if ((uint64_t)acc == 0x123456789ull || sacc == 0x987654321ull) atomicAdd(sink, 1ull);
}


// hol: head-of-line test.  L2-resident windows (4 MiB per XCD) as in reqpath, but every MISS-th
// window comes from a 1 GiB region (an HBM miss), and/or every step also streams one coalesced
// 8-byte-per-lane load from a 1 GiB buffer (the walk's key staging).
template <int VEC, bool LDSDMA, int MISS, bool STREAM>
__global__ __launch_bounds__(256) void hol(const int64_t *table, const int64_t *big, int iters, unsigned long long *sink) {
  __shared__ __attribute__((aligned(16))) int64_t s_win[4 * 64 * VEC];
  const uint32_t xcd = blockIdx.x & 7u;
  const int64_t *base = table + ((uint64_t)xcd << 19);
  const uint32_t lane = threadIdx.x & 63u, sub = lane & 1u, wave = threadIdx.x >> 6;
  uint32_t st = mix32(blockIdx.x * 256u + threadIdx.x / 2 + 7u);
  int64_t acc = 0;
  uint64_t spos = ((uint64_t)(blockIdx.x * 4 + wave) * 64 * 1024) & ((1ull << 27) - 1);
  for (int it = 0; it < iters; ++it) {
    int64_t sk = 0;
    if (STREAM) {
      sk = __builtin_nontemporal_load(big + spos + lane);
      spos = (spos + 64 * 1024 * 7 + 64) & ((1ull << 27) - 1);
    }
    longlong2 v[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      st = lcg(st);
      const bool miss = MISS > 0 && ((st >> 3) % MISS) == 0;
      const int64_t *src = miss ? big + (uint64_t)((st >> 4) & ((1u << 25) - 1)) * 4 + 2 * sub
                                : base + (uint64_t)((st >> 8) & ((1u << 17) - 1)) * 4 + 2 * sub;
      if (LDSDMA)
        __builtin_amdgcn_global_load_lds((const void *)src, (__attribute__((address_space(3))) void *)&s_win[(wave * VEC + k) * 128], 16, 0, 0);
      else
        v[k] = *reinterpret_cast<const longlong2 *>(src);
    }
    if (LDSDMA) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      acc ^= s_win[(wave * VEC) * 128 + 2 * lane];
    } else {
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc ^= v[k].x ^ v[k].y;
    }
    acc ^= sk;
  }
  if ((uint64_t)acc == 0x123456789ull) atomicAdd(sink, 1ull);
}

template <int VEC, bool LDSDMA, int MISS, bool STREAM>
void run_hol(const int64_t *table, const int64_t *big, int wg_per_cu, int iters, unsigned long long *sink) {
  const unsigned grid = 256u * wg_per_cu;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((hol<VEC, LDSDMA, MISS, STREAM>), dim3(grid), dim3(256), 0, 0, table, big, iters, sink);
  CK(hipEventRecord(a));
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((hol<VEC, LDSDMA, MISS, STREAM>), dim3(grid), dim3(256), 0, 0, table, big, iters, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= 5;
  const double w = (double)grid * 4 * 32 * VEC * iters;
  printf("{\"test\": \"hol\", \"vec\": %d, \"lds\": %d, \"miss_1_in\": %d, \"stream\": %d, \"wg_per_cu\": %d, \"ms\": %.3f, \"G_windows_s\": %.1f}\n",
         VEC, (int)LDSDMA, MISS, (int)STREAM, wg_per_cu, ms, w / ms / 1e6);
  fflush(stdout);
}

template <int VEC, int SC, bool LDSDMA, int LN = 2, int VL = 0>
void run(const char *name, const int64_t *table, uint32_t region_log2, int wg_per_cu, int iters,
         unsigned long long *sink) {
  const uint32_t region_mask = (1u << (region_log2 - 2)) - 1u;
  const unsigned grid = 256u * wg_per_cu;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((reqpath<VEC, SC, LDSDMA, LN, VL>), dim3(grid), dim3(256), 0, 0, table, region_log2, region_mask, iters, sink);
  CK(hipEventRecord(a));
  const int reps = 5;
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((reqpath<VEC, SC, LDSDMA, LN, VL>), dim3(grid), dim3(256), 0, 0, table, region_log2, region_mask, iters,
                       sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  const double vreq = (double)grid * 4 * (64 / LN) * VEC * iters + (double)grid * 4 * 32 * VL * iters;  // windows
  const double sreq = (double)grid * 4 * SC * iters;        // windows by scalar loads
  printf("{\"test\": \"%s\", \"ln\": %d, \"vl\": %d, \"vec\": %d, \"scal\": %d, \"lds\": %d, \"region_KiB\": %u, \"wg_per_cu\": %d, \"ms\": %.3f, "
         "\"G_vec_windows_s\": %.1f, \"G_scal_windows_s\": %.1f, \"G_total_s\": %.1f}\n",
         name, LN, VL, VEC, SC, (int)LDSDMA, (1u << region_log2) * 8u / 1024u, wg_per_cu, ms, vreq / ms / 1e6, sreq / ms / 1e6,
         (vreq + sreq) / ms / 1e6);
  fflush(stdout);
}

int main() {
  const uint64_t tbytes = 1ull << 30;  // region 2^27 slots x 8 XCDs wraps: use 2^27 slots = 1 GiB shared
  int64_t *table;
  unsigned long long *sink;
  CK(hipMalloc(&table, tbytes));
  CK(hipMemset(table, 1, tbytes));
  CK(hipMalloc(&sink, 8));
  const int it = 256;
  int64_t *big;
  CK(hipMalloc(&big, 1ull << 30));
  CK(hipMemset(big, 2, 1ull << 30));
  run_hol<3, false, 0, false>(table, big, 6, it, sink);
  run_hol<3, true, 0, false>(table, big, 6, it, sink);
  run_hol<3, false, 10, false>(table, big, 6, it, sink);
  run_hol<3, true, 10, false>(table, big, 6, it, sink);
  run_hol<3, false, 30, false>(table, big, 6, it, sink);
  run_hol<3, true, 30, false>(table, big, 6, it, sink);
  run_hol<3, false, 0, true>(table, big, 6, it, sink);
  run_hol<3, true, 0, true>(table, big, 6, it, sink);
  run_hol<3, false, 10, true>(table, big, 6, it, sink);
  run_hol<3, true, 10, true>(table, big, 6, it, sink);
  run_hol<6, true, 10, false>(table, big, 4, it, sink);
  run_hol<6, false, 10, false>(table, big, 6, it, sink);
  return 0;
}
