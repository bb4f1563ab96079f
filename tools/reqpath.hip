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


// One LDS-DMA wave-instruction (lane L's 16 bytes at g land at LDS byte lds + 16 L).  M0 is saved and
// restored around it: the compiler treats M0 as reserved and does not honour a clobber of it.
__device__ __forceinline__ void dma16(const void *g, uint32_t lds) {
  uint32_t saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(saved)
               : "v"(g), "s"(lds)
               : "memory");
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
          const uint32_t w = (st >> 8) & region_mask & ~(uint32_t)((LN >= 2 ? LN / 2 : 1) - 1);
          const int64_t *src = base + (uint64_t)w * 4 + 2 * sub;
          // inline asm: the builtin's address computation was hoisted out of the loop by the compiler
          // (every iteration re-read the same windows: round 3's first "2x" reading was that artifact)
          const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane(
              (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) int64_t *)&s_win[(wave * VEC + k) * 128]);
          dma16(src, lds);
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
      if (LDSDMA) {
        const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) int64_t *)&s_win[(wave * VEC + k) * 128]);
        dma16(src, lds);
      }
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

// verify: one LDS-DMA of random 16-byte pieces per lane (table[i] = i), read back and checked
__global__ __launch_bounds__(256) void dma_verify(const int64_t *table, uint32_t mask, unsigned long long *bad,
                                                  unsigned long long *good) {
  __shared__ __attribute__((aligned(16))) int64_t s_win[4 * 128];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t st = mix32(blockIdx.x * 256u + threadIdx.x / 2 + 7u);
  const uint32_t w = (st >> 4) & mask;
  const int64_t *src = table + (uint64_t)w * 4 + 2 * (lane & 1u);
  s_win[wave * 128 + 2 * lane] = -5;
  s_win[wave * 128 + 2 * lane + 1] = -5;
  __syncthreads();
  __builtin_amdgcn_global_load_lds((const void *)src, (__attribute__((address_space(3))) void *)&s_win[wave * 128], 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int64_t e0 = (int64_t)w * 4 + 2 * (lane & 1u);
  const bool ok = s_win[wave * 128 + 2 * lane] == e0 && s_win[wave * 128 + 2 * lane + 1] == e0 + 1;
  if (ok) atomicAdd(good, 1ull); else atomicAdd(bad, 1ull);
}
__global__ void iota64(int64_t *p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[i] = (int64_t)i;
}

// verify2: the throughput kernel's shape (VEC DMAs in flight per wave, many iterations) with every
// landed window checked against table[i] = i; counts bad / good lanes
template <int VEC>
__global__ __launch_bounds__(256) void dma_verify2(const int64_t *table, uint32_t mask, int iters,
                                                   unsigned long long *bad, unsigned long long *good) {
  __shared__ __attribute__((aligned(16))) int64_t s_win[4 * 128 * VEC];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t st = mix32(blockIdx.x * 256u + threadIdx.x / 2 + 7u);
  uint32_t nb = 0, ng = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t w[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      st = lcg(st);
      w[k] = (st >> 8) & mask;
      const int64_t *src = table + (uint64_t)w[k] * 4 + 2 * (lane & 1u);
      const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane(
          (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) int64_t *)&s_win[(wave * VEC + k) * 128]);
      dma16(src, lds);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const int64_t e0 = (int64_t)w[k] * 4 + 2 * (lane & 1u);
      const int64_t *x = &s_win[(wave * VEC + k) * 128 + 2 * lane];
      if (x[0] == e0 && x[1] == e0 + 1) ++ng; else ++nb;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  atomicAdd(bad, (unsigned long long)nb);
  atomicAdd(good, (unsigned long long)ng);
}

// policy: random 64-byte rows (4 lanes x 16 B) from a 1 GiB region by buffer loads with cache
// policy AUX (1 sc0, 2 nt, 16 sc1): which policies make the L2 fetch less than a 128-byte line?
template <int AUX>
__global__ __launch_bounds__(256) void policy_read(const int64_t *table, int iters, unsigned long long *sink) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t st = mix32(blockIdx.x * 256u + threadIdx.x / 4 + 7u);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)table, (short)0, 0x7FFFFFFF, 0x00020000);
  int64_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      st = lcg(st);
      w[k] = (st >> 8) & ((1u << 24) - 1);  // 2^24 rows of 64 B = 1 GiB
    }
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    i32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(w[k] * 64u + (lane & 3u) * 16u), 0, AUX);
#pragma unroll
    for (int k = 0; k < 4; ++k) acc ^= (int64_t)v[k].x ^ v[k].w;
  }
  if (acc == 0x123456789ll) atomicAdd(sink, 1ull);
}
template <int AUX>
void run_policy(const int64_t *table, unsigned long long *sink) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((policy_read<AUX>), dim3(1536), dim3(256), 0, 0, table, 64, sink);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL((policy_read<AUX>), dim3(1536), dim3(256), 0, 0, table, 64, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double rows = 1536.0 * 256 / 4 * 4 * 64;
  printf("{\"test\": \"policy\", \"aux\": %d, \"ms\": %.3f, \"G_rows_s\": %.1f}\n", AUX, ms, rows / ms / 1e6);
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
  const char *mode = getenv("REQPATH_MODE");
  if (mode && !strcmp(mode, "verify")) {
    hipLaunchKernelGGL(iota64, dim3(4096), dim3(256), 0, 0, table, tbytes / 8);
    unsigned long long *cnt;
    CK(hipMalloc(&cnt, 16));
    CK(hipMemset(cnt, 0, 16));
    hipLaunchKernelGGL(dma_verify, dim3(4096), dim3(256), 0, 0, table, (1u << 25) - 1, cnt, cnt + 1);
    unsigned long long h[2];
    CK(hipMemcpy(h, cnt, 16, hipMemcpyDeviceToHost));
    printf("{\"test\": \"dma_verify\", \"bad_lanes\": %llu, \"good_lanes\": %llu}\n", h[0], h[1]);
    CK(hipMemset(cnt, 0, 16));
    hipLaunchKernelGGL((dma_verify2<3>), dim3(1536), dim3(256), 0, 0, table, (1u << 25) - 1, 64, cnt, cnt + 1);
    CK(hipMemcpy(h, cnt, 16, hipMemcpyDeviceToHost));
    printf("{\"test\": \"dma_verify2\", \"bad_lanes\": %llu, \"good_lanes\": %llu}\n", h[0], h[1]);
    return 0;
  }
  if (mode && !strcmp(mode, "policy")) {
    run_policy<0>(table, sink);
    run_policy<1>(table, sink);
    run_policy<2>(table, sink);
    run_policy<3>(table, sink);
    run_policy<16>(table, sink);
    run_policy<17>(table, sink);
    run_policy<18>(table, sink);
    run_policy<19>(table, sink);
    return 0;
  }
  if (mode && !strcmp(mode, "lanes")) {  // LDS-DMA lanes per window: 16 / 32 / 64 / 128-byte windows
    run<3, 0, true, 1>("lds16B", table, 19u, 6, it, sink);
    run<3, 0, true, 2>("lds32B", table, 19u, 6, it, sink);
    run<3, 0, true, 4>("lds64B", table, 19u, 6, it, sink);
    run<3, 0, true, 8>("lds128B", table, 19u, 6, it, sink);
    run<1, 0, true, 1>("lds16B_1", table, 19u, 6, it, sink);
    run<1, 0, true, 2>("lds32B_1", table, 19u, 6, it, sink);
    run<3, 0, false, 1>("vec16B", table, 19u, 6, it, sink);
    run<3, 0, false, 2>("vec32B", table, 19u, 6, it, sink);
    return 0;
  }
  if (mode && !strcmp(mode, "sizes")) {  // request sizes from HBM (run under rocprofv3 --pmc)
    run<3, 0, false>("vec", table, 27u, 6, it, sink);
    run<3, 0, true>("lds", table, 27u, 6, it, sink);
    run<3, 0, true, 4>("lds64B", table, 27u, 6, it, sink);
    return 0;
  }
  int64_t *big;
  CK(hipMalloc(&big, 1ull << 30));
  CK(hipMemset(big, 2, 1ull << 30));
  run_hol<3, false, 0, false>(table, big, 6, it, sink);
  run_hol<3, true, 0, false>(table, big, 6, it, sink);
  run_hol<3, false, 10, false>(table, big, 6, it, sink);
  run_hol<3, true, 10, false>(table, big, 6, it, sink);
  return 0;
}
