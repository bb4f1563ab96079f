// tools/l2coop.hip — ceilings for the slot-partitioned probe:
//  (1) random reads of a W-byte window from an L2-resident table, the window loaded cooperatively
//      by G lanes (16 B each, one load instruction) or by one lane (W/16 instructions);
//  (2) streaming read, write and copy ceilings of HBM with wide per-thread accesses.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/l2coop tools/l2coop.hip
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

typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// G lanes share one window of 16*G*LPL bytes; every group performs PER independent window reads.
// LPL > 1: each lane loads LPL consecutive 16-B pieces (separate instructions).
template <int G, int LPL, int PER>
__global__ __launch_bounds__(256) void coop_read(const int4 *table, uint32_t n_windows, unsigned long long *sink) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t grp = t / G;
  const uint32_t part = (uint32_t)(t % G);
  int acc = 0;
  int4 v[PER][LPL];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t w = (uint32_t)(mix(grp * PER + k + 99) % n_windows);
    const int4 *p = table + (uint64_t)w * G * LPL + part * LPL;
#pragma unroll
    for (int q = 0; q < LPL; ++q) v[k][q] = p[q];
  }
#pragma unroll
  for (int k = 0; k < PER; ++k)
#pragma unroll
    for (int q = 0; q < LPL; ++q) acc ^= v[k][q].x ^ v[k][q].w;
  if (acc == 0x1234567) atomicAdd(sink, 1ull);
}

// one lane, one 16-byte window at an 8-byte-aligned (not 16-aligned) random slot
template <int PER>
__global__ __launch_bounds__(256) void unaligned_read(const int64_t *table, uint32_t n_slots, unsigned long long *sink) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t acc = 0;
  int64_t v[PER][2];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t s = (uint32_t)(mix(t * PER + k + 7) % (n_slots - 1));
    const int64_t *p = table + s;
    v[k][0] = p[0];
    v[k][1] = p[1];
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) acc ^= v[k][0] ^ v[k][1];
  if (acc == 0x1234567) atomicAdd(sink, 1ull);
}

template <int U>
__global__ __launch_bounds__(256) void stream_read(const v4i *src, uint64_t n, unsigned long long *sink) {
  int acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * U;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x * U + threadIdx.x; i < n; i += stride) {
    v4i v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + i + (uint64_t)u * blockDim.x);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x1234567) atomicAdd(sink, 1ull);
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void stream_write(v4i *dst, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * U;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x * U + threadIdx.x; i < n; i += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const v4i v = v4i{(int)i, u, 1, 2};
      if (NT) __builtin_nontemporal_store(v, dst + i + (uint64_t)u * blockDim.x);
      else dst[i + (uint64_t)u * blockDim.x] = v;
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void stream_copy(const v4i *src, v4i *dst, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * U;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x * U + threadIdx.x; i < n; i += stride) {
    v4i v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + i + (uint64_t)u * blockDim.x);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], dst + i + (uint64_t)u * blockDim.x);
  }
}

struct Timer {
  hipEvent_t a, b;
  Timer() {
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
  }
  void start() { CK(hipEventRecord(a)); }
  float stop(int reps) {
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
  }
};

template <int G, int LPL, int PER>
void run_coop(const int4 *table, uint64_t table_bytes, unsigned long long *sink, uint64_t windows) {
  const uint32_t n_windows = (uint32_t)(table_bytes / (16ull * G * LPL));
  const uint64_t threads = windows / PER * G;
  const unsigned grid = (unsigned)((threads + 255) / 256);
  Timer t;
  hipLaunchKernelGGL((coop_read<G, LPL, PER>), dim3(grid), dim3(256), 0, 0, table, n_windows, sink);
  t.start();
  for (int i = 0; i < 5; ++i)
    hipLaunchKernelGGL((coop_read<G, LPL, PER>), dim3(grid), dim3(256), 0, 0, table, n_windows, sink);
  const float ms = t.stop(5);
  printf("{\"test\": \"coop_read\", \"window_B\": %d, \"lanes_per_window\": %d, \"loads_per_lane\": %d, \"per\": %d, "
         "\"table_KiB\": %llu, \"windows\": %llu, \"ms\": %.3f, \"Gwindows_per_s\": %.1f, \"GBps\": %.0f}\n",
         16 * G * LPL, G, LPL, PER, (unsigned long long)(table_bytes >> 10), (unsigned long long)windows, ms,
         windows / ms / 1e6, windows * 16.0 * G * LPL / ms / 1e6);
}

int main() {
  unsigned long long *sink;
  CK(hipMalloc(&sink, 8));
  const uint64_t big = 4ull << 30;
  int4 *a, *b;
  CK(hipMalloc(&a, big));
  CK(hipMalloc(&b, big));
  CK(hipMemset(a, 1, big));
  CK(hipMemset(b, 2, big));
  const uint64_t W = 1ull << 28;  // windows per launch
  for (uint64_t tb : {2ull << 20, 1ull << 20}) {
    run_coop<1, 1, 4>(a, tb, sink, W);
    run_coop<1, 1, 8>(a, tb, sink, W);
    run_coop<2, 1, 4>(a, tb, sink, W);
    run_coop<2, 1, 8>(a, tb, sink, W);
    run_coop<1, 2, 4>(a, tb, sink, W);
    run_coop<4, 1, 4>(a, tb, sink, W);
    run_coop<4, 1, 8>(a, tb, sink, W);
    run_coop<2, 2, 4>(a, tb, sink, W);
    run_coop<1, 4, 2>(a, tb, sink, W);
    run_coop<8, 1, 4>(a, tb, sink, W);
    run_coop<4, 2, 4>(a, tb, sink, W);
    Timer t;
    const unsigned grid = (unsigned)(W / 4 / 256);
    hipLaunchKernelGGL(unaligned_read<4>, dim3(grid), dim3(256), 0, 0, (const int64_t *)a, (uint32_t)(tb / 8), sink);
    t.start();
    for (int i = 0; i < 5; ++i)
      hipLaunchKernelGGL(unaligned_read<4>, dim3(grid), dim3(256), 0, 0, (const int64_t *)a, (uint32_t)(tb / 8), sink);
    const float ms = t.stop(5);
    printf("{\"test\": \"unaligned16_read\", \"table_KiB\": %llu, \"ms\": %.3f, \"Gwindows_per_s\": %.1f}\n",
           (unsigned long long)(tb >> 10), ms, W / ms / 1e6);
  }
  const uint64_t n = big / 16;
  const unsigned grids[] = {1024, 4096, 16384};
  for (unsigned g : grids) {
    Timer t;
    hipLaunchKernelGGL(stream_read<4>, dim3(g), dim3(256), 0, 0, (const v4i *)a, n, sink);
    t.start();
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(stream_read<4>, dim3(g), dim3(256), 0, 0, (const v4i *)a, n, sink);
    float ms = t.stop(5);
    printf("{\"test\": \"stream_read\", \"grid\": %u, \"GBps\": %.0f}\n", g, big / ms / 1e6);
    hipLaunchKernelGGL((stream_write<4, true>), dim3(g), dim3(256), 0, 0, (v4i *)b, n);
    t.start();
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((stream_write<4, true>), dim3(g), dim3(256), 0, 0, (v4i *)b, n);
    ms = t.stop(5);
    printf("{\"test\": \"stream_write_nt\", \"grid\": %u, \"GBps\": %.0f}\n", g, big / ms / 1e6);
    t.start();
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((stream_write<4, false>), dim3(g), dim3(256), 0, 0, (v4i *)b, n);
    ms = t.stop(5);
    printf("{\"test\": \"stream_write\", \"grid\": %u, \"GBps\": %.0f}\n", g, big / ms / 1e6);
    t.start();
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(stream_copy<4>, dim3(g), dim3(256), 0, 0, (const v4i *)a, (v4i *)b, n);
    ms = t.stop(5);
    printf("{\"test\": \"stream_copy\", \"grid\": %u, \"GBps\": %.0f}\n", g, 2.0 * big / ms / 1e6);
  }
  return 0;
}
