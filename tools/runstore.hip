// runstore.hip — measurement tool (not product): how the one-pass split's store phase
// (csrc/ccj_partition.hip slot_split_pipe) depends on the length and alignment of its runs.
// 256 persistent 1024-thread workgroups (tile group g = blockIdx & 7 as the XCD), tiles of L x 512
// entries: every partition gets a run of exactly L entries per tile, reserved by one device atomic
// per partition in segment (partition, g); each thread stores image entries q = it * 1024 + tid
// (8-byte key + 4-byte row) at their run's destination.  2^30 entries per launch.
//   runstore L off [what [P [G]]]  off = 0: every segment cursor starts at 0 (runs of 16 / 32 are
//                             aligned to 128-byte key lines); off = 1: cursors start at a
//                             per-segment offset in [1, 15] (runs never line-aligned)
//   runstore L off what P G pad: pad entries added to every segment's capacity (segment stride)
//   what = both | keys | rows | read (both, plus each entry's 8-byte key read linearly from its tile,
//   right before its store) | pref (the same with the split's schedule: the next tile's keys in
//   flight while this tile's entries are stored; L x P must be 11264) | pref16 (pref, keys loaded as
//   16-byte pairs);  P partitions (default 512, <= 1024);  G tile groups: 8 (a segment
//   per partition and XCD, the split's layout: P x 8 write streams) or 1 (P streams, every XCD
//   writing into every segment)
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

constexpr int T = 1024, PMAX = 1024;

template <int WHAT>  // 0 both, 1 keys, 2 rows, 3 both + the tile's 8-byte keys read linearly (the split's loads)
__global__ __launch_bounds__(T) void stores(int64_t *out_k, uint32_t *out_r, uint32_t *cur, uint64_t n_tiles,
                                            uint64_t cap, uint32_t L, uint32_t P, uint32_t G, const int64_t *src) {
  __shared__ uint64_t s_dst[PMAX];
  const uint32_t tid = threadIdx.x, g = G == 8 ? blockIdx.x & 7u : 0u, bpg = G == 8 ? gridDim.x >> 3 : gridDim.x;
  const uint32_t tile = L * P;
  const uint64_t tend = (g + 1) * n_tiles / G;
  for (uint64_t t = g * n_tiles / G + (G == 8 ? blockIdx.x >> 3 : blockIdx.x); t < tend; t += bpg) {
    if (tid < P) {
      const uint32_t r = atomicAdd(&cur[g * P + tid], L);
      s_dst[tid] = ((uint64_t)tid * G + g) * cap + (r < cap - 64 ? r : 0u) - (uint64_t)tid * L;
    }
    __syncthreads();
    for (uint32_t q = tid; q < tile; q += T) {
      const uint64_t dest = s_dst[q / L] + q;
      const int64_t v = WHAT == 3 ? __builtin_nontemporal_load(src + t * tile + q) : (int64_t)q;
      if (WHAT != 2) out_k[dest] = v;
      if (WHAT != 1) out_r[dest] = q;
    }
    __syncthreads();
  }
}

// pref: the split's own load schedule — the next tile's 11 keys per thread are loaded while this
// tile's entries are stored (tiles of exactly 11 x 1024 entries: L x P = 11264)
__global__ __launch_bounds__(T) void stores_pref(int64_t *out_k, uint32_t *out_r, uint32_t *cur, uint64_t n_tiles,
                                                 uint64_t cap, uint32_t L, uint32_t P, uint32_t G, const int64_t *src) {
  constexpr int PER = 11;
  __shared__ uint64_t s_dst[PMAX];
  const uint32_t tid = threadIdx.x, g = G == 8 ? blockIdx.x & 7u : 0u, bpg = G == 8 ? gridDim.x >> 3 : gridDim.x;
  const uint32_t tile = L * P;  // == PER * T
  const uint64_t tend = (g + 1) * n_tiles / G;
  uint64_t t = g * n_tiles / G + (G == 8 ? blockIdx.x >> 3 : blockIdx.x);
  if (t >= tend) return;
  int64_t kc[PER], kn[PER];
#pragma unroll
  for (int it = 0; it < PER; ++it) kc[it] = __builtin_nontemporal_load(src + t * tile + it * T + tid);
  for (; t < tend; t += bpg) {
    const uint64_t tn = t + bpg < tend ? t + bpg : t;
#pragma unroll
    for (int it = 0; it < PER; ++it) kn[it] = __builtin_nontemporal_load(src + tn * tile + it * T + tid);
    if (tid < P) {
      const uint32_t r = atomicAdd(&cur[g * P + tid], L);
      s_dst[tid] = ((uint64_t)tid * G + g) * cap + (r < cap - 64 ? r : 0u) - (uint64_t)tid * L;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const uint32_t q = (uint32_t)it * T + tid;
      const uint64_t dest = s_dst[q / L] + q;
      out_k[dest] = kc[it];
      out_r[dest] = q;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < PER; ++it) kc[it] = kn[it];
  }
}

// pref16: pref with the keys loaded as 16-byte pairs (2 tid, 2 tid + 1 of each 2048-entry block, the
// 11th key per thread as one 8-byte load); the stores as in pref (their addresses do not depend on
// how the keys were loaded: in the split they come from the LDS image)
__global__ __launch_bounds__(T) void stores_pref16(int64_t *out_k, uint32_t *out_r, uint32_t *cur, uint64_t n_tiles,
                                                   uint64_t cap, uint32_t L, uint32_t P, uint32_t G, const int64_t *src) {
  constexpr int PER = 11;
  typedef long long i64x2 __attribute__((ext_vector_type(2)));
  __shared__ uint64_t s_dst[PMAX];
  const uint32_t tid = threadIdx.x, g = G == 8 ? blockIdx.x & 7u : 0u, bpg = G == 8 ? gridDim.x >> 3 : gridDim.x;
  const uint32_t tile = L * P;  // == PER * T
  const uint64_t tend = (g + 1) * n_tiles / G;
  uint64_t t = g * n_tiles / G + (G == 8 ? blockIdx.x >> 3 : blockIdx.x);
  if (t >= tend) return;
  int64_t kc[PER], kn[PER];
  auto load = [&](uint64_t tt, int64_t(&kk)[PER]) {
#pragma unroll
    for (int j = 0; j < PER / 2; ++j) {
      const i64x2 v = __builtin_nontemporal_load(reinterpret_cast<const i64x2 *>(src + tt * tile + j * 2 * T + 2 * tid));
      kk[2 * j] = v.x;
      kk[2 * j + 1] = v.y;
    }
    kk[PER - 1] = __builtin_nontemporal_load(src + tt * tile + (PER - 1) * T + tid);
  };
  load(t, kc);
  for (; t < tend; t += bpg) {
    const uint64_t tn = t + bpg < tend ? t + bpg : t;
    load(tn, kn);
    if (tid < P) {
      const uint32_t r = atomicAdd(&cur[g * P + tid], L);
      s_dst[tid] = ((uint64_t)tid * G + g) * cap + (r < cap - 64 ? r : 0u) - (uint64_t)tid * L;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const uint32_t q = (uint32_t)it * T + tid;
      const uint64_t dest = s_dst[q / L] + q;
      out_k[dest] = kc[it];
      out_r[dest] = q;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < PER; ++it) kc[it] = kn[it];
  }
}

__global__ void init_cur(uint32_t *cur, uint32_t off) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < PMAX * 8) cur[i] = off ? 1u + (i * 7u) % 15u : 0u;
}

int main(int argc, char **argv) {
  const uint32_t L = argc > 1 ? (uint32_t)atoi(argv[1]) : 22;
  const uint32_t off = argc > 2 ? (uint32_t)atoi(argv[2]) : 0;
  const int what = argc > 3 ? (!strcmp(argv[3], "keys") ? 1 : !strcmp(argv[3], "rows") ? 2 : !strcmp(argv[3], "read") ? 3
                                : !strcmp(argv[3], "pref") ? 4 : !strcmp(argv[3], "pref16") ? 5 : 0) : 0;
  const uint32_t P = argc > 4 ? (uint32_t)atoi(argv[4]) : 512;
  const uint32_t G = argc > 5 && atoi(argv[5]) == 1 ? 1u : 8u;
  const uint64_t pad = argc > 6 ? (uint64_t)atoll(argv[6]) : 0;  // entries added to every segment's capacity
  if (P == 0 || P > (uint32_t)PMAX) return 2;
  const uint64_t n = 1ull << 30;
  const uint64_t tile = (uint64_t)L * P;
  const uint64_t n_tiles = (n + tile - 1) / tile;
  const uint64_t cap = (uint64_t)((double)n / ((double)G * P) * 1.0625 + 8000 + 256) / 2048 * 2048 + 2048 + pad;
  const uint64_t positions = (uint64_t)P * G * cap + 64;
  int64_t *k;
  uint32_t *r, *cur;
  CK(hipMalloc(&k, positions * 8));
  CK(hipMalloc(&r, positions * 4));
  CK(hipMalloc(&cur, PMAX * 8 * 4));
  int64_t *src = nullptr;
  if (what >= 4 && L * P != 11264) return 2;
  if (what >= 3) {
    CK(hipMalloc(&src, (n_tiles * tile) * 8));
    CK(hipMemset(src, 3, (n_tiles * tile) * 8));
  }
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned grid = cus / 8 * 8;
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipLaunchKernelGGL(init_cur, dim3((PMAX * 8 + 255) / 256), dim3(256), 0, 0, cur, off);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    if (what == 0) hipLaunchKernelGGL(stores<0>, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap, L, P, G, src);
    if (what == 1) hipLaunchKernelGGL(stores<1>, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap, L, P, G, src);
    if (what == 2) hipLaunchKernelGGL(stores<2>, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap, L, P, G, src);
    if (what == 3) hipLaunchKernelGGL(stores<3>, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap, L, P, G, src);
    if (what == 4) hipLaunchKernelGGL(stores_pref, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap, L, P, G, src);
    if (what == 5) hipLaunchKernelGGL(stores_pref16, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap, L, P, G, src);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep) best = ms < best ? ms : best;
  }
  const double bytes = (what == 0 ? 12.0 : what == 1 ? 8.0 : what == 2 ? 4.0 : 20.0) * (double)n_tiles * tile;
  const char *wn[6] = {"both", "keys", "rows", "read", "pref", "pr16"};
  printf("L %3u off %u %-4s P %4u G %u pad %5lu  %.3f ms  %.2f TB/s\n", L, off,
         wn[what], P, G, (unsigned long)pad, best,
         bytes / (best * 1e-3) / 1e12);
  return 0;
}
