// storebench.hip — measurement tool (not product): the store phase of the one-pass slot split
// (csrc/ccj_partition.hip slot_split_pipe) in isolation.  256 persistent 1024-thread workgroups
// (one per CU, tile group g = blockIdx & 7 as the XCD), tiles of 11264 entries spread over 512
// partitions (runs of ~22 entries, pseudo-random lengths), per tile one device atomic per partition
// reserving its run in segment (partition, g); then every thread stores image entries
// q = it * 1024 + tid to their destinations.  Variants (rate = 2^30 entries / time):
//   split     8-byte key + 4-byte row per entry at its run destination (the split's stores)
//   keys      only the 8-byte keys;  rows: only the 4-byte rows
//   linear    both, at tile-linear destinations (t * 11264 + q): perfectly sequential
//   vec16     the same bytes as 16-byte stores (2 keys / 4 rows per lane, destination rounded down)
//   storebench [variant...]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int T = 1024, PER = 11, P = 512;
constexpr uint32_t TILE = T * PER;
typedef long long i64x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  return (uint32_t)x;
}

template <int MODE>  // 0 split, 1 keys, 2 rows, 3 linear, 4 vec16
__global__ __launch_bounds__(T) void stores(int64_t *out_k, uint32_t *out_r, uint32_t *cur, uint64_t n_tiles,
                                            uint64_t cap) {
  __shared__ uint32_t s_len[P], s_loc[P];
  __shared__ uint64_t s_dst[P];
  __shared__ uint16_t s_part[TILE];
  const uint32_t tid = threadIdx.x, g = blockIdx.x & 7u, bpg = gridDim.x >> 3;
  const uint64_t tend = (g + 1) * n_tiles / 8;
  for (uint64_t t = g * n_tiles / 8 + (blockIdx.x >> 3); t < tend; t += bpg) {
    // runs of TILE / P = 22 entries per partition (the split's mean run); the cursors make each
    // run's destination offset arbitrary
    if (tid < P) {
      s_len[tid] = TILE / P;
      s_loc[tid] = tid * (TILE / P);
    }
    __syncthreads();
    if (tid < P) {
      const uint32_t h = s_len[tid];
      const uint32_t r = h ? atomicAdd(&cur[g * P + tid], h) : 0u;
      s_dst[tid] = ((uint64_t)tid * 8 + g) * cap + (r < cap - 64 ? r : 0u) - s_loc[tid];
      for (uint32_t i = 0; i < h; ++i) s_part[s_loc[tid] + i] = (uint16_t)tid;
    }
    __syncthreads();
    if (MODE == 4) {
#pragma unroll
      for (int it = 0; it < (PER + 1) / 2; ++it) {
        const uint32_t q = 2u * ((uint32_t)it * T + tid);
        if (q + 1 < TILE) {
          const uint64_t dest = (s_dst[s_part[q]] + q) & ~1ull;
          const i64x2 kv = {(long long)q, (long long)q + 1};
          *reinterpret_cast<i64x2 *>(out_k + dest) = kv;
        }
      }
#pragma unroll
      for (int it = 0; it < (PER + 3) / 4; ++it) {
        const uint32_t q = 4u * ((uint32_t)it * T + tid);
        if (q + 3 < TILE) {
          const uint64_t dest = (s_dst[s_part[q]] + q) & ~3ull;
          const u32x4 rv = {q, q + 1, q + 2, q + 3};
          *reinterpret_cast<u32x4 *>(out_r + dest) = rv;
        }
      }
    } else {
#pragma unroll
      for (int it = 0; it < PER; ++it) {
        const uint32_t q = (uint32_t)it * T + tid;
        const uint64_t dest = MODE == 3 ? t * TILE + q : s_dst[s_part[q]] + q;
        if (MODE != 2) out_k[dest] = (int64_t)q;
        if (MODE != 1) out_r[dest] = q;
      }
    }
    __syncthreads();
  }
}

int main(int argc, char **argv) {
  const uint64_t n = 1ull << 30;
  const uint64_t n_tiles = (n + TILE - 1) / TILE;
  const uint64_t cap = (uint64_t)((double)n / (8.0 * P) * 1.0625 + 8.0 * 1000 + 256) / 2048 * 2048 + 2048;
  const uint64_t positions = (uint64_t)P * 8 * cap + 64;
  int64_t *k;
  uint32_t *r, *cur;
  CK(hipMalloc(&k, positions * 8));
  CK(hipMalloc(&r, positions * 4));
  CK(hipMalloc(&cur, P * 8 * 4));
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned grid = cus / 8 * 8;
  const char *names[5] = {"split", "keys", "rows", "linear", "vec16"};
  for (int m = 0; m < 5; ++m) {
    bool want = argc == 1;
    for (int a = 1; a < argc; ++a) want |= !strcmp(argv[a], names[m]);
    if (!want) continue;
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipMemset(cur, 0, P * 8 * 4));
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a, 0));
      switch (m) {
        case 0: hipLaunchKernelGGL(stores<0>, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap); break;
        case 1: hipLaunchKernelGGL(stores<1>, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap); break;
        case 2: hipLaunchKernelGGL(stores<2>, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap); break;
        case 3: hipLaunchKernelGGL(stores<3>, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap); break;
        case 4: hipLaunchKernelGGL(stores<4>, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap); break;
      }
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep) best = ms < best ? ms : best;
    }
    printf("%-8s %.3f ms  (%.2f TB/s of key+row bytes)\n", names[m], best, 12.0 * n / (best * 1e-3) / 1e12);
    fflush(stdout);
  }
  return 0;
}
