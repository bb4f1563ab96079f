// runstore.hip — measurement tool (not product): how the one-pass split's store phase
// (csrc/ccj_partition.hip slot_split_pipe) depends on the length and alignment of its runs.
// 256 persistent 1024-thread workgroups (tile group g = blockIdx & 7 as the XCD), tiles of L x 512
// entries: every partition gets a run of exactly L entries per tile, reserved by one device atomic
// per partition in segment (partition, g); each thread stores image entries q = it * 1024 + tid
// (8-byte key + 4-byte row) at their run's destination.  2^30 entries per launch.
//   runstore L off [what]     off = 0: every segment cursor starts at 0 (runs of 16 / 32 are
//                             aligned to 128-byte key lines); off = 1: cursors start at a
//                             per-segment offset in [1, 15] (runs never line-aligned)
//   what = both | keys | rows
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

constexpr int T = 1024, P = 512;

template <int WHAT>  // 0 both, 1 keys, 2 rows
__global__ __launch_bounds__(T) void stores(int64_t *out_k, uint32_t *out_r, uint32_t *cur, uint64_t n_tiles,
                                            uint64_t cap, uint32_t L) {
  __shared__ uint64_t s_dst[P];
  const uint32_t tid = threadIdx.x, g = blockIdx.x & 7u, bpg = gridDim.x >> 3;
  const uint32_t tile = L * P;
  const uint64_t tend = (g + 1) * n_tiles / 8;
  for (uint64_t t = g * n_tiles / 8 + (blockIdx.x >> 3); t < tend; t += bpg) {
    if (tid < P) {
      const uint32_t r = atomicAdd(&cur[g * P + tid], L);
      s_dst[tid] = ((uint64_t)tid * 8 + g) * cap + (r < cap - 64 ? r : 0u) - (uint64_t)tid * L;
    }
    __syncthreads();
    for (uint32_t q = tid; q < tile; q += T) {
      const uint64_t dest = s_dst[q / L] + q;
      if (WHAT != 2) out_k[dest] = (int64_t)q;
      if (WHAT != 1) out_r[dest] = q;
    }
    __syncthreads();
  }
}

__global__ void init_cur(uint32_t *cur, uint32_t off) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < P * 8) cur[i] = off ? 1u + (i * 7u) % 15u : 0u;
}

int main(int argc, char **argv) {
  const uint32_t L = argc > 1 ? (uint32_t)atoi(argv[1]) : 22;
  const uint32_t off = argc > 2 ? (uint32_t)atoi(argv[2]) : 0;
  const int what = argc > 3 ? (!strcmp(argv[3], "keys") ? 1 : !strcmp(argv[3], "rows") ? 2 : 0) : 0;
  const uint64_t n = 1ull << 30;
  const uint64_t tile = (uint64_t)L * P;
  const uint64_t n_tiles = (n + tile - 1) / tile;
  const uint64_t cap = (uint64_t)((double)n / (8.0 * P) * 1.0625 + 8000 + 256) / 2048 * 2048 + 2048;
  const uint64_t positions = (uint64_t)P * 8 * cap + 64;
  int64_t *k;
  uint32_t *r, *cur;
  CK(hipMalloc(&k, positions * 8));
  CK(hipMalloc(&r, positions * 4));
  CK(hipMalloc(&cur, P * 8 * 4));
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned grid = cus / 8 * 8;
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipLaunchKernelGGL(init_cur, dim3((P * 8 + 255) / 256), dim3(256), 0, 0, cur, off);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    if (what == 0) hipLaunchKernelGGL(stores<0>, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap, L);
    if (what == 1) hipLaunchKernelGGL(stores<1>, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap, L);
    if (what == 2) hipLaunchKernelGGL(stores<2>, dim3(grid), dim3(T), 0, 0, k, r, cur, n_tiles, cap, L);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep) best = ms < best ? ms : best;
  }
  const double bytes = (what == 0 ? 12.0 : what == 1 ? 8.0 : 4.0) * (double)n_tiles * tile;
  printf("L %3u off %u %-4s %.3f ms  %.2f TB/s\n", L, off, what == 0 ? "both" : what == 1 ? "keys" : "rows", best,
         bytes / (best * 1e-3) / 1e12);
  return 0;
}
