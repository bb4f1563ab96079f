// overlap_emu.hip — measurement tool (not product): can the C2 walk's L2-request-bound work and the
// split's HBM-bound store pattern share the chip?  Two LDS-light kernels that emulate them:
//   walk   one 256-thread workgroup per 2048-row chunk, chunks of a partition consecutive and
//          dealt XCD by XCD (the walk's swizzle); per row an 8-byte key read (streamed) and one
//          random 32-byte window of the partition's 4 MiB table slice (lane pairs, 16 B each);
//          2^30 rows, 512 partitions of a 2 GiB table
//   split  tools/runstore's "read" pattern: 256 persistent 1024-thread workgroups, 11264-entry
//          tiles, runs of 22 over 512 partitions x 8 XCD groups, 8-byte key read + 12 bytes
//          stored per entry (2^30 entries)
// Each alone, then both at once on two streams (the split's grid capped so walk workgroups keep
// room on every CU).   overlap_emu [split_wgs]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

constexpr uint32_t kChunk = 2048, kParts = 512, kWinSlots = 1u << 19;  // 4 MiB of 8-byte slots

// walk: chunk order swizzled so that XCD x walks partitions [64x, 64x + 64) in order.
// KEYS: 0 no key loads (windows only), 1 one 8-byte key per lane and row (the walk's form),
// 2 two keys per 16-byte load (half the key load instructions, same lines)
template <int KEYS>
__global__ __launch_bounds__(256) void walk_emu(const int64_t *keys, const u32x4 *table, uint64_t n_chunks,
                                                uint32_t *sink) {
  const uint64_t per = n_chunks / 8;
  const uint64_t c = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  if (c >= n_chunks) return;
  const uint32_t part = (uint32_t)(c * kParts / n_chunks);
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t acc = 0;
  int64_t kk[8];
  if (KEYS == 2) {  // lane L loads rows 2L, 2L + 1 of each 512-row half: kk[j] for row j * 256 + tid
    typedef long long i64x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const i64x2 v = __builtin_nontemporal_load(reinterpret_cast<const i64x2 *>(keys + c * kChunk + h * 512) + threadIdx.x);
      kk[2 * h] = v.x;
      kk[2 * h + 1] = v.y;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {  // 8 rows per thread, one window per row (lane pairs)
    const uint64_t row = c * kChunk + (uint32_t)j * 256 + threadIdx.x;
    const int64_t k = KEYS == 1 ? __builtin_nontemporal_load(keys + row) : KEYS == 2 ? kk[j] : (int64_t)row;
    // a random 32-byte window of the partition's slice (the row index mixed in: the key column
    // is constant here, its load only carries the walk's 8 bytes of key traffic)
    const uint32_t w = mix32((uint32_t)row * 0x9E3779B9u ^ (uint32_t)k) & (kWinSlots / 4 - 1);
    // lanes 2q, 2q + 1 load the two 16-byte halves of lane 2q's window, then of lane 2q + 1's
    const uint32_t w0 = (uint32_t)__shfl((int)w, (int)(lane & ~1u)), w1 = (uint32_t)__shfl((int)w, (int)(lane | 1u));
    const u32x4 v0 = table[((uint64_t)part * kWinSlots / 4 + w0) * 2 + (lane & 1u)];
    const u32x4 v1 = table[((uint64_t)part * kWinSlots / 4 + w1) * 2 + (lane & 1u)];
    acc += v0.x ^ v1.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(1024) void split_emu(const int64_t *src, int64_t *out_k, uint32_t *out_r, uint32_t *cur,
                                                  uint64_t n_tiles, uint64_t cap) {
  constexpr uint32_t L = 22, P = 512, T = 1024;
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
      out_k[dest] = __builtin_nontemporal_load(src + t * tile + q);
      out_r[dest] = q;
    }
    __syncthreads();
  }
}

__global__ void init_cur(uint32_t *cur) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 512 * 8) cur[i] = 1u + (i * 7u) % 15u;
}

int main(int argc, char **argv) {
  const uint64_t n = 1ull << 30;
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned split_wgs = argc > 1 ? (unsigned)atoi(argv[1]) / 8 * 8 : (unsigned)cus / 8 * 8;
  int64_t *keys, *src, *ok;
  u32x4 *table;
  uint32_t *orr, *cur, *sink;
  const uint64_t tile = 22 * 512, n_tiles = (n + tile - 1) / tile;
  const uint64_t cap = (uint64_t)((double)n / 4096.0 * 1.0625 + 8000 + 256) / 2048 * 2048 + 2048;
  CK(hipMalloc(&keys, n * 8));
  CK(hipMalloc(&src, n_tiles * tile * 8));
  CK(hipMalloc(&table, (size_t)kParts * kWinSlots * 8));
  CK(hipMalloc(&ok, (4096 * cap + 64) * 8));
  CK(hipMalloc(&orr, (4096 * cap + 64) * 4));
  CK(hipMalloc(&cur, 4096 * 4));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(keys, 7, n * 8));
  CK(hipMemset(src, 3, n_tiles * tile * 8));
  CK(hipMemset(table, 1, (size_t)kParts * kWinSlots * 8));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  const uint64_t n_chunks = n / kChunk;
  int kmode = 1;
  auto walk = [&](hipStream_t s) {
    if (kmode == 0) hipLaunchKernelGGL(walk_emu<0>, dim3((unsigned)n_chunks), dim3(256), 0, s, keys, table, n_chunks, sink);
    if (kmode == 1) hipLaunchKernelGGL(walk_emu<1>, dim3((unsigned)n_chunks), dim3(256), 0, s, keys, table, n_chunks, sink);
    if (kmode == 2) hipLaunchKernelGGL(walk_emu<2>, dim3((unsigned)n_chunks), dim3(256), 0, s, keys, table, n_chunks, sink);
  };
  auto split = [&](hipStream_t s) {
    hipLaunchKernelGGL(init_cur, dim3(16), dim3(256), 0, s, cur);
    hipLaunchKernelGGL(split_emu, dim3(split_wgs), dim3(1024), 0, s, src, ok, orr, cur, n_tiles, cap);
  };
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timed = [&](int mode) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a, 0));
      CK(hipStreamWaitEvent(s0, a, 0));
      CK(hipStreamWaitEvent(s1, a, 0));
      if (mode & 1) split(s1);
      if (mode & 2) walk(s0);
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, s0));
      CK(hipEventRecord(e1, s1));
      CK(hipStreamWaitEvent(0, e0, 0));
      CK(hipStreamWaitEvent(0, e1, 0));
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep) best = ms < best ? ms : best;
    }
    return best;
  };
  if (argc > 2) {  // overlap_emu WGS keys: the walk alone with each key-load form
    for (kmode = 0; kmode < 3; ++kmode)
      printf("walk alone, keys %s: %.3f ms\n", kmode == 0 ? "none" : kmode == 1 ? "8-byte loads" : "16-byte loads",
             timed(2));
    return 0;
  }
  const float ts = timed(1), tw = timed(2), tb = timed(3);
  printf("split_wgs %u  split alone %.3f ms  walk alone %.3f ms  both %.3f ms  (sum %.3f, max %.3f)\n", split_wgs, ts,
         tw, tb, ts + tw, ts > tw ? ts : tw);
  return 0;
}
