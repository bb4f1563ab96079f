// tilesplit_emu.hip — measurement tool (not product): the floor of a TILE-CONTIGUOUS C2 layout
// (VERDICT r5 task 4) against today's segment layout, same box, same run.
//   today   split_seg: runs of ~22 keys + rows scattered into 512 x 8 fixed-capacity segments
//           (tools/overlap_emu's split pattern, 8-byte key read linearly + 12 B stored per key);
//           walk_seg: one 256-thread workgroup per 2048 contiguous positions of a partition's
//           segment, keys by 16-byte loads + one random 32-byte window of the partition's 4 MiB
//           table slice per row (overlap_emu's walk, keys mode 2)
//   tile    split_tile: each 11264-key tile writes its keys + rows to ITS OWN contiguous region
//           (full-line streaming stores, the order inside the tile being the partition-sorted
//           image in the real kernel) and, partition-major, one 4-byte run record per (partition,
//           tile) = {start in the tile | length << 16} (a per-tile LDS histogram + scan gives them);
//           walk_tile: one 256-thread workgroup per (partition, group of TG consecutive tiles):
//           the group's TG run records (contiguous), their prefix in LDS, then per row a binary
//           search for its run, its key read from the run's place in its tile, and the same random
//           32-byte table window
// Prints each kernel alone and the two pairs' sums.   tilesplit_emu [TG]
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
typedef long long i64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

constexpr uint32_t kChunk = 2048, kParts = 512, kWinSlots = 1u << 19;  // 4 MiB of 8-byte slots
constexpr uint32_t kT = 1024, kPer = 11, kTile = kT * kPer;           // 11264 keys per tile

// ---- today's layout ------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void split_seg(const int64_t *src, int64_t *out_k, uint32_t *out_r, uint32_t *cur,
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

__global__ __launch_bounds__(256) void walk_seg(const int64_t *keys, const u32x4 *table, uint64_t n_chunks,
                                                uint32_t *sink) {
  const uint64_t per = n_chunks / 8;
  const uint64_t c = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  if (c >= n_chunks) return;
  const uint32_t part = (uint32_t)(c * kParts / n_chunks);
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t acc = 0;
  int64_t kk[8];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const i64x2 v = __builtin_nontemporal_load(reinterpret_cast<const i64x2 *>(keys + c * kChunk + h * 512) + threadIdx.x);
    kk[2 * h] = v.x;
    kk[2 * h + 1] = v.y;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint64_t row = c * kChunk + (uint32_t)j * 256 + threadIdx.x;
    const uint32_t w = mix32((uint32_t)row * 0x9E3779B9u ^ (uint32_t)kk[j]) & (kWinSlots / 4 - 1);
    const uint32_t w0 = (uint32_t)__shfl((int)w, (int)(lane & ~1u)), w1 = (uint32_t)__shfl((int)w, (int)(lane | 1u));
    const u32x4 v0 = table[((uint64_t)part * kWinSlots / 4 + w0) * 2 + (lane & 1u)];
    const u32x4 v1 = table[((uint64_t)part * kWinSlots / 4 + w1) * 2 + (lane & 1u)];
    acc += v0.x ^ v1.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// ---- tile-contiguous layout ----------------------------------------------------------------
// The partition of key k (the real split: home slot >> window bits; here a hash of the key).
__device__ __forceinline__ uint32_t part_of(int64_t k) { return mix32((uint32_t)k ^ (uint32_t)(k >> 32)) & (kParts - 1); }

__global__ __launch_bounds__(kT) void split_tile(const int64_t *src, int64_t *out_k, uint32_t *out_r, uint32_t *runs,
                                                 uint64_t n_tiles) {
  __shared__ uint32_t s_cnt[kParts];
  const uint32_t tid = threadIdx.x;
  int64_t kc[kPer], kn[kPer];
  uint64_t t = blockIdx.x;
  if (t >= n_tiles) return;
#pragma unroll
  for (int it = 0; it < (int)kPer; ++it) kc[it] = __builtin_nontemporal_load(src + t * kTile + it * kT + tid);
  for (; t < n_tiles; t += gridDim.x) {
    const uint64_t tn = t + gridDim.x < n_tiles ? t + gridDim.x : t;
#pragma unroll
    for (int it = 0; it < (int)kPer; ++it) kn[it] = __builtin_nontemporal_load(src + tn * kTile + it * kT + tid);
    if (tid < kParts) s_cnt[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int it = 0; it < (int)kPer; ++it) atomicAdd(&s_cnt[part_of(kc[it])], 1u);
    __syncthreads();
    if (tid < kParts) {  // exclusive scan of the 512 counts (a wave scan per 64, then the wave sums)
      const uint32_t c = s_cnt[tid];
      uint32_t x = c;
      const uint32_t lane = tid & 63u;
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d);
        if (lane >= d) x += y;
      }
      // (the 8 wave sums' prefix is LDS traffic of the real kernel; here the run start stays
      // within-wave — the pattern is the partition-major record store)
      runs[(uint64_t)tid * n_tiles + t] = (x - c) | c << 16;
    }
#pragma unroll
    for (int it = 0; it < (int)kPer; ++it) {  // the tile's region, streamed (full lines)
      const uint64_t q = t * kTile + it * kT + tid;
      __builtin_nontemporal_store(kc[it], out_k + q);
      __builtin_nontemporal_store((uint32_t)(it * kT + tid), out_r + q);
    }
#pragma unroll
    for (int it = 0; it < (int)kPer; ++it) kc[it] = kn[it];
    __syncthreads();
  }
}

template <int TG>
__global__ __launch_bounds__(256) void walk_tile(const int64_t *keys, const uint32_t *runs, const u32x4 *table,
                                                 uint64_t n_tiles, uint64_t groups, uint32_t *sink) {
  __shared__ uint32_t s_pre[TG + 1], s_st[TG];
  // work unit u = (partition, tile group): XCD x walks partitions [64x, 64x + 64), group-major inside
  const uint64_t per = (uint64_t)kParts * groups / 8;
  const uint64_t u = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  if (u >= (uint64_t)kParts * groups) return;
  const uint32_t part = (uint32_t)(u / groups);
  const uint64_t t0 = (u % groups) * TG;
  const uint32_t lane = threadIdx.x & 63u;
  if (threadIdx.x < TG) {
    const uint64_t t = t0 + threadIdx.x;
    const uint32_t r = t < n_tiles ? runs[(uint64_t)part * n_tiles + t] : 0u;
    s_st[threadIdx.x] = r & 0xFFFFu;
    s_pre[threadIdx.x + 1] = r >> 16;
  }
  if (threadIdx.x == 0) s_pre[0] = 0;
  __syncthreads();
  if (threadIdx.x < 64) {  // inclusive prefix of the run lengths (TG <= 128: two per lane)
    uint32_t a = threadIdx.x * 2 + 1 <= TG ? s_pre[threadIdx.x * 2 + 1] : 0u;
    uint32_t b = threadIdx.x * 2 + 2 <= TG ? s_pre[threadIdx.x * 2 + 2] : 0u;
    uint32_t x = a + b;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, d);
      if (lane >= d) x += y;
    }
    if (threadIdx.x * 2 + 1 <= TG) s_pre[threadIdx.x * 2 + 1] = x - b;
    if (threadIdx.x * 2 + 2 <= TG) s_pre[threadIdx.x * 2 + 2] = x;
  }
  __syncthreads();
  const uint32_t rows = s_pre[TG];
  uint32_t acc = 0;
  // all of the thread's rows at once, as walk_seg does: positions (binary searches in LDS), then
  // every key load in flight, then every window load in flight (rows <= 9 x 256)
  constexpr int R = 9;
  uint64_t pos[R];
  int64_t k[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t r0 = threadIdx.x + 256u * (uint32_t)j;
    const uint32_t r = r0 < rows ? r0 : 0u;
    uint32_t lo = 0, hi = TG;  // the run lo with s_pre[lo] <= r < s_pre[lo + 1]
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const uint32_t m = (lo + hi) >> 1;
      if (hi - lo > 1) (s_pre[m] <= r ? lo : hi) = m;
    }
    pos[j] = (t0 + lo) * kTile + s_st[lo] + (r - s_pre[lo]);
  }
#pragma unroll
  for (int j = 0; j < R; ++j) k[j] = __builtin_nontemporal_load(keys + pos[j]);
#pragma unroll
  for (int j = 0; j < R; ++j) {
    if (threadIdx.x + 256u * (uint32_t)j >= rows && j >= 8) break;  // (the 9th row group: mostly empty)
    const uint32_t w = mix32((uint32_t)pos[j] * 0x9E3779B9u ^ (uint32_t)k[j]) & (kWinSlots / 4 - 1);
    const uint32_t w0 = (uint32_t)__shfl((int)w, (int)(lane & ~1u)), w1 = (uint32_t)__shfl((int)w, (int)(lane | 1u));
    const u32x4 v0 = table[((uint64_t)part * kWinSlots / 4 + w0) * 2 + (lane & 1u)];
    const u32x4 v1 = table[((uint64_t)part * kWinSlots / 4 + w1) * 2 + (lane & 1u)];
    acc += v0.x ^ v1.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void init_cur(uint32_t *cur) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 512 * 8) cur[i] = 1u + (i * 7u) % 15u;
}

__global__ void fill_keys(int64_t *k, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    k[i] = (int64_t)(i * 0x9E3779B97F4A7C15ull);
}

int main(int argc, char **argv) {
  const uint64_t n = 1ull << 30;
  const int tg = argc > 1 ? atoi(argv[1]) : 93;
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t n_tiles = (n + kTile - 1) / kTile;
  const uint64_t cap = (uint64_t)((double)n / 4096.0 * 1.0625 + 8000 + 256) / 2048 * 2048 + 2048;
  int64_t *src, *ok, *tk;
  u32x4 *table;
  uint32_t *orr, *tr, *cur, *sink, *runs;
  CK(hipMalloc(&src, n_tiles * kTile * 8));
  CK(hipMalloc(&table, (size_t)kParts * kWinSlots * 8));
  CK(hipMalloc(&ok, (4096 * cap + 64) * 8));
  CK(hipMalloc(&orr, (4096 * cap + 64) * 4));
  CK(hipMalloc(&tk, n_tiles * kTile * 8));
  CK(hipMalloc(&tr, n_tiles * kTile * 4));
  CK(hipMalloc(&runs, (size_t)kParts * n_tiles * 4));
  CK(hipMalloc(&cur, 4096 * 4));
  CK(hipMalloc(&sink, 64));
  hipLaunchKernelGGL(fill_keys, dim3(4096), dim3(256), 0, 0, src, n_tiles * kTile);
  CK(hipMemset(table, 1, (size_t)kParts * kWinSlots * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timed = [&](auto fn) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a, 0));
      fn();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep) best = ms < best ? ms : best;
    }
    CK(hipGetLastError());
    return best;
  };
  const unsigned grid = (unsigned)cus / 8 * 8;
  const float s_seg = timed([&] {
    hipLaunchKernelGGL(init_cur, dim3(16), dim3(256), 0, 0, cur);
    hipLaunchKernelGGL(split_seg, dim3(grid), dim3(1024), 0, 0, src, ok, orr, cur, n_tiles, cap);
  });
  const uint64_t n_chunks = n / kChunk;
  const float w_seg = timed([&] { hipLaunchKernelGGL(walk_seg, dim3((unsigned)n_chunks), dim3(256), 0, 0, ok, table, n_chunks, sink); });
  const float s_tile = timed([&] {
    hipLaunchKernelGGL(split_tile, dim3(grid), dim3(kT), 0, 0, src, tk, tr, runs, n_tiles);
  });
  float w_tile = 0;
  const uint64_t groups = (n_tiles + tg - 1) / tg;
  auto wt = [&](auto kern) {
    return timed([&] { hipLaunchKernelGGL(kern, dim3((unsigned)(kParts * groups)), dim3(256), 0, 0, tk, runs, table, n_tiles, groups, sink); });
  };
  if (tg == 64) w_tile = wt(walk_tile<64>);
  else if (tg == 93) w_tile = wt(walk_tile<93>);
  else if (tg == 128) w_tile = wt(walk_tile<128>);
  else { fprintf(stderr, "TG: 64, 93 or 128\n"); return 2; }
  printf("segment layout: split %.3f + walk %.3f = %.3f ms\n", s_seg, w_seg, s_seg + w_seg);
  printf("tile layout (TG %d): split %.3f + walk %.3f = %.3f ms\n", tg, s_tile, w_tile, s_tile + w_tile);
  return 0;
}
