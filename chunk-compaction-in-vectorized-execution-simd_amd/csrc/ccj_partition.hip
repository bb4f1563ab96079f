// ccj_partition.hip — owner partitioning of a probe (or build) key column for the multi-GPU join
// (SURVEY §8e): owner(k) = murmurhash64(k) >> (64 - log2 P), the TOP hash bits, disjoint from the
// low bits every GPU's local table uses for its slot/bucket, so shard tables stay evenly loaded.
//
// Stable multisplit in two passes: (1) per-tile destination counts, written destination-major;
// (2) after an exclusive scan of those counts, every tile re-reads its keys and scatters them in
// row order (ballot + mbcnt ranks inside a wave, LDS-scanned across the tile's waves), so each
// destination segment keeps the source row order: deterministic send buffers.
#include <hipcub/hipcub.hpp>

#include "ccj_internal.h"

namespace ccj {
namespace {

constexpr int kTileThreads = 256;
constexpr int kTileIters = 32;
constexpr uint64_t kTile = (uint64_t)kTileThreads * kTileIters;  // 8192 keys per tile

__device__ __forceinline__ uint32_t owner_of(int64_t k, uint32_t shift) {
  return shift >= 64 ? 0u : (uint32_t)(murmurhash64((uint64_t)k) >> shift);
}

__global__ __launch_bounds__(kTileThreads) void part_count(const int64_t *keys, uint64_t n, uint32_t parts,
                                                           uint32_t shift, uint64_t n_tiles, uint64_t *cnt) {
  __shared__ uint32_t s_cnt[kMaxParts];
  const uint64_t tile = blockIdx.x;
  if (threadIdx.x < kMaxParts) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  for (int it = 0; it < kTileIters; ++it) {
    const uint64_t i = tile * kTile + (uint64_t)it * kTileThreads + threadIdx.x;
    if (i < n) atomicAdd(&s_cnt[owner_of(keys[i], shift)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < parts) cnt[(uint64_t)threadIdx.x * n_tiles + tile] = s_cnt[threadIdx.x];
}

__global__ __launch_bounds__(kTileThreads) void part_scatter(const int64_t *keys, uint64_t n, uint32_t parts,
                                                             uint32_t shift, uint64_t n_tiles, const uint64_t *off,
                                                             uint64_t row_base, int64_t *out_keys,
                                                             uint64_t *out_rows) {
  __shared__ uint64_t s_base[kMaxParts];
  __shared__ uint32_t s_wave[kTileThreads / 64][kMaxParts];
  const uint64_t tile = blockIdx.x;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  if (threadIdx.x < parts) s_base[threadIdx.x] = off[(uint64_t)threadIdx.x * n_tiles + tile];
  __syncthreads();
  for (int it = 0; it < kTileIters; ++it) {
    const uint64_t i = tile * kTile + (uint64_t)it * kTileThreads + threadIdx.x;
    const bool valid = i < n;
    const int64_t k = valid ? keys[i] : 0;
    const uint32_t d = valid ? owner_of(k, shift) : 0xFFFFFFFFu;
    uint32_t rank = 0;
    for (uint32_t p = 0; p < parts; ++p) {
      const uint64_t m = __ballot(d == p);
      if (d == p) rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (lane == 0) s_wave[wave][p] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (valid) {
      uint64_t pos = s_base[d] + rank;
      for (uint32_t w = 0; w < wave; ++w) pos += s_wave[w][d];
      out_keys[pos] = k;
      out_rows[pos] = row_base + i;
    }
    __syncthreads();
    if (threadIdx.x < parts) {
      uint32_t t = 0;
      for (uint32_t w = 0; w < kTileThreads / 64; ++w) t += s_wave[w][threadIdx.x];
      s_base[threadIdx.x] += t;
    }
    __syncthreads();
  }
}

__global__ void part_totals(const uint64_t *cnt, const uint64_t *off, uint32_t parts, uint64_t n_tiles,
                            uint64_t *out_counts) {
  const uint32_t p = threadIdx.x;
  if (p < parts) {
    const uint64_t last = (uint64_t)p * n_tiles + n_tiles - 1;
    const uint64_t first = (uint64_t)p * n_tiles;
    out_counts[p] = off[last] + cnt[last] - off[first];
  }
}

size_t scan_bytes(uint64_t n) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint64_t *)nullptr, (uint64_t *)nullptr, (int)n);
  return (b + 255) & ~(size_t)255;
}

}  // namespace

size_t partition_workspace(uint64_t n, uint32_t parts) {
  const uint64_t n_tiles = (n + kTile - 1) / kTile;
  const uint64_t m = n_tiles * parts;
  return 2 * ((m * 8 + 255) & ~255ull) + scan_bytes(m ? m : 1);
}

hipError_t launch_partition(const int64_t *keys, uint64_t n, uint32_t parts, uint64_t row_base, int64_t *out_keys,
                            uint64_t *out_rows, uint64_t *out_counts, void *ws, hipStream_t s) {
  uint32_t log2p = 0;
  while ((1u << log2p) < parts) ++log2p;
  const uint32_t shift = 64 - log2p;  // 64 -> every key to part 0
  const uint64_t n_tiles = (n + kTile - 1) / kTile;
  const uint64_t m = n_tiles * parts;
  if (n == 0) return hipMemsetAsync(out_counts, 0, parts * 8, s);
  char *w = (char *)ws;
  uint64_t *cnt = (uint64_t *)w;
  w += (m * 8 + 255) & ~255ull;
  uint64_t *off = (uint64_t *)w;
  w += (m * 8 + 255) & ~255ull;
  size_t tb = scan_bytes(m);
  hipLaunchKernelGGL(part_count, dim3((unsigned)n_tiles), dim3(kTileThreads), 0, s, keys, n, parts, shift, n_tiles, cnt);
  hipError_t e = hipGetLastError();
  if (e) return e;
  e = hipcub::DeviceScan::ExclusiveSum(w, tb, cnt, off, (int)m, s);
  if (e) return e;
  hipLaunchKernelGGL(part_scatter, dim3((unsigned)n_tiles), dim3(kTileThreads), 0, s, keys, n, parts, shift, n_tiles,
                     off, row_base, out_keys, out_rows);
  hipLaunchKernelGGL(part_totals, dim3(1), dim3(64), 0, s, cnt, off, parts, n_tiles, out_counts);
  return hipGetLastError();
}

}  // namespace ccj
