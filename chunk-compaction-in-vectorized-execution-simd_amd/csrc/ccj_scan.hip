// ccj_scan.hip — exclusive prefix sums of u64 / u32 arrays on the device (the compactor's per-chunk
// row and pass-through counts, compactor.cpp:5-41's running `tmp` offsets made parallel; the
// pipeline's level sizes; the exact multisplit's per-(digit, tile) counts; the chaining build's
// bucket offsets, chaining_ht.cpp:25-36).  Hand-written in place of a library
// scan: tiles of 2048 values per 256-thread workgroup (8 consecutive values per thread, a wave scan
// by shuffles, one LDS word per wave), a reduce pass writing each tile's sum, the tile sums
// scanned by the same routine one level up (recursively, until one workgroup holds them all), then
// an apply pass adding each tile's offset.  No spin-waits on other workgroups (every dependency is a
// kernel boundary), so nothing relies on cross-XCD visibility inside a launch.
#include <hip/hip_runtime.h>

#include "ccj_internal.h"

namespace ccj {
namespace {

constexpr uint32_t kScanThreads = 256, kScanItems = 8, kScanTile = kScanThreads * kScanItems;
constexpr uint32_t kScanWaves = kScanThreads / 64;

__device__ __forceinline__ uint64_t wave_incl_u64(uint64_t x, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t t = __shfl_up(x, d);
    if (lane >= d) x += t;
  }
  return x;
}

// exclusive prefix of v over the workgroup's threads; total = the sum of all v
__device__ __forceinline__ uint64_t block_excl(uint64_t v, uint64_t *s_w, uint64_t &total) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint64_t incl = wave_incl_u64(v, lane);
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  uint64_t pre = 0;
  total = 0;
#pragma unroll
  for (uint32_t w = 0; w < kScanWaves; ++w) {
    const uint64_t x = s_w[w];
    pre += w < wave ? x : 0u;
    total += x;
  }
  return pre + incl - v;
}

// tile b's sum -> bsum[b]
template <typename T>
__global__ __launch_bounds__(kScanThreads) void scan_reduce(const T *in, uint64_t n, T *bsum) {
  __shared__ uint64_t s_w[kScanWaves];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  uint64_t v = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {  // coalesced: value base + k * 256 + tid
    const uint64_t i = base + k * kScanThreads + threadIdx.x;
    v += i < n ? in[i] : 0u;
  }
  uint64_t total;
  (void)block_excl(v, s_w, total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = (T)total;
}

// out[i] = bpre[tile] + the exclusive prefix of in inside its tile (bpre null: one tile, offset 0);
// *total (optional) = the sum of the whole array (written by the one-tile launch only).  in may be
// out: every thread reads its values before any is written.
template <typename T>
__global__ __launch_bounds__(kScanThreads) void scan_apply(const T *in, T *out, uint64_t n, const T *bpre,
                                                           T *total_out) {
  __shared__ uint64_t s_w[kScanWaves];
  const uint64_t i0 = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  uint64_t v[kScanItems], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {
    v[k] = i0 + k < n ? in[i0 + k] : 0u;
    sum += v[k];
  }
  uint64_t total;
  uint64_t run = block_excl(sum, s_w, total) + (bpre ? bpre[blockIdx.x] : 0u);
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {
    if (i0 + k < n) out[i0 + k] = (T)run;
    run += v[k];
  }
  if (total_out && threadIdx.x == 0) *total_out = (T)total;
}

uint64_t tiles_of(uint64_t n) { return (n + kScanTile - 1) / kScanTile; }

}  // namespace

namespace {
template <typename T>
hipError_t scan_exclusive(const T *in, T *out, uint64_t n, T *total, void *tmp, hipStream_t s) {
  if (n == 0) return total ? hipMemsetAsync(total, 0, sizeof(T), s) : hipSuccess;
  if (n <= kScanTile) {
    hipLaunchKernelGGL(scan_apply<T>, dim3(1), dim3(kScanThreads), 0, s, in, out, n, (const T *)nullptr, total);
    return hipGetLastError();
  }
  const uint64_t nb = tiles_of(n);
  T *bsum = (T *)tmp;
  hipLaunchKernelGGL(scan_reduce<T>, dim3((unsigned)nb), dim3(kScanThreads), 0, s, in, n, bsum);
  hipError_t e = hipGetLastError();
  if (e) return e;
  // the tile sums, scanned in place one level up (its temp space follows this level's)
  e = scan_exclusive<T>(bsum, bsum, nb, total, (char *)tmp + ((nb * 8 + 255) & ~(size_t)255), s);
  if (e) return e;
  hipLaunchKernelGGL(scan_apply<T>, dim3((unsigned)nb), dim3(kScanThreads), 0, s, in, out, n, (const T *)bsum,
                     (T *)nullptr);
  return hipGetLastError();
}
}  // namespace

size_t scan_u64_temp_bytes(uint64_t n) {
  size_t b = 0;
  for (uint64_t m = n; m > kScanTile; m = tiles_of(m)) b += (tiles_of(m) * 8 + 255) & ~(size_t)255;
  return b ? b : 256;
}

hipError_t scan_exclusive_u64(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *total, void *tmp,
                              hipStream_t s) {
  return scan_exclusive<uint64_t>(in, out, n, total, tmp, s);
}

hipError_t scan_exclusive_u32(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *total, void *tmp,
                              hipStream_t s) {
  return scan_exclusive<uint32_t>(in, out, n, total, tmp, s);
}

}  // namespace ccj
