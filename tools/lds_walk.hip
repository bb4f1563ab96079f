// tools/lds_walk.hip — prototype of the north star's "LDS-staged bucket windows" for the C2 linear
// probe: how fast is the walk once every row's table window sits in LDS?
//
// Setup (untimed): the C2 table (2^26 keys 0..2^26-1 inserted by atomicCAS linear probing into
// 2^28 slots, murmurhash64 home slots), 2^30 SplitMix64(42) probe keys % 2^26, then the probe column
// sorted by home slot (hipcub radix sort) — i.e. the input a perfect split into 2^(28-WBITS)
// windows of 2^WBITS slots would produce, at no cost to this measurement.
// Timed: one workgroup (1024 threads) per window: the window (+ a 64-slot halo for runs that cross
// its end) is loaded into LDS with 16-byte loads, then the workgroup streams the window's rows
// (8-byte keys, coalesced), walks each run in LDS and writes (u32 position, i64 payload) per match
// at the row's position (every C2 row matches exactly once; runs that leave the halo continue in
// the global table).  Matches are counted and checked against 2^30.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I chunk-compaction-in-vectorized-execution-simd_amd/csrc \
//          -o tools/lds_walk tools/lds_walk.hip
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstdlib>

#include "ccj_internal.h"

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);     \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

using ccj::murmurhash64;

__device__ __forceinline__ uint64_t splitmix_at(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__global__ void fill(int64_t *p, uint64_t n, int64_t v) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[i] = v;
}

__global__ void build(int64_t *slots, uint64_t n_build, uint32_t mask) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_build; i += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t k = (int64_t)i;
    uint32_t s = (uint32_t)murmurhash64((uint64_t)k) & mask;
    while (true) {
      const unsigned long long old = atomicCAS((unsigned long long *)&slots[s], ~0ull, (unsigned long long)k);
      if (old == ~0ull) break;
      s = (s + 1) & mask;
    }
  }
}

__global__ void gen(int64_t *keys, uint32_t *home, uint64_t n, uint64_t range, uint32_t mask) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t k = (int64_t)(splitmix_at(42, i) % range);
    keys[i] = k;
    home[i] = (uint32_t)murmurhash64((uint64_t)k) & mask;
  }
}

__global__ void win_count(const uint32_t *home, uint64_t n, uint32_t wbits, uint32_t *cnt) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[home[i] >> wbits], 1u);
}

constexpr int kThreads = 1024;
constexpr uint32_t kHalo = 64;

template <uint32_t WBITS>
__global__ __launch_bounds__(kThreads) void lds_walk(const int64_t *table, uint32_t mask, const int64_t *keys,
                                                     const uint64_t *start, uint32_t *out_sel, int64_t *out_pay,
                                                     unsigned long long *matches) {
  constexpr uint32_t W = 1u << WBITS;
  __shared__ int64_t win[W + kHalo];
  const uint32_t w = blockIdx.x, tid = threadIdx.x;
  const uint32_t s0 = w << WBITS;
  for (uint32_t q = tid; q < (W + kHalo) / 2; q += kThreads) {
    const uint32_t s = (s0 + 2 * q) & mask;
    const longlong2 v = *reinterpret_cast<const longlong2 *>(table + s);
    win[2 * q] = v.x;
    win[2 * q + 1] = v.y;
  }
  __syncthreads();
  const uint64_t r0 = start[w], r1 = start[w + 1];
  uint32_t m = 0;
  for (uint64_t r = r0 + tid; r < r1; r += kThreads) {
    const int64_t k = __builtin_nontemporal_load(keys + r);
    uint32_t s = ((uint32_t)murmurhash64((uint64_t)k) & mask) - s0;
    int64_t hit = 0;
    uint32_t n = 0;
    for (;; ++s) {
      const int64_t v = s < W + kHalo ? win[s] : table[(s0 + s) & mask];
      if (v == -1) break;
      if (v == k) {
        hit = v;
        ++n;
      }
    }
    if (n) {
      __builtin_nontemporal_store((uint32_t)r, out_sel + r);
      __builtin_nontemporal_store(hit, out_pay + r);
    }
    m += n;
  }
  for (int d = 32; d > 0; d >>= 1) m += (uint32_t)__shfl_xor((int)m, d);
  if ((tid & 63) == 0 && m) atomicAdd(matches, (unsigned long long)m);
}

template <uint32_t WBITS>
static void run(const int64_t *table, uint32_t mask, const int64_t *keys, const uint32_t *home, uint64_t n,
                uint32_t *sel, int64_t *pay, unsigned long long *d_m) {
  const uint32_t n_win = (mask + 1) >> WBITS;
  uint32_t *cnt;
  uint64_t *start;
  CK(hipMalloc(&cnt, (n_win + 1) * 4ull));
  CK(hipMalloc(&start, (n_win + 1) * 8ull));
  CK(hipMemset(cnt, 0, (n_win + 1) * 4ull));
  win_count<<<4096, 256>>>(home, n, WBITS, cnt);
  uint64_t *h = (uint64_t *)malloc((n_win + 1) * 8ull);
  uint32_t *c = (uint32_t *)malloc(n_win * 4ull);
  CK(hipMemcpy(c, cnt, n_win * 4ull, hipMemcpyDeviceToHost));
  h[0] = 0;
  for (uint32_t i = 0; i < n_win; ++i) h[i + 1] = h[i] + c[i];
  CK(hipMemcpy(start, h, (n_win + 1) * 8ull, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e9f, sum = 0.f;
  const int reps = 6;
  unsigned long long m = 0;
  for (int it = 0; it < reps + 1; ++it) {
    CK(hipMemset(d_m, 0, 8));
    CK(hipEventRecord(a));
    lds_walk<WBITS><<<n_win, kThreads>>>(table, mask, keys, start, sel, pay, d_m);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (it) {
      best = ms < best ? ms : best;
      sum += ms;
    }
    CK(hipMemcpy(&m, d_m, 8, hipMemcpyDeviceToHost));
  }
  printf("{\"wbits\": %u, \"windows\": %u, \"window_kib\": %u, \"lds_walk_ms_min\": %.3f, \"lds_walk_ms_avg\": %.3f, "
         "\"matches\": %llu, \"matches_ok\": %s}\n",
         WBITS, n_win, (8u << WBITS) / 1024u, best, sum / reps, m, m == n ? "true" : "false");
  fflush(stdout);
  free(h);
  free(c);
  CK(hipFree(cnt));
  CK(hipFree(start));
}

int main() {
  const uint64_t n_build = 1ull << 26, n = 1ull << 30;
  const uint32_t mask = (1u << 28) - 1;
  int64_t *table, *keys, *keys2, *pay;
  uint32_t *home, *home2, *sel;
  unsigned long long *d_m;
  CK(hipMalloc(&table, (mask + 1ull) * 8));
  CK(hipMalloc(&keys, n * 8));
  CK(hipMalloc(&keys2, n * 8));
  CK(hipMalloc(&home, n * 4));
  CK(hipMalloc(&home2, n * 4));
  CK(hipMalloc(&d_m, 8));
  fill<<<4096, 256>>>(table, mask + 1ull, -1);
  build<<<4096, 256>>>(table, n_build, mask);
  gen<<<4096, 256>>>(keys, home, n, n_build, mask);
  size_t tmp_bytes = 0;
  CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, home, home2, keys, keys2, n, 0, 28));
  void *tmp;
  CK(hipMalloc(&tmp, tmp_bytes));
  CK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, home, home2, keys, keys2, n, 0, 28));
  CK(hipDeviceSynchronize());
  CK(hipFree(tmp));
  CK(hipFree(keys));
  CK(hipFree(home));
  CK(hipMalloc(&sel, n * 4));
  CK(hipMalloc(&pay, n * 8));
  printf("[setup] table built, 2^30 probe keys sorted by home slot\n");
  fflush(stdout);
  run<14>(table, mask, keys2, home2, n, sel, pay, d_m);  // 128 KiB windows: the largest that fits LDS
  run<13>(table, mask, keys2, home2, n, sel, pay, d_m);  // 64 KiB
  return 0;
}
