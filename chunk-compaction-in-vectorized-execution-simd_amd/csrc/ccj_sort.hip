// ccj_sort.hip — hand-written stable LSD radix sort for the chaining build.
//
// HashTable::HashTable (chaining_ht.cpp:29-35) appends tuple t to the END of bucket h(k_t)'s
// std::list, so a chain lists its keys in generator order: the CSR form is a STABLE sort of the
// tuples by bucket.  Each pass sorts by one 8-bit digit, keeping the order of the previous pass
// among equal digits:
//   1. sort_digits_hist: per 4096-key tile, a histogram of the pass's digit (LDS atomics), written
//      digit-major: cnt[d * tiles + tile];
//   2. the hand-written exclusive scan (ccj_scan.hip) of that array: off[d * tiles + tile] is where
//      tile `tile`'s keys of digit d start in the output — digit order first, tile order second;
//   3. sort_digits_scatter: each wave ranks its 1024 consecutive keys by digit in order (wave64
//      ballots on the 8 digit bits: the lanes of equal digit and their order in one step, a running
//      per-wave digit count in LDS across the 16 steps); the tile's keys are then placed in LDS in
//      (digit, wave, step, lane) order = (digit, input position) order and written out in runs that
//      continue at off[d * tiles + tile] — so equal digits keep input order inside a tile (the ranks)
//      and across tiles (the scan's tile order).
// Digits whose bits are equal in every key are skipped (one OR / AND reduction of the keys first):
// the bucket sort of n keys into 2^b buckets takes ceil(b / 8) passes, the max_dup sort of small
// reference keys skips its zero high bytes.  Untimed, like the reference's build (main.cpp:62-68).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <utility>

#include "ccj_internal.h"

namespace ccj {
namespace {

constexpr uint32_t kSortThreads = 256, kSortWaves = kSortThreads / 64;
constexpr uint32_t kSortSteps = 16;                             // 64-key steps per wave
constexpr uint32_t kSortTile = kSortThreads * kSortSteps;       // 4096 keys per workgroup
constexpr uint32_t kDigitBits = 8, kDigits = 1u << kDigitBits;

__device__ __forceinline__ uint32_t digit_of(uint64_t k, uint32_t shift, uint32_t dmask) {
  return (uint32_t)(k >> shift) & dmask;
}

// OR and AND of all keys: bits equal in every key give passes that move nothing.
template <typename K>
__global__ __launch_bounds__(256) void sort_key_bits(const K *keys, uint64_t n, unsigned long long *or_and) {
  uint64_t o = 0, a = ~0ull;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = (uint64_t)keys[i];
    o |= k;
    a &= k;
  }
  for (int d = 32; d > 0; d >>= 1) {
    o |= (uint64_t)__shfl_xor((long long)o, d);
    a &= (uint64_t)__shfl_xor((long long)a, d);
  }
  if ((threadIdx.x & 63u) == 0) {
    atomicOr(or_and, (unsigned long long)o);
    atomicAnd(or_and + 1, (unsigned long long)a);
  }
}

template <typename K>
__global__ __launch_bounds__(kSortThreads) void sort_digits_hist(const K *keys, uint64_t n, uint32_t shift,
                                                                 uint32_t dmask, uint32_t tiles, uint32_t *cnt) {
  __shared__ uint32_t s_h[kDigits];
  s_h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
#pragma unroll 4
  for (uint32_t k = 0; k < kSortSteps; ++k) {
    const uint64_t i = base + k * kSortThreads + threadIdx.x;
    if (i < n) atomicAdd(&s_h[digit_of((uint64_t)keys[i], shift, dmask)], 1u);
  }
  __syncthreads();
  cnt[(uint64_t)threadIdx.x * tiles + blockIdx.x] = s_h[threadIdx.x];
}

template <typename K, bool VALS>
__global__ __launch_bounds__(kSortThreads) void sort_digits_scatter(const K *keys, const uint32_t *vals, uint64_t n,
                                                                    uint32_t shift, uint32_t dmask, uint32_t tiles,
                                                                    const uint32_t *off, K *out_keys,
                                                                    uint32_t *out_vals) {
  __shared__ uint32_t s_wcnt[kSortWaves][kDigits];  // running, then exclusive-over-waves, digit counts
  __shared__ uint32_t s_tpre[kDigits];              // the tile's exclusive prefix over digits
  __shared__ uint32_t s_gpre[kDigits];              // off[d * tiles + tile]
  __shared__ uint32_t s_wsum[kSortWaves];
  __shared__ K s_key[kSortTile];
  __shared__ uint32_t s_val[VALS ? kSortTile : 1];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
  for (uint32_t w = 0; w < kSortWaves; ++w) s_wcnt[w][tid] = 0;
  s_gpre[tid] = off[(uint64_t)tid * tiles + blockIdx.x];
  __syncthreads();

  // wave `wave` owns keys [base + wave * 1024, + 1024): step k covers 64 consecutive keys
  const uint64_t base = (uint64_t)blockIdx.x * kSortTile + (uint64_t)wave * 64u * kSortSteps;
  K key[kSortSteps];
  uint32_t val[VALS ? kSortSteps : 1];
  uint32_t rank[kSortSteps];
  uint32_t *wcnt = s_wcnt[wave];
#pragma unroll
  for (uint32_t k = 0; k < kSortSteps; ++k) {
    const uint64_t i = base + k * 64u + lane;
    const bool live = i < n;
    key[k] = live ? keys[i] : (K)0;
    if (VALS) val[VALS ? k : 0] = live ? vals[i] : 0u;
    const uint32_t d = digit_of((uint64_t)key[k], shift, dmask);
    // lanes of the same digit: AND of the ballots of each digit bit (or its complement)
    uint64_t peers = __ballot(live);
#pragma unroll
    for (uint32_t b = 0; b < kDigitBits; ++b) {
      const uint64_t on = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? on : ~on;
    }
    const uint32_t before = (uint32_t)__popcll(peers & lt);
    const uint32_t c = live ? wcnt[d] : 0u;  // every lane reads before the group's first lane writes
    rank[k] = c + before;
    __builtin_amdgcn_wave_barrier();
    if (live && before == 0) wcnt[d] = c + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();

  // thread tid = digit tid: per-wave exclusive offsets, the tile total, its prefix over digits
  uint32_t tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < kSortWaves; ++w) {
    const uint32_t c = s_wcnt[w][tid];
    s_wcnt[w][tid] = tot;
    tot += c;
  }
  uint32_t incl = tot;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)incl, d);
    if (lane >= d) incl += t;
  }
  if (lane == 63) s_wsum[wave] = incl;
  __syncthreads();
  uint32_t pre = 0;
#pragma unroll
  for (uint32_t w = 0; w < kSortWaves; ++w) pre += w < wave ? s_wsum[w] : 0u;
  s_tpre[tid] = pre + incl - tot;
  __syncthreads();

  // the tile in (digit, input position) order in LDS
  const uint64_t tile0 = (uint64_t)blockIdx.x * kSortTile;
  const uint32_t live_n = (uint32_t)(n - tile0 < kSortTile ? n - tile0 : kSortTile);
#pragma unroll
  for (uint32_t k = 0; k < kSortSteps; ++k) {
    if (base + k * 64u + lane < n) {
      const uint32_t d = digit_of((uint64_t)key[k], shift, dmask);
      const uint32_t p = s_tpre[d] + s_wcnt[wave][d] + rank[k];
      s_key[p] = key[k];
      if (VALS) s_val[p] = val[VALS ? k : 0];
    }
  }
  __syncthreads();
  // out: position p of the tile goes to off[d * tiles + tile] + (p - the tile's first p of digit d)
  for (uint32_t p = tid; p < live_n; p += kSortThreads) {
    const K kk = s_key[p];
    const uint32_t d = digit_of((uint64_t)kk, shift, dmask);
    const uint64_t o = (uint64_t)s_gpre[d] + (p - s_tpre[d]);
    out_keys[o] = kk;
    if (VALS) out_vals[o] = s_val[p];
  }
}

template <typename K, bool VALS>
hipError_t radix_sort(K *keys, K *keys_alt, uint32_t *vals, uint32_t *vals_alt, uint64_t n, uint32_t end_bit,
                      void *tmp, hipStream_t s, bool *in_alt) {
  *in_alt = false;
  if (n < 2 || end_bit == 0) return hipSuccess;
  if (n > 0xFFFFFFFFull) return hipErrorInvalidValue;  // u32 offsets
  const uint64_t tiles = (n + kSortTile - 1) / kSortTile;
  if (tiles > (1u << 22)) return hipErrorInvalidValue;
  char *w = (char *)tmp;
  unsigned long long *or_and = (unsigned long long *)w;
  uint32_t *cnt = (uint32_t *)(w + 256);
  void *scan_tmp = w + 256 + ((kDigits * tiles * 4 + 255) & ~(uint64_t)255);
  unsigned long long got[2];
  // OR starts at 0, AND at all ones (memsets: no host buffer that must outlive the call)
  hipError_t e = hipMemsetAsync(or_and, 0, 8, s);
  if (!e) e = hipMemsetAsync(or_and + 1, 0xFF, 8, s);
  if (e) return e;
  const unsigned grid = (unsigned)std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(sort_key_bits<K>, dim3(grid), dim3(256), 0, s, keys, n, or_and);
  if ((e = hipGetLastError())) return e;
  if ((e = hipMemcpyAsync(got, or_and, sizeof(got), hipMemcpyDeviceToHost, s))) return e;
  if ((e = hipStreamSynchronize(s))) return e;
  const uint64_t varying = got[0] ^ got[1];  // bits that differ between some two keys
  K *src_k = keys, *dst_k = keys_alt;
  uint32_t *src_v = vals, *dst_v = vals_alt;
  for (uint32_t shift = 0; shift < end_bit; shift += kDigitBits) {
    const uint32_t width = end_bit - shift < kDigitBits ? end_bit - shift : kDigitBits;
    const uint32_t dmask = (1u << width) - 1u;
    if (((varying >> shift) & dmask) == 0) continue;  // one digit value: the pass is the identity
    hipLaunchKernelGGL((sort_digits_hist<K>), dim3((unsigned)tiles), dim3(kSortThreads), 0, s, src_k, n, shift, dmask,
                       (uint32_t)tiles, cnt);
    if ((e = hipGetLastError())) return e;
    if ((e = scan_exclusive_u32(cnt, cnt, kDigits * tiles, nullptr, scan_tmp, s))) return e;
    hipLaunchKernelGGL((sort_digits_scatter<K, VALS>), dim3((unsigned)tiles), dim3(kSortThreads), 0, s, src_k, src_v,
                       n, shift, dmask, (uint32_t)tiles, cnt, dst_k, dst_v);
    if ((e = hipGetLastError())) return e;
    std::swap(src_k, dst_k);
    std::swap(src_v, dst_v);
    *in_alt = !*in_alt;
  }
  return hipSuccess;
}

}  // namespace

size_t radix_sort_temp_bytes(uint64_t n) {
  const uint64_t tiles = (n + kSortTile - 1) / kSortTile;
  const uint64_t m = kDigits * (tiles ? tiles : 1);
  return 256 + ((m * 4 + 255) & ~(uint64_t)255) + scan_u64_temp_bytes(m);
}

hipError_t radix_sort_pairs_u32(uint32_t *keys, uint32_t *keys_alt, uint32_t *vals, uint32_t *vals_alt, uint64_t n,
                                uint32_t end_bit, void *tmp, hipStream_t s, bool *in_alt) {
  return radix_sort<uint32_t, true>(keys, keys_alt, vals, vals_alt, n, end_bit, tmp, s, in_alt);
}

hipError_t radix_sort_keys_u64(uint64_t *keys, uint64_t *keys_alt, uint64_t n, void *tmp, hipStream_t s,
                               bool *in_alt) {
  return radix_sort<uint64_t, false>(keys, keys_alt, nullptr, nullptr, n, 64, tmp, s, in_alt);
}

}  // namespace ccj
