// ccj_build.hip — the chaining hash table built on the device.
//
// HashTable::HashTable (chaining_ht.cpp:4-36) puts build tuple t at the END of the std::list of
// bucket h(k_t) & mask (:29-35), so a chain lists its keys in generator order.  The CSR form of
// that is a STABLE counting sort of the tuples by bucket:
//   1. bucket ids b_t = murmurhash64(k_t) & mask and a histogram of them (one atomic per tuple);
//   2. off = exclusive scan of the histogram (ccj_scan.hip) — the chain ranges, off[size] = n;
//   3. (b_t, t) sorted by b_t with the hand-written stable LSD radix sort (ccj_sort.hip) over the
//      log2(size) bucket bits, so equal buckets keep ascending t: position j of the chain array
//      holds tuple idx[j] — exactly the std::list order;
//   4. chain[j] = k_idx[j], row[j] = idx[j] (padded to a multiple of 4 with -1 / kNoRow: the probes
//      read aligned 4-key windows);
//   5. per bucket the 16-byte record {start | len << 32, first key} and the 8-byte record
//      {start | len << 32 | fp(node 0) << 40 | fp(node 1) << 52} (kept when the longest chain is
//      < 255), plus the longest chain (max_rounds);
//   6. max_dup (largest multiplicity of one key, which sizes every probe output): known from the
//      generator for reference builds; otherwise from a copy of the keys sorted by the same radix
//      sort (as 64-bit patterns: equal keys adjacent) — the largest L with some i such that
//      sorted[i] == sorted[i + L - 1], found by doubling then bisection.
// Every array is byte-identical to the host build (ccj_api.hip build_chain_host, kept for
// ccj_table_build_from_host); tests/test_build_gpu.py compares them.  Build time is untimed, as in
// the reference (main.cpp:62-68 builds before the timer at :92-94).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <memory>
#include <vector>

#include "ccj_internal.h"

namespace ccj {
namespace {

unsigned grid_of(uint64_t n, unsigned threads) {
  const uint64_t g = (n + threads - 1) / threads;
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, 1u << 20));
}

// Step 1: bucket id + tuple index per build tuple, histogram of the buckets.
__global__ void chain_bucket_ids(const int64_t *keys, uint64_t n, uint32_t mask, uint32_t *bid, uint32_t *idx,
                                 uint32_t *cnt) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t b = (uint32_t)murmurhash64((uint64_t)keys[t]) & mask;
    bid[t] = b;
    idx[t] = (uint32_t)t;
    atomicAdd(cnt + b, 1u);
  }
}

// Step 4: the chain array in bucket-major, insertion order, and its row map (+ padding).
__global__ void chain_gather(const int64_t *keys, const uint32_t *idx, uint64_t n, uint64_t n_pad, int64_t *chain,
                             uint32_t *row) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n_pad;
       j += (uint64_t)gridDim.x * blockDim.x) {
    if (j < n) {
      const uint32_t t = idx[j];
      chain[j] = keys[t];
      row[j] = t;
    } else {
      chain[j] = -1;
      row[j] = kNoRow;
    }
  }
}

// Step 5: bucket records and the longest chain.  rec8 has n_rec8 >= max(size, 2) entries (the
// walks read them as aligned 16-byte pairs); entries past size are empty records.
__global__ __launch_bounds__(256) void chain_records(const uint32_t *off, const int64_t *chain, uint64_t size,
                                                     longlong2 *rec16, uint64_t *rec8, uint64_t n_rec8,
                                                     uint32_t *longest) {
  uint32_t best = 0;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n_rec8;
       b += (uint64_t)gridDim.x * blockDim.x) {
    if (b >= size) {
      rec8[b] = 0;
      continue;
    }
    const uint64_t lo = off[b], len = off[b + 1] - lo;
    best = (uint32_t)len > best ? (uint32_t)len : best;
    const int64_t k0 = len ? chain[lo] : -1;
    rec16[b] = make_longlong2((long long)(lo | (len << 32)), (long long)k0);
    const uint64_t fp0 = len ? bucket_fp(murmurhash64((uint64_t)k0)) : 0u;
    const uint64_t fp1 = len > 1 ? bucket_fp(murmurhash64((uint64_t)chain[lo + 1])) : 0u;
    rec8[b] = lo | (len & 0xFFull) << 32 | fp0 << 40 | fp1 << 52;
  }
  // one atomic per workgroup (the grid is capped, so a few thousand): one per wave of a
  // one-bucket-per-thread grid queued 2^21 atomics on one address (round 4: 23.8 ms for C3's table)
  for (int d = 32; d > 0; d >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)best, d);
    best = o > best ? o : best;
  }
  __shared__ uint32_t s_best[4];
  if ((threadIdx.x & 63u) == 0) s_best[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < blockDim.x / 64; ++w) best = s_best[w] > best ? s_best[w] : best;
    if (best) atomicMax(longest, best);
  }
}

// The bucket filter (probe_chain_filt): 2 bits per bucket, 16 buckets per word.  One thread per
// bucket (coalesced offset reads), the 16 codes of a word OR-ed across 16 lanes; a thread per word
// reading 16 strided offsets took 1.5 ms for C3's 2^27 buckets.
__global__ void chain_filter(const uint32_t *off, const int64_t *chain, uint64_t size, uint32_t *filt) {
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x; b0 < size; b0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = b0 + threadIdx.x;  // size: a power of two >= 128; blockDim 256
    uint32_t v = 0;
    if (b < size) {
      const uint32_t lo = off[b], len = off[b + 1] - lo;
      const uint32_t code = len == 0 ? 0u : len == 1 ? 1u + (uint32_t)((murmurhash64((uint64_t)chain[lo]) >> 40) & 1u) : 3u;
      v = code << (2 * (lane & 15u));
    }
    for (int d = 1; d < 16; d <<= 1) v |= (uint32_t)__shfl_xor((int)v, d);
    if (b < size && (lane & 15u) == 0) filt[b / 16] = v;
  }
}

// Step 6: *flag = 1 if some run of equal keys in the sorted column is at least L long.
__global__ void has_run(const int64_t *sorted, uint64_t n, uint64_t L, uint32_t *flag) {
  if (L < 2 || L > n) return;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i + L - 1 < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    if (sorted[i] == sorted[i + L - 1]) {
      *flag = 1u;
      return;
    }
}

// Device memory that frees itself (the build's scratch and, on failure, the table's arrays).
struct DevBuf {
  void *p = nullptr;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 8); }
  template <class T> T *as() const { return static_cast<T *>(p); }
  void *release() {
    void *q = p;
    p = nullptr;
    return q;
  }
};

int hip_err(hipError_t e, const char *what) {
  return api_fail(e == hipErrorOutOfMemory ? CCJ_ERR_OOM : CCJ_ERR_HIP,
                  std::string("device chaining build: ") + what + ": " + hipGetErrorString(e));
}

#define BUILD_TRY(expr, what)                  \
  do {                                         \
    hipError_t e_ = (expr);                    \
    if (e_ != hipSuccess) return hip_err(e_, what); \
  } while (0)

// Largest multiplicity of one key among d_keys[0, n): radix-sort a copy, then find the largest L with
// a run of L equal keys (doubling, then bisection; one pass for distinct keys).
int max_multiplicity(const int64_t *d_keys, uint64_t n, hipStream_t s, uint64_t *out) {
  *out = n ? 1 : 0;
  if (n < 2) return CCJ_OK;
  DevBuf a, b, tmp, flag;
  BUILD_TRY(a.alloc(n * sizeof(int64_t)), "sorted keys");
  BUILD_TRY(b.alloc(n * sizeof(int64_t)), "sorted keys (alt)");
  BUILD_TRY(tmp.alloc(radix_sort_temp_bytes(n)), "sort scratch");
  BUILD_TRY(flag.alloc(sizeof(uint32_t)), "flag");
  BUILD_TRY(hipMemcpyAsync(a.p, d_keys, n * sizeof(int64_t), hipMemcpyDeviceToDevice, s), "key copy");
  bool in_alt = false;
  BUILD_TRY(radix_sort_keys_u64(a.as<uint64_t>(), b.as<uint64_t>(), n, tmp.p, s, &in_alt), "sort keys");
  const int64_t *sorted = in_alt ? b.as<int64_t>() : a.as<int64_t>();
  auto test = [&](uint64_t L, bool *yes) -> int {
    uint32_t h = 0;
    BUILD_TRY(hipMemsetAsync(flag.p, 0, sizeof(uint32_t), s), "flag reset");
    hipLaunchKernelGGL(has_run, dim3(grid_of(n, 256)), dim3(256), 0, s, sorted, n, L, flag.as<uint32_t>());
    BUILD_TRY(hipGetLastError(), "has_run");
    BUILD_TRY(hipMemcpyAsync(&h, flag.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "flag read");
    BUILD_TRY(hipStreamSynchronize(s), "flag sync");
    *yes = h != 0;
    return CCJ_OK;
  };
  uint64_t lo = 1, hi = 2;  // a run of lo exists; hi is the next length tried
  while (true) {
    bool yes = false;
    if (int rc = test(hi, &yes)) return rc;
    if (!yes) break;
    lo = hi;
    if (hi == n) break;
    hi = std::min<uint64_t>(2 * hi, n);
  }
  if (lo < hi) {  // the answer is in [lo, hi)
    uint64_t a = lo, b = hi;  // run of a exists, run of b does not (unless lo == n)
    while (b - a > 1) {
      const uint64_t m = a + (b - a) / 2;
      bool yes = false;
      if (int rc = test(m, &yes)) return rc;
      (yes ? a : b) = m;
    }
    lo = a;
  }
  *out = lo;
  return CCJ_OK;
}

}  // namespace

hipError_t build_chain_filter(ccj_table *t, hipStream_t s) {
  const uint64_t size = t->info.size;
  if (size < 128 || t->d_filt) return hipSuccess;  // (the filter walk needs >= 8 partitions of >= 16 buckets)
  const uint64_t words = size / 16;
  hipError_t e = hipMalloc((void **)&t->d_filt, words * 4);
  if (e != hipSuccess) {
    t->d_filt = nullptr;
    return e;
  }
  hipLaunchKernelGGL(chain_filter, dim3(std::min<unsigned>(grid_of(size, 256), 8192)), dim3(256), 0, s, t->d_off,
                     t->d_table, size, t->d_filt);
  return hipGetLastError();
}

int build_chain_device(const int64_t *d_keys, uint64_t n, hipStream_t s, uint64_t known_dup, ccj_table **out) {
  uint64_t size = 1;
  while (size < 2 * n) size *= 2;  // chaining_ht.cpp:5-6
  if (size > (1ull << 31)) return api_fail(CCJ_ERR_LIMIT, "device chaining build: more than 2^31 buckets");
  const uint64_t n_pad = ((n + 3) / 4) * 4 + (n == 0 ? 4 : 0);
  const uint64_t n_rec8 = size < 2 ? 2 : size;
  uint32_t bits = 0;
  while ((1ull << bits) < size) ++bits;

  DevBuf chain, off, row, rec16, rec8, cnt, bid, bid_s, idx, idx_s, sort_tmp, scan_tmp, d_longest;
  BUILD_TRY(chain.alloc(n_pad * sizeof(int64_t)), "chain keys");
  BUILD_TRY(off.alloc((size + 1) * sizeof(uint32_t)), "chain offsets");
  BUILD_TRY(row.alloc(n_pad * sizeof(uint32_t)), "chain rows");
  BUILD_TRY(rec16.alloc(size * 16), "bucket records");
  BUILD_TRY(rec8.alloc(n_rec8 * 8), "bucket records (8 B)");
  BUILD_TRY(cnt.alloc((size + 1) * sizeof(uint32_t)), "histogram");
  BUILD_TRY(d_longest.alloc(sizeof(uint32_t)), "longest");
  BUILD_TRY(hipMemsetAsync(cnt.p, 0, (size + 1) * sizeof(uint32_t), s), "histogram reset");
  BUILD_TRY(hipMemsetAsync(d_longest.p, 0, sizeof(uint32_t), s), "longest reset");
  if (n) {
    BUILD_TRY(bid.alloc(n * 4), "bucket ids");
    BUILD_TRY(idx.alloc(n * 4), "tuple ids");
    BUILD_TRY(bid_s.alloc(n * 4), "sorted bucket ids");
    BUILD_TRY(idx_s.alloc(n * 4), "sorted tuple ids");
    hipLaunchKernelGGL(chain_bucket_ids, dim3(grid_of(n, 256)), dim3(256), 0, s, d_keys, n, (uint32_t)(size - 1),
                       bid.as<uint32_t>(), idx.as<uint32_t>(), cnt.as<uint32_t>());
    BUILD_TRY(hipGetLastError(), "bucket ids");
  }
  BUILD_TRY(scan_tmp.alloc(scan_u64_temp_bytes(size + 1)), "scan scratch");
  BUILD_TRY(scan_exclusive_u32(cnt.as<uint32_t>(), off.as<uint32_t>(), size + 1, nullptr, scan_tmp.p, s), "offset scan");
  const uint32_t *idx_sorted = idx.as<uint32_t>();
  if (n) {
    // stable LSD radix sort by bucket: equal buckets keep ascending tuple order (push_back order)
    bool in_alt = false;
    BUILD_TRY(sort_tmp.alloc(radix_sort_temp_bytes(n)), "sort scratch");
    BUILD_TRY(radix_sort_pairs_u32(bid.as<uint32_t>(), bid_s.as<uint32_t>(), idx.as<uint32_t>(), idx_s.as<uint32_t>(), n,
                                   bits ? bits : 1, sort_tmp.p, s, &in_alt),
              "bucket sort");
    if (in_alt) idx_sorted = idx_s.as<uint32_t>();
  }
  hipLaunchKernelGGL(chain_gather, dim3(grid_of(n_pad, 256)), dim3(256), 0, s, d_keys, idx_sorted, n, n_pad,
                     chain.as<int64_t>(), row.as<uint32_t>());
  BUILD_TRY(hipGetLastError(), "chain gather");
  hipLaunchKernelGGL(chain_records, dim3(std::min<unsigned>(grid_of(n_rec8, 256), 4096)), dim3(256), 0, s, off.as<uint32_t>(),
                     chain.as<int64_t>(), size, rec16.as<longlong2>(), rec8.as<uint64_t>(), n_rec8,
                     d_longest.as<uint32_t>());
  BUILD_TRY(hipGetLastError(), "bucket records");
  uint32_t longest = 0;
  BUILD_TRY(hipMemcpyAsync(&longest, d_longest.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "longest read");
  BUILD_TRY(hipStreamSynchronize(s), "build sync");
  uint64_t dup = known_dup;
  if (!dup) {
    if (int rc = max_multiplicity(d_keys, n, s, &dup)) return rc;
  }

  std::unique_ptr<ccj_table> t(new ccj_table());
  t->info.kind = CCJ_TABLE_CHAIN;
  t->info.layout = CCJ_LAYOUT_DEVICE;
  t->info.n_keys = n;
  t->info.size = size;
  t->info.max_rounds = longest;
  t->info.max_dup = n ? (dup ? dup : 1) : 0;
  t->positions = n_pad;
  t->d_table = (int64_t *)chain.release();
  t->d_off = (uint32_t *)off.release();
  t->d_row = (uint32_t *)row.release();
  t->d_bucket = (int64_t *)rec16.release();
  if (longest < 0xFFu) t->d_bucket8 = (uint64_t *)rec8.release();  // len fits the record's 8 bits
  t->info.d_table = t->d_table;
  t->info.d_bucket_off = t->d_off;
  (void)hipGetDevice(&t->device);
  hipError_t fe = build_chain_filter(t.get(), s);
  if (fe == hipSuccess) fe = hipStreamSynchronize(s);
  if (fe != hipSuccess) {
    for (void *q : {(void *)t->d_table, (void *)t->d_off, (void *)t->d_row, (void *)t->d_bucket, (void *)t->d_bucket8,
                    (void *)t->d_filt})
      if (q) (void)hipFree(q);
    return hip_err(fe, "bucket filter");
  }
  *out = t.release();
  return CCJ_OK;
}

}  // namespace ccj
