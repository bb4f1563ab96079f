// ccj_compact.hip — device chunk compaction (NaiveCompactor::Compact/Flush, compactor.cpp:5-41,
// with the fresh-temp-chunk fix of :36) over the Next results of a ccj_probe output.
//
// The reference compacts sequentially: a cache of up to `chunk` rows absorbs each Next result;
// a full result bypasses the cache (:6); an overflowing result tops the cache up, the cache is
// emitted, and the rest becomes the new cache (:22-35).  That order is a closed form of two
// prefix sums, so it runs in parallel:
//   pass-through results: the non-empty ones of >= T rows (T = threshold; T = chunk: the
//   reference's full-chunk rule, compactor.cpp:6)
//   P-stream  = rows of the other results, concatenated in pipeline order (t = position in it)
//   F_s       = pass-through results before result s;  E(t) = t == 0 ? 0 : ceil(t / chunk) - 1
//   pass-through result s   -> output chunk E(t_s) + F_s (keeping its own row count)
//   P-row u (chunk k = u/B)  -> output chunk k + #{pass-through s : E(t_s) <= k}, row u % B
// Kernels: per-chunk segment sums -> exclusive scans (ccj_scan.hip) -> full-result E list -> one wave
// per probe chunk copies its rows (DataChunk::Append's gather, base.cpp:15-27) -> chunk counts.

#include <cstdlib>

#include "ccj_internal.h"

namespace ccj {
namespace {

struct CompactParams {
  ccj_compact_args a;
  uint64_t *nonfull;  // [n_chunks] -> exclusive scan in place (t at chunk start)
  uint64_t *full;     // [n_chunks] -> exclusive scan in place (F at chunk start)
  uint64_t *totals;   // [2]: T_total, F_total
  uint32_t *fullE;    // [max full results]
  uint64_t max_full;
  uint32_t thr;       // pass-through threshold (>= 1)
  __device__ __forceinline__ bool bypass(uint32_t rc) const { return rc != 0 && rc >= thr; }
};

__global__ void seg_sums(CompactParams p) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= p.a.n_chunks) return;
  const uint32_t rounds = p.a.rounds[c];
  uint64_t nf = 0, f = 0;
  for (uint32_t r = 0; r < rounds && r < p.a.max_rounds; ++r) {
    const uint32_t rc = p.a.round_counts[c * p.a.max_rounds + r];
    if (p.bypass(rc)) ++f;
    else nf += rc;
  }
  p.nonfull[c] = nf;
  p.full[c] = f;
}

__global__ void seg_totals(CompactParams p, const uint64_t *nf_last, const uint64_t *f_last) {
  // called after the exclusive scans: totals = scan[last] + value[last]
  p.totals[0] = p.nonfull[p.a.n_chunks - 1] + nf_last[0];
  p.totals[1] = p.full[p.a.n_chunks - 1] + f_last[0];
  const uint64_t T = p.totals[0], F = p.totals[1], B = p.a.chunk;
  const uint64_t n_out = F + (T + B - 1) / B;
  if (p.a.out_n_chunks) *p.a.out_n_chunks = n_out;
  if (n_out * B > p.a.out_cap_rows && p.a.status) atomicOr(p.a.status, CCJ_FLAG_CAP_OVERFLOW);
  if (F > p.max_full && p.a.status) atomicOr(p.a.status, CCJ_FLAG_CAP_OVERFLOW);
}

__device__ __forceinline__ uint64_t e_of(uint64_t t, uint64_t B) { return t == 0 ? 0 : (t + B - 1) / B - 1; }

__global__ void full_list(CompactParams p) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= p.a.n_chunks) return;
  const uint32_t rounds = p.a.rounds[c];
  uint64_t t = p.nonfull[c], f = p.full[c];
  for (uint32_t r = 0; r < rounds && r < p.a.max_rounds; ++r) {
    const uint32_t rc = p.a.round_counts[c * p.a.max_rounds + r];
    if (p.bypass(rc)) {
      if (f < p.max_full) {
        const uint64_t e = e_of(t, p.a.chunk);
        p.fullE[f] = (uint32_t)e;
        if ((e + f + 1) * p.a.chunk <= p.a.out_cap_rows) p.a.out_chunk_counts[e + f] = rc;  // its own count
      }
      ++f;
    } else {
      t += rc;
    }
  }
}

// #{full results s : E(t_s) <= k}: fullE is non-decreasing.
__device__ __forceinline__ uint64_t full_before(const CompactParams &p, uint64_t F, uint64_t k) {
  uint64_t lo = 0, hi = F;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (p.fullE[mid] <= k) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// One wave per probe chunk with at most 64 Next results: lane r holds round r's count,
// its P-stream start, its pass-through index and its source offset (wave prefix sums); every lane
// then copies matches m = lane, lane + 64, ... of the chunk, finding m's round by a binary search
// over the lanes.  All 64 lanes stay busy however the matches spread over rounds.
__global__ __launch_bounds__(256) void copy_rows_flat(CompactParams p) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t c = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= p.a.n_chunks) return;
  const uint64_t B = p.a.chunk;
  const uint64_t F = p.totals[1] < p.max_full ? p.totals[1] : p.max_full;
  const uint64_t cap_rows = p.a.out_cap_rows;
  const uint32_t rounds = p.a.rounds[c] < p.a.max_rounds ? p.a.rounds[c] : p.a.max_rounds;
  const uint32_t total = p.a.count[c];
  if (rounds > 64) {  // rare: a per-round loop (the round-wise form measured 4.20 vs 3.83 ms, main.cpp pipeline)
    uint64_t t = p.nonfull[c], f = p.full[c], src = c * p.a.cap;
    for (uint32_t r = 0; r < rounds; ++r) {
      const uint32_t rc = p.a.round_counts[c * p.a.max_rounds + r];
      const bool is_full = p.bypass(rc);
      const uint64_t fbase = (e_of(t, B) + f) * B;
      for (uint32_t j = lane; j < rc; j += 64) {
        if (src + j >= c * p.a.cap + total) break;
        uint64_t dest;
        if (is_full) {
          dest = fbase + j;
        } else {
          const uint64_t u = t + j, k = u / B;
          dest = (k + (F ? full_before(p, F, k) : 0)) * B + (u - k * B);
        }
        if (dest >= cap_rows) continue;
        const uint64_t row = c * B + p.a.sel[src + j];
        for (uint32_t q = 0; q < p.a.n_cols; ++q)
          p.a.out_cols[q][dest] = (p.a.key_cols >> q) & 1u ? p.a.payload[src + j] : p.a.cols[q][row];
        if (p.a.out_payload) p.a.out_payload[dest] = p.a.payload[src + j];
        if (p.a.out_row) p.a.out_row[dest] = row;
      }
      src += rc;
      if (is_full) ++f;
      else t += rc;
    }
    return;
  }
  const bool b2 = (B & (B - 1)) == 0;  // a power-of-two chunk (every bench chunk): shifts, not divisions
  const uint32_t bl2 = (uint32_t)__builtin_ctzll(B);
  const uint64_t obase = c * p.a.cap;
  // One round (every chunk of the partitioned probe: its matches are one compactor input): round 0's
  // values are wave-uniform — no scans or searches over the lanes.  The match's row and payload are
  // read once, before any store (the stores may alias them for the compiler).
  if (rounds <= 1) {
    const uint32_t rc0 = rounds ? p.a.round_counts[c * p.a.max_rounds] : 0u;
    const bool rb0 = rounds && p.bypass(rc0);
    const uint64_t tr0 = p.nonfull[c], fb0 = (e_of(tr0, B) + p.full[c]) * B;
    for (uint32_t m = lane; m < total; m += 64) {
      uint64_t dest;
      if (rb0) {
        dest = fb0 + m;
      } else {
        const uint64_t u = tr0 + m, k = b2 ? u >> bl2 : u / B;
        dest = (k + (F ? full_before(p, F, k) : 0)) * B + (u - k * B);
      }
      if (dest >= cap_rows) continue;
      const uint64_t row = c * B + p.a.sel[obase + m];
      const int64_t pay = p.a.payload[obase + m];
      for (uint32_t q = 0; q < p.a.n_cols; ++q)
        p.a.out_cols[q][dest] = (p.a.key_cols >> q) & 1u ? pay : p.a.cols[q][row];
      if (p.a.out_payload) p.a.out_payload[dest] = pay;
      if (p.a.out_row) p.a.out_row[dest] = row;
    }
    return;
  }
  const uint32_t rc = lane < rounds ? p.a.round_counts[c * p.a.max_rounds + lane] : 0u;
  const bool byp = lane < rounds && p.bypass(rc);
  // exclusive prefixes over rounds: source offset, P-stream rows, pass-through results
  uint32_t src = rc, ps = byp ? 0u : rc, fs = byp ? 1u : 0u;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t a = (uint32_t)__shfl_up((int)src, d), b = (uint32_t)__shfl_up((int)ps, d),
                   e = (uint32_t)__shfl_up((int)fs, d);
    if (lane >= (uint32_t)d) {
      src += a;
      ps += b;
      fs += e;
    }
  }
  src -= rc;
  ps -= byp ? 0u : rc;
  fs -= byp ? 1u : 0u;
  const uint64_t t_r = p.nonfull[c] + ps, f_r = p.full[c] + fs;
  const uint64_t fbase = (e_of(t_r, B) + f_r) * B;  // lane r's pass-through destination
  // Every lane runs every iteration (cross-lane reads need the source lanes active).
  for (uint32_t m0 = 0; m0 < total; m0 += 64) {
    const uint32_t m = m0 + lane;
    // round of match m: the last r < rounds with src_r <= m (src is non-decreasing, src_0 = 0)
    uint32_t r = 0;
#pragma unroll
    for (uint32_t step = 32; step >= 1; step >>= 1) {
      const uint32_t cand = r + step;
      const uint32_t v = (uint32_t)__shfl((int)src, (int)(cand < rounds ? cand : 0u));
      if (cand < rounds && v <= m) r = cand;
    }
    const uint32_t j = m - (uint32_t)__shfl((int)src, (int)r);
    const bool rb = __shfl((int)byp, (int)r) != 0;
    const uint64_t fb = (uint64_t)__shfl((long long)fbase, (int)r);
    const uint64_t tr = (uint64_t)__shfl((long long)t_r, (int)r);
    if (m >= total) continue;
    uint64_t dest;
    if (rb) {
      dest = fb + j;
    } else {
      const uint64_t u = tr + j, k = b2 ? u >> bl2 : u / B;
      dest = (k + (F ? full_before(p, F, k) : 0)) * B + (u - k * B);
    }
    if (dest >= cap_rows) continue;
    const uint64_t row = c * B + p.a.sel[obase + m];
    const int64_t pay = p.a.payload[obase + m];
    // (a join-key column equals the payload on every output row: read densely, not gathered)
    for (uint32_t q = 0; q < p.a.n_cols; ++q)
      p.a.out_cols[q][dest] = (p.a.key_cols >> q) & 1u ? pay : p.a.cols[q][row];
    if (p.a.out_payload) p.a.out_payload[dest] = pay;
    if (p.a.out_row) p.a.out_row[dest] = row;
  }
}

__global__ void chunk_counts(CompactParams p) {
  // P-chunks (compacted): all full except the last; pass-through chunks were counted by full_list.
  const uint64_t T = p.totals[0], B = p.a.chunk;
  const uint64_t F = p.totals[1] < p.max_full ? p.totals[1] : p.max_full;
  const uint64_t n_p = (T + B - 1) / B;
  const uint64_t lim = p.a.out_cap_rows / B;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_p;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t q = k + (F ? full_before(p, F, k) : 0);
    if (q >= lim) continue;
    p.a.out_chunk_counts[q] = k + 1 < n_p ? (uint32_t)B : (uint32_t)(T - k * B);
  }
}

size_t scan_temp_bytes(uint64_t n) { return scan_u64_temp_bytes(n); }

}  // namespace

// Pass-through results per probe chunk: at most cap / T of them (each has >= T rows) and at most
// one per round.
uint64_t max_bypass(uint64_t n_chunks, uint64_t cap, uint32_t chunk, uint32_t max_rounds, uint32_t threshold) {
  const uint64_t t = threshold ? threshold : chunk;
  uint64_t per = cap / t + 1;
  if (max_rounds && max_rounds < per) per = max_rounds;
  return n_chunks * per;
}

size_t compact_workspace(uint64_t n_chunks, uint64_t cap, uint32_t chunk, uint32_t max_rounds, uint32_t threshold) {
  const uint64_t max_full = max_bypass(n_chunks, cap, chunk, max_rounds, threshold);
  return 256 + 4 * ((n_chunks * 8 + 255) & ~255ull) + ((max_full * 4 + 255) & ~255ull) + scan_temp_bytes(n_chunks);
}

hipError_t launch_compact(const ccj_compact_args &a, hipStream_t s) {
  CompactParams p{};
  p.a = a;
  char *w = (char *)a.workspace;
  auto take = [&](size_t bytes) {
    char *r = w;
    w += (bytes + 255) & ~(size_t)255;
    return r;
  };
  p.totals = (uint64_t *)take(256);
  p.nonfull = (uint64_t *)take(a.n_chunks * 8);
  p.full = (uint64_t *)take(a.n_chunks * 8);
  uint64_t *nf_raw = (uint64_t *)take(a.n_chunks * 8);
  uint64_t *f_raw = (uint64_t *)take(a.n_chunks * 8);
  p.max_full = max_bypass(a.n_chunks, a.cap, a.chunk, a.max_rounds, a.threshold);
  p.thr = a.threshold ? (a.threshold < a.chunk ? a.threshold : a.chunk) : a.chunk;
  p.fullE = (uint32_t *)take(p.max_full * 4);
  void *tmp = take(scan_temp_bytes(a.n_chunks));
  const unsigned g = (unsigned)((a.n_chunks + 255) / 256);
  CompactParams q = p;
  q.nonfull = nf_raw;
  q.full = f_raw;
  hipLaunchKernelGGL(seg_sums, dim3(g), dim3(256), 0, s, q);
  hipError_t e = hipGetLastError();
  if (e) return e;
  e = scan_exclusive_u64(nf_raw, p.nonfull, a.n_chunks, nullptr, tmp, s);
  if (e) return e;
  e = scan_exclusive_u64(f_raw, p.full, a.n_chunks, nullptr, tmp, s);
  if (e) return e;
  hipLaunchKernelGGL(seg_totals, dim3(1), dim3(1), 0, s, p, nf_raw + a.n_chunks - 1, f_raw + a.n_chunks - 1);
  hipLaunchKernelGGL(full_list, dim3(g), dim3(256), 0, s, p);
  hipLaunchKernelGGL(copy_rows_flat, dim3((unsigned)((a.n_chunks + 3) / 4)), dim3(256), 0, s, p);
  hipLaunchKernelGGL(chunk_counts, dim3(1024), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace ccj
