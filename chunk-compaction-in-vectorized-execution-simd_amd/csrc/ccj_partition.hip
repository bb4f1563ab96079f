// ccj_partition.hip — multisplits of a key column by a digit of its murmurhash64 value.
//
//  - owner partitioning for the multi-GPU join: digit = h >> (64 - log2 P), the TOP
//    hash bits, disjoint from the low bits every GPU's local table uses, so shards stay balanced;
//  - slot-range partitioning for the L2-resident probe (ccj_probe_partitioned): the slot index
//    h & (n_slots - 1) above the window bits, split in ONE pass into fixed-capacity segments
//    (slot_split_fixed, below), or exactly in two LSD passes (low digit, then high) as the
//    fallback for key skew that overflows a segment.
//
// Each exact pass is a multisplit in two kernels: (1) per-tile digit counts, written digit-major;
// (2) after an exclusive scan of those counts, every tile re-reads its keys, builds an LDS image
// of itself grouped by digit, and writes each digit segment whole; tiles are dealt to XCDs in
// contiguous ranges so the lines where neighbouring tiles' segments meet are completed in one L2.
// The exact-size owner split (build-side sharding, exchange fallback) ranks keys stably (ballot +
// mbcnt), so its output is deterministic; the fixed-capacity owner split and the slot split rank
// them with LDS atomics (grouping exact, order inside a tile's segment not), which is all the
// probe needs — the second LSD pass still leaves every slot partition contiguous.

#include <cmath>
#include <type_traits>

#include "ccj_internal.h"
#include "ccj_tuning.h"

namespace ccj {
namespace {

extern "C" __device__ uint32_t __ockl_wfscan_add_u32(uint32_t, bool);
// Inclusive prefix sum over the wave's lanes (DPP row shifts + permlane, no LDS).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) { return __ockl_wfscan_add_u32(x, true); }

constexpr int kTileThreads = 256;
constexpr int kTileIters = 8;
constexpr uint64_t kTile = (uint64_t)kTileThreads * kTileIters;  // 2048 keys per tile (24 KB of LDS image)

struct Digit {
  uint32_t shift;  // >= 64: every key to digit 0
  uint32_t mask;   // parts - 1
  __device__ __forceinline__ uint32_t operator()(int64_t k) const {
    return shift >= 64 ? 0u : (uint32_t)(murmurhash64((uint64_t)k) >> shift) & mask;
  }
};

__global__ __launch_bounds__(kTileThreads) void part_count(const int64_t *keys, uint64_t n, uint32_t parts, Digit dg,
                                                           uint64_t n_tiles, uint64_t *cnt) {
  __shared__ uint32_t s_cnt[kMaxParts];
  const uint64_t tile = blockIdx.x;
  if (threadIdx.x < kMaxParts) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  for (int it = 0; it < kTileIters; ++it) {
    const uint64_t i = tile * kTile + (uint64_t)it * kTileThreads + threadIdx.x;
    if (i < n) atomicAdd(&s_cnt[dg(keys[i])], 1u);
  }
  __syncthreads();
  if (threadIdx.x < parts) cnt[(uint64_t)threadIdx.x * n_tiles + tile] = s_cnt[threadIdx.x];
}

// Scatter of one tile: keys are ranked stably per digit (ballot + mbcnt inside a wave, LDS scan
// across the tile's waves and iterations) into an LDS image of the tile sorted by digit, which is
// then written out digit segment by digit segment: consecutive threads write consecutive
// addresses of one segment, so every destination line is written whole (a direct scatter of
// 8-byte stores to up to 64 destinations leaves partial lines in L2 and measured 2-3x slower).
template <typename RowT, bool STABLE>
__global__ __launch_bounds__(kTileThreads) void part_scatter(const int64_t *keys, const RowT *in_rows, uint64_t n,
                                                             uint32_t parts, Digit dg, uint64_t n_tiles,
                                                             const uint64_t *cnt, const uint64_t *off,
                                                             uint64_t row_base, int64_t *out_keys, RowT *out_rows,
                                                             uint64_t stride, uint32_t *status) {
  __shared__ int64_t s_k[kTile];
  __shared__ RowT s_r[kTile];
  __shared__ uint64_t s_glob[kMaxParts];
  __shared__ uint32_t s_loc[kMaxParts], s_run[kMaxParts];
  __shared__ uint32_t s_wave[kTileThreads / 64][kMaxParts];
  // XCD-aware tile order: workgroups are dealt round-robin to the 8 XCDs; block b takes tile
  // (b % 8) * (n8 / 8) + b / 8, so each XCD writes a contiguous range of tiles and the partial
  // lines where one tile's digit segment meets the next one's are completed in one XCD's L2.
  uint64_t tile = blockIdx.x;
  {
    const uint64_t n8 = n_tiles & ~7ull;
    if (tile < n8) tile = (tile & 7) * (n8 >> 3) + (tile >> 3);
  }
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t t0 = tile * kTile;
  const uint32_t tn = (uint32_t)(n - t0 < kTile ? n - t0 : kTile);
  if (threadIdx.x < parts) {
    const uint64_t d = threadIdx.x;
    // compact: digit segments back to back; fixed (stride > 0): digit d owns [d*stride, (d+1)*stride)
    s_glob[d] = stride ? d * stride + (off[d * n_tiles + tile] - off[d * n_tiles]) : off[d * n_tiles + tile];
    s_run[d] = (uint32_t)cnt[d * n_tiles + tile];
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // local exclusive offsets of the digit segments inside the tile image
    uint32_t acc = 0;
    for (uint32_t d = 0; d < parts; ++d) {
      s_loc[d] = acc;
      acc += s_run[d];
    }
  }
  __syncthreads();
  if (threadIdx.x < parts) s_run[threadIdx.x] = s_loc[threadIdx.x];
  __syncthreads();
  if (STABLE) {
    for (int it = 0; it < kTileIters; ++it) {
      const uint32_t li = (uint32_t)it * kTileThreads + threadIdx.x;
      const bool valid = li < tn;
      const int64_t k = valid ? keys[t0 + li] : 0;
      const uint32_t d = valid ? dg(k) : 0xFFFFFFFFu;
      uint32_t rank = 0;
      for (uint32_t q = 0; q < parts; ++q) {
        const uint64_t m = __ballot(d == q);
        if (d == q) rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (lane == 0) s_wave[wave][q] = (uint32_t)__popcll(m);
      }
      __syncthreads();
      if (valid) {
        uint32_t pos = s_run[d] + rank;
        for (uint32_t w = 0; w < wave; ++w) pos += s_wave[w][d];
        s_k[pos] = k;
        s_r[pos] = in_rows ? in_rows[t0 + li] : (RowT)(row_base + t0 + li);
      }
      __syncthreads();
      if (threadIdx.x < parts) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < kTileThreads / 64; ++w) t += s_wave[w][threadIdx.x];
        s_run[threadIdx.x] += t;
      }
      __syncthreads();
    }
  } else {
    // Unstable: the position inside a digit segment comes from an LDS atomic (one per key).
    // Grouping is exact; the order inside a (tile, digit) segment is not reproducible.
    // All of the tile's loads are issued before the first LDS atomic (latency hidden once).
    int64_t kk[kTileIters];
    RowT rr[kTileIters];
#pragma unroll
    for (int it = 0; it < kTileIters; ++it) {
      const uint32_t li = (uint32_t)it * kTileThreads + threadIdx.x;
      kk[it] = li < tn ? __builtin_nontemporal_load(keys + t0 + li) : 0;
      rr[it] = li < tn ? (in_rows ? __builtin_nontemporal_load(in_rows + t0 + li) : (RowT)(row_base + t0 + li)) : 0;
    }
#pragma unroll
    for (int it = 0; it < kTileIters; ++it) {
      const uint32_t li = (uint32_t)it * kTileThreads + threadIdx.x;
      if (li < tn) {
        const uint32_t pos = atomicAdd(&s_run[dg(kk[it])], 1u);
        s_k[pos] = kk[it];
        s_r[pos] = rr[it];
      }
    }
    __syncthreads();
  }
  bool dropped = false;
  for (uint32_t q = threadIdx.x; q < tn; q += kTileThreads) {
    const int64_t k = s_k[q];
    const uint32_t d = dg(k);
    const uint64_t dest = s_glob[d] + (q - s_loc[d]);
    if (stride && dest >= (uint64_t)(d + 1) * stride) {  // destination segment full
      dropped = true;
      continue;
    }
    out_keys[dest] = k;
    out_rows[dest] = s_r[q];
  }
  if (dropped && status) atomicOr(status, CCJ_FLAG_CAP_OVERFLOW);
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

size_t scan_bytes(uint64_t n) { return scan_u64_temp_bytes(n); }

size_t pass_workspace(uint64_t n, uint32_t parts) {
  const uint64_t n_tiles = (n + kTile - 1) / kTile;
  const uint64_t m = n_tiles * parts;
  return 2 * ((m * 8 + 255) & ~255ull) + scan_bytes(m ? m : 1);
}

// One multisplit pass (STABLE: ballot ranking; else LDS atomics).  out_counts (digit totals) may be
// NULL; stride > 0 gives destination d the fixed segment [d*stride, (d+1)*stride).
template <typename RowT, bool STABLE>
hipError_t split_pass(const int64_t *keys, const RowT *in_rows, uint64_t n, uint32_t parts, Digit dg,
                      uint64_t row_base, int64_t *out_keys, RowT *out_rows, uint64_t *out_counts, void *ws,
                      hipStream_t s, uint64_t stride = 0, uint32_t *status = nullptr) {
  const uint64_t n_tiles = (n + kTile - 1) / kTile;
  const uint64_t m = n_tiles * parts;
  if (n == 0) return out_counts ? hipMemsetAsync(out_counts, 0, parts * 8, s) : hipSuccess;
  char *w = (char *)ws;
  uint64_t *cnt = (uint64_t *)w;
  w += (m * 8 + 255) & ~255ull;
  uint64_t *off = (uint64_t *)w;
  w += (m * 8 + 255) & ~255ull;
  hipLaunchKernelGGL(part_count, dim3((unsigned)n_tiles), dim3(kTileThreads), 0, s, keys, n, parts, dg, n_tiles, cnt);
  hipError_t e = hipGetLastError();
  if (e) return e;
  e = scan_exclusive_u64(cnt, off, m, nullptr, w, s);
  if (e) return e;
  hipLaunchKernelGGL((part_scatter<RowT, STABLE>), dim3((unsigned)n_tiles), dim3(kTileThreads), 0, s, keys, in_rows, n, parts,
                     dg, n_tiles, cnt, off, row_base, out_keys, out_rows, stride, status);
  if (out_counts) hipLaunchKernelGGL(part_totals, dim3(1), dim3(64), 0, s, cnt, off, parts, n_tiles, out_counts);
  return hipGetLastError();
}

uint32_t log2u(uint64_t x) {
  uint32_t l = 0;
  while ((1ull << l) < x) ++l;
  return l;
}

}  // namespace

size_t partition_workspace(uint64_t n, uint32_t parts) { return pass_workspace(n, parts); }

hipError_t launch_partition(const int64_t *keys, uint64_t n, uint32_t parts, uint64_t row_base, int64_t *out_keys,
                            uint64_t *out_rows, uint64_t *out_counts, void *ws, hipStream_t s) {
  const uint32_t lp = log2u(parts);
  const Digit dg{lp == 0 ? 64u : 64u - lp, parts - 1};
  return split_pass<uint64_t, true>(keys, nullptr, n, parts, dg, row_base, out_keys, out_rows, out_counts, ws, s);
}

hipError_t launch_partition_fixed(const int64_t *keys, uint64_t n, uint32_t parts, uint32_t row_base, uint64_t seg_cap,
                                  int64_t *out_keys, uint32_t *out_rows, uint64_t *out_counts, uint32_t *status,
                                  void *ws, hipStream_t s) {
  const uint32_t lp = log2u(parts);
  const Digit dg{lp == 0 ? 64u : 64u - lp, parts - 1};
  // order inside a destination segment does not matter to the probe: rank with LDS atomics
  return split_pass<uint32_t, false>(keys, nullptr, n, parts, dg, row_base, out_keys, out_rows, out_counts, ws, s,
                                     seg_cap, status);
}

namespace {
// cursors[seg_cursor_index(parts, g, d)] (u32, group-major, group stride max(parts, 32)) ->
// counts[d * 8 + g] (u64, destination-major)
__global__ void grouped_counts(const uint32_t *cur, uint32_t parts, uint64_t *out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < parts * 8) out[i] = cur[seg_cursor_index(parts, i % 8, i / 8)];
}
}  // namespace

// cursors, then the pipelined split's sink
static size_t grouped_cursor_bytes(uint32_t parts) { return (split_cursor_count(parts) * 4 + 255) & ~(size_t)255; }
size_t partition_grouped_workspace(uint32_t parts) { return grouped_cursor_bytes(parts) + kSplitSinkBytes; }

uint64_t partition_grouped_sub_cap(uint64_t n, uint32_t parts, uint32_t chunk) {
  // tile group g takes tiles [g * n_tiles / 8, (g + 1) * n_tiles / 8): at most ceil(n_tiles / 8)
  const uint64_t tile = slot_split_tile_keys(parts), n_tiles = (n + tile - 1) / tile;
  const uint64_t g_rows = std::min<uint64_t>(n, (n_tiles + 7) / 8 * tile);
  const double m = (double)g_rows / parts;
  const uint64_t c = (uint64_t)(m + 8.0 * std::sqrt(m) + chunk);
  return chunk ? (c + chunk - 1) / chunk * chunk : c;
}

static hipError_t launch_owner_split_small(const int64_t *keys, uint64_t n, uint32_t parts, uint32_t shift,
                                          uint64_t sub_cap, uint32_t *cur, int64_t *out_keys, uint32_t *out_rows,
                                          uint32_t *status, uint32_t row_base, void *sink, hipStream_t s,
                                          uint32_t self_last);

hipError_t launch_partition_grouped(const int64_t *keys, uint64_t n, uint32_t parts, uint32_t row_base,
                                    uint64_t sub_cap, int64_t *out_keys, uint32_t *out_rows, uint64_t *out_counts,
                                    uint32_t *status, void *ws, hipStream_t s, uint32_t self_last) {
  // the slot split's one-pass kernel with partition = the owner (top log2(parts) hash bits) and no
  // overflow area: a sub-segment that overflows drops rows and raises CCJ_FLAG_PART_OVERFLOW
  SlotPlan pl{};
  pl.lo_bits = log2u(parts);
  pl.hi_bits = 0;
  const uint32_t shift = parts > 1 ? 64u - pl.lo_bits : 0u;
  uint32_t *cur = (uint32_t *)ws;
  // Half the CUs: the multi-GPU step runs this beside the previous batch's all-to-all and the
  // local probe, and a persistent one-workgroup-per-CU grid would hold every CU (its LDS).
  static const uint32_t half = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return (uint32_t)(n >= 16 ? n / 16 * 8 : 8);
  }();
  const uint32_t wgs = (uint32_t)ccj_tune_int("CCJ_OWNER_WGS", (int)half);
  hipError_t e;
  if (ccj_tune_int("CCJ_OWNER_SMALL", 1) && parts <= 64) {
    e = launch_owner_split_small(keys, n, parts, shift, sub_cap, cur, out_keys, out_rows, status, row_base,
                                 (char *)ws + grouped_cursor_bytes(parts), s, self_last);
  } else {
    e = launch_slot_split_fixed(keys, n, pl, sub_cap, 0, 0, 0, cur, out_keys, out_rows, status, s, nullptr, 0,
                                nullptr, nullptr, row_base, shift, wgs, (char *)ws + grouped_cursor_bytes(parts),
                                self_last);
  }
  if (e) return e;
  hipLaunchKernelGGL(grouped_counts, dim3((parts * 8 + 255) / 256), dim3(256), 0, s, cur, parts, out_counts);
  return hipGetLastError();
}

namespace {
// Chunk counts of fixed-capacity segments: segment g holds counts[g] live rows at the front of its
// seg_cap slots; chunk j of segment g is rows [j*chunk, (j+1)*chunk) of it.
__global__ void seg_chunk_counts(const uint64_t *counts, uint32_t n_segs, uint64_t seg_cap, uint32_t chunk,
                                 uint32_t *out, uint32_t *status) {
  const uint64_t per = seg_cap / chunk;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= per * n_segs) return;
  const uint64_t g = i / per, j = i - g * per;
  uint64_t live = counts[g];
  if (live > seg_cap) {
    if (j == 0 && status) atomicOr(status, CCJ_FLAG_CAP_OVERFLOW);
    live = seg_cap;
  }
  const uint64_t lo = j * chunk;
  out[i] = live <= lo ? 0u : (uint32_t)(live - lo < chunk ? live - lo : chunk);
}
}  // namespace

hipError_t launch_segment_chunk_counts(const uint64_t *counts, uint32_t n_segs, uint64_t seg_cap, uint32_t chunk,
                                       uint32_t *out, uint32_t *status, hipStream_t s) {
  const uint64_t n = seg_cap / chunk * n_segs;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(seg_chunk_counts, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, counts, n_segs, seg_cap,
                     chunk, out, status);
  return hipGetLastError();
}

// ---- slot-range partitioning for the L2-resident probe ------------------------------------------
SlotPlan slot_plan(uint64_t table_size, int kind) {
  // log2 slots of table per partition (the tuning build sweeps CCJ_WINDOW_BITS)
  const uint32_t wbits = (uint32_t)ccj_tune_int("CCJ_WINDOW_BITS", (int)kWindowBits);
  SlotPlan pl{};
  const uint32_t sbits = log2u(table_size);  // table_size is a power of two
  const uint32_t wb = kind == CCJ_TABLE_CHAIN && wbits > 0 ? wbits - 1 : wbits;
  pl.window_bits = wb < sbits ? wb : sbits;
  if (sbits - pl.window_bits > kSplitPartBits) pl.window_bits = sbits - kSplitPartBits;
  const uint32_t dbits = sbits - pl.window_bits;
  pl.lo_bits = (dbits + 1) / 2;  // exact form: two balanced LSD passes of <= 32 digits
  pl.hi_bits = dbits - pl.lo_bits;
  return pl;
}

// ---- one-pass fixed-capacity slot split (ccj_probe_partitioned's default form) -----------------
//
// Every probe key goes to segment (partition d, tile group g) = position range
// [(d*8 + g) * cap, (d*8 + g + 1) * cap): g = the XCD the tile's workgroup runs on, so each
// segment is written from one L2 only.  A persistent workgroup per CU walks its group's tiles
// (11264 keys); per tile it ranks the keys by partition with LDS atomics, reserves every
// partition's run in its segment with ONE device atomic per partition (group-major cursors, so a
// wave's 64 reservations are 256 contiguous bytes), builds the tile's image grouped by partition in
// LDS while those atomics fly, loads the next tile's keys into registers, and writes the runs out.
// One pass of 8 B read + 12 B written per key replaces the exact form's two count passes and two
// scatter passes (measured at C2: 6.5 ms vs 1.8 + 1.9 + 5.5 + 4.9 ms).  Runs that do not fit their
// segment are dropped and CCJ_FLAG_PART_OVERFLOW is raised: the caller re-runs with the exact form
// (only heavy key skew does this; cap leaves 8 standard deviations of room).
namespace {
constexpr int kSplitThreads = 1024;
#ifndef CCJ_SPLIT_PER_KEYS
#define CCJ_SPLIT_PER_KEYS 11
#endif
#ifndef CCJ_SPLIT_NARROW
#define CCJ_SPLIT_NARROW 0
#endif
// keys per thread of the pipelined split (CCJ_SPLIT_PER sweep at C2, round 1's fixed form: 8-13 keys
// -> 6.35 6.12 5.98 5.90 6.34 7.11 ms); the fixed form (slot_split_fixed) keeps 11
constexpr int kSplitPer = CCJ_SPLIT_PER_KEYS;
constexpr int kSplitPerFixed = 11;
// CCJ_SPLIT_NARROW: the pipelined split's image holds each entry's tile row in 16 bits and the
// stores re-derive its partition from the key (one hash more per key, 2 bytes less LDS per key)
constexpr bool kSplitNarrow = CCJ_SPLIT_NARROW != 0;
constexpr uint32_t kSplitParts = 1u << kSplitPartBits;
static_assert(kSplitParts <= (uint32_t)kSplitThreads, "one partition per thread in the scan");

// The owner split's partition -> slot map for the multi-GPU exchange: the rank's own partition
// (self_last) goes to the last slot and the partitions above it move down one, so the N - 1 peer
// segments are contiguous in rank order (one all-to-all with a zero self split) and the self
// segment sits after them, copied locally instead of through RCCL.  self_last >= parts: identity.
__device__ __forceinline__ uint32_t self_slot(uint32_t d, uint32_t self_last, uint32_t parts) {
  return d == self_last ? parts - 1u : d - (d > self_last ? 1u : 0u);
}

template <bool COUNTS, int THREADS, int MAXP, int PER>
__global__ __launch_bounds__(THREADS) void slot_split_fixed(const int64_t *keys, uint64_t n, uint32_t shift,
                                                                 uint32_t parts, uint64_t n_tiles, uint32_t *cur,
                                                                 uint64_t cap, uint64_t ovf_base, uint64_t ovf_cap,
                                                                 int64_t *out_k, uint32_t *out_r, uint32_t *status,
                                                                 uint32_t ablate, const uint32_t *counts, uint32_t chunk,
                                                                 uint2 *runs, uint32_t *ovf_runs, uint32_t row_base,
                                                                 uint32_t self_last, uint32_t ovf_pg) {
  constexpr uint32_t kTileKeys = (uint32_t)THREADS * PER;
  static_assert(MAXP <= THREADS, "one partition per thread in the scan");
  __shared__ int64_t s_k[kTileKeys];
  __shared__ uint32_t s_ovf[MAXP], s_olim[MAXP];  // overflow-area run: start, length
  // image entry: tile-local row (low 16 bits) | partition << 16, so the write phase does not hash the
  // key again (C2: 5.57 ms against 6.03 with the second hash; tools/hashbench: 46 SIMD cycles per
  // wave-hash)
  __shared__ uint32_t s_i[kTileKeys];
  __shared__ uint32_t s_hist[MAXP], s_loc[MAXP], s_lim[MAXP];
  __shared__ uint64_t s_dst[MAXP];
  __shared__ uint32_t s_wsum[THREADS / 64], s_tot;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t g = blockIdx.x & 7u, bpg = gridDim.x >> 3;  // gridDim.x is a multiple of 8
  const uint32_t mask = parts - 1;
  // group g's tiles: [g * n_tiles / 8, (g + 1) * n_tiles / 8); this workgroup takes every bpg-th
  const uint64_t tend = (g + 1) * n_tiles / 8;
  uint64_t tile = g * n_tiles / 8 + (blockIdx.x >> 3);
  int64_t kk[PER];
  uint32_t live = 0;  // bit it: row it of this thread is in the column (counts: within its chunk's count)
  // COUNTS (fixed-capacity input segments: chunk c's first counts[c] rows are live): the counts of
  // a tile's chunks travel through LDS (thread j loads chunk c0 + j's beside the keys), so every key
  // load is unconditional and in flight at once — a per-row counts load ahead of a conditional key
  // load made each row a dependent round trip
  __shared__ uint32_t s_ccnt[COUNTS ? THREADS : 1];
  uint32_t cpre = 0;
  auto tile_rows = [&](uint64_t t) { return (uint32_t)(n - t * kTileKeys < kTileKeys ? n - t * kTileKeys : kTileKeys); };
  auto load = [&](uint64_t t) {
    const uint64_t t0 = t * kTileKeys;
    const uint32_t tn = tile_rows(t);
    live = 0;
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const uint32_t li = (uint32_t)it * THREADS + tid;
      const bool in = li < tn;
      if (!COUNTS) live |= (in ? 1u : 0u) << it;
      if CCJ_ABLATED(ablate, 0x20u) kk[it] = (int64_t)((t0 + li) * 0x9E3779B97F4A7C15ull >> 20);  // timing only: no key reads
      else kk[it] = __builtin_nontemporal_load(keys + t0 + (in ? li : 0u));
    }
    if (COUNTS) {
      const uint64_t c0 = t0 / chunk, nc = (t0 + tn - 1) / chunk - c0 + 1;
      cpre = tid < nc ? counts[c0 + tid] : 0u;
    }
  };
  if (tile < tend) load(tile);
  bool dropped = false;
  for (; tile < tend; tile += bpg) {
    const uint64_t t0 = tile * kTileKeys;
    if (COUNTS) s_ccnt[tid] = cpre;
    if (tid < MAXP) s_hist[tid] = 0;
    __syncthreads();
    if (COUNTS) {
      const uint32_t tn = tile_rows(tile);
      const uint64_t c0 = t0 / chunk;
      live = 0;
#pragma unroll
      for (int it = 0; it < PER; ++it) {
        const uint32_t li = (uint32_t)it * THREADS + tid;
        const uint64_t pos = t0 + li, c = pos / chunk;
        live |= (li < tn && pos - c * chunk < s_ccnt[c - c0] ? 1u : 0u) << it;
      }
    }
    uint32_t dd[PER], rk[PER];
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      dd[it] = self_slot((uint32_t)(murmurhash64((uint64_t)kk[it]) >> shift) & mask, self_last, parts);
      rk[it] = (live >> it) & 1u ? atomicAdd(&s_hist[dd[it]], 1u) : 0u;
    }
    __syncthreads();
    // thread tid owns partition tid: block-wide exclusive scan + the segment reservation
    const uint32_t h = tid < parts ? s_hist[tid] : 0u;
    uint32_t incl = wave_incl_scan(h);
    if (lane == 63) s_wsum[wave] = incl;
    uint32_t r = h && !CCJ_ABLATED(ablate, 0x40u) ? atomicAdd(&cur[seg_cursor_index(parts, g, tid)], h) : 0u;  // flies during the image build
    // (timing only, 0xC0: no reservation atomics, runs at their expected offsets: 9.5 ms, not less —
    // the atomics keep one segment's runs written close together in time, so its L2 merges them)
    if CCJ_ABLATED(ablate, 0x80u) r = (uint32_t)(((tile - g * n_tiles / 8) * (kTileKeys / parts)) % cap);
    __syncthreads();
    uint32_t wpre = 0;
    for (uint32_t w = 0; w < wave; ++w) wpre += s_wsum[w];
    if (tid < parts) s_loc[tid] = wpre + incl - h;
    if (tid == THREADS - 1) s_tot = wpre + incl;  // rows in the image (live rows of the tile)
    __syncthreads();
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const uint32_t li = (uint32_t)it * THREADS + tid;
      if ((live >> it) & 1u) {
        const uint32_t pos = s_loc[dd[it]] + rk[it];
        s_k[pos] = kk[it];
        s_i[pos] = li | dd[it] << 16;
      }
    }
    if (tid < parts) {
      const uint64_t seg = (uint64_t)tid * 8 + g;
      const uint32_t lim = r >= cap ? 0u : (uint32_t)(cap - r < h ? cap - r : h);
      s_dst[tid] = seg * cap + r;
      s_lim[tid] = lim;
      uint32_t olim = 0, r2 = 0;
      if (lim < h) {  // the rest of the run goes to one of group g's overflow sub-areas (key skew)
        const uint32_t extra = h - lim;
        if (ovf_cap) {
          const uint32_t sub = g * ovf_pg + (tid + (blockIdx.x >> 3)) % ovf_pg;
          r2 = atomicAdd(&cur[ovf_cursor_index(parts, sub)], extra);
          olim = r2 >= ovf_cap ? 0u : (uint32_t)(ovf_cap - r2 < extra ? ovf_cap - r2 : extra);
          r2 += sub * (uint32_t)ovf_cap;
        }
        dropped |= olim < extra;
      }
      s_ovf[tid] = r2;
      s_olim[tid] = olim;
      if (runs) {  // where this tile's rows of partition tid went (the ordered probe maps them back)
        runs[tile * parts + tid] = make_uint2((uint32_t)(seg * cap + r), lim | olim << 16);
        if (olim) ovf_runs[tile * parts + tid] = (uint32_t)(ovf_base + r2);
      }
    }
    __syncthreads();
    if (tile + bpg < tend) load(tile + bpg);  // next tile's keys arrive while this one is written
    // (An unrolled write loop with a fixed store count, so that the next tile's keys are awaited
    // with vmcnt(2 * PER) and these stores drain under the next tile's ranking, measured 7.8 ms
    // against 5.6: the reservation atomics then queue behind the stores.)
    const uint32_t tl = s_tot;  // rows in the image
    for (uint32_t q = tid; q < tl; q += THREADS) {
      const int64_t k = s_k[q];
      const uint32_t si = s_i[q], d = si >> 16;
      const uint32_t o = q - s_loc[d];
      const uint32_t lim = s_lim[d];
      if (runs && !CCJ_ABLATED(ablate, 0x10u))
        // the ordered probe: the row inside its tile (16 bits) at the entry's IMAGE index t0 + q,
        // exactly as slot_split_pipe writes it (unsplit_words reads row_loc[t0 + j])
        reinterpret_cast<uint16_t *>(out_r)[t0 + q] = (uint16_t)(si & 0xFFFFu);
      if ((o < lim || o - lim < s_olim[d]) && !CCJ_ABLATED(ablate, 0x10u)) {  // (0x10: timing only, no stores)
        const uint64_t dest = o < lim ? s_dst[d] + o : ovf_base + s_ovf[d] + (o - lim);
        out_k[dest] = k;  // plain stores: the L2 merges neighbouring runs' partial lines
        if (!runs) out_r[dest] = row_base + (uint32_t)(t0 + (si & 0xFFFFu));  // (non-temporal stores measured the same)
      }
    }
    __syncthreads();
  }
  if (dropped && status) atomicOr(status, CCJ_FLAG_PART_OVERFLOW);
}

// A uniform value the compiler cannot fold (keeps the prologue's sink stores below real stores).
__device__ __forceinline__ uint32_t opaque_u32(uint32_t x) {
  asm volatile("" : "+s"(x));
  return x;
}
// A lane value the compiler must recompute from here on (rematerialises addresses derived from it).
__device__ __forceinline__ uint32_t opaque_v32(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

// slot_split_pipe: slot_split_fixed's tile work software-pipelined so that a tile's stores drain
// while the next tile is ranked.  Per iteration (tile t, the previous tile's image in LDS):
//   load keys of t + 1 | rank t (LDS atomics) | barrier | scan t + reservation atomics t |
//   store the previous tile's image | barrier | t's run table | barrier | t's image
// The keys of t + 1 and the reservation atomics are issued BEFORE the stores, so neither wait
// (vmcnt counts in issue order) has to drain the stores; every load and store is
// unconditional (a clamped tile, a per-XCD sink position for inactive lanes), so the waits the
// compiler derives are the same on every path (a prologue issues the sink stores of "tile -1").
// The sink: 64 positions at the end of the overflow area, or caller memory (kSplitSinkBytes).
template <bool COUNTS, int THREADS, int MAXP, int PER, bool RUNS>
__global__ __launch_bounds__(THREADS) void slot_split_pipe(const int64_t *keys, uint64_t n, uint32_t shift,
                                                                uint32_t parts, uint64_t n_tiles, uint32_t *cur,
                                                                uint64_t cap, uint64_t ovf_base, uint64_t ovf_cap,
                                                                int64_t *out_k, uint32_t *out_r, uint32_t *status,
                                                                const uint32_t *counts, uint32_t chunk, uint2 *runs,
                                                                uint32_t *ovf_runs, uint32_t row_base, int64_t *sink_k,
                                                                uint32_t *sink_r, uint32_t ablate, uint32_t self_last,
                                                                uint32_t ovf_pg) {
  constexpr uint32_t kTileKeys = (uint32_t)THREADS * PER;
  static_assert(MAXP <= THREADS, "one partition per thread in the scan");
  static_assert(kTileKeys <= 65536u, "tile rows in 16 bits");
  using ImgT = typename std::conditional<kSplitNarrow, uint16_t, uint32_t>::type;
  __shared__ int64_t s_k[kTileKeys];
  __shared__ ImgT s_i[kTileKeys];  // tile-local row | partition << 16 (narrow: the row only)
  __shared__ uint32_t s_hist[MAXP], s_loc[MAXP];
  // per partition, for the stores: {dest - image index (u64), segment end, overflow end} (image
  // indices) and the overflow area's dest - image index: two LDS reads per stored key
  __shared__ uint4 s_rec[MAXP];
  __shared__ uint64_t s_oadj[MAXP];
  __shared__ uint32_t s_wsum[THREADS / 64], s_tot;
  __shared__ uint32_t s_ccnt[COUNTS ? THREADS : 1];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t g = blockIdx.x & 7u, bpg = gridDim.x >> 3;
  const uint32_t mask = parts - 1;
  const uint64_t tend = (g + 1) * n_tiles / 8;
  uint64_t tile = g * n_tiles / 8 + (blockIdx.x >> 3);
  if (tile >= tend) return;
  // a key's destination partition (the owner split's small forms — launch_owner_split_small only:
  // shift = 64 - log2(parts) or mask 0 — need only the hash's high word: one 32-bit product fewer)
  auto dest_of = [&](int64_t k) -> uint32_t {
    constexpr bool kOwnerHi = MAXP <= 64 && THREADS <= 512;
    const uint32_t d0 = CCJ_ABLATED(ablate, 0x2000u) ? (uint32_t)((uint64_t)k >> shift) & mask  // (timing: no hash)
                        : kOwnerHi ? (murmurhash64_hi((uint64_t)k) >> ((shift - 32u) & 31u)) & mask
                                   : (uint32_t)(murmurhash64((uint64_t)k) >> shift) & mask;
    if constexpr (MAXP <= 64) return self_slot(d0, self_last, parts);  // (the owner split: own rank's segment last)
    else return d0;
  };
  sink_k += g * 8;  // inactive lanes store here (8 positions per XCD group)
  sink_r += g * 8;
  if (tid < MAXP) s_hist[tid] = 0;
  auto tile_rows = [&](uint64_t t) { return (uint32_t)(n - t * kTileKeys < kTileKeys ? n - t * kTileKeys : kTileKeys); };
  auto load = [&](uint64_t t, int64_t(&kk)[PER], uint32_t &cp) {
    const uint64_t tt = t < tend ? t : tend - 1;  // the last prefetch re-reads a valid tile
    const uint64_t t0 = tt * kTileKeys;
    const uint32_t tn = tile_rows(tt);
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const uint32_t li = (uint32_t)it * THREADS + tid;
      if CCJ_ABLATED(ablate, 0x20u) kk[it] = (int64_t)((t0 + li) * 0x9E3779B97F4A7C15ull >> 20);  // (timing: no key reads)
      else kk[it] = __builtin_nontemporal_load(keys + t0 + (li < tn ? li : 0u));
    }
    if (COUNTS) {
      const uint64_t c0 = t0 / chunk, nc = (t0 + tn - 1) / chunk - c0 + 1;
      cp = counts[c0 + (tid < nc ? tid : 0u)];  // masked where used
    }
  };
  uint32_t have_prev = opaque_u32(0u), p_tl = 0;
  uint64_t p_t0 = 0;
  auto store_one = [&](int it) {
    {
      const uint32_t q = (uint32_t)it * THREADS + tid;
      const int64_t k = s_k[q];
      const uint32_t si = s_i[q], d = kSplitNarrow ? dest_of(k) : (si >> 16) & (uint32_t)(MAXP - 1);
      const uint4 rc = s_rec[d];
      const uint64_t oadj = s_oadj[d];
      const bool act = have_prev && q < p_tl && q < rc.w;
      const uint64_t dest = q < rc.z ? (rc.x | (uint64_t)rc.y << 32) + q : oadj + q;
      if CCJ_ABLATED(ablate, 0x10u) return;  // (timing: no stores)
      *(act ? out_k + dest : sink_k) = k;
      if constexpr (RUNS)  // the ordered probe: the row inside its tile (16 bits) at the entry's IMAGE index
        // (tile-major, sequential: the unsplit reads it with whole lines, not from the runs' partial ones)
        *(have_prev && q < p_tl ? reinterpret_cast<uint16_t *>(out_r) + p_t0 + q : reinterpret_cast<uint16_t *>(sink_r)) =
            (uint16_t)(si & 0xFFFFu);
      else
        *(act ? out_r + dest : sink_r) = row_base + (uint32_t)(p_t0 + (si & 0xFFFFu));
      __builtin_amdgcn_sched_barrier(0);  // keep the LDS reads of later entries below (registers)
    }
  };
  auto stores = [&]() {
#pragma unroll
    for (int it = 0; it < PER; ++it) store_one(it);
  };
  // The previous tile's first KS entries are stored between the rankings of this tile's keys, so
  // their issue overlaps the hash / LDS-atomic work; the rest after the segment reservations,
  // which they hide as before.  C2, same box, interleaved 3x: all stores after the reservations
  // 5.51-5.54 ms, KS = 7 4.76-4.77 (KS 4 / 10 on another box 4.90 / 4.94 against 4.84 at 7).
  // (-DCCJ_SPLIT_KS=k builds other values for A/B; 0 = all after the reservations.)
#ifndef CCJ_SPLIT_KS
#define CCJ_SPLIT_KS 7
#endif
#ifndef CCJ_SPLIT_KS_OWNER
#define CCJ_SPLIT_KS_OWNER 0  // (the owner split's ballot ranking: -DCCJ_SPLIT_KS_OWNER=k for A/B)
#endif
  constexpr int kKSw = MAXP > 64 ? CCJ_SPLIT_KS : CCJ_SPLIT_KS_OWNER;
  constexpr int kKS = kKSw < PER ? kKSw : 0;
#ifdef CCJ_SPLIT_STORES16
  // (timing only, an experiment build (-DCCJ_SPLIT_STORES16): the same bytes stored as 16-byte stores — two keys / four rows
  // per lane at their first entry's destination, rounded down to 16 bytes: wrong layout; does the
  // split's time follow its store-instruction count?)
  auto stores16 = [&]() {
    typedef long long i64x2 __attribute__((ext_vector_type(2)));
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int it = 0; it < (PER + 1) / 2; ++it) {
      const uint32_t q = 2u * ((uint32_t)it * THREADS + tid);
      const uint32_t qq = q < kTileKeys - 1 ? q : 0u;
      const i64x2 kv = {s_k[qq], s_k[qq + 1]};
      const uint32_t si = s_i[qq], d = (si >> 16) & (uint32_t)(MAXP - 1);
      const uint4 rc = s_rec[d];
      const bool act = have_prev && q + 1 < p_tl && q < rc.z;
      const uint64_t dest = ((rc.x | (uint64_t)rc.y << 32) + q) & ~1ull;
      *(act ? reinterpret_cast<i64x2 *>(out_k + dest) : reinterpret_cast<i64x2 *>(sink_k)) = kv;
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int it = 0; it < (PER + 3) / 4; ++it) {
      const uint32_t q = 4u * ((uint32_t)it * THREADS + tid);
      const uint32_t qq = q < kTileKeys - 3 ? q : 0u;
      const u32x4 rv = {s_i[qq] & 0xFFFFu, s_i[qq + 1] & 0xFFFFu, s_i[qq + 2] & 0xFFFFu, s_i[qq + 3] & 0xFFFFu};
      const uint32_t d = (s_i[qq] >> 16) & (uint32_t)(MAXP - 1);
      const uint4 rc = s_rec[d];
      const bool act = have_prev && q + 3 < p_tl && q < rc.z;
      const uint64_t dest = ((rc.x | (uint64_t)rc.y << 32) + q) & ~3ull;
      *(act ? reinterpret_cast<u32x4 *>(out_r + dest) : reinterpret_cast<u32x4 *>(sink_r)) = rv;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
#endif
  bool dropped = false;
  // partition ptid's store records from its reservation r, run length h and image offset loc
  auto records = [&](uint32_t ptid, uint32_t r, uint32_t h, uint32_t loc, uint64_t t) {
    const uint64_t seg = (uint64_t)ptid * 8 + g;
    const uint32_t lim = r >= cap ? 0u : (uint32_t)(cap - r < h ? cap - r : h);
    uint32_t olim = 0, r2 = 0;
    if (lim < h) {  // the rest of the run goes to one of group g's overflow sub-areas (key skew)
      const uint32_t extra = h - lim;
      if (ovf_cap) {
        const uint32_t sub = g * ovf_pg + (ptid + (blockIdx.x >> 3)) % ovf_pg;
        r2 = atomicAdd(&cur[ovf_cursor_index(parts, sub)], extra);
        olim = r2 >= ovf_cap ? 0u : (uint32_t)(ovf_cap - r2 < extra ? ovf_cap - r2 : extra);
        r2 += sub * (uint32_t)ovf_cap;  // (the sub-area's place in the overflow area)
      }
      dropped |= olim < extra;
    }
    const uint64_t dadj = seg * cap + r - loc;  // mod 2^64: + the image index gives the dest
    s_rec[ptid] = make_uint4((uint32_t)dadj, (uint32_t)(dadj >> 32), loc + lim, loc + lim + olim);
    s_oadj[ptid] = ovf_base + r2 - (loc + lim);
    if constexpr (RUNS) {  // (a compile-time switch: the C2 kernel carries no run-record state)
      runs[t * parts + ptid] = make_uint2((uint32_t)(seg * cap + r), lim | olim << 16);
      if (olim) ovf_runs[t * parts + ptid] = (uint32_t)(ovf_base + r2);
    }
  };
  auto step = [&](uint64_t t, int64_t(&kc)[PER], uint32_t cc, int64_t(&kn)[PER], uint32_t &cn) {
    load(t + bpg, kn, cn);  // kn held the previous tile's keys, already in its image: a whole step of latency
    if (kKS) __syncthreads();  // (the previous image is complete before any of it is stored)
    const uint64_t t0 = t * kTileKeys;
    const uint32_t tn = tile_rows(t);
    uint32_t live = 0;
    if (COUNTS) {
      const uint64_t c0 = t0 / chunk, nc = (t0 + tn - 1) / chunk - c0 + 1;
      s_ccnt[tid] = tid < nc ? cc : 0u;
      __syncthreads();
#pragma unroll
      for (int it = 0; it < PER; ++it) {
        const uint32_t li = (uint32_t)it * THREADS + tid;
        const uint64_t pos = t0 + li, c = pos / chunk;
        live |= (li < tn && pos - c * chunk < s_ccnt[c - c0] ? 1u : 0u) << it;
      }
    } else {
#pragma unroll
      for (int it = 0; it < PER; ++it) live |= ((uint32_t)it * THREADS + tid < tn ? 1u : 0u) << it;
    }
    uint32_t dr[PER];  // partition | rank in it << 10 (one register per key: no spills at 11 keys)
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const uint32_t d = dest_of(kc[it]);
      if constexpr (MAXP <= 64) {
        // few partitions (the owner split: one per rank): an LDS atomic per key would queue the
        // wave's 64 lanes on at most `parts` addresses (one address at N = 1).  Instead one ballot
        // per partition ranks the wave's keys, lane p adds partition p's wave count to s_hist[p]
        // (distinct addresses), and each lane takes its partition's base from that lane.
        const bool lv = (live >> it) & 1u;
        // bit-sliced: one ballot per partition-index bit; a lane's mask keeps the live lanes that
        // agree with its partition (mine) / with partition `lane` (pm) on every bit — log2(parts)
        // ballots instead of parts (owner split alone, 8 owners, ranking only: see DESIGN §5)
        uint64_t mine = __ballot(lv), pm = mine;
        for (uint32_t b = 0; (1u << b) < parts; ++b) {
          const uint64_t bb = __ballot((d >> b) & 1u);
          mine &= (d >> b) & 1u ? bb : ~bb;
          pm &= (lane >> b) & 1u ? bb : ~bb;
        }
        const uint32_t wcnt = (uint32_t)__popcll(pm);
        const uint32_t base = lane < parts && wcnt ? atomicAdd(&s_hist[lane], wcnt) : 0u;
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
        const uint32_t rk = (uint32_t)__shfl((int)base, (int)d) + below;
        dr[it] = d | (lv ? rk : 0u) << 10;
        if (it < kKS) store_one(it);
      } else {
        dr[it] = d | ((live >> it) & 1u ? atomicAdd(&s_hist[d], 1u) : 0u) << 10;
        if (it < kKS) store_one(it);
      }
    }
    __syncthreads();
    const uint32_t h = tid < parts ? s_hist[tid] : 0u;
    if (tid < MAXP) s_hist[tid] = 0;  // for the next tile (ranked after two more barriers)
    const uint32_t incl = wave_incl_scan(h);
    if (lane == 63) s_wsum[wave] = incl;
    uint32_t r = 0;
    if (h) {
      if CCJ_ABLATED(ablate, 0x100000u)  // (timing: no reservation atomics — each tile an expected-size run)
        r = (uint32_t)(((t - g * n_tiles / 8) * (kTileKeys / parts)) % (cap > 2 * kTileKeys ? cap - 2 * kTileKeys : 1));
      else
        r = atomicAdd(&cur[seg_cursor_index(parts, g, opaque_v32(tid))], h);  // awaited after the stores are issued
    }
#ifdef CCJ_SPLIT_STORES16
    stores16();
#else
    if (kKS) {
#pragma unroll
      for (int it = kKS; it < PER; ++it) store_one(it);
    } else {
      stores();
    }
#endif
    __syncthreads();  // the previous image is read; s_wsum is complete
    uint32_t wpre = 0;
    for (uint32_t w = 0; w < wave; ++w) wpre += s_wsum[w];
    const uint32_t ptid = opaque_v32(tid);  // recomputed addresses instead of registers held all loop
    if (ptid < parts) {
      const uint32_t loc = wpre + incl - h;
      s_loc[tid] = loc;
      // (round 5: this step's records from the previous step's reservation, so that the atomic's
      // round trip hides under the image scatter — C2 split 4.94 / 4.93 -> 4.97 / 4.97 ms at 11 keys
      // per thread, where carrying (r, h, loc) across the step spilled; not kept)
      records(ptid, r, h, loc, t);
    }
    if (tid == THREADS - 1) s_tot = wpre + incl;
    __syncthreads();
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      if (((live >> it) & 1u) && !CCJ_ABLATED(ablate, 0x200000u)) {  // (timing: 0x200000 no image scatter)
        const uint32_t d = dr[it] & 1023u;
        const uint32_t pos = s_loc[d] + (dr[it] >> 10);
        s_k[pos] = kc[it];
        s_i[pos] = (ImgT)(((uint32_t)it * THREADS + tid) | (kSplitNarrow ? 0u : d << 16));
      }
    }
    p_tl = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tot);
    p_t0 = t0;
    have_prev = 1u;
  };
  if CCJ_ABLATED(ablate, 0x200000u) {  // (timing, no image scatter: every image entry names partition 0,
    // whose run bounds every store, so the stale image stays inside reserved space)
    for (uint32_t q = tid; q < kTileKeys; q += THREADS) {
      s_k[q] = 0;
      s_i[q] = (ImgT)(q & 0xFFFFu);
    }
  }
  int64_t kA[PER], kB[PER];
  uint32_t cA = 0, cB = 0;
  load(tile, kA, cA);
  stores();  // "tile -1": all to the sink, so the loop is entered with the waits it has inside
  for (;;) {
    step(tile, kA, cA, kB, cB);
    tile += bpg;
    if (tile >= tend) break;
    step(tile, kB, cB, kA, cA);
    tile += bpg;
    if (tile >= tend) break;
  }
  __syncthreads();
  stores();
  if (dropped && status) atomicOr(status, CCJ_FLAG_PART_OVERFLOW);
}

// owner_split_direct: the owner split (<= 64 destinations) without the workgroup's tile image.
// Per tile:
//   rank (ATOM: an LDS atomic on the wave's counter of the key's destination; else one ballot per
//   destination-index bit, the wave's running count of destination p in lane p) | the wave's
//   64 x PER keys written to its own LDS image in destination order | barrier |
//   one reservation atomic per destination for the workgroup's whole run, split into the waves'
//   runs | barrier | each wave stores its image in order
// A wave's image holds whole runs of ~64 x PER / parts keys, as slot_split_pipe's image does for
// the workgroup — but it is the wave's own (written and read back by the same wave: no barrier
// guards it), and there are two barriers per tile instead of four.  (Round 5: lanes storing their
// keys where they rank, with no image — 8-key pieces per store instruction — measured slower,
// 0.182-0.197 against 0.165 ms per 2^25 keys.)  Same tiles, tile groups and segment layout as
// slot_split_pipe's small form (partition_grouped_sub_cap sizes them); the order inside a
// segment is free ("in any order").  Inactive lanes store to the per-XCD sink, so every store is
// unconditional (as in the pipe).
template <int PER, bool ATOM>
__global__ __launch_bounds__(256) void owner_split_direct(const int64_t *keys, uint64_t n, uint32_t shift,
                                                          uint32_t parts, uint64_t n_tiles, uint32_t *cur,
                                                          uint64_t cap, int64_t *out_k, uint32_t *out_r,
                                                          uint32_t *status, uint32_t row_base, int64_t *sink_k,
                                                          uint32_t *sink_r, uint32_t self_last, uint32_t ablate) {
  constexpr uint32_t T = 256, kTile = T * PER, kWaves = T / 64, kWaveKeys = 64 * PER;
  __shared__ uint32_t s_cnt[kWaves][64];   // wave w's keys of destination p in this tile
  __shared__ uint32_t s_base[kWaves][64];  // their run's first position in segment (p, g)
  __shared__ int64_t s_wk[kWaves][kWaveKeys];   // the waves' images: key
  __shared__ uint32_t s_wr[kWaves][kWaveKeys];  // and row in the wave's block | destination << 16
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t g = blockIdx.x & 7u, bpg = gridDim.x >> 3;
  const uint32_t mask = parts - 1;
  const uint64_t tend = (g + 1) * n_tiles / 8;
  uint64_t tile = g * n_tiles / 8 + (blockIdx.x >> 3);
  if (tile >= tend) return;
  sink_k += g * 8;
  sink_r += g * 8;
  // wave w takes the tile's keys [w * 64 * PER, (w + 1) * 64 * PER): key it of lane L at it * 64 + L
  auto load = [&](uint64_t t, int64_t(&kk)[PER]) {
    const uint64_t tt = t < tend ? t : tend - 1;  // the last prefetch re-reads a valid tile
    const uint64_t i0 = tt * kTile + wave * kWaveKeys + lane;
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const uint64_t i = i0 + (uint32_t)it * 64u;
      kk[it] = __builtin_nontemporal_load(keys + (i < n ? i : 0u));
    }
  };
  bool dropped = false;
  int64_t kA[PER], kB[PER];
  auto step = [&](uint64_t t, int64_t(&kc)[PER], int64_t(&kn)[PER]) {
    load(t + bpg, kn);
    const uint64_t w0 = t * kTile + wave * kWaveKeys;  // the wave's first key
    uint32_t dr[PER];  // destination | rank in the wave's run << 8 (0xFFFFFFFF: no key)
    uint32_t cum = 0;  // lane p < parts: the wave's keys of destination p so far
    if (ATOM) {
      // ranks from LDS atomics on the wave's own counters (the LDS runs one wave's operations in
      // order: the zeroing lands before the adds, the adds before the read of the totals; the
      // previous tile's reservation read the counters before the barrier that ended it)
      if (lane < parts) s_cnt[wave][lane] = 0;
#pragma unroll
      for (int it = 0; it < PER; ++it) {
        const bool lv = w0 + (uint32_t)it * 64u + lane < n;
        const uint32_t d =
            self_slot((murmurhash64_hi((uint64_t)kc[it]) >> ((shift - 32u) & 31u)) & mask, self_last, parts);
        dr[it] = lv ? d | atomicAdd(&s_cnt[wave][d], 1u) << 8 : 0xFFFFFFFFu;
      }
      cum = lane < parts ? s_cnt[wave][lane] : 0u;
    } else {
#pragma unroll
      for (int it = 0; it < PER; ++it) {
        const bool lv = w0 + (uint32_t)it * 64u + lane < n;
        const uint32_t d =
            self_slot((murmurhash64_hi((uint64_t)kc[it]) >> ((shift - 32u) & 31u)) & mask, self_last, parts);
        uint64_t mine = __ballot(lv), pm = mine;
        for (uint32_t b = 0; (1u << b) < parts; ++b) {
          const uint64_t bb = __ballot((d >> b) & 1u);
          mine &= (d >> b) & 1u ? bb : ~bb;
          pm &= (lane >> b) & 1u ? bb : ~bb;
        }
        const uint32_t below =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
        const uint32_t pre = (uint32_t)__shfl((int)cum, (int)d);
        dr[it] = lv ? d | (pre + below) << 8 : 0xFFFFFFFFu;
        cum += (uint32_t)__popcll(pm);
      }
    }
    // lane p: destination p's offset in the wave image (wloc); the image's length (wtot)
    const uint32_t mine_cnt = lane < parts ? cum : 0u;
    const uint32_t incl = wave_incl_scan(mine_cnt);
    const uint32_t wloc = incl - mine_cnt, wtot = (uint32_t)__shfl((int)incl, 63);
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      // (the shuffle with every lane active: a lane reading an inactive lane's value gets 0)
      const uint32_t d = dr[it] & 63u;
      const uint32_t q = (uint32_t)__shfl((int)wloc, (int)d) + (dr[it] >> 8);
      if (dr[it] != 0xFFFFFFFFu) {
        s_wk[wave][q] = kc[it];
        s_wr[wave][q] = ((uint32_t)it * 64u + lane) | d << 16;
      }
    }
    if (!ATOM && lane < parts) s_cnt[wave][lane] = cum;
    __syncthreads();
    if (tid < parts) {
      uint32_t tot = 0;
#pragma unroll
      for (uint32_t w = 0; w < kWaves; ++w) tot += s_cnt[w][tid];
      uint32_t r = 0;
      if (tot) {
        if CCJ_ABLATED(ablate, 0x100000u)  // (timing: no reservation atomics)
          r = (uint32_t)(((t - g * n_tiles / 8) * (kTile / parts)) % (cap > 2 * kTile ? cap - 2 * kTile : 1));
        else
          r = atomicAdd(&cur[seg_cursor_index(parts, g, tid)], tot);
      }
#pragma unroll
      for (uint32_t w = 0; w < kWaves; ++w) {
        s_base[w][tid] = r;
        r += s_cnt[w][tid];
      }
    }
    __syncthreads();
    // lane p < parts: its run's base minus its image offset, so entry q of destination d is stored
    // at position base_d + q (mod 2^32).  (Round 6: each wave reserving its own runs, no barriers,
    // measured 0.156 -> 0.204 ms per 2^25 keys at 8 owners — runs of 64 keys instead of 256.)
    const uint32_t adj = lane < parts ? s_base[wave][lane] - wloc : 0u;
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const uint32_t q = (uint32_t)it * 64u + lane;
      const uint32_t e = s_wr[wave][q];
      const uint32_t d = (e >> 16) & 63u;
      const uint32_t base = (uint32_t)__shfl((int)adj, (int)d);  // (every lane active)
      const uint32_t pos = q < wtot ? base + q : 0xFFFFFFFFu;
      const bool act = pos < cap;
      dropped |= q < wtot && !act;
      const uint64_t dest = ((uint64_t)d * 8 + g) * cap + pos;
      if CCJ_ABLATED(ablate, 0x10u) continue;  // (timing: no stores)
      *(act ? out_k + dest : sink_k) = s_wk[wave][q];
      *(act ? out_r + dest : sink_r) = row_base + (uint32_t)(w0 + (e & 0xFFFFu));
    }
  };
  load(tile, kA);
  for (;;) {
    step(tile, kA, kB);
    tile += bpg;
    if (tile >= tend) break;
    step(tile, kB, kA);
    tile += bpg;
    if (tile >= tend) break;
  }
  if (dropped && status) atomicOr(status, CCJ_FLAG_PART_OVERFLOW);
}

}  // namespace

// The owner split (the multi-GPU step) in small workgroups: 256 threads and 2048-key tiles (~26 KB
// of LDS) instead of one 1024-thread, 149 KB workgroup per CU.  The step runs it beside the local
// probe: a workgroup that needs a whole CU's LDS waits until no walk workgroup is left on some CU,
// i.e. until the walk's ~3·10^5 workgroups have drained (round-3 kernel trace of the one-rank
// rehearsal: no partition ran during any walk), while 26 KB workgroups take the slots the walk's
// retiring workgroups free.  Persistent, kOwnerDirectPerCu per CU of the stream (a multiple of 8:
// one tile group per XCD; 87 VGPRs: 5 waves per SIMD).  owner_split_direct since round 5 (DESIGN
// §3.6: 0.177 -> 0.165 ms per 2^25 keys at 8 owners); the tuning build's CCJ_OWNER_DIRECT=0 runs
// round 4's form, slot_split_pipe's ballot-ranked small instantiation, for A/B.
constexpr uint32_t kOwnerDirectPerCu = 5;

static hipError_t launch_owner_split_small(const int64_t *keys, uint64_t n, uint32_t parts, uint32_t shift,
                                          uint64_t sub_cap, uint32_t *cur, int64_t *out_keys, uint32_t *out_rows,
                                          uint32_t *status, uint32_t row_base, void *sink, hipStream_t s,
                                          uint32_t self_last) {
  constexpr int kT = 256, kPer = 8;
  constexpr uint32_t kTile = (uint32_t)kT * kPer;
  hipError_t e = hipMemsetAsync(cur, 0, split_cursor_count(parts) * 4, s);
  if (e || n == 0) return e;
  const uint64_t n_tiles = (n + kTile - 1) / kTile;
  int64_t *sink_k = (int64_t *)sink;
  uint32_t *sink_r = (uint32_t *)((char *)sink + kSplitSinkBytes / 16 * 8);
  const uint32_t abl = (uint32_t)ccj_tune_int("CCJ_OWNER_ABLATE", 0);  // (timing ablations, tuning build)
  // per_cu = 0: one workgroup per tile (not persistent)
  const uint32_t per_cu = (uint32_t)ccj_tune_int("CCJ_OWNER_PER_CU", kOwnerDirectPerCu);
  uint64_t grid = per_cu ? (uint64_t)stream_cus(s) * per_cu / 8 * 8 : (n_tiles + 7) / 8 * 8;
  grid = grid < 8 ? 8 : grid;
  // ranks: LDS atomics from 4 destinations up (8 owners 0.161 -> 0.154 ms per 2^25 keys, same box,
  // profiles/r6_ab_owner_rank.log); one or two destinations by ballots (one owner: 64 lanes on one
  // counter made the atomics 0.144 -> 0.177 ms)
  const bool atom = parts >= 4 && ccj_tune_int("CCJ_OWNER_RANK", 1);
  // (Round 6, same box: 4096-key tiles — PER 16, 137 VGPRs, three workgroups per CU — 0.155 ->
  // 0.157 ms per 2^25 keys at 8 owners; not kept.)
  if (ccj_tune_int("CCJ_OWNER_DIRECT", 1) && atom)
    hipLaunchKernelGGL((owner_split_direct<kPer, true>), dim3((unsigned)grid), dim3(kT), 0, s, keys, n, shift, parts,
                       n_tiles, cur, sub_cap, out_keys, out_rows, status, row_base, sink_k, sink_r, self_last, abl);
  else if (ccj_tune_int("CCJ_OWNER_DIRECT", 1))
    hipLaunchKernelGGL((owner_split_direct<kPer, false>), dim3((unsigned)grid), dim3(kT), 0, s, keys, n, shift, parts,
                       n_tiles, cur, sub_cap, out_keys, out_rows, status, row_base, sink_k, sink_r, self_last, abl);
  else
    hipLaunchKernelGGL((slot_split_pipe<false, kT, 64, kPer, false>), dim3((unsigned)grid), dim3(kT), 0, s, keys, n,
                       shift, parts, n_tiles, cur, sub_cap, (uint64_t)0, (uint64_t)0, out_keys, out_rows, status,
                       nullptr, 0u, nullptr, nullptr, row_base, sink_k, sink_r, abl, self_last, 1u);
  return hipGetLastError();
}

uint64_t slot_seg_cap(uint64_t n, const SlotPlan &pl, uint32_t chunk) {
  const uint32_t parts = 1u << (pl.lo_bits + pl.hi_bits);
  const double m = (double)n / (8.0 * parts);
  // 6.25 % for the uneven key -> partition map of a finite key range, + 8 binomial sigmas
  const uint64_t c = (uint64_t)(m * 1.0625 + 8.0 * std::sqrt(m) + 256.0);
  return (c + chunk - 1) / chunk * chunk;
}

// keys per thread per tile: 11 (11264-key tiles, 149 KB of LDS with <= 512 partitions); 1024
// partitions leave room for 10 (the tuning build sweeps 10 / 11 below that)
static int split_per(uint32_t parts) {
  // (only 10 and 11 are instantiated below: any other value must not size the tiles)
  const int per = ccj_tune_int("CCJ_SPLIT_PER", kSplitPer) == 10 ? 10 : kSplitPer;
  return parts > kSplitParts / 2 ? 10 : per;
}

// With run records (the ordered probe) the pipelined split holds 10 keys per thread: at 11 its
// 128 VGPRs spill the run-record pointers, and every reload waits for the stores in flight.
uint32_t slot_split_tile_keys(uint32_t parts, bool runs) {
  return (uint32_t)kSplitThreads * (runs ? 10u : (uint32_t)split_per(parts));
}

hipError_t launch_slot_split_fixed(const int64_t *keys, uint64_t n, const SlotPlan &pl, uint64_t cap,
                                   uint64_t ovf_base, uint64_t ovf_cap, uint64_t ovf_sub, uint32_t *cursors, int64_t *out_keys,
                                   uint32_t *out_rows, uint32_t *status, hipStream_t s, const uint32_t *counts,
                                   uint32_t chunk, uint2 *runs, uint32_t *ovf_runs, uint32_t row_base,
                                   uint32_t shift, uint32_t wgs, void *sink, uint32_t self_last, uint32_t ovf_per_group) {
  const uint32_t ovf_pg = ovf_per_group ? ovf_per_group : 1u;
  const uint32_t parts = 1u << (pl.lo_bits + pl.hi_bits);
  // counts: a tile's chunks (tile / chunk + 2 at most) fit one count per thread
  if (counts && (chunk == 0 || slot_split_tile_keys(parts, runs != nullptr) / chunk + 2 > (uint32_t)kSplitThreads))
    return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(cursors, 0, split_cursor_count(parts) * 4, s);
  if (e || n == 0) return e;
  // One persistent 1024-thread workgroup per CU (<= 149 KB of LDS), a multiple of 8 (one tile group
  // per XCD).  Two 512-thread workgroups per CU on 6144-key tiles (same run length at 512
  // partitions, phases overlapping between the two) measured 7.8 ms against 6.5 at C2.
  static const unsigned cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return (unsigned)(n >= 8 ? n / 8 * 8 : 8);
  }();
  const uint32_t ablate = (uint32_t)ccj_tune_int("CCJ_ABLATE", 0);  // timing-only (tuning build)
  const int per = runs ? 10 : split_per(parts);
  const uint32_t tile = slot_split_tile_keys(parts, runs != nullptr);
  if (shift == ~0u) shift = pl.window_bits;  // the slot split: partition = home slot >> window bits
  const uint64_t n_tiles = (n + tile - 1) / tile;
  // wgs: leave CUs to kernels of other streams; a CU-masked stream: one workgroup per CU it may use
  // (a grid larger than that would run its last workgroups after the first ones: a persistent
  // grid's whole work again)
  if (!wgs) wgs = (uint32_t)ccj_tune_int("CCJ_SPLIT_WGS", 0);  // (tuning build: a smaller persistent grid)
  const uint32_t scus = std::max<uint32_t>(8u, stream_cus(s) / 8 * 8);
  const unsigned grid = std::min<unsigned>(wgs ? (wgs + 7) / 8 * 8 : cus, scus);
  // the pipelined form needs a sink for its inactive lanes' stores: 64 positions of the overflow
  // area (8 per XCD group), or the caller's kSplitSinkBytes
  if ((ovf_cap >= 128 || sink) && ccj_tune_int("CCJ_SPLIT_PIPE", 1)) {
    // (the kOvfSubs overflow sub-areas of ovf_sub positions end at least 64 positions before the area's end)
    const uint64_t oc = ovf_sub;
    // only the <= 64-partition instantiation (the owner split's) maps the own rank's partition last
    // (dest_of); refuse self_last for any other route rather than ignore it
    if (self_last < parts && (runs || parts > 64 || per != kSplitPer)) return hipErrorInvalidValue;
    int64_t *sink_k = sink ? (int64_t *)sink : out_keys + ovf_base + ovf_cap - 64;
    uint32_t *sink_r = sink ? (uint32_t *)((char *)sink + kSplitSinkBytes / 16 * 8) : out_rows + ovf_base + ovf_cap - 64;
#define CCJ_PIPE_LAUNCH(C, MAXP, P)                                                                                   \
  do {                                                                                                              \
    if (runs)                                                                                                       \
      hipLaunchKernelGGL((slot_split_pipe<C, kSplitThreads, MAXP, P, true>), dim3(grid), dim3(kSplitThreads), 0, s,  \
                         keys, n, shift, parts, n_tiles, cursors, cap, ovf_base, oc, out_keys, out_rows, status,     \
                         counts, chunk, runs, ovf_runs, row_base, sink_k, sink_r, ablate, self_last, ovf_pg);                \
    else                                                                                                            \
      hipLaunchKernelGGL((slot_split_pipe<C, kSplitThreads, MAXP, P, false>), dim3(grid), dim3(kSplitThreads), 0, s, \
                         keys, n, shift, parts, n_tiles, cursors, cap, ovf_base, oc, out_keys, out_rows, status,     \
                         counts, chunk, runs, ovf_runs, row_base, sink_k, sink_r, ablate, self_last, ovf_pg);                \
  } while (0)
#ifdef CCJ_TUNING
    // (tuning build: two workgroups per CU instead of one lock-stepped 1024-thread workgroup —
    // CCJ_SPLIT_T = 512: 512 threads x 10 keys; 1025: 1024 threads x 4 keys; both <= 76 KB of LDS)
    const int st = ccj_tune_int("CCJ_SPLIT_T", 1024);
    if ((st == 512 || st == 1025) && !runs && parts > 64 && parts <= kSplitParts / 2) {
      const uint32_t tk = st == 512 ? 512u * 10u : 1024u * 4u;
      const uint64_t nt = (n + tk - 1) / tk;
      const unsigned g2 = std::min<unsigned>(2 * grid, 2 * scus);
      if (st == 512) {
        if (counts)
          hipLaunchKernelGGL((slot_split_pipe<true, 512, kSplitParts / 2, 10, false>), dim3(g2), dim3(512), 0, s, keys, n,
                             shift, parts, nt, cursors, cap, ovf_base, oc, out_keys, out_rows, status, counts, chunk,
                             runs, ovf_runs, row_base, sink_k, sink_r, ablate, self_last, ovf_pg);
        else
          hipLaunchKernelGGL((slot_split_pipe<false, 512, kSplitParts / 2, 10, false>), dim3(g2), dim3(512), 0, s, keys,
                             n, shift, parts, nt, cursors, cap, ovf_base, oc, out_keys, out_rows, status, counts, chunk,
                             runs, ovf_runs, row_base, sink_k, sink_r, ablate, self_last, ovf_pg);
      } else {
        if (counts)
          hipLaunchKernelGGL((slot_split_pipe<true, 1024, kSplitParts / 2, 4, false>), dim3(g2), dim3(1024), 0, s, keys,
                             n, shift, parts, nt, cursors, cap, ovf_base, oc, out_keys, out_rows, status, counts, chunk,
                             runs, ovf_runs, row_base, sink_k, sink_r, ablate, self_last, ovf_pg);
        else
          hipLaunchKernelGGL((slot_split_pipe<false, 1024, kSplitParts / 2, 4, false>), dim3(g2), dim3(1024), 0, s, keys,
                             n, shift, parts, nt, cursors, cap, ovf_base, oc, out_keys, out_rows, status, counts, chunk,
                             runs, ovf_runs, row_base, sink_k, sink_r, ablate, self_last, ovf_pg);
      }
      return hipGetLastError();
    }
#endif
    if (parts <= 64 && !runs && per == kSplitPer) {  // the owner split: ballot ranking (above)
      if (counts) CCJ_PIPE_LAUNCH(true, 64, kSplitPer);
      else CCJ_PIPE_LAUNCH(false, 64, kSplitPer);
    } else if (parts > kSplitParts / 2) {
      if (counts) CCJ_PIPE_LAUNCH(true, kSplitParts, 10);
      else CCJ_PIPE_LAUNCH(false, kSplitParts, 10);
    } else if (per == 10) {
      if (counts) CCJ_PIPE_LAUNCH(true, kSplitParts / 2, 10);
      else CCJ_PIPE_LAUNCH(false, kSplitParts / 2, 10);
    } else {
      if (counts) CCJ_PIPE_LAUNCH(true, kSplitParts / 2, kSplitPer);
      else CCJ_PIPE_LAUNCH(false, kSplitParts / 2, kSplitPer);
    }
#undef CCJ_PIPE_LAUNCH
    return hipGetLastError();
  }
  // the fixed form: at most kSplitPerFixed keys per thread (its LDS holds 32-bit rows), own tile count
  const int fper = per < kSplitPerFixed ? per : kSplitPerFixed;
  const uint64_t f_tiles = (n + (uint64_t)kSplitThreads * fper - 1) / ((uint64_t)kSplitThreads * fper);
#define CCJ_SPLIT_LAUNCH(C, MAXP, P)                                                                              \
  hipLaunchKernelGGL((slot_split_fixed<C, kSplitThreads, MAXP, P>), dim3(grid), dim3(kSplitThreads), 0, s, keys, n,      \
                     shift, parts, f_tiles, cursors, cap, ovf_base, ovf_sub, out_keys, out_rows, status, ablate,         \
                     counts, chunk, runs, ovf_runs, row_base, self_last, ovf_pg)
  if (parts > kSplitParts / 2) {  // 1024 partitions: 10 keys per thread
    if (counts) CCJ_SPLIT_LAUNCH(true, kSplitParts, 10);
    else CCJ_SPLIT_LAUNCH(false, kSplitParts, 10);
  } else if (per == 10) {
    if (counts) CCJ_SPLIT_LAUNCH(true, kSplitParts / 2, 10);
    else CCJ_SPLIT_LAUNCH(false, kSplitParts / 2, 10);
  } else {
    if (counts) CCJ_SPLIT_LAUNCH(true, kSplitParts / 2, kSplitPerFixed);
    else CCJ_SPLIT_LAUNCH(false, kSplitParts / 2, kSplitPerFixed);
  }
#undef CCJ_SPLIT_LAUNCH
  return hipGetLastError();
}

size_t slot_partition_workspace(uint64_t n, const SlotPlan &pl) {
  if (pl.lo_bits == 0) return 256;
  // pass buffers (keys + u32 rows) + the larger of the two passes' count/scan scratch
  const size_t buf = ((n * 8 + 255) & ~255ull) + ((n * 4 + 255) & ~255ull);
  const size_t a = pass_workspace(n, 1u << pl.lo_bits);
  const size_t b = pl.hi_bits ? pass_workspace(n, 1u << pl.hi_bits) : 0;
  return buf + (a > b ? a : b);
}

hipError_t launch_slot_partition(const int64_t *keys, uint64_t n, const SlotPlan &pl, int64_t *out_keys,
                                 uint32_t *out_rows, void *ws, hipStream_t s) {
  if (pl.lo_bits == 0) return hipSuccess;
  char *w = (char *)ws;
  int64_t *tk = (int64_t *)w;
  w += (n * 8 + 255) & ~255ull;
  uint32_t *tr = (uint32_t *)w;
  w += (n * 4 + 255) & ~255ull;
  const Digit lo{pl.window_bits, (1u << pl.lo_bits) - 1};
  if (pl.hi_bits == 0)
    return split_pass<uint32_t, false>(keys, nullptr, n, 1u << pl.lo_bits, lo, 0, out_keys, out_rows, nullptr, w, s);
  const Digit hi{pl.window_bits + pl.lo_bits, (1u << pl.hi_bits) - 1};
  hipError_t e = split_pass<uint32_t, false>(keys, nullptr, n, 1u << pl.lo_bits, lo, 0, tk, tr, nullptr, w, s);
  if (e) return e;
  return split_pass<uint32_t, false>(tk, tr, n, 1u << pl.hi_bits, hi, 0, out_keys, out_rows, nullptr, w, s);
}

}  // namespace ccj
