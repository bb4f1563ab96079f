// ccj_pipeline.hip — the reference's multi-join pipeline (main.cpp:119-191) on the device.
//
// The reference runs ExecutePipeline depth-first: every Next result of join l is handed to join
// l+1 (through the compactor when one is configured) before join l produces its next result.
// Join l+1 therefore sees join l's results in a fixed order — input chunk by input chunk, Next by
// Next — and each compactor sees only its own join's stream.  So the same result comes out of a
// breadth-first schedule: join l probes all of its input chunks in one ccj probe launch, then its
// output is either
//   - concatenated (CCJ_COMPACT_NONE): every non-empty Next result becomes one input chunk of
//     join l+1 (rows packed back to back; chunk_base / out_base give each chunk its rows), or
//   - compacted (CCJ_COMPACT_FULL): ccj_compact's closed form of NaiveCompactor::Compact + Flush.
// The final level's output is the ResultCollector's table (main.cpp:125-128) in append order.

#include <memory>
#include <vector>

#include "ccj_internal.h"
#include "ccj_tuning.h"

namespace ccj {
namespace {

constexpr uint32_t kCarry = CCJ_MAX_COLS;  // carried columns per level (n_joins + joins so far)

struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t ensure(size_t n) {
    if (n <= bytes && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    const size_t want = n ? (n + 255) & ~(size_t)255 : 256;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) bytes = want;
    return e;
  }
  template <typename T>
  T *as() const {
    return static_cast<T *>(p);
  }
};

// Per chunk of a probe output: its matches and its non-empty Next results.
__global__ void level_sizes(const uint32_t *count, const uint32_t *rounds, const uint32_t *round_counts,
                            uint32_t max_rounds, uint64_t n_chunks, uint64_t *rows, uint64_t *segs) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_chunks) return;
  const uint32_t r = rounds[c] < max_rounds ? rounds[c] : max_rounds;
  uint64_t k = 0;
  for (uint32_t i = 0; i < r; ++i) k += round_counts[c * max_rounds + i] != 0;
  rows[c] = count[c];
  segs[c] = k;
}

__global__ void level_totals(const uint64_t *rows, const uint64_t *rows_pre, const uint64_t *segs,
                             const uint64_t *segs_pre, uint64_t n_chunks, uint64_t *tot) {
  tot[0] = rows_pre[n_chunks - 1] + rows[n_chunks - 1];
  tot[1] = segs_pre[n_chunks - 1] + segs[n_chunks - 1];
}

struct ConcatParams {
  const uint32_t *count, *sel, *rounds, *round_counts;
  const int64_t *payload;
  const uint64_t *chunk_base, *out_base;  // probe input geometry (NULL: c * chunk, c * cap)
  uint64_t n_chunks, cap;
  uint32_t max_rounds, chunk;
  const uint64_t *rows_pre, *segs_pre;
  uint32_t n_cols;
  uint64_t next_dup;  // max_dup of the next join's table (its per-row output bound)
  const int64_t *cols[kCarry];
  int64_t *out_cols[kCarry + 1];  // carried columns, then this join's payload
  uint64_t *seg_base, *seg_obase;
  uint32_t *seg_count;
};

// CCJ_COMPACT_NONE: one wave per probe chunk appends its matches (already in Next order) at
// rows_pre[c] — DataChunk::Append's gather of every carried column through the selection
// vector — and lane 0 emits one next-level chunk per non-empty Next result.
__global__ __launch_bounds__(256) void concat_rows(ConcatParams p) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t c = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= p.n_chunks) return;
  const uint64_t obase = p.out_base ? p.out_base[c] : c * p.cap;
  const uint64_t ibase = p.chunk_base ? p.chunk_base[c] : c * p.chunk;
  const uint32_t cnt = p.count[c];
  const uint64_t d0 = p.rows_pre[c];
  for (uint32_t j = lane; j < cnt; j += 64) {
    const uint64_t row = ibase + p.sel[obase + j];
    for (uint32_t q = 0; q < p.n_cols; ++q) p.out_cols[q][d0 + j] = p.cols[q][row];
    p.out_cols[p.n_cols][d0 + j] = p.payload[obase + j];
  }
  if (lane == 0 && p.seg_base) {
    const uint32_t r = p.rounds[c] < p.max_rounds ? p.rounds[c] : p.max_rounds;
    uint64_t k = p.segs_pre[c], acc = d0;
    for (uint32_t i = 0; i < r; ++i) {
      const uint32_t rc = p.round_counts[c * p.max_rounds + i];
      if (!rc) continue;
      p.seg_base[k] = acc;
      p.seg_count[k] = rc;
      if (p.seg_obase) p.seg_obase[k] = acc * p.next_dup;
      ++k;
      acc += rc;
    }
  }
}

__device__ __forceinline__ uint64_t fmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct SinkParams {
  const int64_t *cols[CCJ_MAX_JOINS];
  const int64_t *pay[CCJ_MAX_JOINS];
  uint32_t joins;
  uint64_t n;
};

__global__ __launch_bounds__(256) void pipeline_sink(SinkParams p, unsigned long long *acc) {
  uint64_t sum = 0, cnt = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t t = 0x51ED27ull;
    uint32_t k = 0;
    for (uint32_t j = 0; j < p.joins; ++j, ++k) t = fmix64(t ^ (uint64_t)p.cols[j][i]) + k;
    for (uint32_t l = 0; l < p.joins; ++l) {
      t = fmix64(t) + k++;  // column m of join l: never written, 0
      t = fmix64(t ^ (uint64_t)p.pay[l][i]) + k++;
    }
    sum += fmix64(t);
    ++cnt;
  }
  for (int d = 32; d > 0; d >>= 1) {
    sum += __shfl_xor(sum, d);
    cnt += __shfl_xor(cnt, d);
  }
  if ((threadIdx.x & 63u) == 0 && cnt) {
    atomicAdd(acc, (unsigned long long)cnt);
    atomicAdd(acc + 1, (unsigned long long)sum);
  }
}

// Result collection (DataCollection::AppendChunk, data_collection.cpp:10-21): chunk by chunk, the
// live rows of every column appended densely.  Needed after a threshold-gated compactor, whose
// pass-through chunks are not full.
__global__ void widen_counts(const uint32_t *c, uint64_t n, uint64_t *w) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) w[i] = c[i];
}

struct PackParams {
  const int64_t *src[kCarry + 1];
  int64_t *dst[kCarry + 1];
  uint32_t n_cols, chunk;
  uint64_t n_chunks;
  const uint32_t *counts;
  const uint64_t *pre;
};

__global__ __launch_bounds__(256) void dense_pack(PackParams p) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t c = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= p.n_chunks) return;
  const uint32_t n = p.counts[c];
  const uint64_t d0 = p.pre[c], s0 = c * p.chunk;
  for (uint32_t q = 0; q < p.n_cols; ++q)
    for (uint32_t j = lane; j < n; j += 64) p.dst[q][d0 + j] = p.src[q][s0 + j];
}

size_t scan_bytes(uint64_t n) { return scan_u64_temp_bytes(n); }

}  // namespace
}  // namespace ccj

struct ccj_pipeline {
  struct Level {
    ccj::DevBuf count, sel, payload, rounds, round_counts;  // probe output of this join
    ccj::DevBuf rows, rows_pre, segs, segs_pre, scan_tmp;   // sizes
    ccj::DevBuf cols[ccj::kCarry + 1];                      // this join's output rows (next input)
    ccj::DevBuf next_counts, seg_base, seg_obase;           // next join's chunks
    ccj::DevBuf compact_ws;
    ccj::DevBuf ordered_ws;  // ccj_probe_ordered's workspace (large tables)
  };
  std::vector<const ccj_table *> tables;
  uint32_t joins = 0, chunk = 0;
  int mode = CCJ_COMPACT_NONE;
  std::vector<std::unique_ptr<Level>> lv;
  std::vector<uint32_t> thresholds;  // CCJ_COMPACT_FULL pass-through threshold per join (0 = chunk)
  ccj::DevBuf tot;  // [0] rows, [1] segments, [2] compact out chunks, [3] status
  ccj::DevBuf res_cols[2 * CCJ_MAX_JOINS], pack_w, pack_pre, pack_tmp;  // dense result after gated compaction
  hipEvent_t ev[CCJ_MAX_JOINS + 1] = {};
  ~ccj_pipeline() {
    for (auto e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};

namespace {
#define PL_TRY(expr, what)                                                                        \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess)                                                                         \
      return ccj::api_fail(e_ == hipErrorOutOfMemory ? CCJ_ERR_OOM : CCJ_ERR_HIP,                 \
                           std::string(what) + ": " + hipGetErrorString(e_));                     \
  } while (0)
}  // namespace

extern "C" int ccj_pipeline_create(const ccj_table *const *tables, uint32_t n_joins, uint32_t chunk, int compact_mode,
                                   ccj_pipeline **out) {
  if (!out || !tables) return ccj::api_fail(CCJ_ERR_INVALID, "ccj_pipeline_create: null argument");
  *out = nullptr;
  if (n_joins == 0 || n_joins > CCJ_MAX_JOINS) return ccj::api_fail(CCJ_ERR_INVALID, "ccj_pipeline_create: n_joins must be 1..8");
  if (chunk == 0 || chunk > ccj::kMaxChunk) return ccj::api_fail(CCJ_ERR_INVALID, "ccj_pipeline_create: chunk must be 1..2048");
  if (compact_mode != CCJ_COMPACT_NONE && compact_mode != CCJ_COMPACT_FULL)
    return ccj::api_fail(CCJ_ERR_INVALID, "ccj_pipeline_create: bad compact mode");
  for (uint32_t l = 0; l < n_joins; ++l)
    if (!tables[l]) return ccj::api_fail(CCJ_ERR_INVALID, "ccj_pipeline_create: null table");
  if (int rc = ccj::api_check_device()) return rc;
  auto *pl = new (std::nothrow) ccj_pipeline;
  if (!pl) return ccj::api_fail(CCJ_ERR_OOM, "ccj_pipeline_create: out of host memory");
  pl->tables.assign(tables, tables + n_joins);
  pl->joins = n_joins;
  pl->chunk = chunk;
  pl->mode = compact_mode;
  for (uint32_t l = 0; l < n_joins; ++l) pl->lv.emplace_back(new ccj_pipeline::Level);
  pl->thresholds.assign(n_joins, 0);
  for (uint32_t l = 0; l <= n_joins; ++l) {
    if (hipEventCreate(&pl->ev[l]) != hipSuccess) {
      delete pl;
      return ccj::api_fail(CCJ_ERR_HIP, "ccj_pipeline_create: hipEventCreate failed");
    }
  }
  *out = pl;
  return CCJ_OK;
}

extern "C" int ccj_pipeline_set_thresholds(ccj_pipeline *pl, const uint32_t *thresholds) {
  if (!pl) return ccj::api_fail(CCJ_ERR_INVALID, "ccj_pipeline_set_thresholds: null pipeline");
  for (uint32_t l = 0; l < pl->joins; ++l) pl->thresholds[l] = thresholds ? thresholds[l] : 0;
  return CCJ_OK;
}

extern "C" int ccj_pipeline_free(ccj_pipeline *pl) {
  delete pl;
  return CCJ_OK;
}

extern "C" int ccj_pipeline_run(ccj_pipeline *pl, const int64_t *const *d_cols, uint64_t n_rows, ccj_stream stream,
                                ccj_pipeline_result *res) {
  if (!pl || !res || (n_rows && !d_cols)) return ccj::api_fail(CCJ_ERR_INVALID, "ccj_pipeline_run: null argument");
  const uint32_t J = pl->joins, B = pl->chunk;
  for (uint32_t j = 0; j < J && n_rows; ++j)
    if (!d_cols[j]) return ccj::api_fail(CCJ_ERR_INVALID, "ccj_pipeline_run: null column");
  if (n_rows >= (1ull << 40)) return ccj::api_fail(CCJ_ERR_LIMIT, "ccj_pipeline_run: too many rows");
  *res = ccj_pipeline_result{};
  hipStream_t s = (hipStream_t)stream;
  PL_TRY(pl->tot.ensure(4 * sizeof(uint64_t)), "alloc");
  uint64_t *tot = pl->tot.as<uint64_t>();

  // Input of the current join.
  const int64_t *in_cols[ccj::kCarry] = {};
  for (uint32_t j = 0; j < J; ++j) in_cols[j] = n_rows ? d_cols[j] : nullptr;
  uint32_t in_ncols = J;
  uint64_t in_rows = n_rows, in_chunks = (n_rows + B - 1) / B;
  uint64_t in_phys = n_rows;  // physical extent of the input columns (chunk-major after compaction)
  const uint32_t *in_counts = nullptr;       // NULL: every physical row of the chunk
  const uint64_t *in_base = nullptr, *in_obase = nullptr;

  PL_TRY(hipEventRecord(pl->ev[0], s), "event");
  uint32_t levels_run = 0;
  bool gaps = false;           // the last compaction left pass-through chunks that are not full
  uint64_t last_out_chunks = 0;
  for (uint32_t l = 0; l < J; ++l) {
    res->chunks_in[l] = in_chunks;
    res->rows_in[l] = in_rows;
    if (in_chunks == 0) break;
    levels_run = l + 1;
    ccj_pipeline::Level &L = *pl->lv[l];
    const ccj_table *t = pl->tables[l];
    const uint64_t dup = t->info.max_dup ? t->info.max_dup : 1;
    const uint32_t R = t->info.max_rounds + 1;
    const uint64_t cap = (uint64_t)B * dup;
    const uint64_t out_slots = in_obase ? in_rows * dup : in_chunks * cap;
    PL_TRY(L.count.ensure(in_chunks * 4), "alloc");
    PL_TRY(L.rounds.ensure(in_chunks * 4), "alloc");
    PL_TRY(L.round_counts.ensure(in_chunks * R * 4), "alloc");
    PL_TRY(L.sel.ensure(out_slots * 4), "alloc");
    PL_TRY(L.payload.ensure(out_slots * 8), "alloc");
    PL_TRY(hipMemsetAsync(tot + 3, 0, 8, s), "memset");

    ccj::ProbeParams p{};
    p.table = t->d_table;
    p.off = t->d_off;
    p.bucket = reinterpret_cast<const longlong2 *>(t->d_bucket);
    p.bucket8 = nullptr;  // the chunk probe reads the 16-byte records (round 0's candidate inside)
    p.mask = (uint32_t)(t->info.size - 1);
    p.keys = in_cols[l];
    p.counts = in_counts;
    p.n_rows = in_phys;
    p.n_chunks = in_chunks;
    p.chunk = B;
    p.max_rounds = R;
    p.cap = cap;
    p.out_count = L.count.as<uint32_t>();
    p.out_sel = L.sel.as<uint32_t>();
    p.out_payload = L.payload.as<int64_t>();
    p.out_rounds = L.rounds.as<uint32_t>();
    p.out_round_counts = L.round_counts.as<uint32_t>();
    p.status = (uint32_t *)(tot + 3);
    p.chunk_base = in_base;
    p.out_base = in_obase;
    // Tables past L2 / the Infinity Cache (>= 2^22 slots or buckets) and inputs of whole chunks
    // (the first join, or compacted chunks): ccj_probe_ordered — the same per-Next outputs as the
    // chunk probe, through the slot / bucket partitioned layout, so the table reads are L2 hits
    // instead of random HBM lines.  Its rare skew overflow re-runs the chunk probe.  Only where the
    // input fills the split's fixed-capacity segments (positions <= 4/3 rows): a short input spread over
    // many partitions walks mostly empty chunks (2^25 LHS rows per join, same box: 2^25-key tables
    // 5.68 / 5.27 ms per pipeline step against 6.24 / 5.36 for chaining / LP, but 2^27-key tables
    // 7.19 / 6.00 against 6.63 / 5.66 — positions 1.5 x rows there).
    const size_t ows = in_base || in_obase ? 0 : ccj_probe_ordered_workspace_size(t, in_phys, B);
    const bool dense = ows && ccj_probe_partitioned_positions(t, in_phys, B) * 3 <= in_phys * 4;
    const bool ordered = dense && ccj_tune_int("CCJ_PIPE_ORDERED", 1);
    if (ordered) {
      PL_TRY(L.ordered_ws.ensure(ows), "alloc");
      ccj_probe_args a{};
      a.keys = p.keys;
      a.counts = in_counts;
      a.n_rows = in_phys;
      a.chunk = B;
      a.max_rounds = R;
      a.cap = cap;
      a.out_count = p.out_count;
      a.out_sel = p.out_sel;
      a.out_payload = p.out_payload;
      a.out_rounds = p.out_rounds;
      a.out_round_counts = p.out_round_counts;
      a.status = p.status;
      if (int rc = ccj_probe_ordered(t, &a, L.ordered_ws.p, L.ordered_ws.bytes, stream)) return rc;
    } else {
      PL_TRY(ccj::launch_probe(t->info.kind, p, s), "pipeline probe");
    }

    // Output sizes: matches and non-empty Next results, per chunk and in total (one D2H copy and
    // synchronisation per join; the ordered route's skew-overflow flag rides in the same copy, so
    // it costs a second one only when it fired: the chunk probe re-runs, the sizes are recomputed).
    PL_TRY(L.rows.ensure(in_chunks * 8), "alloc");
    PL_TRY(L.rows_pre.ensure(in_chunks * 8), "alloc");
    PL_TRY(L.segs.ensure(in_chunks * 8), "alloc");
    PL_TRY(L.segs_pre.ensure(in_chunks * 8), "alloc");
    size_t tb = ccj::scan_bytes(in_chunks);
    PL_TRY(L.scan_tmp.ensure(tb), "alloc");
    uint64_t h[4];
    auto sizes = [&]() -> int {
      const unsigned g = (unsigned)((in_chunks + 255) / 256);
      hipLaunchKernelGGL(ccj::level_sizes, dim3(g), dim3(256), 0, s, p.out_count, p.out_rounds, p.out_round_counts, R,
                         in_chunks, L.rows.as<uint64_t>(), L.segs.as<uint64_t>());
      PL_TRY(hipGetLastError(), "level sizes");
      PL_TRY(ccj::scan_exclusive_u64(L.rows.as<uint64_t>(), L.rows_pre.as<uint64_t>(), in_chunks, nullptr, L.scan_tmp.p, s),
             "scan");
      PL_TRY(ccj::scan_exclusive_u64(L.segs.as<uint64_t>(), L.segs_pre.as<uint64_t>(), in_chunks, nullptr, L.scan_tmp.p, s),
             "scan");
      hipLaunchKernelGGL(ccj::level_totals, dim3(1), dim3(1), 0, s, L.rows.as<uint64_t>(), L.rows_pre.as<uint64_t>(),
                         L.segs.as<uint64_t>(), L.segs_pre.as<uint64_t>(), in_chunks, tot);
      PL_TRY(hipGetLastError(), "level totals");
      PL_TRY(hipMemcpyAsync(h, tot, sizeof(h), hipMemcpyDeviceToHost, s), "copy sizes");
      PL_TRY(hipStreamSynchronize(s), "sync");
      return CCJ_OK;
    };
    if (int rc = sizes()) return rc;
    if (ordered && (h[3] & CCJ_FLAG_PART_OVERFLOW)) {  // key skew filled the split's overflow area
      PL_TRY(hipMemsetAsync(tot + 3, 0, 8, s), "memset");
      PL_TRY(ccj::launch_probe(t->info.kind, p, s), "pipeline probe");
      if (int rc = sizes()) return rc;
    }
    if (h[3]) return ccj::api_fail(CCJ_ERR_LIMIT, "ccj_pipeline_run: probe status flags " + std::to_string(h[3]));
    const uint64_t T = h[0], S = h[1];
    res->rows_out[l] = T;

    // Next join's input: this join's carried columns + its payload.
    const uint32_t ncols = in_ncols + 1;
    const bool last = l + 1 == J;
    const uint64_t next_dup =
        last ? 1 : (pl->tables[l + 1]->info.max_dup ? pl->tables[l + 1]->info.max_dup : 1);
    if (pl->mode == CCJ_COMPACT_FULL) {
      const uint32_t thr = pl->thresholds[l];
      // compacted chunks (all full but the last) + pass-through chunks (at most one per
      // non-empty Next result, only when the threshold is below a full chunk)
      const uint64_t out_chunks = (T + B - 1) / B + (thr != 0 && thr < B ? S : 0);
      const uint64_t cap_rows = out_chunks * B;
      for (uint32_t q = 0; q < ncols; ++q) PL_TRY(L.cols[q].ensure(cap_rows * 8), "alloc");
      PL_TRY(L.next_counts.ensure(out_chunks * 4), "alloc");
      const size_t wsb = ccj::compact_workspace(in_chunks, cap, B, R, thr);
      PL_TRY(L.compact_ws.ensure(wsb), "alloc");
      ccj_compact_args a{};
      a.count = p.out_count;
      a.sel = p.out_sel;
      a.payload = p.out_payload;
      a.rounds = p.out_rounds;
      a.round_counts = p.out_round_counts;
      a.n_chunks = in_chunks;
      a.cap = cap;
      a.max_rounds = R;
      a.chunk = B;
      a.n_cols = in_ncols;
      a.threshold = thr;
      for (uint32_t q = 0; q < in_ncols; ++q) {
        a.cols[q] = in_cols[q];
        a.out_cols[q] = L.cols[q].as<int64_t>();
      }
      a.out_payload = L.cols[in_ncols].as<int64_t>();
      a.out_chunk_counts = L.next_counts.as<uint32_t>();
      a.out_cap_rows = cap_rows;
      a.out_n_chunks = tot + 2;
      a.workspace = L.compact_ws.p;
      a.workspace_bytes = L.compact_ws.bytes;
      a.status = (uint32_t *)(tot + 3);
      if (T) PL_TRY(ccj::launch_compact(a, s), "pipeline compact");
      gaps = thr != 0 && thr < B;
      if (gaps) {  // pass-through chunks add output chunks beyond ceil(T / B): read the number
        PL_TRY(hipMemcpyAsync(h, tot, sizeof(h), hipMemcpyDeviceToHost, s), "copy sizes");
        PL_TRY(hipStreamSynchronize(s), "sync");
        if (h[3]) return ccj::api_fail(CCJ_ERR_LIMIT, "ccj_pipeline_run: compaction status flags " + std::to_string(h[3]));
        in_chunks = T ? h[2] : 0;
      } else {  // NaiveCompactor: every output chunk is full but the last (status checked later)
        in_chunks = out_chunks;
      }
      last_out_chunks = in_chunks;
      in_counts = L.next_counts.as<uint32_t>();
      in_base = in_obase = nullptr;
    } else {
      for (uint32_t q = 0; q < ncols; ++q) PL_TRY(L.cols[q].ensure(T * 8), "alloc");
      PL_TRY(L.seg_base.ensure(S * 8), "alloc");
      PL_TRY(L.seg_obase.ensure(S * 8), "alloc");
      PL_TRY(L.next_counts.ensure(S * 4), "alloc");
      ccj::ConcatParams c{};
      c.count = p.out_count;
      c.sel = p.out_sel;
      c.rounds = p.out_rounds;
      c.round_counts = p.out_round_counts;
      c.payload = p.out_payload;
      c.chunk_base = in_base;
      c.out_base = in_obase;
      c.n_chunks = in_chunks;
      c.cap = cap;
      c.max_rounds = R;
      c.chunk = B;
      c.rows_pre = L.rows_pre.as<uint64_t>();
      c.segs_pre = L.segs_pre.as<uint64_t>();
      c.n_cols = in_ncols;
      c.next_dup = next_dup;
      for (uint32_t q = 0; q < in_ncols; ++q) c.cols[q] = in_cols[q];
      for (uint32_t q = 0; q < ncols; ++q) c.out_cols[q] = L.cols[q].as<int64_t>();
      c.seg_base = L.seg_base.as<uint64_t>();
      c.seg_obase = L.seg_obase.as<uint64_t>();
      c.seg_count = L.next_counts.as<uint32_t>();
      if (T) {
        hipLaunchKernelGGL(ccj::concat_rows, dim3((unsigned)((in_chunks + 3) / 4)), dim3(256), 0, s, c);
        PL_TRY(hipGetLastError(), "pipeline concat");
      }
      in_chunks = T ? S : 0;
      in_counts = L.next_counts.as<uint32_t>();
      in_base = L.seg_base.as<uint64_t>();
      in_obase = L.seg_obase.as<uint64_t>();
    }
    for (uint32_t q = 0; q < ncols; ++q) in_cols[q] = L.cols[q].as<int64_t>();
    in_ncols = ncols;
    in_rows = T;
    in_phys = pl->mode == CCJ_COMPACT_FULL ? in_chunks * B : T;
    PL_TRY(hipEventRecord(pl->ev[l + 1], s), "event");
    if (last) {
      PL_TRY(hipMemcpyAsync(h, tot, sizeof(h), hipMemcpyDeviceToHost, s), "copy status");
      PL_TRY(hipStreamSynchronize(s), "sync");
      if (h[3]) return ccj::api_fail(CCJ_ERR_LIMIT, "ccj_pipeline_run: compaction status flags " + std::to_string(h[3]));
      res->n_out = T;
      if (gaps && T) {  // collect the result densely, chunk by chunk
        const uint64_t n = last_out_chunks;
        PL_TRY(pl->pack_w.ensure(n * 8), "alloc");
        PL_TRY(pl->pack_pre.ensure(n * 8), "alloc");
        size_t tb = ccj::scan_bytes(n);
        PL_TRY(pl->pack_tmp.ensure(tb), "alloc");
        hipLaunchKernelGGL(ccj::widen_counts, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in_counts, n,
                           pl->pack_w.as<uint64_t>());
        PL_TRY(hipGetLastError(), "widen");
        PL_TRY(ccj::scan_exclusive_u64(pl->pack_w.as<uint64_t>(), pl->pack_pre.as<uint64_t>(), n, nullptr, pl->pack_tmp.p, s),
               "scan");
        ccj::PackParams pp{};
        pp.n_cols = 2 * J;
        pp.chunk = B;
        pp.n_chunks = n;
        pp.counts = in_counts;
        pp.pre = pl->pack_pre.as<uint64_t>();
        for (uint32_t q = 0; q < 2 * J; ++q) {
          PL_TRY(pl->res_cols[q].ensure(T * 8), "alloc");
          pp.src[q] = in_cols[q];
          pp.dst[q] = pl->res_cols[q].as<int64_t>();
          in_cols[q] = pp.dst[q];
        }
        hipLaunchKernelGGL(ccj::dense_pack, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, pp);
        PL_TRY(hipGetLastError(), "dense pack");
        PL_TRY(hipEventRecord(pl->ev[l + 1], s), "event");
      }
      for (uint32_t j = 0; j < J; ++j) {
        res->cols[j] = in_cols[j];
        res->payload[j] = in_cols[J + j];
      }
    }
  }
  PL_TRY(hipEventSynchronize(pl->ev[levels_run]), "sync");
  for (uint32_t l = 0; l < levels_run; ++l) {
    float ms = 0;
    PL_TRY(hipEventElapsedTime(&ms, pl->ev[l], pl->ev[l + 1]), "event time");
    res->level_ms[l] = ms;
  }
  return CCJ_OK;
}

extern "C" int ccj_pipeline_checksum(const ccj_pipeline_result *res, uint32_t n_joins, uint64_t *d_acc,
                                     ccj_stream stream) {
  if (!res || !d_acc || n_joins == 0 || n_joins > CCJ_MAX_JOINS)
    return ccj::api_fail(CCJ_ERR_INVALID, "ccj_pipeline_checksum: bad argument");
  if (res->n_out == 0) return CCJ_OK;
  ccj::SinkParams p{};
  for (uint32_t j = 0; j < n_joins; ++j) {
    if (!res->cols[j] || !res->payload[j]) return ccj::api_fail(CCJ_ERR_INVALID, "ccj_pipeline_checksum: null column");
    p.cols[j] = res->cols[j];
    p.pay[j] = res->payload[j];
  }
  p.joins = n_joins;
  p.n = res->n_out;
  const uint64_t want = (res->n_out + 255) / 256;
  hipLaunchKernelGGL(ccj::pipeline_sink, dim3((unsigned)(want < 4096 ? want : 4096)), dim3(256), 0, (hipStream_t)stream,
                     p, (unsigned long long *)d_acc);
  PL_TRY(hipGetLastError(), "pipeline checksum");
  return CCJ_OK;
}
