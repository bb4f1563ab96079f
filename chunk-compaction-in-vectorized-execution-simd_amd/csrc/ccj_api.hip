// ccj_api.hip — the C ABI (include/ccj.h): device selection, table builds, probe dispatch.
//
// No CPU fallback: every entry point requires a gfx950 device and reports CCJ_ERR_NO_DEVICE
// otherwise.  Host-side work here is limited to building tables in the reference's sequential
// insertion order (CCJ_LAYOUT_REFERENCE), which is inherently serial and untimed in the
// reference too (main.cpp:62-68 builds tables before the timed loop at :92-94).
#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "ccj_internal.h"
#include "ccj_tuning.h"

namespace {

thread_local std::string g_err;

// Phase boundary events (ccj_set_phase_events): the reference's CycleProfiler slots
// (profiler.h:262-290) mapped onto this thread's next probe call's kernels.
// One-shot: the probe call that sees them armed records all four — every return path,
// the early ones too (PhaseScope) — and then clears them, so a later call can never record on
// events the caller has since destroyed, and phases never mix two calls.
thread_local hipEvent_t g_phase[4] = {};
thread_local uint32_t g_n_phase = 0;
thread_local uint32_t g_phase_next = 0;  // the next boundary this call has not recorded yet
void phase_mark(hipStream_t s, uint32_t i) {
  if (i < g_n_phase && g_phase[i]) (void)hipEventRecord(g_phase[i], s);
  if (i + 1 > g_phase_next) g_phase_next = i + 1;
}
void phase_marks(hipStream_t s, uint32_t from, uint32_t to) {
  for (uint32_t i = from; i <= to; ++i) phase_mark(s, i);
}
// Scope of one probe API call: on exit, the boundaries the call did not reach (an empty input, a
// one-pass fallback, an error) are recorded at the stream's current point and the events cleared.
// A nested probe call (ccj_probe_ordered's fallback to ccj_probe) consumes them itself.
struct PhaseScope {
  hipStream_t s;
  bool outer;
  explicit PhaseScope(hipStream_t st) : s(st), outer(g_n_phase != 0) {
    if (outer) g_phase_next = 0;
  }
  ~PhaseScope() {
    if (!outer || !g_n_phase) return;
    for (uint32_t i = g_phase_next; i < 4; ++i) phase_mark(s, i);
    for (auto &e : g_phase) e = nullptr;
    g_n_phase = 0;
    g_phase_next = 0;
  }
};


int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char *what) {
  return fail(CCJ_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr, what)                  \
  do {                                       \
    hipError_t e_ = (expr);                  \
    if (e_ != hipSuccess) return hip_fail(e_, what); \
  } while (0)

int check_device() {
  int dev = -1;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return fail(CCJ_ERR_NO_DEVICE, std::string("no HIP device: ") + hipGetErrorString(e));
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return fail(CCJ_ERR_NO_DEVICE, std::string("no HIP device: ") + hipGetErrorString(e));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(CCJ_ERR_NO_DEVICE, std::string("device is ") + prop.gcnArchName + ", need gfx950");
  return CCJ_OK;
}

}  // namespace

namespace ccj {
int api_fail(int code, const std::string &msg) { return fail(code, msg); }
int api_check_device() { return check_device(); }
}  // namespace ccj

namespace {

uint64_t lp_num_slots(uint64_t n) {  // linear_probing_ht.cpp:5-6
  uint64_t s = 1;
  while (s < (n << 2)) s <<= 1;
  return s;
}
uint64_t chain_num_buckets(uint64_t n) {  // chaining_ht.cpp:5-6
  uint64_t b = 1;
  while (b < 2 * n) b *= 2;
  return b;
}

std::vector<int64_t> reference_keys(uint64_t n, uint64_t cf) {  // linear_probing_ht.cpp:14-25
  std::vector<int64_t> k(n);
  const uint64_t num_unique = n / cf + (n % cf != 0);
  const uint64_t step = n / num_unique;
  for (uint64_t t = 0; t < n; ++t) k[t] = (int64_t)((t / cf) * step);
  return k;
}

// Longest occupied run (circular) and largest multiplicity of one key inside a run.
void lp_host_stats(const std::vector<int64_t> &slots, uint32_t *max_run, uint64_t *max_dup) {
  const uint64_t n = slots.size();
  uint64_t start = 0;
  while (start < n && slots[start] != -1) ++start;  // an empty slot always exists (alpha <= 1/4)
  uint64_t best = 0, dup = slots.empty() ? 0 : 1;
  uint64_t run = 0;
  std::vector<int64_t> cl;
  for (uint64_t t = 1; t <= n; ++t) {
    const uint64_t i = (start + t) % n;
    if (slots[i] != -1) {
      ++run;
      cl.push_back(slots[i]);
    } else {
      best = std::max(best, run);
      if (cl.size() > 1) {
        std::sort(cl.begin(), cl.end());
        uint64_t r = 1;
        for (size_t a = 1; a < cl.size(); ++a) {
          r = cl[a] == cl[a - 1] ? r + 1 : 1;
          dup = std::max(dup, r);
        }
      }
      cl.clear();
      run = 0;
    }
  }
  *max_run = (uint32_t)best;
  *max_dup = dup;
}

int upload(void **dst, const void *src, size_t bytes, const char *what) {
  if (bytes == 0) bytes = 8;
  hipError_t e = hipMalloc(dst, bytes);
  if (e != hipSuccess) return fail(CCJ_ERR_OOM, std::string(what) + ": hipMalloc failed");
  if (src) HIP_TRY(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice), what);
  return CCJ_OK;
}

#ifdef CCJ_RANK_WALK
// The rank walk's window index (ccj_rank.hip), built on the device from the finished slot array for
// tables the partitioned probe splits into windows the LDS can hold (<= 2^19 slots).  Build-time
// work like the table itself (main.cpp:62-68 times neither).  Without it the slot-array walk runs.
bool rank_index_applies(const ccj_table *t) {
  const ccj::SlotPlan pl = ccj::slot_plan(t->info.size, CCJ_TABLE_LP);
  const uint64_t size = t->info.size;
  return t->info.kind == CCJ_TABLE_LP && pl.lo_bits && ccj::rank_walk_fits(pl.window_bits) && size % 128 == 0 &&
         size <= (1ull << 32);
}
int build_rank_index(ccj_table *t, hipStream_t s) {
  if (!rank_index_applies(t) || t->d_ckeys) return CCJ_OK;
  const ccj::SlotPlan pl = ccj::slot_plan(t->info.size, CCJ_TABLE_LP);
  const uint64_t size = t->info.size;
  const uint64_t words = size / 64;
  uint32_t *cnt = nullptr;
  hipError_t e = hipMalloc((void **)&t->d_occ, words * 8);
  if (e == hipSuccess) e = hipMalloc((void **)&t->d_pre, words / 2 * 4);
  if (e == hipSuccess) e = hipMalloc((void **)&cnt, words * 4);
  const uint64_t nck = t->info.n_keys + 32;  // occupied slots <= keys; 4-key windows read past the last
  if (e == hipSuccess) e = hipMalloc((void **)&t->d_ckeys, nck * 8);
  if (e == hipSuccess) e = ccj::launch_fill(t->d_ckeys, nck, -1, s);
  if (e == hipSuccess) e = ccj::launch_rank_index(t->d_table, size, t->d_occ, t->d_pre, cnt, s);
  if (e == hipSuccess) e = ccj::launch_rank_compact_keys(t->d_table, size, t->d_occ, t->d_pre, t->d_ckeys, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (cnt) (void)hipFree(cnt);
  if (e != hipSuccess) {
    for (void *q : {(void *)t->d_occ, (void *)t->d_pre, (void *)t->d_ckeys})
      if (q) (void)hipFree(q);
    t->d_occ = nullptr;
    t->d_pre = nullptr;
    t->d_ckeys = nullptr;
    return hip_fail(e, "LP window index");
  }
  t->rank_wbits = pl.window_bits;
  return CCJ_OK;
}
#else
// The rank walk (ccj_rank.hip, DESIGN §3.3: measured slower than the slot-array walk) is built into
// libccj_tuning.so only; the product library refuses its index and flag.
int build_rank_index(ccj_table *, hipStream_t) {
  return fail(CCJ_ERR_INVALID, "ccj_table_build_rank_index: the rank walk is built into libccj_tuning.so only");
}
#endif

int build_lp_host(const int64_t *keys, uint64_t n, ccj_table **out) {
  const uint64_t size = lp_num_slots(n);
  if (size > (1ull << 32)) return fail(CCJ_ERR_LIMIT, "LP table larger than 2^32 slots");
  std::vector<int64_t> slots(size, -1);
  std::vector<uint32_t> rows(size < 4 ? 4 : size, ccj::kNoRow);
  const uint64_t mask = size - 1;
  for (uint64_t i = 0; i < n; ++i) {  // linear_probing_ht.cpp:28-36
    uint64_t s = ccj::murmurhash64((uint64_t)keys[i]) & mask;
    while (slots[s] != -1) s = (s + 1) & mask;
    slots[s] = keys[i];
    if (keys[i] != -1) rows[s] = (uint32_t)i;
  }
  std::unique_ptr<ccj_table> t(new ccj_table());
  t->info.kind = CCJ_TABLE_LP;
  t->info.layout = CCJ_LAYOUT_REFERENCE;
  t->info.n_keys = n;
  t->info.size = size;
  lp_host_stats(slots, &t->info.max_rounds, &t->info.max_dup);
  // storage padded to >= 4 slots: the probe reads aligned 4-slot windows (n_slots = 1 when n = 0)
  if (slots.size() < 4) slots.resize(4, -1);
  void *d = nullptr;
  int rc = upload(&d, slots.data(), slots.size() * sizeof(int64_t), "LP slots");
  if (rc) return rc;
  t->d_table = (int64_t *)d;
  t->positions = slots.size();
  rc = upload(&d, rows.data(), rows.size() * sizeof(uint32_t), "LP slot rows");
  if (rc) {
    (void)hipFree(t->d_table);
    return rc;
  }
  t->d_row = (uint32_t *)d;
  t->info.d_table = t->d_table;
  (void)hipGetDevice(&t->device);
  *out = t.release();
  return CCJ_OK;
}

int build_chain_host(const int64_t *keys, uint64_t n, ccj_table **out) {
  if (n >= (1ull << 32)) return fail(CCJ_ERR_LIMIT, "chaining table needs < 2^32 keys (uint32 CSR)");
  const uint64_t size = chain_num_buckets(n);
  const uint64_t mask = size - 1;
  // chaining_ht.cpp:29-35: push_back in order == stable counting sort by bucket.
  std::vector<uint32_t> off(size + 1, 0);
  std::vector<uint32_t> bucket(n);
  for (uint64_t i = 0; i < n; ++i) {
    bucket[i] = (uint32_t)(ccj::murmurhash64((uint64_t)keys[i]) & mask);
    off[bucket[i] + 1]++;
  }
  uint32_t longest = 0;
  for (uint64_t b = 0; b < size; ++b) {
    longest = std::max(longest, off[b + 1]);
    off[b + 1] += off[b];
  }
  std::vector<int64_t> chain(n);
  std::vector<uint32_t> rows;
  {
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    rows.assign(((n + 3) / 4) * 4 + (n == 0 ? 4 : 0), ccj::kNoRow);
    for (uint64_t i = 0; i < n; ++i) {
      rows[fill[bucket[i]]] = (uint32_t)i;
      chain[fill[bucket[i]]++] = keys[i];
    }
  }
  uint64_t dup = n ? 1 : 0;
  for (uint64_t b = 0; b < size; ++b) {
    const uint32_t lo = off[b], hi = off[b + 1];
    if (hi - lo < 2) continue;
    std::vector<int64_t> cl(chain.begin() + lo, chain.begin() + hi);
    std::sort(cl.begin(), cl.end());
    uint64_t r = 1;
    for (size_t a = 1; a < cl.size(); ++a) {
      r = cl[a] == cl[a - 1] ? r + 1 : 1;
      dup = std::max(dup, r);
    }
  }
  std::unique_ptr<ccj_table> t(new ccj_table());
  t->info.kind = CCJ_TABLE_CHAIN;
  t->info.layout = CCJ_LAYOUT_REFERENCE;
  t->info.n_keys = n;
  t->info.size = size;
  t->info.max_rounds = longest;
  t->info.max_dup = dup;
  // padded to a multiple of 4 keys (>= 4): the probe reads aligned 4-key windows
  chain.resize(((n + 3) / 4) * 4 + (n == 0 ? 4 : 0), -1);
  void *d = nullptr;
  int rc = upload(&d, chain.data(), chain.size() * sizeof(int64_t), "chain keys");
  if (rc) return rc;
  t->d_table = (int64_t *)d;
  rc = upload(&d, off.data(), (size + 1) * sizeof(uint32_t), "chain offsets");
  if (rc) {
    (void)hipFree(t->d_table);
    return rc;
  }
  t->d_off = (uint32_t *)d;
  t->positions = chain.size();
  rc = upload(&d, rows.data(), rows.size() * sizeof(uint32_t), "chain rows");
  if (rc) {
    (void)hipFree(t->d_table);
    (void)hipFree(t->d_off);
    return rc;
  }
  t->d_row = (uint32_t *)d;
  {  // bucket records: the chain's range and first key in one 16-byte load
    std::vector<int64_t> rec(2 * size);
    for (uint64_t b = 0; b < size; ++b) {
      const uint64_t lo = off[b], len = off[b + 1] - off[b];
      rec[2 * b] = (int64_t)(lo | (len << 32));
      rec[2 * b + 1] = len ? chain[lo] : -1;
    }
    rc = upload(&d, rec.data(), rec.size() * sizeof(int64_t), "chain bucket records");
    if (rc) {
      (void)hipFree(t->d_table);
      (void)hipFree(t->d_off);
      (void)hipFree(t->d_row);
      return rc;
    }
    t->d_bucket = (int64_t *)d;
  }
  if (longest < 0xFFu) {  // 8-byte records {start | len << 32 | fp(node 0) << 40 | fp(node 1) << 52}
    std::vector<uint64_t> rec(size < 2 ? 2 : size, 0);  // read as aligned 16-byte pairs: >= 2 records
    for (uint64_t b = 0; b < size; ++b) {
      const uint64_t lo = off[b], len = off[b + 1] - off[b];
      const uint64_t fp0 = len ? ccj::bucket_fp(ccj::murmurhash64((uint64_t)chain[lo])) : 0u;
      const uint64_t fp1 = len > 1 ? ccj::bucket_fp(ccj::murmurhash64((uint64_t)chain[lo + 1])) : 0u;
      rec[b] = lo | len << 32 | fp0 << 40 | fp1 << 52;
    }
    rc = upload(&d, rec.data(), rec.size() * sizeof(uint64_t), "chain bucket records (8 B)");
    if (rc) {
      (void)hipFree(t->d_table);
      (void)hipFree(t->d_off);
      (void)hipFree(t->d_row);
      (void)hipFree(t->d_bucket);
      return rc;
    }
    t->d_bucket8 = (uint64_t *)d;
  }
  t->info.d_table = t->d_table;
  t->info.d_bucket_off = t->d_off;
  (void)hipGetDevice(&t->device);
  hipError_t fe = ccj::build_chain_filter(t.get(), nullptr);  // (from the uploaded CSR, on the device)
  if (fe == hipSuccess) fe = hipDeviceSynchronize();
  if (fe != hipSuccess) {
    ccj_table_free(t.release());
    return hip_fail(fe, "chain bucket filter");
  }
  *out = t.release();
  return CCJ_OK;
}

int build_lp_device(const int64_t *d_keys, uint64_t n, hipStream_t s, uint64_t known_dup, ccj_table **out) {
  const uint64_t size = lp_num_slots(n);
  if (size > (1ull << 32)) return fail(CCJ_ERR_LIMIT, "LP table larger than 2^32 slots");
  std::unique_ptr<ccj_table> t(new ccj_table());
  void *d = nullptr;
  const uint64_t alloc = size < 4 ? 4 : size;  // aligned 4-slot windows
  if (hipMalloc(&d, alloc * sizeof(int64_t)) != hipSuccess) return fail(CCJ_ERR_OOM, "LP slots: hipMalloc failed");
  t->d_table = (int64_t *)d;
  auto cleanup = [&]() {
    (void)hipFree(t->d_table);
    if (t->d_row) (void)hipFree(t->d_row);
  };
  t->positions = alloc;
  if (hipMalloc(&d, alloc * sizeof(uint32_t)) != hipSuccess) {
    cleanup();
    return fail(CCJ_ERR_OOM, "LP slot rows: hipMalloc failed");
  }
  t->d_row = (uint32_t *)d;
  hipError_t e = ccj::launch_fill(t->d_table, alloc, -1, s);
  if (e == hipSuccess) e = hipMemsetAsync(t->d_row, 0xFF, alloc * sizeof(uint32_t), s);
  if (e == hipSuccess) e = ccj::launch_lp_insert(d_keys, n, t->d_table, t->d_row, (uint32_t)(size - 1), s);
  const uint64_t n_seg = (size + ccj::kRunSegment - 1) / ccj::kRunSegment;
  uint32_t *d_stats = nullptr;
  if (e == hipSuccess) e = hipMalloc(&d_stats, n_seg * 4 * sizeof(uint32_t));
  if (e == hipSuccess) e = ccj::launch_lp_runs(t->d_table, size, d_stats, s);
  std::vector<uint32_t> st(n_seg * 4);
  if (e == hipSuccess) e = hipMemcpyAsync(st.data(), d_stats, st.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (d_stats) (void)hipFree(d_stats);
  if (e != hipSuccess) {
    cleanup();
    return hip_fail(e, "device LP build");
  }
  // combine per-segment run stats (circular)
  uint64_t best = 0, carry = 0;
  for (uint64_t g = 0; g < n_seg; ++g) {
    const uint32_t lead = st[g * 4], trail = st[g * 4 + 1], inner = st[g * 4 + 2], full = st[g * 4 + 3];
    if (full) {
      carry += lead;
      continue;
    }
    best = std::max<uint64_t>(best, std::max<uint64_t>(inner, carry + lead));
    carry = trail;
  }
  if (n_seg) best = std::max<uint64_t>(best, carry + st[0]);
  t->info.kind = CCJ_TABLE_LP;
  t->info.layout = CCJ_LAYOUT_DEVICE;
  t->info.n_keys = n;
  t->info.size = size;
  t->info.max_rounds = (uint32_t)best;
  // Largest multiplicity of one key: it sizes every probe output (cap = chunk * max_dup).
  uint64_t dup = known_dup;
  if (!dup && n) {
    uint32_t *d_dup = nullptr, h_dup = 0;
    e = hipMalloc(&d_dup, sizeof(uint32_t));
    if (e == hipSuccess) e = ccj::launch_lp_max_dup(t->d_table, size, (uint32_t)std::min<uint64_t>(best, size), d_dup, s);
    if (e == hipSuccess) e = hipMemcpyAsync(&h_dup, d_dup, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (d_dup) (void)hipFree(d_dup);
    if (e != hipSuccess) {
      cleanup();
      return hip_fail(e, "device LP build (max dup)");
    }
    dup = h_dup;
  }
  t->info.max_dup = dup ? dup : 1;
  t->info.d_table = t->d_table;
  (void)hipGetDevice(&t->device);
  *out = t.release();
  return CCJ_OK;
}

// Zipf s = 1 over ranks 1..n as a 2^16-bucket inverse CDF: t[j] = the smallest rank whose CDF
// H_r / H_n exceeds j / 2^16, t[2^16] = n + 1 (the same IEEE-double construction as the test
// oracle's ccj_zipf_table, so host and device streams agree bit for bit).
void zipf_table(uint64_t n, uint32_t *t) {
  double hn = 0.0;
  for (uint64_t r = 1; r <= n; ++r) hn += 1.0 / (double)r;
  uint32_t j = 0;
  double h = 0.0;
  for (uint64_t r = 1; r <= n && j < ccj::kZipfBuckets; ++r) {
    h += 1.0 / (double)r;
    while (j < ccj::kZipfBuckets && h * (double)ccj::kZipfBuckets > (double)j * hn) t[j++] = (uint32_t)r;
  }
  while (j < ccj::kZipfBuckets) t[j++] = (uint32_t)(n ? n : 1);
  t[ccj::kZipfBuckets] = (uint32_t)(n + 1);
}

}  // namespace

extern "C" {

const char *ccj_last_error(void) { return g_err.c_str(); }

int ccj_set_phase_events(void *const *events, uint32_t n) {
  if (n > 4 || (n && !events)) return fail(CCJ_ERR_INVALID, "ccj_set_phase_events: at most 4 events");
  for (uint32_t i = 0; i < 4; ++i) g_phase[i] = i < n ? (hipEvent_t)events[i] : nullptr;
  g_n_phase = n;
  g_phase_next = 0;
  return CCJ_OK;
}

int ccj_abi_version(void) { return CCJ_ABI_VERSION; }

#ifndef CCJ_SRC_HASH
#define CCJ_SRC_HASH "unknown"
#endif
const char *ccj_build_hash(void) { return CCJ_SRC_HASH; }

const char *ccj_last_gather_kernel(void) { return ccj::last_gather_kernel(); }

int ccj_device_init(int device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) return fail(CCJ_ERR_NO_DEVICE, "no HIP device visible");
  if (device < 0 || device >= n) return fail(CCJ_ERR_INVALID, "device index out of range");
  HIP_TRY(hipSetDevice(device), "hipSetDevice");
  return check_device();
}

int ccj_table_build_reference(int kind, uint64_t n, uint64_t cf, int layout, ccj_stream stream, ccj_table **out) {
  if (!out || cf == 0) return fail(CCJ_ERR_INVALID, "ccj_table_build_reference: bad argument");
  if (kind != CCJ_TABLE_LP && kind != CCJ_TABLE_CHAIN) return fail(CCJ_ERR_INVALID, "bad table kind");
  if (int rc = check_device()) return rc;
  *out = nullptr;
  if (layout != CCJ_LAYOUT_REFERENCE && layout != CCJ_LAYOUT_DEVICE) return fail(CCJ_ERR_INVALID, "bad layout");
  if (layout == CCJ_LAYOUT_REFERENCE && kind == CCJ_TABLE_LP) {  // sequential insert order (L3 layout)
    std::vector<int64_t> keys = reference_keys(n, cf);
    return build_lp_host(keys.data(), n, out);
  }
  hipStream_t s = (hipStream_t)stream;
  int64_t *d_keys = nullptr;
  if (hipMalloc(&d_keys, std::max<uint64_t>(n, 1) * sizeof(int64_t)) != hipSuccess)
    return fail(CCJ_ERR_OOM, "reference keys: hipMalloc failed");
  hipError_t e = ccj::launch_gen_reference_keys(d_keys, 0, n, n, cf, s);
  if (e != hipSuccess) {
    (void)hipFree(d_keys);
    return hip_fail(e, "gen reference keys");
  }
  const uint64_t dup = std::max<uint64_t>(1, std::min<uint64_t>(cf, n));  // first group: min(cf, n) copies
  // chaining: the device's stable bucket sort gives the reference's chain order whatever the
  // layout asked for (both layouts are the same table)
  int rc = kind == CCJ_TABLE_LP ? build_lp_device(d_keys, n, s, dup, out) : ccj::build_chain_device(d_keys, n, s, dup, out);
  if (rc == CCJ_OK && kind == CCJ_TABLE_CHAIN) (*out)->info.layout = layout;
  (void)hipStreamSynchronize(s);
  (void)hipFree(d_keys);
  return rc;
}

int ccj_table_build_from_host(int kind, const int64_t *h_keys, uint64_t n, ccj_table **out) {
  if (!out || (!h_keys && n)) return fail(CCJ_ERR_INVALID, "ccj_table_build_from_host: bad argument");
  if (int rc = check_device()) return rc;
  *out = nullptr;
  if (kind == CCJ_TABLE_LP) return build_lp_host(h_keys, n, out);
  if (kind == CCJ_TABLE_CHAIN) return build_chain_host(h_keys, n, out);
  return fail(CCJ_ERR_INVALID, "bad table kind");
}

int ccj_table_build_on_device(int kind, const int64_t *d_keys, uint64_t n, ccj_stream stream, ccj_table **out) {
  if (!out || (!d_keys && n)) return fail(CCJ_ERR_INVALID, "ccj_table_build_on_device: bad argument");
  if (int rc = check_device()) return rc;
  *out = nullptr;
  if (kind == CCJ_TABLE_LP) return build_lp_device(d_keys, n, (hipStream_t)stream, 0, out);
  if (kind == CCJ_TABLE_CHAIN) return ccj::build_chain_device(d_keys, n, (hipStream_t)stream, 0, out);
  return fail(CCJ_ERR_INVALID, "bad table kind");
}

int ccj_table_get_info(const ccj_table *t, ccj_table_info *info) {
  if (!t || !info) return fail(CCJ_ERR_INVALID, "ccj_table_get_info: null");
  *info = t->info;
  return CCJ_OK;
}

int ccj_table_get_arrays(const ccj_table *t, ccj_table_arrays *a) {
  if (!t || !a) return fail(CCJ_ERR_INVALID, "ccj_table_get_arrays: null");
  *a = ccj_table_arrays{};
  a->d_table = t->d_table;
  a->positions = t->positions;
  a->d_row = t->d_row;
  a->d_bucket_off = t->d_off;
  a->d_bucket16 = t->d_bucket;
  a->d_bucket8 = t->d_bucket8;
  a->n_bucket8 = t->d_bucket8 ? (t->info.size < 2 ? 2 : t->info.size) : 0;
  a->d_bucket_filter = t->d_filt;
  a->n_filter_words = t->d_filt ? t->info.size / 16 : 0;
  return CCJ_OK;
}

int ccj_table_set_payload(ccj_table *t, const int64_t *d_payload, uint32_t n_cols, ccj_stream stream) {
  if (!t || n_cols == 0 || n_cols > CCJ_MAX_PAYLOAD_COLS || (!d_payload && t->info.n_keys))
    return fail(CCJ_ERR_INVALID, "ccj_table_set_payload: bad argument");
  if (!t->d_row) return fail(CCJ_ERR_INVALID, "ccj_table_set_payload: table has no row map");
  void *d = nullptr;
  if (hipMalloc(&d, t->positions * n_cols * sizeof(int64_t)) != hipSuccess)
    return fail(CCJ_ERR_OOM, "payload: hipMalloc failed");
  hipError_t e = ccj::launch_scatter_payload(d_payload, n_cols, t->d_row, t->positions, (int64_t *)d,
                                             (hipStream_t)stream);
  if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess) {
    (void)hipFree(d);
    return hip_fail(e, "payload scatter");
  }
  if (t->d_pay) (void)hipFree(t->d_pay);
  t->d_pay = (int64_t *)d;
  t->n_pay = n_cols;
  return CCJ_OK;
}

int ccj_table_build_rank_index(ccj_table *t, ccj_stream stream) {
  if (!t) return fail(CCJ_ERR_INVALID, "ccj_table_build_rank_index: null table");
  return build_rank_index(t, (hipStream_t)stream);
}

int ccj_table_free(ccj_table *t) {
  if (!t) return CCJ_OK;
  if (t->d_table) (void)hipFree(t->d_table);
  if (t->d_off) (void)hipFree(t->d_off);
  if (t->d_bucket) (void)hipFree(t->d_bucket);
  if (t->d_bucket8) (void)hipFree(t->d_bucket8);
  if (t->d_filt) (void)hipFree(t->d_filt);
  if (t->d_row) (void)hipFree(t->d_row);
  if (t->d_pay) (void)hipFree(t->d_pay);
  if (t->d_occ) (void)hipFree(t->d_occ);
  if (t->d_pre) (void)hipFree(t->d_pre);
  if (t->d_ckeys) (void)hipFree(t->d_ckeys);
  delete t;
  return CCJ_OK;
}

namespace {
int fill_probe_params(const ccj_table *t, const ccj_probe_args *a, ccj::ProbeParams &p) {
  if (!t || !a) return fail(CCJ_ERR_INVALID, "ccj_probe: null table/args");
  if (a->chunk == 0 || a->chunk > ccj::kMaxChunk) return fail(CCJ_ERR_INVALID, "ccj_probe: chunk must be 1..2048");
  if (a->out_round_counts && a->max_rounds == 0) return fail(CCJ_ERR_INVALID, "ccj_probe: max_rounds == 0");
  if (a->n_rows && (!a->out_count || !a->out_sel || !a->keys))
    return fail(CCJ_ERR_INVALID, "ccj_probe: missing buffer");
  p = ccj::ProbeParams{};
  p.table = t->d_table;
  p.off = t->d_off;
  p.bucket = reinterpret_cast<const longlong2 *>(t->d_bucket);
  p.bucket8 = ccj_tune_int("CCJ_BUCKET8", 1) ? t->d_bucket8 : nullptr;
  p.filt = t->d_filt;
  p.filt_wb = t->info.kind == CCJ_TABLE_CHAIN ? ccj::slot_plan(t->info.size, CCJ_TABLE_CHAIN).window_bits : 0u;
  p.mask = (uint32_t)(t->info.size - 1);
  p.keys = a->keys;
  p.sel = a->sel;
  p.counts = a->counts;
  p.n_rows = a->n_rows;
  p.n_chunks = (a->n_rows + a->chunk - 1) / a->chunk;
  p.chunk = a->chunk;
  p.max_rounds = a->max_rounds;
  p.cap = a->cap;
  p.out_count = a->out_count;
  p.out_sel = a->out_sel;
  p.out_payload = a->out_payload;
  p.out_rounds = a->out_rounds;
  p.out_round_counts = a->out_round_counts;
  p.status = a->status;
  p.out_pos = a->out_pos;
  if (a->n_payload_cols > t->n_pay) return fail(CCJ_ERR_INVALID, "ccj_probe: table has fewer payload columns");
  p.pay = t->d_pay;
  p.n_pay = a->n_payload_cols;
  p.pay_stride = t->n_pay;
  for (uint32_t c = 0; c < a->n_payload_cols; ++c) {
    if (!a->out_payload_cols[c]) return fail(CCJ_ERR_INVALID, "ccj_probe: null payload column");
    p.out_cols[c] = a->out_payload_cols[c];
  }
  return CCJ_OK;
}
}  // namespace

namespace {
// Layout of the partitioned column: identity (table = one window), or the fixed-capacity split's
// parts * 8 segments of seg_cap positions (the exact split uses a prefix of the same positions).
struct PartLayout {
  ccj::SlotPlan pl;
  uint32_t parts;
  uint64_t seg_cap, positions;
  uint64_t ovf_base, ovf_cap;  // overflow area after the segments (runs that do not fit: key skew)
  uint64_t ovf_sub;            // its 8 x ovf_per_group sub-areas (a multiple of chunk each; the last 64 positions: the sink)
  uint32_t ovf_per_group;      // overflow sub-areas (cursors) per XCD group: 1 or kOvfPerGroup
};
PartLayout part_layout(const ccj_table *t, uint64_t n_rows, uint32_t chunk) {
  PartLayout L{};
  L.pl = ccj::slot_plan(t->info.size, t->info.kind);
  L.parts = 1u << (L.pl.lo_bits + L.pl.hi_bits);
  if (L.pl.lo_bits == 0 || n_rows == 0 || chunk == 0) {
    L.positions = n_rows;
    return L;
  }
  L.seg_cap = ccj::slot_seg_cap(n_rows, L.pl, chunk);
  L.ovf_base = (uint64_t)L.parts * 8 * L.seg_cap;
  // Per tile group (XCD) g, a sub-area of 1/16 of the most rows one group can receive — tile group
  // g splits tiles [g n_tiles / 8, (g + 1) n_tiles / 8), so with few tiles one group may get all
  // of them (1/8 of n / 16 each sent skewed small inputs to the exact fallback early) —
  // at least one chunk each, then the split's 64-position sink.
  uint64_t g_rows = 0;
  for (const bool runs : {false, true}) {
    const uint64_t tile = ccj::slot_split_tile_keys(L.parts, runs), n_tiles = (n_rows + tile - 1) / tile;
    g_rows = std::max<uint64_t>(g_rows, std::min<uint64_t>(n_rows, (n_tiles + 7) / 8 * tile));
  }
  // A group's room, 1/16 of its rows + one chunk, split over kOvfPerGroup sub-areas (cursors) only
  // where each can hold a whole tile (one partition's run of a skewed tile may need it); the area
  // keeps its size either way (ccj_pipeline_run's route gate, positions <= 4/3 of the rows,
  // depends on it).
  const uint64_t room = g_rows / 16 + chunk;
  L.ovf_per_group = room / ccj::kOvfPerGroup >= ccj::slot_split_tile_keys(L.parts) ? ccj::kOvfPerGroup : 1u;
  L.ovf_sub = (room / L.ovf_per_group + chunk - 1) / chunk * chunk;
  L.ovf_cap = (8 * L.ovf_per_group * L.ovf_sub + 64 + chunk - 1) / chunk * chunk;
  L.positions = L.ovf_base + L.ovf_cap;
  return L;
}
uint64_t align256(uint64_t b) { return (b + 255) & ~255ull; }
}  // namespace

uint64_t ccj_probe_partitioned_positions(const ccj_table *t, uint64_t n_rows, uint32_t chunk) {
  if (!t) return 0;
  return part_layout(t, n_rows, chunk).positions;
}

namespace {
// The partitioned probe's workspace without the C5 sub-range starts (part_ws_sub_bytes), which
// follow it: partitioned keys (positions) + the fixed split's cursors, or the exact split's pass
// scratch, + the rank walk's per-block hit masks, hit counts and partition counters.
size_t part_ws_base_bytes(const ccj_table *t, const PartLayout &L, uint64_t n_rows) {
  const size_t fixed = align256(ccj::split_cursor_count(L.parts) * 4);
  const size_t exact = ccj::slot_partition_workspace(n_rows, L.pl);
#ifdef CCJ_RANK_WALK
  const size_t rank = t->d_ckeys && L.pl.lo_bits ? ccj::rank_workspace(L.positions, L.parts) : 0;
#else
  const size_t rank = 0;
  (void)t;
#endif
  return align256(L.positions * 8) + align256(fixed > exact ? fixed : exact) + rank;
}
// 8 u32 sub-range starts per output chunk (walk_emit_pos_sub), for tables with payload columns
size_t part_ws_sub_bytes(const ccj_table *t, const PartLayout &L, uint32_t chunk) {
  if (!t->n_pay || !L.pl.lo_bits) return 0;
  const uint64_t out_chunks = (L.positions + chunk - 1) / chunk;
  return align256(out_chunks * 8 * 4);
}
}  // namespace

size_t ccj_probe_partitioned_workspace_size(const ccj_table *t, uint64_t n_rows, uint32_t chunk) {
  if (!t) return 0;
  const PartLayout L = part_layout(t, n_rows, chunk);
  return part_ws_base_bytes(t, L, n_rows) + part_ws_sub_bytes(t, L, chunk);
}

int ccj_probe_partitioned(const ccj_table *t, const ccj_probe_args *a, uint32_t flags, uint32_t *out_row_map,
                          void *ws, size_t ws_bytes, ccj_stream stream) {
  PhaseScope phase_scope((hipStream_t)stream);
  ccj::ProbeParams p;
  if (int rc = fill_probe_params(t, a, p)) return rc;
  if (t->info.kind == CCJ_TABLE_CHAIN && (a->out_pos || a->n_payload_cols))
    return fail(CCJ_ERR_INVALID, "ccj_probe_partitioned: positions / payload columns need an LP table");
  if (a->sel) return fail(CCJ_ERR_INVALID, "ccj_probe_partitioned: sel must be NULL");
  if (a->counts && (flags & CCJ_PART_EXACT))
    return fail(CCJ_ERR_INVALID, "ccj_probe_partitioned: input chunk counts need the one-pass split (no CCJ_PART_EXACT)");
  if (a->out_round_counts)
    return fail(CCJ_ERR_INVALID, "ccj_probe_partitioned: no round counts (no Next boundaries in partition order)");
  if ((a->out_pos || a->n_payload_cols) && t->info.size < 16)
    return fail(CCJ_ERR_INVALID, "ccj_probe_partitioned: positions / payload columns need a table of >= 16 slots");
  if (a->n_rows >= (1ull << 32)) return fail(CCJ_ERR_LIMIT, "ccj_probe_partitioned: n_rows must be < 2^32");
  if (flags & ~(CCJ_PART_EXACT | CCJ_PART_ROWS | CCJ_PART_RANK | CCJ_PART_SHARE))
    return fail(CCJ_ERR_INVALID, "ccj_probe_partitioned: unknown flags");
#ifdef CCJ_RANK_WALK
  if ((flags & CCJ_PART_RANK) && !t->d_ckeys && rank_index_applies(t))  // refused before any launch
    return fail(CCJ_ERR_INVALID, "ccj_probe_partitioned: CCJ_PART_RANK needs ccj_table_build_rank_index first");
#else
  if (flags & CCJ_PART_RANK)
    return fail(CCJ_ERR_INVALID, "ccj_probe_partitioned: CCJ_PART_RANK: the rank walk is built into libccj_tuning.so only");
#endif
  const bool rows = (flags & CCJ_PART_ROWS) != 0;
  // (with positions / payload columns the walk packs matched | slot into 32 bits: <= 2^31 slots)
  if (rows && (!a->out_payload || p.cap != a->chunk || t->info.max_dup > 1 || t->info.kind != CCJ_TABLE_LP ||
               t->info.size < 16 || ((a->out_pos || a->n_payload_cols) && t->info.size > (1ull << 31))))
    return fail(CCJ_ERR_INVALID, "ccj_probe_partitioned: CCJ_PART_ROWS needs an LP table of >= 16 slots with distinct "
                                 "keys, cap == chunk, out_payload (with positions / payload columns: <= 2^31 slots)");
  if (a->n_rows == 0) return CCJ_OK;
  const PartLayout L = part_layout(t, a->n_rows, a->chunk);
  const size_t ws_base = part_ws_base_bytes(t, L, a->n_rows);
  if ((!out_row_map && !rows) || !ws || ws_bytes < ws_base)
    return fail(CCJ_ERR_INVALID, "ccj_probe_partitioned: missing row map or workspace too small");
  const bool exact = (flags & CCJ_PART_EXACT) != 0;
  if (L.pl.lo_bits && !exact && !a->status)
    return fail(CCJ_ERR_INVALID, "ccj_probe_partitioned: the fixed-capacity split needs args->status");
  hipStream_t s = (hipStream_t)stream;
  // With one output slot per position (cap == chunk) the partitioned keys are written straight
  // into out_payload: a matched row's payload is its key (an LP match means slot value == key), so
  // the walk writes payloads only for chunks where some row missed (in place, compacted).
  // With CCJ_PART_ROWS the split likewise writes each position's original row into out_sel.
  const bool alias = rows || (a->out_payload && p.cap == a->chunk && p.n_pay == 0 && !a->out_pos &&
                              t->info.kind == CCJ_TABLE_LP && t->info.size >= 16 &&
                              ccj_tune_int("CCJ_KEYS_IN_OUT", 1));
  int64_t *pkeys = alias ? a->out_payload : (int64_t *)ws;
  p.keys_in_out = alias ? 1u : 0u;
  p.rows_in_sel = rows ? 1u : 0u;
  if (rows) out_row_map = a->out_sel;
  void *rest = (char *)ws + align256(L.positions * 8);
  const uint64_t out_chunks = L.positions / a->chunk + (L.positions % a->chunk ? 1 : 0);
  phase_mark(s, 0);
  if (L.pl.lo_bits == 0) {  // the whole table is one window: identity order
    HIP_TRY(hipMemcpyAsync(pkeys, a->keys, a->n_rows * 8, hipMemcpyDeviceToDevice, s), "copy");
    HIP_TRY(ccj::launch_iota_u32(out_row_map, a->n_rows, s), "iota");
  } else if (!exact) {
    uint32_t *cursors = (uint32_t *)rest;
    // CCJ_PART_SHARE: 3/4 of the stream's CUs (a multiple of 8), the rest left to other streams
    const uint32_t share = (flags & CCJ_PART_SHARE) ? std::max<uint32_t>(8u, ccj::stream_cus(s) * 3 / 4 / 8 * 8) : 0u;
    HIP_TRY(ccj::launch_slot_split_fixed(a->keys, a->n_rows, L.pl, L.seg_cap, L.ovf_base, L.ovf_cap, L.ovf_sub, cursors, pkeys,
                                         out_row_map, a->status, s, a->counts, a->chunk, nullptr, nullptr, 0, ~0u,
                                         share, nullptr, ~0u, L.ovf_per_group),
            "slot split");
    p.seg_count = cursors;
    p.counts = nullptr;  // the input's chunk counts were applied by the split
    p.seg_parts = L.parts;
    p.seg_cap = L.seg_cap;
    p.ovf_base = L.ovf_base;
    p.ovf_sub = L.ovf_sub;
    p.swz_chunks = L.ovf_base / a->chunk;
    p.n_rows = L.positions;
    p.n_chunks = out_chunks;
  } else {
    p.counts = nullptr;
    HIP_TRY(ccj::launch_slot_partition(a->keys, a->n_rows, L.pl, pkeys, out_row_map, rest, s), "slot partition");
    if (out_chunks > p.n_chunks)  // the layout's trailing chunks are empty in the exact form
      HIP_TRY(hipMemsetAsync(a->out_count + p.n_chunks, 0, (out_chunks - p.n_chunks) * 4, s), "count tail");
  }
  phase_mark(s, 1);  // hash + home partition of every key (and, CCJ_PART_ROWS, keys + rows written out)
  p.keys = pkeys;
  p.xcd_swizzle = 1;  // consecutive chunks (one partition's rows) go to one XCD: its L2 holds the window
  // distinct build keys and no per-chunk rounds: the walk ends a row at its match (C2: 1.168 -> 1.013
  // windows per row in a host simulation of the walk's windows)
  p.first_match = t->info.max_dup <= 1 && !a->out_rounds && ccj_tune_int("CCJ_FIRST_MATCH", 1) ? 1u : 0u;
  // probe_walk's emit: the chunk's matches staged in LDS, 16-byte non-temporal stores (C2 walk
  // 14.04-14.07 ms per step against 14.19-14.20 with per-wave 4/8-byte stores; write-through sc1
  // 16-byte stores 14.6, plain 15.2; CCJ_EMIT_POL = -1 is the per-wave form)
  p.emit_pol = (uint32_t)ccj_tune_int("CCJ_EMIT_POL", 2);
#ifdef CCJ_TUNING
  p.ablate = (uint32_t)ccj_tune_int("CCJ_ABLATE", 0);
  // CCJ_PREFETCH = distance in eighths of a partition's chunks (probe_walk1's window prefetch),
  // CCJ_PF_MULT = slices of lines per chunk
  if (!exact && L.pl.lo_bits && t->info.kind == CCJ_TABLE_LP && L.pl.window_bits >= 4) {
    p.kp_dist = (uint32_t)ccj_tune_int("CCJ_KEYPF", 64);
    p.key_aux = (uint32_t)ccj_tune_int("CCJ_KEY_AUX", 0);
    const int pf8 = ccj_tune_int("CCJ_PREFETCH", 0);
    if (pf8 > 0) {
      const uint64_t K = 8 * (L.seg_cap / a->chunk);
      const uint64_t wl = (1ull << L.pl.window_bits) / 16;
      p.pf_dist = K * (uint64_t)pf8 / 8;
      p.pf_lines = (uint32_t)std::min<uint64_t>(64, (wl + K - 1) / K * (uint64_t)ccj_tune_int("CCJ_PF_MULT", 1));
    }
  }
#endif
#ifdef CCJ_RANK_WALK
  // The rank walk (CCJ_PART_RANK, ccj_rank.hip): the window index in LDS, candidate keys from the
  // compact array.  Distinct keys (a row matches at most once), the keys in out_payload (cap ==
  // chunk), blocks of 512 rows inside chunks, the index built for this window size.
  const bool rank = !exact && L.pl.lo_bits && L.ovf_base && t->d_ckeys && t->rank_wbits == L.pl.window_bits &&
                    p.keys_in_out && t->info.max_dup <= 1 && p.n_pay == 0 && !p.out_pos && !p.out_rounds &&
                    a->chunk % ccj::kRankChunkMultiple == 0 && ((flags & CCJ_PART_RANK) || ccj_tune_int("CCJ_RANK", 0));
  if (rank) {
    const ccj::RankIndex ix{t->d_occ, t->d_pre, t->d_ckeys, t->rank_wbits};
    const size_t fixed = align256(ccj::split_cursor_count(L.parts) * 4);
    const size_t exact_ws = ccj::slot_partition_workspace(a->n_rows, L.pl);
    void *rws = (char *)rest + align256(fixed > exact_ws ? fixed : exact_ws);
    HIP_TRY(ccj::launch_probe_rank(p, ix, rws, s), "rank walk launch");
    phase_marks(s, 2, 3);
    return CCJ_OK;
  }
#endif
  if (p.n_pay == 0) {
#ifdef CCJ_TUNING
    // CCJ_STATS: per-phase cycle sums of the walk's waves, printed per launch (tuning only)
    static unsigned long long *stats = nullptr;
    if (ccj_tune_env("CCJ_STATS")) {
      if (!stats) HIP_TRY(hipMalloc((void **)&stats, 8 * sizeof(unsigned long long)), "stats");
      HIP_TRY(hipMemsetAsync(stats, 0, 8 * sizeof(unsigned long long), s), "stats");
      p.stats = stats;
    }
#endif
    HIP_TRY(ccj::launch_probe_flat(t->info.kind, p, s), "probe launch");
    phase_marks(s, 2, 3);  // match + advance (the walk, which also writes the chunks with misses)
#ifdef CCJ_TUNING
    if (p.stats) {
      unsigned long long h[8];
      HIP_TRY(hipMemcpyAsync(h, p.stats, sizeof(h), hipMemcpyDeviceToHost, s), "stats");
      HIP_TRY(hipStreamSynchronize(s), "stats");
      const double w = h[4] ? (double)h[4] : 1.0;
      fprintf(stderr, "[walk stats] waves %llu  per wave: stage %.0f  walk %.0f  emit %.0f cycles, %.2f steps\n",
              h[4], h[0] / w, h[1] / w, h[2] / w, h[3] / w);
    }
#endif
    return CCJ_OK;
  }
  // Wide payload (C5): the walk records every match's table position, a second pass gathers rows
  // (consecutive chunks share a table window, so their payload rows stay in the Infinity Cache).
  uint32_t *pos = p.out_pos;
  if (!pos) HIP_TRY(hipMallocAsync((void **)&pos, p.n_chunks * p.cap * sizeof(uint32_t), s), "payload positions");
  ccj::ProbeParams q = p;
  q.out_pos = pos;
  q.n_pay = 0;
  // Slab order (round 6): the walk writes each chunk's matches by sub-range of their slot — 8 per
  // partition window, a 4 MiB slab of payload rows at C5 — and the gather takes one slab per XCD at
  // a time, so the rows it reads stay in that XCD's L2.  Where the 16-byte column form applies:
  // rows mode, the fixed split's segments (>= 8 partitions, one XCD's range each), 8 columns,
  // unpacked even-capacity outputs, and the workspace holds the sub-range starts.
  bool sub = rows && !exact && L.pl.lo_bits && L.parts >= 8 && L.parts % 8 == 0 && L.pl.window_bits >= 3 &&
             p.n_pay == 8 && p.cap % 2 == 0 && !p.out_base && t->n_pay % 2 == 0 && (uintptr_t)t->d_pay % 16 == 0 &&
             ws_bytes >= ws_base + part_ws_sub_bytes(t, L, a->chunk) && ccj_tune_int("CCJ_GATHER_SUB", 1);
  for (uint32_t c = 0; c < p.n_pay; ++c) sub = sub && (uintptr_t)p.out_cols[c] % 16 == 0;
  if (sub) {
    q.out_sub = p.out_sub = (uint32_t *)((char *)ws + ws_base);
    q.sub_shift = p.sub_shift = L.pl.window_bits - 3;
  }
  hipError_t e = ccj::launch_probe_flat(t->info.kind, q, s);
  phase_mark(s, 2);
  if (e == hipSuccess)
    e = sub ? ccj::launch_gather_payload(p, pos, s, L.parts, L.seg_cap / a->chunk * 8)
            : ccj::launch_gather_payload(p, pos, s);
  phase_mark(s, 3);
  if (!p.out_pos) (void)hipFreeAsync(pos, s);
  HIP_TRY(e, "partitioned probe + payload gather launch");
  return CCJ_OK;
}

}  // extern "C"

namespace {
// Ordered probe (ccj_probe_ordered): tables of at least this many LP slots take the partitioned
// route (below it the table sits in L2 / the Infinity Cache and probe_chunks' random reads hit).
constexpr uint64_t kOrderedMinSlots = 1ull << 22;

struct OrderedLayout {
  bool partitioned = false;
  PartLayout L{};
  uint32_t tile = 0;
  uint64_t n_tiles = 0;
  size_t pkeys = 0, row_map = 0, w_pos = 0, w_row = 0, cursors = 0, runs = 0, ovf_runs = 0, total = 0;
};

OrderedLayout ordered_layout(const ccj_table *t, uint64_t n_rows, uint32_t chunk) {
  OrderedLayout O;
  if (!t || t->info.size < kOrderedMinSlots || n_rows == 0 || chunk == 0 || n_rows >= (1ull << 32) ||
      (t->info.kind == CCJ_TABLE_CHAIN && !t->d_bucket))
    return O;
  O.L = part_layout(t, n_rows, chunk);
  // the split's run records and the unsplit address positions as u32: beyond 2^32 positions
  // (about 3.8e9 rows: segments + the n/16 overflow area) the one-pass route would wrap them
  if (O.L.pl.lo_bits == 0 || O.L.positions >= (1ull << 32)) return O;
  O.partitioned = true;
  O.tile = ccj::slot_split_tile_keys(1u << (O.L.pl.lo_bits + O.L.pl.hi_bits), true);
  O.n_tiles = (n_rows + O.tile - 1) / O.tile;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t at = off;
    off += align256(bytes);
    return at;
  };
  O.pkeys = take(O.L.positions * 8);
  O.row_map = take(O.L.positions * 4);
  O.w_pos = take(O.L.positions * 4);
  O.w_row = take(n_rows * 4);
  O.cursors = take(ccj::split_cursor_count(O.L.parts) * 4);
  O.runs = take(O.n_tiles * O.L.parts * 8);
  O.ovf_runs = take(O.n_tiles * O.L.parts * 4);
  O.total = off;
  return O;
}
}  // namespace

extern "C" {

size_t ccj_probe_ordered_workspace_size(const ccj_table *t, uint64_t n_rows, uint32_t chunk) {
  const OrderedLayout O = ordered_layout(t, n_rows, chunk);
  return O.partitioned ? O.total : 0;
}

int ccj_probe_ordered(const ccj_table *t, const ccj_probe_args *a, void *ws, size_t ws_bytes, ccj_stream stream) {
  PhaseScope phase_scope((hipStream_t)stream);
  ccj::ProbeParams p;
  if (int rc = fill_probe_params(t, a, p)) return rc;
  if (a->n_rows == 0) return CCJ_OK;
  hipStream_t s = (hipStream_t)stream;
  const OrderedLayout O = ordered_layout(t, a->n_rows, a->chunk);
  if (!O.partitioned || a->sel || a->out_pos || a->n_payload_cols) {  // small table / gathered input: one pass
    if (p.n_pay == 0) {
      HIP_TRY(ccj::launch_probe(t->info.kind, p, s), "probe launch");
      return CCJ_OK;
    }
    return ccj_probe(t, a, stream);
  }
  if (!ws || ws_bytes < O.total)
    return fail(CCJ_ERR_INVALID, "ccj_probe_ordered: workspace missing or smaller than ccj_probe_ordered_workspace_size");
  if (!a->status) return fail(CCJ_ERR_INVALID, "ccj_probe_ordered: the partitioned route needs args->status");
  char *w = (char *)ws;
  int64_t *pkeys = (int64_t *)(w + O.pkeys);
  uint32_t *row_map = (uint32_t *)(w + O.row_map), *w_pos = (uint32_t *)(w + O.w_pos);
  uint32_t *w_row = (uint32_t *)(w + O.w_row), *cursors = (uint32_t *)(w + O.cursors);
  uint2 *runs = (uint2 *)(w + O.runs);
  uint32_t *ovf_runs = (uint32_t *)(w + O.ovf_runs);
  const PartLayout &L = O.L;
  phase_mark(s, 0);
  // 1. one-pass slot split of the live rows, recording where every tile's runs went
  HIP_TRY(ccj::launch_slot_split_fixed(a->keys, a->n_rows, L.pl, L.seg_cap, L.ovf_base, L.ovf_cap, L.ovf_sub, cursors, pkeys,
                                       row_map, a->status, s, a->counts, a->chunk, runs, ovf_runs, 0, ~0u, 0, nullptr,
                                       ~0u, L.ovf_per_group),
          "slot split");
  phase_mark(s, 1);
  // 2. walk with the table window L2-resident: every row's Next-round word at its position
  ccj::ProbeParams q = p;
  q.keys = pkeys;
  q.counts = nullptr;
  q.seg_count = cursors;
  q.seg_parts = L.parts;
  q.seg_cap = L.seg_cap;
  q.ovf_base = L.ovf_base;
  q.ovf_sub = L.ovf_sub;
  q.swz_chunks = L.ovf_base / a->chunk;
  q.n_rows = L.positions;
  q.n_chunks = L.positions / a->chunk + (L.positions % a->chunk ? 1 : 0);
  q.xcd_swizzle = 1;
  q.out_w = w_pos;
  // distinct build keys: a row matches in at most one round, so 16-bit words carry it (halves the
  // words' three HBM crossings: walk -> unsplit -> emit)
  const uint32_t w16 = t->info.max_dup <= 1 && ccj_tune_int("CCJ_W16", 1) ? 1u : 0u;
  q.w16 = w16;
  HIP_TRY(ccj::launch_ordered_walk(t->info.kind, q, s), "ordered walk");
  phase_mark(s, 2);
  // 3. the words back into row order, one split tile per workgroup
  HIP_TRY(ccj::launch_unsplit_words(runs, ovf_runs, reinterpret_cast<const uint16_t *>(row_map), w_pos, w_row,
                                    a->n_rows, L.parts, O.tile, a->status, s,
                                    w16 != 0),
          "unsplit");
  // 4. per chunk: the reference's per-Next stream from its rows' words (probe_chunks' emit)
  p.in_w = w_row;
  p.w16 = w16;
  p.xcd_swizzle = 0;
  HIP_TRY(ccj::launch_ordered_emit(t->info.kind, p, s), "ordered emit");
  phase_mark(s, 3);  // gather: the round words back in row order + the reference-order emit
  return CCJ_OK;
}

int ccj_probe(const ccj_table *t, const ccj_probe_args *a, ccj_stream stream) {
  PhaseScope phase_scope((hipStream_t)stream);
  ccj::ProbeParams p;
  if (int rc = fill_probe_params(t, a, p)) return rc;
  if (a->n_rows == 0) return CCJ_OK;  // no chunks: nothing to launch
  hipStream_t s = (hipStream_t)stream;
  phase_mark(s, 0);
  if (p.n_pay == 0) {
    HIP_TRY(ccj::launch_probe(t->info.kind, p, s), "probe launch");
    phase_marks(s, 1, 3);  // probe_chunks fuses hash, match, gather and advance
    return CCJ_OK;
  }
  // Wide payload: the probe records every match's table position, a second pass gathers rows.
  uint32_t *pos = p.out_pos;
  if (!pos) HIP_TRY(hipMallocAsync((void **)&pos, p.n_chunks * p.cap * sizeof(uint32_t), s), "payload positions");
  ccj::ProbeParams q = p;
  q.out_pos = pos;
  q.n_pay = 0;
  hipError_t e = ccj::launch_probe(t->info.kind, q, s);
  phase_marks(s, 1, 2);
  if (e == hipSuccess) e = ccj::launch_gather_payload(p, pos, s);
  phase_mark(s, 3);
  if (!p.out_pos) (void)hipFreeAsync(pos, s);
  HIP_TRY(e, "probe + payload gather launch");
  return CCJ_OK;
}

size_t ccj_compact_workspace_size(uint64_t n_chunks, uint64_t cap, uint32_t chunk, uint32_t max_rounds,
                                  uint32_t threshold) {
  if (chunk == 0) return 0;
  return ccj::compact_workspace(n_chunks, cap, chunk, max_rounds, threshold);
}

int ccj_compact(const ccj_compact_args *a, ccj_stream stream) {
  if (!a) return fail(CCJ_ERR_INVALID, "ccj_compact: null args");
  if (a->chunk == 0 || a->chunk > ccj::kMaxChunk) return fail(CCJ_ERR_INVALID, "ccj_compact: chunk must be 1..2048");
  if (a->n_cols > CCJ_MAX_COLS) return fail(CCJ_ERR_INVALID, "ccj_compact: too many columns");
  if (a->out_cap_rows % a->chunk) return fail(CCJ_ERR_INVALID, "ccj_compact: out_cap_rows must be a multiple of chunk");
  if (a->n_chunks == 0) {
    if (a->out_n_chunks) HIP_TRY(hipMemsetAsync(a->out_n_chunks, 0, 8, (hipStream_t)stream), "memset");
    return CCJ_OK;
  }
  if (!a->count || !a->sel || !a->rounds || !a->round_counts || !a->out_chunk_counts || !a->workspace)
    return fail(CCJ_ERR_INVALID, "ccj_compact: missing buffer (round counts are required)");
  if (a->out_payload && !a->payload) return fail(CCJ_ERR_INVALID, "ccj_compact: out_payload needs payload");
  if (a->key_cols >> a->n_cols) return fail(CCJ_ERR_INVALID, "ccj_compact: key_cols names a column past n_cols");
  if (a->key_cols && !a->payload) return fail(CCJ_ERR_INVALID, "ccj_compact: key_cols needs payload");
  for (uint32_t q = 0; q < a->n_cols; ++q)
    if ((!a->cols[q] && !((a->key_cols >> q) & 1u)) || !a->out_cols[q])
      return fail(CCJ_ERR_INVALID, "ccj_compact: null column");
  if (a->workspace_bytes < ccj::compact_workspace(a->n_chunks, a->cap, a->chunk, a->max_rounds, a->threshold))
    return fail(CCJ_ERR_INVALID, "ccj_compact: workspace too small");
  HIP_TRY(ccj::launch_compact(*a, (hipStream_t)stream), "compact launch");
  return CCJ_OK;
}

size_t ccj_partition_workspace_size(uint64_t n, uint32_t parts) {
  return parts ? ccj::partition_workspace(n, parts) : 0;
}

int ccj_partition_by_owner(const int64_t *d_keys, uint64_t n, uint32_t parts, uint64_t row_base, int64_t *d_out_keys,
                           uint64_t *d_out_rows, uint64_t *d_out_counts, void *d_workspace, size_t workspace_bytes,
                           ccj_stream stream) {
  if (parts == 0 || parts > ccj::kMaxParts || (parts & (parts - 1)))
    return fail(CCJ_ERR_INVALID, "ccj_partition_by_owner: parts must be a power of two <= 64");
  if (!d_out_counts || (n && (!d_keys || !d_out_keys || !d_out_rows || !d_workspace)))
    return fail(CCJ_ERR_INVALID, "ccj_partition_by_owner: missing buffer");
  if (workspace_bytes < ccj::partition_workspace(n, parts))
    return fail(CCJ_ERR_INVALID, "ccj_partition_by_owner: workspace too small");
  if (n >= (1ull << 31) * 4096) return fail(CCJ_ERR_LIMIT, "ccj_partition_by_owner: too many keys");
  HIP_TRY(ccj::launch_partition(d_keys, n, parts, row_base, d_out_keys, d_out_rows, d_out_counts, d_workspace,
                                (hipStream_t)stream),
          "partition launch");
  return CCJ_OK;
}

int ccj_partition_by_owner_fixed(const int64_t *d_keys, uint64_t n, uint32_t parts, uint32_t row_base,
                                 uint64_t seg_cap, int64_t *d_out_keys, uint32_t *d_out_rows, uint64_t *d_out_counts,
                                 uint32_t *d_status, void *d_workspace, size_t workspace_bytes, ccj_stream stream) {
  if (parts == 0 || parts > ccj::kMaxParts || (parts & (parts - 1)))
    return fail(CCJ_ERR_INVALID, "ccj_partition_by_owner_fixed: parts must be a power of two <= 64");
  if (seg_cap == 0) return fail(CCJ_ERR_INVALID, "ccj_partition_by_owner_fixed: seg_cap == 0");
  if (!d_out_counts || !d_status || (n && (!d_keys || !d_out_keys || !d_out_rows || !d_workspace)))
    return fail(CCJ_ERR_INVALID, "ccj_partition_by_owner_fixed: missing buffer");
  if (workspace_bytes < ccj::partition_workspace(n, parts))
    return fail(CCJ_ERR_INVALID, "ccj_partition_by_owner_fixed: workspace too small");
  if ((uint64_t)row_base + n > (1ull << 32)) return fail(CCJ_ERR_LIMIT, "ccj_partition_by_owner_fixed: rows exceed u32");
  HIP_TRY(ccj::launch_partition_fixed(d_keys, n, parts, row_base, seg_cap, d_out_keys, d_out_rows, d_out_counts,
                                      d_status, d_workspace, (hipStream_t)stream),
          "partition launch");
  return CCJ_OK;
}

size_t ccj_partition_grouped_workspace_size(uint32_t parts) { return ccj::partition_grouped_workspace(parts); }

uint64_t ccj_partition_grouped_sub_cap(uint64_t n, uint32_t parts, uint32_t chunk) {
  return parts ? ccj::partition_grouped_sub_cap(n, parts, chunk) : 0;
}

int ccj_partition_by_owner_grouped(const int64_t *d_keys, uint64_t n, uint32_t parts, uint32_t row_base,
                                   uint64_t sub_cap, uint32_t self_last, int64_t *d_out_keys, uint32_t *d_out_rows,
                                   uint64_t *d_out_counts, uint32_t *d_status, void *d_workspace,
                                   size_t workspace_bytes, ccj_stream stream) {
  if (parts == 0 || parts > ccj::kMaxParts || (parts & (parts - 1)))
    return fail(CCJ_ERR_INVALID, "ccj_partition_by_owner_grouped: parts must be a power of two <= 64");
  if (sub_cap == 0 || sub_cap >= (1ull << 32)) return fail(CCJ_ERR_INVALID, "ccj_partition_by_owner_grouped: bad sub_cap");
  if (!d_out_counts || !d_status || !d_workspace || (n && (!d_keys || !d_out_keys || !d_out_rows)))
    return fail(CCJ_ERR_INVALID, "ccj_partition_by_owner_grouped: missing buffer");
  if (workspace_bytes < ccj::partition_grouped_workspace(parts))
    return fail(CCJ_ERR_INVALID, "ccj_partition_by_owner_grouped: workspace too small");
  if ((uint64_t)row_base + n > (1ull << 32)) return fail(CCJ_ERR_LIMIT, "ccj_partition_by_owner_grouped: rows exceed u32");
  HIP_TRY(ccj::launch_partition_grouped(d_keys, n, parts, row_base, sub_cap, d_out_keys, d_out_rows, d_out_counts,
                                        d_status, d_workspace, (hipStream_t)stream, self_last),
          "grouped partition launch");
  return CCJ_OK;
}

int ccj_segment_chunk_counts(const uint64_t *d_seg_counts, uint32_t n_segs, uint64_t seg_cap, uint32_t chunk,
                             uint32_t *d_out_counts, uint32_t *d_status, ccj_stream stream) {
  if (chunk == 0 || chunk > ccj::kMaxChunk || seg_cap % chunk)
    return fail(CCJ_ERR_INVALID, "ccj_segment_chunk_counts: seg_cap must be a multiple of chunk (1..2048)");
  if (n_segs && (!d_seg_counts || !d_out_counts)) return fail(CCJ_ERR_INVALID, "ccj_segment_chunk_counts: null");
  HIP_TRY(ccj::launch_segment_chunk_counts(d_seg_counts, n_segs, seg_cap, chunk, d_out_counts, d_status,
                                           (hipStream_t)stream),
          "segment chunk counts");
  return CCJ_OK;
}

int ccj_gen_uniform_keys(int64_t *d_out, uint64_t n, uint64_t seed, uint64_t first_row, uint64_t range,
                         ccj_stream stream) {
  if ((!d_out && n) || range == 0) return fail(CCJ_ERR_INVALID, "ccj_gen_uniform_keys: bad argument");
  HIP_TRY(ccj::launch_gen_uniform(d_out, n, seed, first_row, range, (hipStream_t)stream), "gen uniform keys");
  return CCJ_OK;
}

int ccj_copy_device(void *d_dst, const void *d_src, uint64_t bytes, ccj_stream stream) {
  if (bytes % 16 || (bytes && (!d_dst || !d_src)) || ((uintptr_t)d_dst | (uintptr_t)d_src) % 16)
    return fail(CCJ_ERR_INVALID, "ccj_copy_device: buffers must be 16-byte aligned, bytes a multiple of 16");
  if (bytes) HIP_TRY(ccj::launch_copy16(d_src, d_dst, bytes / 16, (hipStream_t)stream), "copy");
  return CCJ_OK;
}

int ccj_gen_c3_keys(int64_t *d_out, uint64_t n, uint64_t seed, uint64_t first_row, uint64_t n_build, uint64_t cf,
                    uint32_t hit_ppm, ccj_stream stream) {
  if ((!d_out && n) || cf == 0 || n_build == 0 || n_build >= (1ull << 62) || hit_ppm > 1000000)
    return fail(CCJ_ERR_INVALID, "ccj_gen_c3_keys: bad argument");
  const uint64_t n_unique = n_build / cf + (n_build % cf != 0);
  if (n_unique >= (1ull << 32)) return fail(CCJ_ERR_LIMIT, "ccj_gen_c3_keys: more than 2^32 distinct build keys");
  // Zipf s = 1 rank table over the n_unique build keys (host, untimed): one device copy per
  // (device, table size), made once and never overwritten, so a generator kernel still running on
  // any stream never sees it change; the map is guarded for concurrent callers.
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev), "zipf table");
  const uint32_t *d_zipf = nullptr;
  {
    static std::mutex mu;
    static std::map<std::pair<int, uint64_t>, uint32_t *> tables;
    std::lock_guard<std::mutex> lock(mu);
    auto it = tables.find({dev, n_unique});
    if (it == tables.end()) {
      std::vector<uint32_t> t(ccj::kZipfBuckets + 1);
      zipf_table(n_unique, t.data());
      uint32_t *d = nullptr;
      HIP_TRY(hipMalloc((void **)&d, t.size() * sizeof(uint32_t)), "zipf table");
      // on the caller's stream, then waited for: the host buffer dies with this scope
      HIP_TRY(hipMemcpyAsync(d, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice, (hipStream_t)stream),
              "zipf table");
      HIP_TRY(hipStreamSynchronize((hipStream_t)stream), "zipf table");
      it = tables.emplace(std::make_pair(dev, n_unique), d).first;
    }
    d_zipf = it->second;
  }
  HIP_TRY(ccj::launch_gen_c3(d_out, n, seed, first_row, n_build, cf, hit_ppm, d_zipf, (hipStream_t)stream),
          "gen c3 keys");
  return CCJ_OK;
}

int ccj_gen_reference_keys(int64_t *d_out, uint64_t first, uint64_t n, uint64_t n_total, uint64_t cf,
                           ccj_stream stream) {
  if ((!d_out && n) || cf == 0 || first + n > n_total) return fail(CCJ_ERR_INVALID, "ccj_gen_reference_keys: bad argument");
  HIP_TRY(ccj::launch_gen_reference_keys(d_out, first, n, n_total, cf, (hipStream_t)stream), "gen reference keys");
  return CCJ_OK;
}

int ccj_probe_cost(const ccj_table *t, const int64_t *d_keys, uint64_t n, uint64_t *d_acc, ccj_stream stream) {
  if (!t || (!d_keys && n) || !d_acc) return fail(CCJ_ERR_INVALID, "ccj_probe_cost: bad argument");
  HIP_TRY(ccj::launch_probe_cost(t->info.kind, t->d_table, t->d_off, (uint32_t)(t->info.size - 1), d_keys, n,
                                 (unsigned long long *)d_acc, (hipStream_t)stream),
          "probe cost");
  return CCJ_OK;
}

int ccj_probe_cost_walk(const ccj_table *t, const int64_t *d_keys, uint64_t n, uint64_t *d_acc, ccj_stream stream) {
  if (!t || (!d_keys && n) || !d_acc) return fail(CCJ_ERR_INVALID, "ccj_probe_cost_walk: bad argument");
  HIP_TRY(ccj::launch_probe_cost(t->info.kind, t->d_table, t->d_off, (uint32_t)(t->info.size - 1), d_keys, n,
                                 (unsigned long long *)d_acc, (hipStream_t)stream, true),
          "probe cost (walk)");
  return CCJ_OK;
}

int ccj_probe_visits(const ccj_table *t, const int64_t *d_keys, const uint32_t *d_sel, uint32_t count,
                     uint32_t max_rounds, int64_t *d_vals, uint32_t *d_len, ccj_stream stream) {
  if (!t || (count && (!d_keys || !d_vals || !d_len || max_rounds == 0)))
    return fail(CCJ_ERR_INVALID, "ccj_probe_visits: bad argument");
  HIP_TRY(ccj::launch_probe_visits(t->info.kind, t->d_table, t->d_off, (uint32_t)(t->info.size - 1), d_keys, d_sel,
                                   count, max_rounds, d_vals, d_len, (hipStream_t)stream),
          "probe visits");
  return CCJ_OK;
}

int ccj_result_checksum(const uint32_t *out_count, const uint32_t *out_sel, const int64_t *out_payload,
                        uint64_t n_chunks, uint64_t cap, uint32_t chunk, uint64_t row_base, uint64_t *d_acc,
                        ccj_stream stream) {
  if ((!out_count || !out_sel || !out_payload) && n_chunks) return fail(CCJ_ERR_INVALID, "ccj_result_checksum: null");
  if (!d_acc) return fail(CCJ_ERR_INVALID, "ccj_result_checksum: null acc");
  HIP_TRY(ccj::launch_result_checksum(out_count, out_sel, out_payload, n_chunks, cap, chunk, row_base, nullptr,
                                      (unsigned long long *)d_acc, (hipStream_t)stream),
          "result checksum");
  return CCJ_OK;
}

int ccj_result_checksum_mapped(const uint32_t *out_count, const uint32_t *out_sel, const int64_t *out_payload,
                               uint64_t n_chunks, uint64_t cap, uint32_t chunk, const uint64_t *row_map,
                               uint64_t *d_acc, ccj_stream stream) {
  if ((!out_count || !out_sel || !out_payload || !row_map) && n_chunks)
    return fail(CCJ_ERR_INVALID, "ccj_result_checksum_mapped: null");
  if (!d_acc) return fail(CCJ_ERR_INVALID, "ccj_result_checksum_mapped: null acc");
  HIP_TRY(ccj::launch_result_checksum(out_count, out_sel, out_payload, n_chunks, cap, chunk, 0, row_map,
                                      (unsigned long long *)d_acc, (hipStream_t)stream),
          "result checksum");
  return CCJ_OK;
}

}  // extern "C"

// ---- CU-masked streams ---------------------------------------------------------------------
namespace {
std::mutex g_mask_mu;
std::unordered_map<hipStream_t, uint32_t> g_mask_cus;  // streams made here -> their CU count

uint32_t device_cus() {
  int dev = 0, n = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
  return (uint32_t)(n > 0 ? n : 1);
}
}  // namespace

uint32_t ccj::stream_cus(hipStream_t s) {
  {
    std::lock_guard<std::mutex> lk(g_mask_mu);
    const auto it = g_mask_cus.find(s);
    if (it != g_mask_cus.end()) return it->second;
  }
  static const uint32_t all = device_cus();
  return all;
}

int ccj_stream_create_cu_masked(const uint32_t *cu_mask, uint32_t mask_words, ccj_stream *out) {
  if (!cu_mask || !out || mask_words == 0) return fail(CCJ_ERR_INVALID, "ccj_stream_create_cu_masked: missing mask");
  const uint32_t n = device_cus();
  uint32_t cus = 0;
  for (uint32_t i = 0; i < n && i / 32 < mask_words; ++i) cus += (cu_mask[i / 32] >> (i % 32)) & 1u;
  if (cus == 0) return fail(CCJ_ERR_INVALID, "ccj_stream_create_cu_masked: the mask selects no CU");
  hipStream_t s = nullptr;
  HIP_TRY(hipExtStreamCreateWithCUMask(&s, mask_words, cu_mask), "hipExtStreamCreateWithCUMask");
  {
    std::lock_guard<std::mutex> lk(g_mask_mu);
    g_mask_cus[s] = cus;
  }
  *out = (ccj_stream)s;
  return CCJ_OK;
}

int ccj_stream_destroy(ccj_stream stream) {
  if (!stream) return fail(CCJ_ERR_INVALID, "ccj_stream_destroy: NULL stream");
  {
    std::lock_guard<std::mutex> lk(g_mask_mu);
    g_mask_cus.erase((hipStream_t)stream);
  }
  HIP_TRY(hipStreamDestroy((hipStream_t)stream), "hipStreamDestroy");
  return CCJ_OK;
}

int ccj_device_cus(uint32_t *out) {
  if (!out) return fail(CCJ_ERR_INVALID, "ccj_device_cus: NULL out");
  *out = device_cus();
  return CCJ_OK;
}
