// ccj_internal.h — shared between the HIP kernels (ccj_kernels.hip) and the C ABI (ccj_api.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "ccj.h"

struct ccj_table {
  ccj_table_info info;
  int64_t *d_table = nullptr;   // LP slots / chain keys
  uint32_t *d_off = nullptr;    // chain CSR offsets (size + 1)
  int64_t *d_bucket = nullptr;  // chain: per bucket {start | len << 32, first chain key} (16 B)
  // chain: per bucket {start | len << 32 | fp0 << 40 | fp1 << 52} (8 B): the 12-bit fingerprints
  // (bucket_fp) of the first two chain keys, len < 2^8 (absent when a chain is longer: the 16-byte
  // records serve alone)
  uint64_t *d_bucket8 = nullptr;
  // chain: 2 bits per bucket, 16 buckets per word — 0 empty, 1 / 2 a one-key chain whose key has hash
  // bit 40 = 0 / 1, 3 a longer chain (probe_chain_filt's LDS filter); absent for tables of < 128 buckets
  uint32_t *d_filt = nullptr;
  uint32_t *d_row = nullptr;    // table position -> build tuple index (LP: kNoRow for empty slots)
  uint64_t positions = 0;       // allocated positions (LP slots / chain keys, padded)
  int64_t *d_pay = nullptr;     // position-major payload rows [positions][n_pay]
  uint32_t n_pay = 0;
  int device = 0;
  // LP window index of the rank walk (ccj_rank.hip; absent: the slot-array walk): occupancy bits,
  // occupied slots before each 64-slot word, occupied slots' keys in slot order; built for windows
  // of rank_wbits slots
  uint64_t *d_occ = nullptr;
  uint32_t *d_pre = nullptr;
  int64_t *d_ckeys = nullptr;
  uint32_t rank_wbits = 0;
};

namespace ccj {

// hash_functions.h:8-16 — the reference's bucket/slot function (NOT MurmurHash3 fmix64).
__host__ __device__ __forceinline__ uint64_t murmurhash64(uint64_t x) {
  x ^= x >> 32;
  x *= 0xd6e8feb86659fd93ULL;
  x ^= x >> 32;
  x *= 0xd6e8feb86659fd93ULL;
  x ^= x >> 32;
  return x;
}

// The high 32 bits of murmurhash64(x) (the last xor-shift leaves them as the second product's
// high word, which needs three 32-bit multiplies, not four).
__host__ __device__ __forceinline__ uint32_t murmurhash64_hi(uint64_t x) {
  constexpr uint64_t kC = 0xd6e8feb86659fd93ULL;
  x ^= x >> 32;
  x *= kC;
  x ^= x >> 32;
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return (uint32_t)(((uint64_t)lo * (uint32_t)kC) >> 32) + lo * (uint32_t)(kC >> 32) + hi * (uint32_t)kC;
}

// Fingerprint of a chain key for the 8-byte bucket records: 12 hash bits far above any bucket index.
__host__ __device__ __forceinline__ uint32_t bucket_fp(uint64_t h) { return (uint32_t)(h >> 52); }
// 8-byte bucket record {start | len << 32 | fp(node 0) << 40 | fp(node 1) << 52} (len < 256): the
// first chain node that can hold a key of fingerprint kfp — nodes 0 and 1 are skipped when their
// fingerprints differ — or start + len when none can (the key is not in the chain).
__host__ __device__ __forceinline__ uint32_t rec8_first(uint64_t r, uint32_t kfp) {
  const uint32_t st = (uint32_t)r, len = (uint32_t)(r >> 32) & 0xFFu;
  const bool m0 = ((uint32_t)(r >> 40) & 0xFFFu) == kfp;
  const bool m1 = len >= 2u && ((uint32_t)(r >> 52) & 0xFFFu) == kfp;
  const uint32_t c = m0 ? st : m1 ? st + 1u : st + 2u;
  return c < st + len ? c : st + len;
}

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr uint32_t kMaxChunk = 2048;
constexpr uint32_t kMaxParts = 64;  // owner partitions (GPUs) per multisplit

struct ProbeParams {
  const int64_t *table;
  const uint32_t *off;
  // chain only, optional: bucket records {start | len << 32, first key} — one 16-byte load gives
  // the chain's range and its round-0 candidate (most chains at load 1/2 have one key)
  const longlong2 *bucket;
  // chain only, optional: 8-byte bucket records {start | len << 32 | fp0 << 40 | fp1 << 52} (the
  // partitioned walks): a key whose fingerprint differs from fp0 / fp1 is not the chain's first /
  // second key, so misses on chains of up to two keys end at the record, and a partition's records
  // take half the L2
  const uint64_t *bucket8;
  uint32_t mask;  // size - 1 (size <= 2^32)
  const int64_t *keys;
  const uint32_t *sel;
  const uint32_t *counts;
  uint64_t n_rows;
  uint64_t n_chunks;
  uint32_t chunk;
  uint32_t max_rounds;
  uint64_t cap;
  uint32_t *out_count;
  uint32_t *out_sel;
  int64_t *out_payload;
  uint32_t *out_rounds;
  uint32_t *out_round_counts;
  uint32_t *status;
  uint32_t *out_pos;
  const int64_t *pay;  // position-major payload rows
  uint32_t n_pay;      // payload columns gathered (<= CCJ_MAX_PAYLOAD_COLS)
  uint32_t pay_stride; // payload columns stored per position
  int64_t *out_cols[CCJ_MAX_PAYLOAD_COLS];
  // Pipeline input (ccj_pipeline, no-compaction mode): chunk c's rows start at chunk_base[c] of
  // `keys` (sel must be NULL, counts required) and its outputs at out_base[c]; NULL = c*chunk, c*cap.
  const uint64_t *chunk_base;
  const uint64_t *out_base;
  // Fixed-capacity partitioned input (ccj_probe_partitioned): chunk c's live rows are the first
  // min(seg_count[seg_cursor_index(seg_parts, g, d)] - offset, chunk) of it, segment d*8+g =
  // positions / seg_cap.
  const uint32_t *seg_count;
  uint32_t seg_parts;
  uint64_t seg_cap;
  // overflow area [ovf_base, n_rows): runs that did not fit their segment (key skew), in 8
  // sub-areas of ovf_sub positions (a multiple of chunk), one per tile group g (XCD) with fill
  // level seg_count[ovf_cursor_index(seg_parts, k)] (k < kOvfSubs).  0 = no overflow area.
  uint64_t ovf_base;
  uint64_t ovf_sub;
  uint64_t swz_chunks;   // chunks dealt to XCDs in contiguous ranges (0: all); the overflow area's
                         // chunks follow in plain order so they do not unbalance the XCDs' shares
  uint32_t xcd_swizzle;  // 1: consecutive chunks go to the same XCD (L2 reuse of partitioned input)
  // probe_walk's emit: kEmitWave = per-wave placement; else the chunk's output staged in LDS in row
  // order and written with 16-byte buffer stores of this cache policy (aux bits: 2 nt, 16 sc1)
  uint32_t emit_pol;
  // 1: keys IS out_payload (ccj_probe_partitioned, cap == chunk): the split wrote every row's key
  // at its own output position, so a chunk whose rows all match once already holds its payload
  uint32_t keys_in_out;
  // 1 (CCJ_PART_ROWS, with keys_in_out): out_sel holds each match's original row, written by the
  // split at every position; the walk only compacts chunks with misses
  uint32_t rows_in_sel;
  uint32_t ablate;       // timing-only ablations (tuning build only: CCJ_ABLATE)
  unsigned long long *stats;  // tuning build only (CCJ_STATS): per-phase cycle sums of the walk
  // Ordered probe (ccj_probe_ordered): round words per position (walk) / per row (emit input)
  uint32_t *out_w;
  const uint32_t *in_w;
  // 1: the round words are 16-bit, L << 7 | the row's match round (127: none) — tables whose keys
  // are distinct (max_dup 1), where a row matches in at most one round
  uint32_t w16;
  // probe_walk: first chunk of the launch (blockIdx.x + chunk0; the rank walk's overflow-area pass)
  uint64_t chunk0;
  // probe_walk1, partitioned input: each workgroup first touches (LDS-DMA into its own scratch)
  // the slice of table lines that the chunk pf_dist chunks later in its XCD's order will need, so a
  // window's first reads hit L2 (0: off); pf_lines lines per chunk
  uint64_t pf_dist;
  uint32_t pf_lines;
  uint32_t kp_dist;  // tuning build (CCJ_ABLATE 0x400): key-line touch distance in chunks
  // probe_walk1: the table's keys are distinct (max_dup 1) and no rounds are asked for, so a row
  // stops at its match instead of walking to the end of its run (same matches and multiplicities)
  uint32_t first_match;
  uint32_t key_aux;  // tuning build (CCJ_KEY_AUX): probe_walk2's key loads as buffer loads, policy key_aux - 1
  // chaining, partitioned walk: the table's bucket filter (2 bits per bucket, 16 per word;
  // ccj_build.hip) and the partitions' window bits — probe_chain_filt holds one partition's filter
  // in LDS; NULL: probe_chain_win
  const uint32_t *filt;
  uint32_t filt_wb;
  // C5 under CCJ_PART_ROWS (walk_emit_pos_sub): each chunk's matches written in order of their slot's
  // sub-range (slot >> sub_shift) & 7 — 8 sub-ranges of a partition's window, each a 4 MiB slab of
  // payload rows at C5 — with out_sub[c * 8 + s] = where sub-range s starts in chunk c, so the payload
  // gather can take one slab of every chunk of a partition at a time (NULL: row order)
  uint32_t *out_sub;
  uint32_t sub_shift;
};
constexpr uint32_t kNoRow = 0xFFFFFFFFu;
constexpr uint32_t kEmitWave = 0xFFFFFFFFu;

// Launchers (ccj_kernels.hip).  Return hipError_t of the launch.
hipError_t launch_probe(int kind, const ProbeParams &p, hipStream_t s);
hipError_t launch_probe_flat(int kind, const ProbeParams &p, hipStream_t s);
// Ordered probe (ccj_probe_ordered, LP or chaining): walk of the slot / bucket partitioned column
// leaving each row's round word at its position (p.out_w); the words back into row order, one
// split tile per workgroup; the reference-order emit of each chunk from its rows' words (p.in_w).
hipError_t launch_ordered_walk(int kind, const ProbeParams &p, hipStream_t s);
// CUs a persistent grid may use on stream s: the popcount of its CU mask for streams made by
// ccj_stream_create_cu_masked, else the device's CU count.
uint32_t stream_cus(hipStream_t s);
hipError_t launch_unsplit_words(const uint2 *runs, const uint32_t *ovf_runs, const uint16_t *row_loc,
                                const void *w_pos, void *w_row, uint64_t n, uint32_t parts, uint32_t tile,
                                uint32_t *status, hipStream_t s, bool w16);
hipError_t launch_ordered_emit(int kind, const ProbeParams &p, hipStream_t s);
// C5 payload columns of a finished probe: out_cols[q][slot] = payload row of pos[slot], column q.
// With p.out_sub (the walk's sub-range order, 8 columns): the partitioned layout's chunks are taken
// slab by slab — XCD x, partition d of its range, sub-range s, a group of the partition's chunks —
// so that the slab's payload rows stay in that XCD's L2 (parts partitions of cpp chunks each, the
// overflow area's chunks after them in plain order).
hipError_t launch_gather_payload(const ProbeParams &p, const uint32_t *pos, hipStream_t s, uint32_t parts = 0,
                                 uint64_t cpp = 0);
// the gather kernel this thread's last launch_gather_payload chose (ccj_last_gather_kernel)
const char *last_gather_kernel();
hipError_t launch_gen_reference_keys(int64_t *out, uint64_t first, uint64_t n, uint64_t n_total, uint64_t cf,
                                     hipStream_t s);
hipError_t launch_fill(int64_t *p, uint64_t n, int64_t v, hipStream_t s);
hipError_t launch_iota_u32(uint32_t *p, uint64_t n, hipStream_t s);
hipError_t launch_copy16(const void *src, void *dst, uint64_t n16, hipStream_t s);
hipError_t launch_lp_insert(const int64_t *keys, uint64_t n, int64_t *slots, uint32_t *slot_row, uint32_t mask,
                            hipStream_t s);
hipError_t launch_scatter_payload(const int64_t *src, uint32_t n_cols, const uint32_t *row, uint64_t positions,
                                  int64_t *dst, hipStream_t s);
// Per-segment run statistics of an LP slot array (segment = 4096 slots): 4 x uint32 per segment:
// {leading run, trailing run, longest run, all occupied}.
// Largest multiplicity of one key (max_run = longest occupied run bounds the walk).
hipError_t launch_lp_max_dup(const int64_t *slots, uint64_t n_slots, uint32_t max_run, uint32_t *out, hipStream_t s);
hipError_t launch_lp_runs(const int64_t *slots, uint64_t n_slots, uint32_t *seg_stats, hipStream_t s);
// The chaining table built on the device (ccj_build.hip): stable bucket sort -> CSR, row map,
// 16- and 8-byte bucket records, longest chain; known_dup = 0: max_dup computed from the keys.
int build_chain_device(const int64_t *d_keys, uint64_t n, hipStream_t s, uint64_t known_dup, ccj_table **out);
// The bucket filter of a finished chaining table (t->d_filt), from its offsets and chain keys.
hipError_t build_chain_filter(ccj_table *t, hipStream_t s);
constexpr uint64_t kRunSegment = 4096;
// C3 probe stream; zipf: device copy of the rank table (kZipfBuckets + 1 entries, zipf_table()).
hipError_t launch_gen_c3(int64_t *out, uint64_t n, uint64_t seed, uint64_t first_row, uint64_t n_build, uint64_t cf,
                         uint32_t hit_ppm, const uint32_t *zipf, hipStream_t s);
constexpr uint32_t kZipfBits = 16, kZipfBuckets = 1u << kZipfBits;
hipError_t launch_gen_uniform(int64_t *out, uint64_t n, uint64_t seed, uint64_t first_row, uint64_t range,
                              hipStream_t s);
hipError_t launch_probe_visits(int kind, const int64_t *table, const uint32_t *off, uint32_t mask,
                               const int64_t *keys, const uint32_t *sel, uint32_t count, uint32_t max_rounds,
                               int64_t *vals, uint32_t *len, hipStream_t s);
hipError_t launch_probe_cost(int kind, const int64_t *table, const uint32_t *off, uint32_t mask,
                             const int64_t *keys, uint64_t n, unsigned long long *acc, hipStream_t s,
                             bool walk = false);
hipError_t launch_result_checksum(const uint32_t *count, const uint32_t *sel, const int64_t *payload,
                                  uint64_t n_chunks, uint64_t cap, uint32_t chunk, uint64_t row_base,
                                  const uint64_t *row_map, unsigned long long *acc, hipStream_t s);

// Error reporting of the C ABI (ccj_api.hip): sets ccj_last_error() and returns code.
int api_fail(int code, const std::string &msg);
int api_check_device();

size_t compact_workspace(uint64_t n_chunks, uint64_t cap, uint32_t chunk, uint32_t max_rounds, uint32_t threshold);
hipError_t launch_compact(const ccj_compact_args &a, hipStream_t s);
size_t partition_workspace(uint64_t n, uint32_t parts);
// Slot-range partitioning for the L2-resident probe: partition p = slot >> window_bits, with the
// partition bits split into a low digit (first LSD pass) and a high digit (second pass).
// 2^19 slots = 4 MiB of LP table per partition (chaining: 2^18 buckets of 16-byte records).  At C2
// windows of 2 / 4 / 8 MiB measured split + walk 7.1 + 10.5 / 6.3 + 10.7 / 5.8 + 12.0 ms: the
// split's runs grow with fewer partitions, the walk's L2 reuse shrinks with bigger windows.
constexpr uint32_t kWindowBits = 19;
constexpr uint32_t kSplitPartBits = 10;  // at most 1024 partitions (larger tables: larger windows)
// The fixed-capacity split's overflow area (key skew): up to kOvfPerGroup sub-areas per tile group
// (XCD), each with its own cursor on its own 128-byte line, so that the Zipf-hot partitions'
// overflow reservations of one XCD's workgroups do not all queue on one address (a partition's
// run takes sub-area (partition + workgroup) mod the group's count: balanced fills).  The layout
// (part_layout) splits a group's room only when each part can still hold a whole tile's run.
constexpr uint32_t kOvfPerGroup = 4;
constexpr uint32_t kOvfSubs = 8 * kOvfPerGroup;
constexpr uint32_t kOvfCurStride = 32;  // u32 cursors between two overflow cursors
// Segment cursors: segment (partition d, tile group g) counts at seg_cursor_index(parts, g, d),
// group-major, each tile group's cursors starting on their own 128-byte line: with few partitions
// (the owner split: one per rank) the XCDs' reservations then never share a line — at one owner
// 0.218 -> 0.145 ms per 2^25 keys (profiles/r5_ab_cursor_lines.log).  Packed within a group: one
// cursor per line instead measured slower for the slot split's 512 partitions (4.85 -> 5.13 ms at
// C2: a wave's 64 reservations then touch 64 lines instead of 2).
// (Spreading the cursors 4 or 8 u32 apart inside a group measured slower too at C2: split 4.85
// -> 5.01 / 4.93 ms, profiles/r5_ab_cursor_spread.log.)
__host__ __device__ constexpr uint64_t seg_group_stride(uint32_t parts) { return parts > 32u ? parts : 32u; }
__host__ __device__ constexpr uint64_t seg_cursor_index(uint32_t parts, uint32_t g, uint32_t d) {
  return (uint64_t)g * seg_group_stride(parts) + d;
}
// cursors of the fixed-capacity split: 8 groups of segment cursors, then the overflow cursors
__host__ __device__ constexpr uint64_t split_cursor_count(uint32_t parts) {
  return 8ull * seg_group_stride(parts) + (uint64_t)kOvfSubs * kOvfCurStride;
}
__host__ __device__ constexpr uint64_t ovf_cursor_index(uint32_t parts, uint32_t sub) {
  return 8ull * seg_group_stride(parts) + (uint64_t)sub * kOvfCurStride;
}
struct SlotPlan {
  uint32_t window_bits, lo_bits, hi_bits;
};
// kind: LP windows are 2^kWindowBits slots (8 B each); chaining windows 2^(kWindowBits-1) buckets
// (16-byte bucket records, plus their chains' keys) — 2 MiB of table either way.
SlotPlan slot_plan(uint64_t table_size, int kind = CCJ_TABLE_LP);
size_t slot_partition_workspace(uint64_t n, const SlotPlan &pl);
hipError_t launch_slot_partition(const int64_t *keys, uint64_t n, const SlotPlan &pl, int64_t *out_keys,
                                 uint32_t *out_rows, void *ws, hipStream_t s);
// One-pass fixed-capacity form: segment (partition d, XCD group g) = positions [(d*8+g)*cap, +cap);
// cursors[seg_cursor_index(parts, g, d)] = rows that went to it (may exceed cap:
// CCJ_FLAG_PART_OVERFLOW raised); the overflow cursors follow at ovf_cursor_index(parts, k).
uint64_t slot_seg_cap(uint64_t n, const SlotPlan &pl, uint32_t chunk);
// Exclusive prefix sums of n values (ccj_scan.hip): out[i] = in[0] + ... + in[i-1] (in may be
// out; u32 sums wrap as the values do); *total (optional, device) = the sum of all n.  tmp:
// scan_u64_temp_bytes(n) bytes (either width).
size_t scan_u64_temp_bytes(uint64_t n);
hipError_t scan_exclusive_u64(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *total, void *tmp,
                              hipStream_t s);
hipError_t scan_exclusive_u32(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *total, void *tmp,
                              hipStream_t s);
// Stable LSD radix sort, 8-bit digits (ccj_sort.hip, the chaining build's bucket sort): sorts by bits
// [0, end_bit) of the keys, ping-ponging between keys/vals and keys_alt/vals_alt; *in_alt = the
// result is in the _alt arrays.  Digits equal in every key are skipped.  tmp: radix_sort_temp_bytes(n).
size_t radix_sort_temp_bytes(uint64_t n);
hipError_t radix_sort_pairs_u32(uint32_t *keys, uint32_t *keys_alt, uint32_t *vals, uint32_t *vals_alt, uint64_t n,
                                uint32_t end_bit, void *tmp, hipStream_t s, bool *in_alt);
hipError_t radix_sort_keys_u64(uint64_t *keys, uint64_t *keys_alt, uint64_t n, void *tmp, hipStream_t s,
                               bool *in_alt);
// cursors[ovf_cursor_index(parts, k)] = rows put in overflow sub-area k < kOvfSubs (tile group
// k / kOvfPerGroup) = [ovf_base + k * ovf_sub, + ovf_sub) (ovf_sub = 0: no overflow area); the last
// 64 positions of the area [ovf_base, ovf_base + ovf_cap) are the pipelined form's sink; cursors
// holds split_cursor_count(parts) entries.
// counts: live rows per input chunk.  runs (optional; the ordered probe): per (tile, partition)
// {segment position of the run, segment length | overflow-area length << 16}; ovf_runs: the
// overflow-area position where that length is non-zero.  Tiles are slot_split_tile_keys(parts, runs) keys.
// With runs, out_rows receives each position's row INSIDE ITS TILE as uint16_t (the unsplit's input).
hipError_t launch_slot_split_fixed(const int64_t *keys, uint64_t n, const SlotPlan &pl, uint64_t cap,
                                   uint64_t ovf_base, uint64_t ovf_cap, uint64_t ovf_sub, uint32_t *cursors, int64_t *out_keys,
                                   uint32_t *out_rows, uint32_t *status, hipStream_t s,
                                   const uint32_t *counts = nullptr, uint32_t chunk = 0, uint2 *runs = nullptr,
                                   uint32_t *ovf_runs = nullptr, uint32_t row_base = 0, uint32_t shift = ~0u,
                                   uint32_t wgs = 0, void *sink = nullptr, uint32_t self_last = ~0u,
                                   uint32_t ovf_per_group = 1);
// Bytes of device memory the split writes its inactive lanes' stores to when the overflow area
// cannot hold them (launch_slot_split_fixed's `sink`; 8 XCD groups x 8 positions of key + row).
constexpr size_t kSplitSinkBytes = 8 * 8 * 16;
size_t partition_grouped_workspace(uint32_t parts);
uint64_t partition_grouped_sub_cap(uint64_t n, uint32_t parts, uint32_t chunk);
hipError_t launch_partition_grouped(const int64_t *keys, uint64_t n, uint32_t parts, uint32_t row_base,
                                    uint64_t sub_cap, int64_t *out_keys, uint32_t *out_rows, uint64_t *out_counts,
                                    uint32_t *status, void *ws, hipStream_t s, uint32_t self_last = ~0u);
uint32_t slot_split_tile_keys(uint32_t parts, bool runs = false);
hipError_t launch_partition_fixed(const int64_t *keys, uint64_t n, uint32_t parts, uint32_t row_base, uint64_t seg_cap,
                                  int64_t *out_keys, uint32_t *out_rows, uint64_t *out_counts, uint32_t *status,
                                  void *ws, hipStream_t s);
// Rank walk (ccj_rank.hip): the LP window index in LDS, keys from the compact key array.
struct RankIndex {
  const uint64_t *occ;
  const uint32_t *pre;
  const int64_t *ckeys;
  uint32_t wbits;
};
bool rank_walk_fits(uint32_t window_bits);
constexpr uint32_t kRankChunkMultiple = 512;
// occ + cnt (per-word occupied counts, scratch) on the device, pre = exclusive scan of cnt
hipError_t launch_rank_index(const int64_t *slots, uint64_t n_slots, uint64_t *occ, uint32_t *pre, uint32_t *cnt,
                             hipStream_t s);
hipError_t launch_rank_compact_keys(const int64_t *slots, uint64_t n_slots, const uint64_t *occ, const uint32_t *pre,
                                    int64_t *ckeys, hipStream_t s);
size_t rank_workspace(uint64_t positions, uint32_t parts);
hipError_t launch_probe_rank(const ProbeParams &p, const RankIndex &ix, void *ws, hipStream_t s);
hipError_t launch_segment_chunk_counts(const uint64_t *counts, uint32_t n_segs, uint64_t seg_cap, uint32_t chunk,
                                       uint32_t *out, uint32_t *status, hipStream_t s);
hipError_t launch_partition(const int64_t *keys, uint64_t n, uint32_t parts, uint64_t row_base, int64_t *out_keys,
                            uint64_t *out_rows, uint64_t *out_counts, void *ws, hipStream_t s);

}  // namespace ccj
