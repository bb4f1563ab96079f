/* ccj.h — C ABI of the MI355X hash-join probe / chunk-compaction engine (libccj.so).
 *
 * This is the drop-in boundary for the reference's hot path.  The reference has
 * no FFI: its operator surface is C++ in namespace simd_compaction.  Each entry point below names
 * the reference interface it replaces; the C++ host facade (host/ccj_operators.h) re-exposes that
 * surface on top of this ABI, and INTEGRATION.md shows the bindings a maintainer would add.
 *
 * Conventions
 *  - C linkage, no exceptions cross the boundary.  Every call returns CCJ_OK (0) or a negative
 *    status; ccj_last_error() (thread-local) describes the last failure.
 *  - Device pointers are caller-owned unless created by ccj_table_*; calls taking a stream are
 *    stream-ordered and never synchronise the host (graph-capturable), except the table builders.
 *  - A built table is immutable: concurrent probes on different streams are allowed.
 *  - There is no CPU fallback.  Without a usable gfx950 device every call fails with
 *    CCJ_ERR_NO_DEVICE.
 *  - All keys are int64; -1 is the reserved empty marker (linear_probing_ht.cpp:7, base.h:52).
 */
#ifndef CCJ_H
#define CCJ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CCJ_ABI_VERSION 15  /* 15: ccj_build_hash, ccj_last_gather_kernel; 14: ccj_partition_by_owner_grouped's self_last (the own rank's segment last); 13: ccj_compact_args.key_cols, per-XCD overflow sub-areas of the partitioned layout; 12: chaining tables built on the device (stable bucket sort), ccj_table_get_arrays; 11: the rank walk in the tuning build only; 10: CCJ_PART_ROWS with positions / payload columns; 9: CCJ_PART_SHARE, CU-masked streams; 8: CCJ_PART_RANK; 7: CCJ_PART_ROWS */

enum ccj_status {
  CCJ_OK = 0,
  CCJ_ERR_INVALID = -1,   /* bad argument */
  CCJ_ERR_HIP = -2,       /* HIP runtime error */
  CCJ_ERR_NO_DEVICE = -3, /* no gfx950 device */
  CCJ_ERR_OOM = -4,       /* device allocation failed */
  CCJ_ERR_LIMIT = -5      /* size outside the supported range */
};

/* Device-side status bits a probe / compaction may raise (ccj_probe_args.status). */
enum ccj_flag {
  CCJ_FLAG_CAP_OVERFLOW = 1u,   /* a chunk produced more than `cap` matches (extra matches dropped) */
  CCJ_FLAG_ROUND_OVERFLOW = 2u, /* a chunk took more than `max_rounds` rounds (counts not recorded) */
  CCJ_FLAG_BAD_INPUT = 4u,      /* count > chunk or a sel entry outside the chunk (rows skipped) */
  CCJ_FLAG_PART_OVERFLOW = 8u,  /* ccj_probe_partitioned: a fixed-capacity partition segment was full
                                   (rows dropped): re-run with CCJ_PART_EXACT */
  CCJ_FLAG_INTERNAL = 16u       /* an internal consistency check failed (raised by libccj_tuning.so's
                                   checked walks only: a DPP address move disagreed with its lanes) */
};

enum ccj_table_kind {
  CCJ_TABLE_LP = 0,   /* LPHashTable      linear_probing_ht.h:56-71 */
  CCJ_TABLE_CHAIN = 1 /* HashTable        chaining_ht.h:86-101      */
};

enum ccj_layout {
  /* Slot/chain order identical to the reference's sequential insertion (L3 parity).
   * LP: inserted on the host, uploaded.  Chain: stable order on device or host. */
  CCJ_LAYOUT_REFERENCE = 0,
  /* Built on the device.  LP: parallel atomicCAS insert — same occupied slots and same per-probe
   * match multiset as the reference, slot order inside a cluster may differ (L1/L2 parity).
   * Chain: stable bucket sort (histogram + scan + stable radix sort by bucket) — identical to the
   * reference order (L3), every array byte-identical to the host build.  Chaining tables are built
   * this way for either layout (the two are the same table). */
  CCJ_LAYOUT_DEVICE = 1
};

typedef void *ccj_stream; /* hipStream_t; NULL = the default stream */
#define CCJ_MAX_PAYLOAD_COLS 8
typedef struct ccj_table ccj_table;

typedef struct ccj_table_info {
  int32_t kind;           /* ccj_table_kind */
  int32_t layout;         /* ccj_layout */
  uint64_t n_keys;        /* build tuples inserted */
  uint64_t size;          /* LP: n_slots (pow2 >= 4n, linear_probing_ht.cpp:5-6);
                             chain: n_buckets (pow2 >= 2n, chaining_ht.cpp:5-6) */
  uint64_t max_dup;       /* largest multiplicity of one key = max matches per probe row */
  uint32_t max_rounds;    /* largest number of Next rounds any probe chunk can take
                             (LP: longest occupied run; chain: longest chain) */
  uint32_t reserved;
  const int64_t *d_table; /* LP: slots int64[size]; chain: chain keys int64[n_keys] */
  const uint32_t *d_bucket_off; /* chain: uint32[size + 1] CSR offsets; LP: NULL */
} ccj_table_info;

/* ---- device / errors ---------------------------------------------------------------------- */
const char *ccj_last_error(void);
int ccj_abi_version(void);
/* 16 hex digits of the SHA-256 of the sources this library was compiled from (the .hip and .h files of csrc,
 * include/ccj.h, in that order; Makefile SRC_HASH): bench.py uses it to refuse a counter profile
 * taken on another build.  No reference counterpart (build bookkeeping). */
const char *ccj_build_hash(void);
/* Name of the payload-gather kernel the calling thread's last probe with payload columns launched
 * ("" if none): the vectorised transposed-store form needs an even cap, no out_base and 16-byte
 * aligned columns, else a fallback runs.  No reference counterpart (the reference has no gather). */
const char *ccj_last_gather_kernel(void);
/* Phase timing in the reference's 4-phase schema (CycleProfiler, profiler.h:262-290: 0 "Hash & Find
 * Bucket", 1 "Match Tuples", 2 "Gather Tuples", 3 "Advance Pointers"): the caller's hipEvent_t
 * handles (n <= 4; NULL / 0 clears), recorded on the call's stream by this thread's later probe
 * calls at their kernel boundaries — events[0] before the first kernel, [1] after hashing and
 * finding every row's bucket (the split of the partitioned / ordered paths), [2] after match +
 * advance (the walk; this design fuses the two), [3] after the gather (C5 payload columns, or the
 * ordered path's unsplit + reference-order emit).  A kernel that fuses several phases records
 * their boundaries together (probe_chunks: [1], [2], [3] after its one launch).  One-shot: the
 * next probe call (ccj_probe, ccj_probe_ordered, ccj_probe_partitioned) records all four on every
 * return path — a boundary it does not reach (empty input, a one-pass route, an error) at the
 * stream's point where it returns — and then clears them. */
int ccj_set_phase_events(void *const *events, uint32_t n);
/* Selects the HIP device for this thread and checks it is gfx950. */
int ccj_device_init(int device);

/* ---- tables ------------------------------------------------------------------------------- */
/* Replaces LPHashTable::LPHashTable(n_rhs_tuples, chunk_factor) (linear_probing_ht.cpp:4-37) and
 * HashTable::HashTable(n_rhs_tuples, chunk_factor) (chaining_ht.cpp:4-36): generates the
 * reference's build keys (:14-25) and builds the table in the requested layout. */
int ccj_table_build_reference(int kind, uint64_t n_rhs_tuples, uint64_t chunk_factor, int layout,
                              ccj_stream stream, ccj_table **out);
/* Same tables from caller keys, inserted in array order (host keys; CCJ_LAYOUT_REFERENCE). */
int ccj_table_build_from_host(int kind, const int64_t *h_keys, uint64_t n, ccj_table **out);
/* Same tables from device-resident keys, built on the device (CCJ_LAYOUT_DEVICE; chaining: the
 * reference's chain order, max_dup computed from the keys). */
int ccj_table_build_on_device(int kind, const int64_t *d_keys, uint64_t n, ccj_stream stream,
                              ccj_table **out);
int ccj_table_get_info(const ccj_table *table, ccj_table_info *info);
/* The table's device arrays (read-only views owned by the table), for checks and external
 * kernels: LP: d_table = slots[positions] (padded to >= 4), d_row = slot -> build tuple (kNoRow
 * 0xFFFFFFFF for empty slots); chaining: d_table = chain keys[positions] (bucket-major, insertion
 * order, padded to a multiple of 4 with -1), d_row = chain position -> build tuple,
 * d_bucket_off = uint32[size + 1] CSR offsets, d_bucket16 = per bucket {start | len << 32, first
 * key} (int64 pairs), d_bucket8 = per bucket {start | len << 32 | fp0 << 40 | fp1 << 52} (n_bucket8
 * = max(size, 2) entries; NULL when a chain has 255 or more keys).  No reference counterpart:
 * the private members HashTable::linked_lists_ (chaining_ht.h:96) and LPHashTable::slots_
 * (linear_probing_ht.h:66). */
typedef struct ccj_table_arrays {
  const int64_t *d_table;
  uint64_t positions;
  const uint32_t *d_row;
  const uint32_t *d_bucket_off;
  const int64_t *d_bucket16;
  const uint64_t *d_bucket8;
  uint64_t n_bucket8;
  const uint32_t *d_bucket_filter; /* chaining: 2 bits per bucket, 16 per word (size / 16 words): 0
                                      empty, 1 / 2 a one-key chain whose key has hash bit 40 = 0 / 1,
                                      3 a longer chain — the partitioned walk's LDS filter; NULL
                                      below 128 buckets */
  uint64_t n_filter_words;
} ccj_table_arrays;
int ccj_table_get_arrays(const ccj_table *table, ccj_table_arrays *arrays);
/* Attaches build-side payload columns (C5): d_payload is row-major int64
 * [n_keys][n_cols] in build-tuple order (the order keys were given to the builder).  The table
 * re-lays them out by table position (slot / chain index) so a match gathers one contiguous row.
 * The reference discards its build payload (linear_probing_ht.cpp:20); this is the wide-payload
 * extension the BASELINE config asks for. */
int ccj_table_set_payload(ccj_table *table, const int64_t *d_payload, uint32_t n_cols, ccj_stream stream);
int ccj_table_free(ccj_table *table);
/* The rank walk's window index (CCJ_PART_RANK): occupancy bits, occupied-slot ranks per 128 slots
 * and the occupied slots' keys in slot order, built on the device from the finished LP table
 * (size/8 + size/32 + n_keys*8 bytes: 560 MiB at C2).  A no-op for tables the rank walk does not
 * serve (chaining, one window, windows > 2^19 slots).  Build-time work, like the table.  Call it
 * before sizing the partitioned workspace (ccj_probe_partitioned_workspace_size grows with it).
 * The rank walk is built into libccj_tuning.so only; libccj.so returns CCJ_ERR_INVALID. */
int ccj_table_build_rank_index(ccj_table *table, ccj_stream stream);

/* ---- probe -------------------------------------------------------------------------------- */
/* Batched form of Probe + the whole `while (HasNext()) Next(...)` loop
 *   LPHashTable::Probe / LPScanStructure::Next   linear_probing_ht.cpp:39-60, :62-115
 *   HashTable::Probe   / ScanStructure::Next     chaining_ht.cpp:38-58,  :60-136
 * over many chunks in one launch (one wavefront per chunk).
 *
 * Input chunk c = physical rows [c*chunk, min((c+1)*chunk, n_rows)) of `keys`; its active rows
 * are sel[c*chunk + i] for i < count_c (sel NULL = identity, counts NULL = all physical rows).
 * Output, per chunk, in the reference's emission order (round-major, idx ascending — L3):
 *   out_sel[c*cap + j]     = result.selection_vector_[...] (chunk-local physical row)
 *   out_payload[c*cap + j] = the matched table value       (result col m+1 at that row)
 *   out_count[c]           = matches;  out_rounds[c] = rounds (LP: Next calls)
 *   out_round_counts[c*max_rounds + r] = matches of round r (optional)
 * cap >= chunk * max_dup can never overflow. */
typedef struct ccj_probe_args {
  const int64_t *keys;       /* device int64[n_rows] */
  const uint32_t *sel;       /* device uint32[n_chunks*chunk] or NULL */
  const uint32_t *counts;    /* device uint32[n_chunks] or NULL */
  uint64_t n_rows;
  uint32_t chunk;            /* kBlockSize, 1..2048 */
  uint32_t max_rounds;       /* stride of out_round_counts (0 if NULL) */
  uint64_t cap;              /* per-chunk output capacity */
  uint32_t *out_count;       /* device uint32[n_chunks] (required) */
  uint32_t *out_sel;         /* device uint32[n_chunks*cap] (required) */
  int64_t *out_payload;      /* device int64[n_chunks*cap] or NULL */
  uint32_t *out_rounds;      /* device uint32[n_chunks] or NULL */
  uint32_t *out_round_counts;/* device uint32[n_chunks*max_rounds] or NULL */
  uint32_t *status;          /* device word, OR-ed with ccj_flag bits, or NULL */
  /* Matched table position (LP slot / chain index), the reference's iterator at the match
   * (GatherResult, chaining_ht.cpp:126-136; slot_ids_, linear_probing_ht.cpp:90-94). Or NULL. */
  uint32_t *out_pos;
  /* Wide payload (C5): the first n_payload_cols of the table's payload columns
   * (ccj_table_set_payload) are gathered for every match: out_payload_cols[c][c*cap + j]. */
  uint32_t n_payload_cols;
  uint32_t reserved2;
  int64_t *out_payload_cols[CCJ_MAX_PAYLOAD_COLS];
} ccj_probe_args;

int ccj_probe(const ccj_table *table, const ccj_probe_args *args, ccj_stream stream);

/* Same outputs as ccj_probe — every chunk's per-Next stream in the reference's order (L3) — for
 * large tables (LP: >= 2^22 slots; chaining: >= 2^22 buckets) with sel == NULL, computed through
 * the slot / bucket partitioned layout:
 *   1. the one-pass split of the live rows (as ccj_probe_partitioned), which also records where
 *      every split tile's run of every partition went;
 *   2. a walk with the table window L2-resident that leaves each row's Next-round word (the
 *      rounds in which it matches + its round count: the run length, or the chain length) at its
 *      partitioned position;
 *   3. the words back into row order, one split tile per workgroup;
 *   4. per chunk, the round-major / idx-ascending emit of linear_probing_ht.cpp:62-115 /
 *      chaining_ht.cpp:60-124 from them.
 * Random slot reads become L2 hits instead of 128-byte HBM lines (C2: 1.24 lines per probe row on
 * ccj_probe).  Other tables, sel != NULL, out_pos or payload columns run ccj_probe itself and need
 * no workspace.  The partitioned route needs args->status: CCJ_FLAG_PART_OVERFLOW there (extreme
 * key skew filled the split's overflow area) means the outputs are incomplete — re-run ccj_probe.
 * ws: device workspace of ccj_probe_ordered_workspace_size bytes (0: no workspace needed).
 * Replaces the same reference interface as ccj_probe. */
size_t ccj_probe_ordered_workspace_size(const ccj_table *table, uint64_t n_rows, uint32_t chunk);
int ccj_probe_ordered(const ccj_table *table, const ccj_probe_args *args, void *ws, size_t ws_bytes,
                      ccj_stream stream);

/* The table values one chunk's rows visit, round by round: the side effect of the reference's
 * InOneNext / SIMDInOneNext, which write the visited slot (LP) or chain key (chaining) into result
 * column m+1 at the row's physical position for EVERY active row, matched or not
 * (linear_probing_ht.cpp:133, :301, :322; chaining_ht.cpp:156, :341, :362).  Row i = keys[sel[i]]
 * (sel NULL: keys[i]), i < count; d_len[i] = the number of rounds it stays active (LP: the
 * non-empty run from its home slot; chaining: its chain's length), capped at max_rounds;
 * d_vals[i * max_rounds + r] = the value visited in round r < d_len[i].  The facade's
 * InOneNext replays these writes (host/ccj_operators.cpp); the batched paths never need them. */
int ccj_probe_visits(const ccj_table *table, const int64_t *d_keys, const uint32_t *d_sel, uint32_t count,
                     uint32_t max_rounds, int64_t *d_vals, uint32_t *d_len, ccj_stream stream);

/* Slot-range-partitioned probe (the throughput path; L1/L2 parity, not L3 order).
 * LP tables only.  The probe column (args->keys, n_rows < 2^32; sel and counts must be NULL) is
 * first split by its home slot's partition (slot >> 19: 4 MiB of table per partition, at most 1024 partitions), then
 * probed chunk by chunk like ccj_probe with consecutive chunks kept on one XCD, so each
 * partition's table window is read from L2 instead of as random HBM lines.
 *
 * The split lays the column out in `positions` slots (ccj_probe_partitioned_positions):
 *   - default: one pass into fixed-capacity segments (partition x XCD group), with gaps, then a
 *     shared overflow area of n_rows / 16 positions for the runs that do not fit their segment
 *     (key skew); only when that fills too (extreme skew) are rows dropped and
 *     CCJ_FLAG_PART_OVERFLOW raised in *args->status (required): re-run with CCJ_PART_EXACT;
 *   - flags & CCJ_PART_EXACT: exact-size two-pass LSD split, no gaps, never overflows.
 * Outputs are ccj_probe's over that layout: args->out_count etc. hold positions / chunk chunks
 * (chunk c = positions [c*chunk, (c+1)*chunk), empty ones report count 0), out_sel indexes
 * positions inside the chunk, and out_row_map[pos] (positions entries) is the original row of a
 * live position.  Same matches, payloads and per-row multiplicities as ccj_probe (L1 + L2);
 * within a chunk the order is unspecified, so out_round_counts is not produced (must be NULL).
 * out_pos (table position of every match) and payload columns (C5: gathered after the walk) are
 * produced as by ccj_probe, for tables of >= 16 slots.  For a table of distinct keys (max_dup 1)
 * without out_rounds the walk ends a row at its match (the rest of its run cannot hold the key);
 * with out_rounds every row is walked to the end of its run, as the reference's Next calls do. */
#define CCJ_PART_EXACT 1u
/* flags & CCJ_PART_ROWS: out_sel receives the ORIGINAL row of every match (u32, row of args->keys)
 * instead of its position inside the chunk, and out_row_map may be NULL.  LP tables of >= 16
 * slots with distinct keys (max_dup 1), cap == chunk, out_payload set; with out_pos / payload
 * columns (C5) the table may have at most 2^31 slots.  The split then writes each position's key
 * into out_payload and its row into out_sel (position p IS output slot p of its chunk: an LP
 * match's payload is the probe key), and the walk only compacts the chunks where some row missed
 * (with positions / payload columns it writes each match's table position at its output slot,
 * which the payload gather then reads).  Without the flag, when cap == chunk the keys still go to
 * out_payload (the workspace's key region is then left untouched). */
#define CCJ_PART_ROWS 2u
/* flags & CCJ_PART_RANK (libccj_tuning.so only — libccj.so, the product, refuses the flag and
 * ccj_table_build_rank_index with CCJ_ERR_INVALID: the rank walk measured slower):
 * the RANK WALK instead of the slot-array walk (LP tables of distinct keys,
 * cap == chunk, chunk a multiple of 512, windows of <= 2^19 slots; otherwise the flag is ignored).
 * Each partition's window index (occupancy bitmap + occupied-slot rank per 128 slots, built with
 * the table) is held in LDS, so a row's run [home, first empty) costs no memory read and its
 * candidate keys come from the table's compact key array (occupied slots' keys in slot order).
 * Same matches, same per-chunk row order.  Measured at C2: fewer L2 requests per row
 * (1.11 vs 1.22), half the HBM lines and 22 % lower L2 latency, but one 768-thread workgroup per
 * CU (the 80 KiB index) keeps half as many requests in flight: 9.9 ms against 7.4 for the slot
 * walk.  Not the default.  Needs ccj_table_build_rank_index (CCJ_ERR_INVALID without it). */
#define CCJ_PART_RANK 4u
/* flags & CCJ_PART_SHARE: the one-pass split runs on 3/4 of the CUs (of the stream's CUs), leaving
 * the rest to kernels of other streams.  The split holds one 1024-thread, ~150 KB-LDS workgroup per
 * CU, so without the flag nothing else — RCCL's kernels, the next batch's owner split — runs while
 * it does.  The multi-GPU step passes it (one-rank rehearsal 32.4 -> 29.2 ms per step). */
#define CCJ_PART_SHARE 8u
uint64_t ccj_probe_partitioned_positions(const ccj_table *table, uint64_t n_rows, uint32_t chunk);
size_t ccj_probe_partitioned_workspace_size(const ccj_table *table, uint64_t n_rows, uint32_t chunk);
int ccj_probe_partitioned(const ccj_table *table, const ccj_probe_args *args, uint32_t flags,
                          uint32_t *out_row_map, void *workspace, size_t workspace_bytes, ccj_stream stream);

/* ---- compaction ------------------------------------------------------------------------- */
/* Replaces NaiveCompactor::Compact + Flush (compactor.cpp:5-41, compactor.h:23) applied to every
 * Next result of a ccj_probe output, in pipeline order (chunk-major, round-major), with the
 * reference's defect fixed (fresh temp chunk, the commented compactor.cpp:36):
 *   - a Next result of exactly `chunk` rows passes through as its own output chunk (:6);
 *     with `threshold` T (the threshold-gated compaction setting.h:20-25 names as
 *     BinaryCompactor / DynamicCompactor but never implements) every non-empty result of at
 *     least T rows passes through as its own chunk, and only smaller ones are compacted:
 *     T = chunk (or 0) is NaiveCompactor, T = 1 compacts nothing;
 *   - other results are appended (DataChunk::Append, base.cpp:15-27: every column gathered
 *     through the selection vector) into a cache that is emitted whenever the next result would
 *     overflow it (:22-35); Flush emits the final partial chunk.
 * Output: dense chunks of `chunk` rows: out_cols[k] = input column k at the matched row,
 * out_payload = the probe payload (reference result column m+1; column m is never written by the
 * reference and is not materialised), out_row = global probe row (c*chunk + sel).
 * key_cols: bit k says input column k is the probe's join-key column.  The join is an equi-join
 * and the payload is the matched build key, so on every output row that column equals the
 * payload: it is filled from the (dense) payload instead of gathered through the selection
 * vector — same output, without reading a 10 %-dense gather's whole lines of the key column
 * (cols[k] may then be NULL; needs payload).
 * Needs out_round_counts from the probe (the Next boundaries). */
#define CCJ_MAX_COLS 16
typedef struct ccj_compact_args {
  const uint32_t *count;        /* ccj_probe outputs (device) */
  const uint32_t *sel;
  const int64_t *payload;       /* or NULL */
  const uint32_t *rounds;
  const uint32_t *round_counts;
  uint64_t n_chunks;
  uint64_t cap;
  uint32_t max_rounds;
  uint32_t chunk;
  uint32_t n_cols;              /* probe-side columns carried along, <= CCJ_MAX_COLS */
  uint32_t threshold;           /* results with >= threshold rows pass through; 0 = chunk (NaiveCompactor) */
  const int64_t *cols[CCJ_MAX_COLS];     /* device int64[n_chunks*chunk] each (chunk-major) */
  int64_t *out_cols[CCJ_MAX_COLS];       /* device int64[out_cap_rows] each */
  int64_t *out_payload;         /* device int64[out_cap_rows] or NULL */
  uint64_t *out_row;            /* device uint64[out_cap_rows] or NULL */
  uint32_t *out_chunk_counts;   /* device uint32[out_cap_rows / chunk]; pass-through chunks keep their count */
  uint64_t out_cap_rows;        /* multiple of chunk */
  uint64_t *out_n_chunks;       /* device word: output chunks written */
  void *workspace;              /* device scratch of ccj_compact_workspace_size(...) bytes */
  size_t workspace_bytes;
  uint32_t *status;             /* device word (ccj_flag bits) or NULL */
  uint32_t key_cols;            /* bit k: column k is the join key (filled from payload; see above) */
} ccj_compact_args;

size_t ccj_compact_workspace_size(uint64_t n_chunks, uint64_t cap, uint32_t chunk, uint32_t max_rounds,
                                  uint32_t threshold);
int ccj_compact(const ccj_compact_args *args, ccj_stream stream);

/* ---- multi-join pipeline ------------------------------------------------------------------ */
/* Replaces main.cpp's ExecutePipeline / FlushPipelineCache (main.cpp:119-191): a chain of joins,
 * join l probing column l of its input with tables[l], and between joins either
 *   CCJ_COMPACT_NONE: every Next result goes on to the next join as its own chunk (main.cpp
 *                     :149-159 with no compactor; LP's empty Next results produce nothing), or
 *   CCJ_COMPACT_FULL: the Next results pass through the NaiveCompactor first (compactor.cpp:5-41
 *                     with the :36 fix, `Compactor` in setting.h), flushed at the end (:172-191).
 * The device runs it join by join: join l probes ALL of its input chunks in one launch, in the
 * order the reference's depth-first recursion would hand them to it, and its output is then
 * concatenated (NONE) or compacted (FULL) into join l+1's chunks.  Both modes materialise the
 * carried columns (DataChunk::Append, base.cpp:15-27); they differ in how rows are chunked, which
 * is what the reference's compaction changes.  The result (the ResultCollector's table,
 * main.cpp:125-128) is, per tuple in the reference's append order: the n_joins probe columns,
 * then per join a zero column (result column m, never written by the reference) and its payload.
 * Synchronises `stream` once per join (output sizes), so it is not graph-capturable. */
#define CCJ_MAX_JOINS 8
enum ccj_compact_mode { CCJ_COMPACT_NONE = 0, CCJ_COMPACT_FULL = 1 };
typedef struct ccj_pipeline ccj_pipeline;
typedef struct ccj_pipeline_result {
  uint64_t n_out;                        /* result tuples */
  const int64_t *cols[CCJ_MAX_JOINS];    /* device int64[n_out]: probe column j of each tuple */
  const int64_t *payload[CCJ_MAX_JOINS]; /* device int64[n_out]: join l's payload (result column n_joins+2l+1) */
  uint64_t chunks_in[CCJ_MAX_JOINS];     /* chunks probed by join l (probe workgroups) */
  uint64_t rows_in[CCJ_MAX_JOINS];       /* tuples probed by join l */
  uint64_t rows_out[CCJ_MAX_JOINS];      /* tuples produced by join l */
  float level_ms[CCJ_MAX_JOINS];         /* device time of join l: probe + sizes + concat/compact */
} ccj_pipeline_result;
/* tables[l] must outlive the pipeline; chunk = kBlockSize (1..2048). */
int ccj_pipeline_create(const ccj_table *const *tables, uint32_t n_joins, uint32_t chunk, int compact_mode,
                        ccj_pipeline **out);
/* d_cols[j] = device int64[n_rows], the probe side (main.cpp:47-55's table, column-major).  Result
 * buffers belong to the pipeline and stay valid until the next run or ccj_pipeline_free. */
int ccj_pipeline_run(ccj_pipeline *pl, const int64_t *const *d_cols, uint64_t n_rows, ccj_stream stream,
                     ccj_pipeline_result *res);
/* CCJ_COMPACT_FULL: join l's compactor lets results of >= thresholds[l] rows pass through and
 * compacts the smaller ones (ccj_compact_args.threshold; 0 = chunk = NaiveCompactor, the
 * default; NULL restores it) — the threshold a DynamicCompactor tunes per run (host/ccj_tuner.h). */
int ccj_pipeline_set_thresholds(ccj_pipeline *pl, const uint32_t *thresholds);
int ccj_pipeline_free(ccj_pipeline *pl);
/* Result verification: d_acc[0] += tuples, d_acc[1] += sum over tuples of fmix64(t), where
 * t = 0x51ED27 folded over the tuple's columns k in order as t = fmix64(t ^ v_k) + k (the
 * order-insensitive checksum host/pipeline_main.cpp and oracle/ref_driver.cpp print). */
int ccj_pipeline_checksum(const ccj_pipeline_result *res, uint32_t n_joins, uint64_t *d_acc, ccj_stream stream);

/* ---- multi-GPU owner partitioning --------------------------------------------------------- */
/* The exchange step of the radix-partitioned multi-GPU join: splits a key column
 * into `parts` (a power of two, one per GPU) by owner(k) = murmurhash64(k) >> (64 - log2 parts),
 * i.e. the top hash bits (the local tables use the low bits), keeping row order inside every
 * destination.  Writes the keys and their global row ids (row_base + i) destination-major and
 * the per-destination counts: the send buffers + split sizes of one all-to-all (RCCL, xGMI).
 * No reference counterpart: the reference is single-threaded. */
size_t ccj_partition_workspace_size(uint64_t n, uint32_t parts);
int ccj_partition_by_owner(const int64_t *d_keys, uint64_t n, uint32_t parts, uint64_t row_base,
                           int64_t *d_out_keys, uint64_t *d_out_rows, uint64_t *d_out_counts,
                           void *d_workspace, size_t workspace_bytes, ccj_stream stream);

/* Fixed-capacity form for a host-synchronisation-free exchange: destination d's keys and their
 * u32 row ids (row_base + i) go to [d*seg_cap, d*seg_cap + count_d) — grouped exactly, in no
 * particular order inside a segment — so every all-to-all split is
 * seg_cap and the send/receive sizes need no host round trip; d_out_counts gets the true counts.
 * Rows of a destination beyond seg_cap are dropped and CCJ_FLAG_CAP_OVERFLOW is OR-ed into
 * *d_status (the caller re-runs that batch with ccj_partition_by_owner). */
int ccj_partition_by_owner_fixed(const int64_t *d_keys, uint64_t n, uint32_t parts, uint32_t row_base,
                                 uint64_t seg_cap, int64_t *d_out_keys, uint32_t *d_out_rows, uint64_t *d_out_counts,
                                 uint32_t *d_status, void *d_workspace, size_t workspace_bytes, ccj_stream stream);
/* One-pass form of the fixed-capacity split (the slot split's kernel with the owner as its
 * partition): destination d's region is CCJ_OWNER_GROUPS sub-segments of sub_cap slots,
 * [(d*G + g)*sub_cap, ... + count_{d,g}), sub-segment g filled only by the workgroups of XCD g (so
 * each is written from one L2); d_out_counts[d*G + g] gets the true counts.  Rows beyond a
 * sub-segment's sub_cap are dropped and CCJ_FLAG_PART_OVERFLOW is OR-ed into *d_status.
 * self_last < parts: destination d's region is placed at slot s(d) instead of d, where
 * s(self_last) = parts - 1 and s(d) = d - (d > self_last) otherwise — the N - 1 peer regions come
 * first, in rank order (one all-to-all with a zero self split sends them), and the rank's own
 * region is last, where a local copy moves it (d_out_counts follows the same slots).
 * self_last >= parts: s(d) = d.
 * Workspace: ccj_partition_grouped_workspace_size(parts) bytes. */
#define CCJ_OWNER_GROUPS 8
size_t ccj_partition_grouped_workspace_size(uint32_t parts);
/* A sub_cap that n uniformly hashed keys overflow with negligible probability: the largest tile
 * group's rows / parts + 8 standard deviations + one chunk, a multiple of chunk. */
uint64_t ccj_partition_grouped_sub_cap(uint64_t n, uint32_t parts, uint32_t chunk);
int ccj_partition_by_owner_grouped(const int64_t *d_keys, uint64_t n, uint32_t parts, uint32_t row_base,
                                   uint64_t sub_cap, uint32_t self_last, int64_t *d_out_keys, uint32_t *d_out_rows,
                                   uint64_t *d_out_counts, uint32_t *d_status, void *d_workspace,
                                   size_t workspace_bytes, ccj_stream stream);
/* Probe chunk counts for n_segs received fixed-capacity segments (seg_cap a multiple of chunk):
 * chunk j of segment g gets min(chunk, max(0, count_g - j*chunk)) live rows, so ccj_probe over the
 * whole receive buffer (counts = this, sel = NULL) skips the padding.  count_g > seg_cap raises
 * CCJ_FLAG_CAP_OVERFLOW. */
int ccj_segment_chunk_counts(const uint64_t *d_seg_counts, uint32_t n_segs, uint64_t seg_cap, uint32_t chunk,
                             uint32_t *d_out_counts, uint32_t *d_status, ccj_stream stream);

/* Streams confined to a subset of the CUs (the multi-GPU step: the local probe, the owner split
 * and RCCL each keep CUs of their own, so that a kernel of 10^5 workgroups on one stream cannot
 * hold every CU until it drains while the others' kernels wait).  cu_mask: mask_words 32-bit
 * words, bit i = CU i in HIP's numbering (hipExtStreamCreateWithCUMask).  The persistent kernels
 * (the one-pass splits) launched on such a stream size their grid to its CUs.  No reference
 * counterpart: plumbing of the sharded path. */
int ccj_stream_create_cu_masked(const uint32_t *cu_mask, uint32_t mask_words, ccj_stream *out);
int ccj_stream_destroy(ccj_stream stream);
/* The device's CU count (hipDeviceAttributeMultiprocessorCount). */
int ccj_device_cus(uint32_t *out);

/* ---- workload + measurement helpers (not on the reference's path) ------------------------- */
/* d_dst[0, bytes) = d_src[0, bytes): 16-byte non-temporal loads and stores (bench.py's measured
 * HBM copy ceiling).  16-byte aligned buffers, bytes a multiple of 16. */
int ccj_copy_device(void *d_dst, const void *d_src, uint64_t bytes, ccj_stream stream);
/* Synthetic probe column: d_out[i] = SplitMix64(seed) output (first_row + i) mod range — the
 * stream of oracle/ccj_gen.h ccj_uniform_key, so any row can be regenerated on the host.
 * Replaces the reference's host-side source (main.cpp:41-55 + DataCollection::FetchChunk). */
int ccj_gen_uniform_keys(int64_t *d_out, uint64_t n, uint64_t seed, uint64_t first_row, uint64_t range,
                         ccj_stream stream);
/* C3 probe column (BASELINE configs[2]): row i is, with probability hit_ppm / 1e6, a
 * build key of the reference generator (n_build, cf) drawn with Zipf s = 1 skew over its distinct
 * keys (a 2^16-bucket inverse-CDF table, ranks spread by a fixed permutation), else a key in
 * [n_build, 2^62) that matches nothing — the stream of oracle/ccj_gen.h ccj_c3_key. */
int ccj_gen_c3_keys(int64_t *d_out, uint64_t n, uint64_t seed, uint64_t first_row, uint64_t n_build, uint64_t cf,
                    uint32_t hit_ppm, ccj_stream stream);
/* Build-side keys first..first+n-1 of the reference generator for n_total tuples
 * (linear_probing_ht.cpp:14-25: key t = (t / cf) * step), e.g. for sharding the build side. */
int ccj_gen_reference_keys(int64_t *d_out, uint64_t first, uint64_t n, uint64_t n_total, uint64_t cf,
                           ccj_stream stream);
/* Work accounting for the roofline: d_acc[0] += table words examined (LP: slots read including
 * the terminating empty; chain: chain keys visited), d_acc[1] += matches, over n probe keys. */
int ccj_probe_cost(const ccj_table *table, const int64_t *d_keys, uint64_t n, uint64_t *d_acc,
                   ccj_stream stream);
/* The same plus what a walk that ends each row at its FIRST match examines (the throughput path's
 * walk on distinct-key tables, ccj_probe_partitioned): d_acc[0..1] as ccj_probe_cost, d_acc[2] +=
 * table words examined through the first match (LP: home slot through the match, or through the
 * terminating empty on a miss; chaining: chain keys through the match, or the whole chain),
 * d_acc[3] += aligned 32-byte windows those words lie in (LP: 4-slot windows; chaining: 2-key
 * windows of the chain array after round 0, which the bucket record serves).  d_acc: 4 words. */
int ccj_probe_cost_walk(const ccj_table *table, const int64_t *d_keys, uint64_t n, uint64_t *d_acc,
                        ccj_stream stream);
/* Result verification without a download: d_acc[0] += matches, d_acc[1] += sum of the L2 term
 * fmix(row * gamma + fmix(payload + 1)) (oracle/ccj_gen.h ccj_l2_term) over every match of a
 * ccj_probe output, row = row_base + c*chunk + out_sel. */
int ccj_result_checksum(const uint32_t *out_count, const uint32_t *out_sel, const int64_t *out_payload,
                        uint64_t n_chunks, uint64_t cap, uint32_t chunk, uint64_t row_base, uint64_t *d_acc,
                        ccj_stream stream);
/* Same, with the probe rows mapped through row_map (row = row_map[c*chunk + sel]), for probes of
 * shuffled columns whose original global rows travel beside the keys. */
int ccj_result_checksum_mapped(const uint32_t *out_count, const uint32_t *out_sel, const int64_t *out_payload,
                               uint64_t n_chunks, uint64_t cap, uint32_t chunk, const uint64_t *row_map,
                               uint64_t *d_acc, ccj_stream stream);

#ifdef __cplusplus
}
#endif
#endif /* CCJ_H */
