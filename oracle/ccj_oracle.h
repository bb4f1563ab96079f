/* ccj_oracle.h — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so,
 * and only as the checker / the timed CPU baseline.  The product library (libccj.so) never links
 * or calls it: it has no CPU fallback and fails loudly without a GPU.
 *
 * Pinning: every function here is checked in tests/test_oracle.py against golden vectors
 * produced by the REFERENCE itself (oracle/_ref/ref_driver, built from /root/reference sources)
 * and committed under tests/golden/ together with tests/golden/make_golden.py.
 *
 * Probe output contract (shared with the device path, include/ccj.h):
 *   chunk c covers physical rows [c*chunk, min((c+1)*chunk, n_rows)) of `keys`;
 *   its active row list is sel[c*chunk + i] (chunk-local physical rows) for i < count_c,
 *   sel == NULL meaning identity and counts == NULL meaning "all physical rows".
 *   For every Next round r (round-major), for every active idx in ascending order whose
 *   candidate equals the probe key, one match is emitted:
 *     out_sel[c*cap + j]     = sel[idx]            (result.selection_vector_ after Slice)
 *     out_payload[c*cap + j] = matched table value (result col m+1 at that row)
 *   out_count[c] = matches, out_rounds[c] = Next rounds, out_round_counts[c*max_rounds + r] = rc_r.
 */
#ifndef CCJ_ORACLE_H
#define CCJ_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

uint64_t ccj_o_murmurhash64(uint64_t x);
uint64_t ccj_o_ref_build_keys(uint64_t n, uint64_t cf, int64_t *out);
uint64_t ccj_o_ref_multiplicity(int64_t k, uint64_t n, uint64_t cf);

uint64_t ccj_o_lp_num_slots(uint64_t n);
void ccj_o_lp_build(const int64_t *keys, uint64_t n, int64_t *slots, uint64_t n_slots);
void ccj_o_lp_build_rows(const int64_t *keys, uint64_t n, int64_t *slots, uint32_t *rows, uint64_t n_slots);
uint64_t ccj_o_chain_num_buckets(uint64_t n);
void ccj_o_chain_build(const int64_t *keys, uint64_t n, uint64_t n_buckets, uint64_t *bucket_off,
                       int64_t *chain_keys);
void ccj_o_chain_build_rows(const int64_t *keys, uint64_t n, uint64_t n_buckets, uint64_t *bucket_off,
                            int64_t *chain_keys, uint32_t *rows);

/* kind 0 = linear probing (table = slots, size = n_slots), 1 = chaining (table = chain_keys,
 * bucket_off[n_buckets+1], size = n_buckets).  Returns 0, or -1 when an output bound
 * (cap / max_rounds) would be exceeded.  threads <= 0: all OpenMP threads. */
int ccj_o_probe(int kind, const int64_t *table, const uint64_t *bucket_off, uint64_t size,
                const int64_t *keys, const uint32_t *sel, const uint32_t *counts, uint64_t n_rows,
                uint32_t chunk, uint64_t cap, uint32_t max_rounds, uint32_t *out_count,
                uint32_t *out_sel, int64_t *out_payload, uint32_t *out_rounds,
                uint32_t *out_round_counts, int threads, uint32_t *out_pos /* matched position or NULL */);

/* Timed CPU baseline: probe n_rows keys chunk by chunk exactly as ccj_o_probe does, but keep only
 * the totals (matches, L2 checksum over global row ids).  Returns matches. */
uint64_t ccj_o_probe_totals(int kind, const int64_t *table, const uint64_t *bucket_off, uint64_t size,
                            const int64_t *keys, uint64_t n_rows, uint32_t chunk, uint64_t row_base,
                            uint64_t *l2_out, int threads);

/* SplitMix64 probe keys rows [row_begin, row_begin + n) (ccj_gen.h ccj_uniform_key), threaded. */
void ccj_o_gen_uniform(uint64_t seed, uint64_t row_begin, uint64_t n, uint64_t range, int64_t *out, int threads);

/* Exact L1/L2 answer for a probe stream of SplitMix64 keys (ccj_gen.h) against the reference
 * generator's build side (n, cf), by membership. Returns matches; *l2 = checksum. */
uint64_t ccj_o_count_uniform(uint64_t seed, uint64_t row_begin, uint64_t row_end, uint64_t range,
                             uint64_t n_build, uint64_t cf, uint64_t *l2, int threads);

/* C3 probe stream (ccj_gen.h ccj_c3_key): rows [row_begin, row_begin + n), and its exact L1/L2
 * answer by membership over rows [row_begin, row_end). */
void ccj_o_gen_c3(uint64_t seed, uint64_t row_begin, uint64_t n, uint64_t n_build, uint64_t cf, uint32_t hit_ppm,
                  int64_t *out, int threads);
uint64_t ccj_o_count_c3(uint64_t seed, uint64_t row_begin, uint64_t row_end, uint64_t n_build, uint64_t cf,
                        uint32_t hit_ppm, uint64_t *l2, int threads);

/* Compaction order of compactor.cpp:5-41 (with the fresh-temp fix of :36).  Segments are the
 * Next results in pipeline order, seg_counts[s] rows each.  For every input row (segments
 * concatenated) writes its destination slot dest[row] = out_chunk * chunk + offset.
 * Returns the number of output chunks (the final partial one included, an empty flush not). */
uint64_t ccj_o_compact_plan(const uint32_t *seg_counts, uint64_t n_segs, uint32_t chunk, uint64_t *dest,
                            uint32_t *out_chunk_counts);
/* Same with a pass-through threshold: non-empty results of >= threshold rows leave as their own
 * chunk (keeping their count), smaller ones are compacted (threshold 0 = chunk: the above). */
uint64_t ccj_o_compact_plan_threshold(const uint32_t *seg_counts, uint64_t n_segs, uint32_t chunk,
                                      uint32_t threshold, uint64_t *dest, uint32_t *out_chunk_counts);

/* The SURVEY §4 driver's probe stream: mt19937_64(seed) % range, n keys (ref_driver.cpp RunProbe
 * gen 1; the reference's own sources draw the keys the same way). */
void ccj_o_gen_mt64(uint64_t seed, uint64_t n, uint64_t range, int64_t *out);
/* The reference driver's sink (ref_driver.cpp Sink::Emit) over a probe output in its stored
 * order: chunk c's matches are sel/payload[c*cap, c*cap + count[c]).  out[0..3] = matches, L2,
 * L3 fold, SURVEY chk (ccj_gen.h), with global row = c * chunk + sel. */
void ccj_o_result_sums(const uint32_t *count, const uint32_t *sel, const int64_t *payload, uint64_t n_chunks,
                       uint64_t cap, uint32_t chunk, uint64_t *out);

#ifdef __cplusplus
}
#endif
#endif
