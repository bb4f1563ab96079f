/* ccj_oracle.c — plain-C restatement of the reference hot path.  TEST INFRASTRUCTURE
 * (header comment of ccj_oracle.h says who may load it).  Every function cites the reference
 * file:line it restates; the reference tree is /root/reference (snapshot 2025-03-04).
 */
#include "ccj_oracle.h"

#include <omp.h>
#include <stdlib.h>
#include <string.h>

#include "ccj_gen.h"

/* hash_functions.h:8-16 — xor-shift-multiply finaliser, constant used twice (not fmix64). */
uint64_t ccj_o_murmurhash64(uint64_t x) {
  x ^= x >> 32;
  x *= 0xd6e8feb86659fd93ULL;
  x ^= x >> 32;
  x *= 0xd6e8feb86659fd93ULL;
  x ^= x >> 32;
  return x;
}

/* linear_probing_ht.cpp:14-25 (== chaining_ht.cpp:16-26): ceil(n/cf) unique values i*step,
 * step = n / num_unique, each repeated cf times (the last group truncated at n).  The payload
 * (cnt + 10000000, :20) is generated and discarded by the reference; only keys are stored. */
uint64_t ccj_o_ref_build_keys(uint64_t n, uint64_t cf, int64_t *out) {
  uint64_t num_unique = n / cf + (n % cf != 0);
  uint64_t step = n / num_unique;
  uint64_t cnt = 0;
  for (uint64_t i = 0; i < num_unique; ++i)
    for (uint64_t j = 0; j < cf && cnt < n; ++j) out[cnt++] = (int64_t)(i * step);
  return cnt;
}

/* Multiplicity of key k in the build side of ccj_o_ref_build_keys(n, cf). */
uint64_t ccj_o_ref_multiplicity(int64_t k, uint64_t n, uint64_t cf) {
  if (k < 0 || n == 0) return 0;
  uint64_t num_unique = n / cf + (n % cf != 0);
  uint64_t step = n / num_unique;
  uint64_t u = (uint64_t)k;
  if (u % step != 0) return 0;
  uint64_t i = u / step;
  if (i >= num_unique) return 0;
  uint64_t left = n - i * cf;
  return left < cf ? left : cf;
}

/* linear_probing_ht.cpp:5-6 — smallest power of two >= 4n. */
uint64_t ccj_o_lp_num_slots(uint64_t n) {
  uint64_t s = 1;
  while (s < (n << 2)) s <<= 1;
  return s;
}

/* linear_probing_ht.cpp:7,28-36 — fill with -1, sequential insert at h(k) & mask, +1 with wrap.
 * Inserting -1 lands in an empty slot and leaves it empty, exactly as the reference does. */
void ccj_o_lp_build(const int64_t *keys, uint64_t n, int64_t *slots, uint64_t n_slots) {
  ccj_o_lp_build_rows(keys, n, slots, NULL, n_slots);
}

/* Same, also recording which build tuple owns each slot (rows[s], UINT32_MAX when empty). */
void ccj_o_lp_build_rows(const int64_t *keys, uint64_t n, int64_t *slots, uint32_t *rows, uint64_t n_slots) {
  uint64_t mask = n_slots - 1;
  for (uint64_t i = 0; i < n_slots; ++i) slots[i] = -1;
  if (rows)
    for (uint64_t i = 0; i < n_slots; ++i) rows[i] = 0xFFFFFFFFu;
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t s = ccj_o_murmurhash64((uint64_t)keys[i]) & mask;
    while (slots[s] != -1) s = (s + 1) & mask;
    slots[s] = keys[i];
    if (rows && keys[i] != -1) rows[s] = (uint32_t)i;
  }
}

/* chaining_ht.cpp:5-6 — smallest power of two >= 2n. */
uint64_t ccj_o_chain_num_buckets(uint64_t n) {
  uint64_t b = 1;
  while (b < 2 * n) b *= 2;
  return b;
}

/* chaining_ht.cpp:29-35 — std::list::push_back in generator order == a stable counting sort by
 * bucket; bucket b's chain is chain_keys[bucket_off[b] .. bucket_off[b+1]). */
void ccj_o_chain_build(const int64_t *keys, uint64_t n, uint64_t n_buckets, uint64_t *bucket_off,
                       int64_t *chain_keys) {
  ccj_o_chain_build_rows(keys, n, n_buckets, bucket_off, chain_keys, NULL);
}

void ccj_o_chain_build_rows(const int64_t *keys, uint64_t n, uint64_t n_buckets, uint64_t *bucket_off,
                            int64_t *chain_keys, uint32_t *rows) {
  uint64_t mask = n_buckets - 1;
  memset(bucket_off, 0, (n_buckets + 1) * sizeof(uint64_t));
  for (uint64_t i = 0; i < n; ++i) bucket_off[(ccj_o_murmurhash64((uint64_t)keys[i]) & mask) + 1]++;
  for (uint64_t b = 0; b < n_buckets; ++b) bucket_off[b + 1] += bucket_off[b];
  uint64_t *fill = (uint64_t *)malloc(n_buckets * sizeof(uint64_t));
  memcpy(fill, bucket_off, n_buckets * sizeof(uint64_t));
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t q = fill[ccj_o_murmurhash64((uint64_t)keys[i]) & mask]++;
    chain_keys[q] = keys[i];
    if (rows) rows[q] = (uint32_t)i;
  }
  free(fill);
}

/* One chunk of Probe + the full Next loop, in the reference's own round structure:
 *   LP     Probe  linear_probing_ht.cpp:39-60  (slot ids, non-empty pack)
 *          Next   :62-115 (match-pack :72-80, Slice :85 + payload :90-94, advance-pack :100-110)
 *   chain  Probe  chaining_ht.cpp:38-58 + ScanStructure ctor chaining_ht.h:31-42
 *          Next   :60-136 (ScanInnerJoin match :88-99, GatherResult :126-136, Advance :109-124)
 * Rounds are recorded one by one (LP: one Next per round; chaining merges empty rounds into the
 * following Next — the host facade reproduces that from out_round_counts).
 * Scratch arrays are chunk-sized; returns -1 on an exceeded output bound. */
static int probe_chunk(int kind, const int64_t *table, const uint64_t *bucket_off, uint64_t size,
                       const int64_t *col, const uint32_t *sel, uint32_t count, uint64_t cap,
                       uint32_t max_rounds, uint64_t *pos, uint64_t *end, uint32_t *act,
                       uint32_t *o_sel, int64_t *o_pay, uint32_t *o_count, uint32_t *o_rounds,
                       uint32_t *o_rc, uint32_t *o_pos) {
  uint64_t mask = size - 1;
  uint32_t n_act = 0;
  for (uint32_t i = 0; i < count; ++i) {
    uint32_t r = sel ? sel[i] : i;
    uint64_t h = ccj_o_murmurhash64((uint64_t)col[r]) & mask;
    if (kind == 0) {
      pos[i] = h;
    } else {
      pos[i] = bucket_off[h];
      end[i] = bucket_off[h + 1];
    }
  }
  for (uint32_t i = 0; i < count; ++i) {
    act[n_act] = i;
    n_act += kind == 0 ? (table[pos[i]] != -1) : (pos[i] != end[i]);
  }
  uint64_t total = 0;
  uint32_t round = 0;
  while (n_act > 0) {
    uint32_t rc = 0;
    for (uint32_t a = 0; a < n_act; ++a) {
      uint32_t idx = act[a];
      uint32_t r = sel ? sel[idx] : idx;
      int64_t cand = table[pos[idx]];
      if (col[r] == cand) {
        if (total >= cap) return -1;
        o_sel[total] = r;
        o_pay[total] = cand;
        if (o_pos) o_pos[total] = (uint32_t)pos[idx];
        ++total;
        ++rc;
      }
    }
    if (o_rc) {
      if (round >= max_rounds) return -1;
      o_rc[round] = rc;
    }
    ++round;
    uint32_t nn = 0;
    for (uint32_t a = 0; a < n_act; ++a) {
      uint32_t idx = act[a];
      act[nn] = idx;
      if (kind == 0) {
        pos[idx] = (pos[idx] + 1) & mask;
        nn += table[pos[idx]] != -1;
      } else {
        pos[idx] += 1;
        nn += pos[idx] != end[idx];
      }
    }
    n_act = nn;
  }
  *o_count = (uint32_t)total;
  *o_rounds = round;
  return 0;
}

int ccj_o_probe(int kind, const int64_t *table, const uint64_t *bucket_off, uint64_t size,
                const int64_t *keys, const uint32_t *sel, const uint32_t *counts, uint64_t n_rows,
                uint32_t chunk, uint64_t cap, uint32_t max_rounds, uint32_t *out_count,
                uint32_t *out_sel, int64_t *out_payload, uint32_t *out_rounds,
                uint32_t *out_round_counts, int threads, uint32_t *out_pos) {
  uint64_t n_chunks = (n_rows + chunk - 1) / chunk;
  int err = 0;
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel num_threads(threads) reduction(| : err)
  {
    uint64_t *pos = (uint64_t *)malloc(chunk * sizeof(uint64_t));
    uint64_t *end = (uint64_t *)malloc(chunk * sizeof(uint64_t));
    uint32_t *act = (uint32_t *)malloc(chunk * sizeof(uint32_t));
#pragma omp for schedule(static)
    for (uint64_t c = 0; c < n_chunks; ++c) {
      uint64_t base = c * (uint64_t)chunk;
      uint32_t phys = (uint32_t)((n_rows - base) < chunk ? (n_rows - base) : chunk);
      uint32_t count = counts ? counts[c] : phys;
      uint32_t rounds = 0;
      int e = probe_chunk(kind, table, bucket_off, size, keys + base, sel ? sel + base : NULL, count, cap,
                          max_rounds, pos, end, act, out_sel + c * cap, out_payload + c * cap, &out_count[c],
                          &rounds, out_round_counts ? out_round_counts + c * (uint64_t)max_rounds : NULL,
                          out_pos ? out_pos + c * cap : NULL);
      if (out_rounds) out_rounds[c] = rounds;
      if (e) err = 1;
    }
    free(pos);
    free(end);
    free(act);
  }
  return err ? -1 : 0;
}

uint64_t ccj_o_probe_totals(int kind, const int64_t *table, const uint64_t *bucket_off, uint64_t size,
                            const int64_t *keys, uint64_t n_rows, uint32_t chunk, uint64_t row_base,
                            uint64_t *l2_out, int threads) {
  uint64_t n_chunks = (n_rows + chunk - 1) / chunk;
  uint64_t matches = 0, l2 = 0;
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel num_threads(threads) reduction(+ : matches, l2)
  {
    uint64_t *pos = (uint64_t *)malloc(chunk * sizeof(uint64_t));
    uint64_t *end = (uint64_t *)malloc(chunk * sizeof(uint64_t));
    uint32_t *act = (uint32_t *)malloc(chunk * sizeof(uint32_t));
    uint32_t *o_sel = (uint32_t *)malloc((uint64_t)chunk * 64 * sizeof(uint32_t));
    int64_t *o_pay = (int64_t *)malloc((uint64_t)chunk * 64 * sizeof(int64_t));
#pragma omp for schedule(static)
    for (uint64_t c = 0; c < n_chunks; ++c) {
      uint64_t base = c * (uint64_t)chunk;
      uint32_t phys = (uint32_t)((n_rows - base) < chunk ? (n_rows - base) : chunk);
      uint32_t cnt = 0, rounds = 0;
      probe_chunk(kind, table, bucket_off, size, keys + base, NULL, phys, (uint64_t)chunk * 64, 0, pos, end,
                  act, o_sel, o_pay, &cnt, &rounds, NULL, NULL);
      matches += cnt;
      for (uint32_t j = 0; j < cnt; ++j) l2 += ccj_l2_term(row_base + base + o_sel[j], o_pay[j]);
    }
    free(pos);
    free(end);
    free(act);
    free(o_sel);
    free(o_pay);
  }
  if (l2_out) *l2_out = l2;
  return matches;
}

void ccj_o_gen_uniform(uint64_t seed, uint64_t row_begin, uint64_t n, uint64_t range, int64_t *out, int threads) {
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for num_threads(threads) schedule(static)
  for (uint64_t i = 0; i < n; ++i) out[i] = ccj_uniform_key(seed, row_begin + i, range);
}

uint64_t ccj_o_count_uniform(uint64_t seed, uint64_t row_begin, uint64_t row_end, uint64_t range,
                             uint64_t n_build, uint64_t cf, uint64_t *l2_out, int threads) {
  uint64_t matches = 0, l2 = 0;
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for num_threads(threads) schedule(static) reduction(+ : matches, l2)
  for (uint64_t i = row_begin; i < row_end; ++i) {
    int64_t k = ccj_uniform_key(seed, i, range);
    uint64_t m = ccj_o_ref_multiplicity(k, n_build, cf);
    matches += m;
    l2 += m * ccj_l2_term(i, k);
  }
  if (l2_out) *l2_out = l2;
  return matches;
}

/* Zipf table of the C3 stream over n_build keys of multiplicity cf (ccj_gen.h ccj_zipf_table). */
static uint32_t *c3_zipf(uint64_t n_build, uint64_t cf) {
  const uint64_t n_unique = n_build / cf + (n_build % cf != 0);
  uint32_t *t = (uint32_t *)malloc((CCJ_ZIPF_BUCKETS + 1) * sizeof(uint32_t));
  ccj_zipf_table(n_unique, t);
  return t;
}

void ccj_o_gen_c3(uint64_t seed, uint64_t row_begin, uint64_t n, uint64_t n_build, uint64_t cf, uint32_t hit_ppm,
                  int64_t *out, int threads) {
  if (threads <= 0) threads = omp_get_max_threads();
  uint32_t *zipf = c3_zipf(n_build, cf);
#pragma omp parallel for num_threads(threads) schedule(static)
  for (uint64_t i = 0; i < n; ++i) out[i] = ccj_c3_key(zipf, seed, row_begin + i, n_build, cf, hit_ppm);
  free(zipf);
}

uint64_t ccj_o_count_c3(uint64_t seed, uint64_t row_begin, uint64_t row_end, uint64_t n_build, uint64_t cf,
                        uint32_t hit_ppm, uint64_t *l2_out, int threads) {
  uint64_t matches = 0, l2 = 0;
  if (threads <= 0) threads = omp_get_max_threads();
  uint32_t *zipf = c3_zipf(n_build, cf);
#pragma omp parallel for num_threads(threads) schedule(static) reduction(+ : matches, l2)
  for (uint64_t i = row_begin; i < row_end; ++i) {
    int64_t k = ccj_c3_key(zipf, seed, i, n_build, cf, hit_ppm);
    uint64_t m = ccj_o_ref_multiplicity(k, n_build, cf);
    matches += m;
    l2 += m * ccj_l2_term(i, k);
  }
  free(zipf);
  if (l2_out) *l2_out = l2;
  return matches;
}

/* compactor.cpp:5-41 simulated literally (with the fresh temp chunk of the commented :36, which
 * removes the aliasing defect of SURVEY §A.3): a full chunk passes through (:6); otherwise rows
 * are appended to the cache (:12-19); on overflow the cache is topped up to `chunk`, emitted,
 * and the remainder becomes the new cache (:22-35).  Flush emits what is cached (compactor.h:23). */
uint64_t ccj_o_compact_plan_threshold(const uint32_t *seg_counts, uint64_t n_segs, uint32_t chunk,
                                      uint32_t threshold, uint64_t *dest, uint32_t *out_chunk_counts) {
  const uint64_t thr = threshold == 0 || threshold > chunk ? chunk : threshold;
  uint64_t *cache = (uint64_t *)malloc((uint64_t)chunk * sizeof(uint64_t));
  uint64_t q = 0, n_out = 0, row = 0;
  for (uint64_t s = 0; s < n_segs; ++s) {
    uint64_t c = seg_counts[s];
    if (c != 0 && c >= thr) {  /* compactor.cpp:6 (thr = chunk); threshold-gated pass-through */
      for (uint64_t j = 0; j < c; ++j) dest[row + j] = n_out * chunk + j;
      if (out_chunk_counts) out_chunk_counts[n_out] = (uint32_t)c;
      ++n_out;
    } else if (c <= chunk - q) {
      for (uint64_t j = 0; j < c; ++j) cache[q++] = row + j;
    } else {
      uint64_t n_move = chunk - q;
      for (uint64_t j = 0; j < n_move; ++j) cache[q++] = row + j;
      for (uint64_t j = 0; j < chunk; ++j) dest[cache[j]] = n_out * chunk + j;
      if (out_chunk_counts) out_chunk_counts[n_out] = chunk;
      ++n_out;
      q = 0;
      for (uint64_t j = n_move; j < c; ++j) cache[q++] = row + j;
    }
    row += c;
  }
  if (q > 0) {
    for (uint64_t j = 0; j < q; ++j) dest[cache[j]] = n_out * chunk + j;
    if (out_chunk_counts) out_chunk_counts[n_out] = (uint32_t)q;
    ++n_out;
  }
  free(cache);
  return n_out;
}

uint64_t ccj_o_compact_plan(const uint32_t *seg_counts, uint64_t n_segs, uint32_t chunk, uint64_t *dest,
                            uint32_t *out_chunk_counts) {
  return ccj_o_compact_plan_threshold(seg_counts, n_segs, chunk, chunk, dest, out_chunk_counts);
}

void ccj_o_gen_mt64(uint64_t seed, uint64_t n, uint64_t range, int64_t *out) {
  ccj_mt19937_64 g;
  ccj_mt19937_64_seed(&g, seed);
  for (uint64_t i = 0; i < n; ++i) out[i] = (int64_t)(ccj_mt19937_64_next(&g) % range);
}

void ccj_o_result_sums(const uint32_t *count, const uint32_t *sel, const int64_t *payload, uint64_t n_chunks,
                       uint64_t cap, uint32_t chunk, uint64_t *out) {
  uint64_t m = 0, l2 = 0, l3 = CCJ_L3_SEED, chk = 0;
  for (uint64_t c = 0; c < n_chunks; ++c) {
    for (uint32_t j = 0; j < count[c]; ++j) {
      const uint32_t s = sel[c * cap + j];
      const int64_t p = payload[c * cap + j];
      const uint64_t row = c * chunk + s;
      ++m;
      l2 += ccj_l2_term(row, p);
      l3 = ccj_l3_fold(l3, row, p);
      chk += (uint64_t)p * 1315423911ULL + s;
    }
  }
  out[0] = m;
  out[1] = l2;
  out[2] = l3;
  out[3] = chk;
}
