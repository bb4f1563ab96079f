// ccj_kernels.hip — gfx950 kernels for the hash-join probe hot path.
//
// probe_chunks<KIND, R>: one wavefront per chunk (up to 64*R rows; lane l owns rows j*64 + l).
// It runs the reference's Probe + Next loop for the whole chunk in one pass:
//   Probe   linear_probing_ht.cpp:45-57 / chaining_ht.cpp:44-55: hash, first candidate, active set
//   Next    match-pack  (:72-80 / :88-99)   -> wave ballot + mbcnt prefix, ordered store
//           payload     (:90-94 / :126-136) -> the matched table value, stored beside the row id
//           advance     (:100-110 / :109-124) -> next slot / next chain node; its candidate is
//                                               compared right away, so the next round's match
//                                               bits are ready without re-reading the table.
// Emission order is round-major, idx ascending within a round: exactly the reference's
// result_vector order (L3).  Per-row state lives in VGPRs (key, slot/chain position, chain end);
// active/match sets are bitmasks over the lane's R rows.
#include <cstdlib>
#include <string>

#include "ccj_internal.h"
#include "ccj_tuning.h"

namespace ccj {
namespace {

__device__ __forceinline__ uint32_t lane_prefix(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Table position of row key k's candidate in round r (LP: home + r; chain: chain start + r) and
// the wide-payload gather (C5) for a match written at output slot o.
template <int KIND>
__device__ __forceinline__ void emit_extra(const ProbeParams &p, uint64_t obase, uint64_t o, int64_t k, uint32_t r) {
  if (!p.out_pos && p.n_pay == 0) return;
  const uint32_t h = (uint32_t)murmurhash64((uint64_t)k) & p.mask;
  const uint32_t pos = KIND == CCJ_TABLE_LP ? ((h + r) & p.mask) : p.off[h] + r;
  if (p.out_pos) p.out_pos[obase + o] = pos;
  if (p.n_pay) {
    const int64_t *row = p.pay + (uint64_t)pos * p.pay_stride;
    for (uint32_t c = 0; c < p.n_pay; ++c) p.out_cols[c][obase + o] = row[c];
  }
}

// Wave reductions over DPP / permlane (ROCm device library ockl), returned wave-uniform (an SGPR
// value: loops over its bits are scalar).  A shuffle tree (__shfl_xor) is 6 dependent
// ds_bpermute round trips through LDS instead.
extern "C" __device__ uint32_t __ockl_wfred_or_u32(uint32_t);
extern "C" __device__ uint32_t __ockl_wfred_max_u32(uint32_t);

__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)__ockl_wfred_or_u32(x));
}

__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)__ockl_wfred_max_u32(x));
}

extern "C" __device__ uint32_t __ockl_wfscan_add_u32(uint32_t, bool);
// Inclusive prefix sum over the wave's lanes (DPP row shifts + permlane, no LDS).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) { return __ockl_wfscan_add_u32(x, true); }

__device__ __forceinline__ void record_round(const ProbeParams &p, uint64_t c, uint32_t r, uint32_t rc,
                                             uint32_t lane, uint32_t &flags) {
  if (p.out_round_counts) {
    if (r < p.max_rounds) {
      if (lane == 0) p.out_round_counts[c * p.max_rounds + r] = rc;
    } else {
      flags |= CCJ_FLAG_ROUND_OVERFLOW;
    }
  }
}

// Generic round-synchronous Next loop for chunks containing a run/chain longer than the
// kMaxFastRounds rounds the windowed path records: round r reads candidate r of every active row
// (position recomputed from the key, no per-row position state).  Rare; correctness path.
__device__ __forceinline__ uint32_t phys_row(const ProbeParams &p, uint64_t base, uint32_t i) {
  return p.sel ? p.sel[base + i] : i;
}

template <int KIND>
__device__ void rounds_generic(const ProbeParams &p, uint64_t c, uint64_t base, uint32_t nj, uint32_t act,
                               const int64_t *s_key, uint32_t &flags, uint64_t &total_out, uint32_t &rounds_out) {
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint64_t obase = p.out_base ? p.out_base[c] : c * p.cap;
  uint64_t total = 0;
  uint32_t round = 0;
  while (true) {
    uint32_t mat = 0;
    for (uint32_t j = 0; j < nj; ++j) {
      if ((act >> j) & 1u) {
        const int64_t k = s_key[j * kWave + lane];
        const uint32_t h = (uint32_t)murmurhash64((uint64_t)k) & p.mask;
        if (KIND == CCJ_TABLE_LP) {
          const int64_t v = p.table[(h + round) & p.mask];
          if (v == -1) act &= ~(1u << j);  // empty slot ends the run
          else if (v == k) mat |= 1u << j;  // (a probe key of -1 never matches)
        } else {
          const uint32_t q = p.off[h] + round;
          if (q >= p.off[h + 1]) act &= ~(1u << j);
          else if (p.table[q] == k) mat |= 1u << j;
        }
      }
    }
    if (wave_or(act) == 0u) break;
    uint32_t rc = 0;
    for (uint32_t any = wave_or(mat); any != 0u; any &= any - 1u) {
      const uint32_t j = (uint32_t)__builtin_ctz(any);
      const bool m = (mat >> j) & 1u;
      const uint64_t mb = __ballot(m);
      if (m) {
        const uint64_t o = total + lane_prefix(mb);
        if (o < p.cap) {
          p.out_sel[obase + o] = phys_row(p, base, j * kWave + lane);
          if (p.out_payload) p.out_payload[obase + o] = s_key[j * kWave + lane];
          emit_extra<KIND>(p, obase, o, s_key[j * kWave + lane], round);
        }
      }
      const uint32_t n = (uint32_t)__popcll(mb);
      total += n;
      rc += n;
    }
    record_round(p, c, round, rc, lane, flags);
    ++round;
  }
  total_out = total;
  rounds_out = round;
}

constexpr int kWin = 4;             // slots (LP) / chain keys per window load: 32 B, one aligned sector
constexpr int kMaxFastRounds = 32;  // rounds recorded by the windowed path (bits of a u32)
// Round words of the ordered probe (probe_walk<..., MM>): mm in bits 0-25, rounds in bits 26-30;
// a row of more than 26 rounds is kMmLong | rounds.
constexpr uint32_t kMmRounds = 26;
constexpr uint32_t kMmLong = 0x80000000u;
// 16-bit form (ProbeParams::w16, distinct build keys: at most one match round per row):
// min(L, 511) << 7 | the match round (127: none).  A row of more than 26 rounds only needs its L
// (its chunk re-walks), so its round field is 127.
__device__ __forceinline__ uint16_t round_word16(uint32_t w) {
  if (w & kMmLong) {
    const uint32_t r = w & ~kMmLong;
    return (uint16_t)((r < 511u ? r : 511u) << 7 | 127u);
  }
  const uint32_t mm = w & ((1u << kMmRounds) - 1u);
  return (uint16_t)((w >> kMmRounds) << 7 | (mm ? (uint32_t)__builtin_ctz(mm) : 127u));
}
__device__ __forceinline__ uint32_t round_word32(uint16_t h) {
  const uint32_t r = (uint32_t)h >> 7, m = h & 127u;
  if (r > kMmRounds) return kMmLong | r;
  return (m < 127u ? 1u << m : 0u) | r << kMmRounds;
}
constexpr int kWalkRows = 2;  // rows per lane walked concurrently (loads in flight)

constexpr int kEmitRows = 4;    // row groups per lane whose sel loads are issued together in the emit
constexpr int kChunkWaves = 4;  // waves cooperating on one chunk
constexpr int kBlock = kWave * kChunkWaves;

// One 256-thread workgroup (4 waves) per chunk of up to 64*nj rows; row (j, lane) = j*64 + lane is
// owned by wave j % 4.  LDS (28 KB): s_key — the chunk's probe keys, staged once with coalesced
// loads; s_mm[row] — bit r set iff the row matches in round r (Next call r); s_off[r*32 + j] —
// matches of (round r, row group j), then their exclusive prefix in round-major order.
//
// Walk: every row's whole run (LP: home slot up to the first empty slot; chain: the bucket's CSR
// range) is read once through aligned 32-byte windows.  G cursors per lane each own every G-th row
// of the lane and move on as soon as their run ends, so ~G window loads per lane stay in flight.
// A continuation reads the line fetched moments earlier (L2-resident), not one fetched a whole
// round of 2048 rows earlier — the reference's round-by-round re-read (linear_probing_ht.cpp:72-80,
// :100-110) loses L2 residency at GPU occupancy.
// Count + scan: per (round, row group) ballot counts, exclusive scan.  Emit: every match goes to
// s_off[r][j] + its ballot prefix — the reference's round-major, idx-ascending result_vector
// order (L3) — with the payload (== probe key) taken from LDS.
// Walk: every row's whole run (LP: home slot up to the first empty slot; chain: the bucket's CSR
// range) through aligned 32-byte windows; s_mm[row] gets bit r for every round r in which the row
// matches.  Lane `lane` of wave `wave` owns rows (q * 4 + wave) * 64 + lane for the q set in
// `act`; G cursors per lane each take every G-th of them and move on as soon as their run ends.
// on_end(row, rounds) reports a finished run (rounds = occupied slots / chain keys walked).
// Returns true if some run is longer than kMaxFastRounds (the caller then uses rounds_generic).
template <int KIND, int G, typename OnEnd>
__device__ __forceinline__ bool walk_rows(const ProbeParams &p, const int64_t *s_key, uint32_t *s_mm, uint32_t act,
                                          uint32_t nq, uint32_t wave, uint32_t lane, OnEnd on_end) {
  bool long_run = false;
  uint32_t q[G], cur[G], r0[G], lim[G], mm[G];
  int64_t kj[G];
  uint32_t live = 0, start = 0;  // bit g: cursor has a row / row still needs its CSR range
  auto next_active = [&](uint32_t from) -> uint32_t {
    for (uint32_t t = from; t < nq; t += G)
      if ((act >> t) & 1u) return t;
    return nq;
  };
  auto begin_row = [&](int g) {
    kj[g] = s_key[(q[g] * kChunkWaves + wave) * kWave + lane];
    const uint32_t h = (uint32_t)murmurhash64((uint64_t)kj[g]) & p.mask;
    cur[g] = h;  // LP: home slot; chain: bucket until its CSR range is loaded
    r0[g] = 0;
    mm[g] = 0;
    live |= 1u << g;
    if (KIND == CCJ_TABLE_CHAIN) start |= 1u << g;
  };
#pragma unroll
  for (int g = 0; g < G; ++g) {
    cur[g] = r0[g] = lim[g] = mm[g] = 0;
    kj[g] = 0;
    q[g] = next_active(g);
    if (q[g] < nq) begin_row(g);
  }
  while (__ballot(live != 0u) != 0ull) {
    longlong2 v[G][kWin / 2];
    uint32_t o0[G], o1[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if ((live >> g) & 1u) {
        if (KIND == CCJ_TABLE_CHAIN && ((start >> g) & 1u)) {
          if (p.bucket) {  // {start | len << 32, first key}: range + round-0 candidate, one load
            const longlong2 rec = p.bucket[cur[g]];
            o0[g] = (uint32_t)rec.x;
            o1[g] = (uint32_t)rec.x + (uint32_t)((uint64_t)rec.x >> 32);
            v[g][0].x = rec.y;
          } else {
            o0[g] = p.off[cur[g]];  // chaining_ht.cpp:46-49: bucket -> chain (CSR range)
            o1[g] = p.off[cur[g] + 1];
          }
        } else {
          const longlong2 *w = reinterpret_cast<const longlong2 *>(p.table + (cur[g] & ~(uint32_t)(kWin - 1)));
#pragma unroll
          for (int t = 0; t < kWin / 2; ++t) v[g][t] = w[t];
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if ((live >> g) & 1u) {
        const uint32_t row = (q[g] * kChunkWaves + wave) * kWave + lane;
        bool done = false;
        if (KIND == CCJ_TABLE_CHAIN && ((start >> g) & 1u)) {
          start &= ~(1u << g);
          cur[g] = o0[g];
          lim[g] = o1[g];
          done = cur[g] == lim[g];  // empty bucket: not in the active set (chaining_ht.cpp:52-55)
          if (!done && p.bucket) {  // round 0 from the record's first key
            if (v[g][0].x == kj[g]) mm[g] |= 1u;
            r0[g] = 1;
            cur[g] = o0[g] + 1;
            if (cur[g] == lim[g]) {  // a one-key chain: one round
              on_end(row, 1u);
              done = true;
            }
          }
        } else {
          const uint32_t blk = cur[g] & ~(uint32_t)(kWin - 1);
          const uint32_t off = cur[g] - blk;
          bool go = true;
#pragma unroll
          for (int t = 0; t < kWin; ++t) {
            const int64_t val = (t & 1) ? v[g][t >> 1].y : v[g][t >> 1].x;
            if (go && (uint32_t)t >= off) {
              const uint32_t r = r0[g] + (uint32_t)t - off;
              const bool stop = KIND == CCJ_TABLE_LP ? (val == -1) : (blk + (uint32_t)t == lim[g]);
              if (stop) {
                go = false;
                on_end(row, r);
              } else if (r >= (uint32_t)kMaxFastRounds) {
                go = false;
                long_run = true;
              } else if (val == kj[g]) {
                mm[g] |= 1u << r;
              }
            }
          }
          if (go) {
            r0[g] += (uint32_t)kWin - off;
            cur[g] = KIND == CCJ_TABLE_LP ? ((blk + kWin) & p.mask) : blk + kWin;
            if (KIND == CCJ_TABLE_CHAIN && cur[g] == lim[g]) {
              on_end(row, r0[g]);
              go = false;
            }
          }
          done = !go;
        }
        if (done) {
          s_mm[row] = mm[g];
          live &= ~(1u << g);
          q[g] = next_active(q[g] + G);
          if (q[g] < nq) begin_row(g);
        }
      }
    }
  }
  return long_run;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int KIND, int G>
__global__ __launch_bounds__(kBlock) void probe_chunks(ProbeParams p) {
  __shared__ int64_t s_key[kMaxChunk];
  __shared__ uint32_t s_mm[kMaxChunk];
  __shared__ uint32_t s_off[kMaxFastRounds * 32];
  __shared__ uint32_t s_red[3 * kChunkWaves];
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  // Optional XCD-aware order (perf only): workgroups are dealt round-robin to the 8 XCDs, so block
  // b takes chunk (b % 8) * (n8 / 8) + b / 8 and each XCD walks a contiguous range of chunks —
  // with slot-partitioned input, the table window those chunks share stays in that XCD's L2.
  uint64_t c = blockIdx.x;
  if (p.xcd_swizzle) {
    const uint64_t n8 = (p.swz_chunks ? p.swz_chunks : p.n_chunks) & ~7ull;
    if (c < n8) c = (c & 7) * (n8 >> 3) + (c >> 3);
  }
  const uint64_t base = p.chunk_base ? p.chunk_base[c] : c * p.chunk;
  const uint64_t rem = p.n_rows - base;
  const uint32_t phys = rem < p.chunk ? (uint32_t)rem : p.chunk;
  const uint32_t nj = (p.chunk + kWave - 1) / kWave;
  uint32_t count = p.counts ? p.counts[c] : phys;
  uint32_t flags = 0;
  if (count > p.chunk) {
    flags |= CCJ_FLAG_BAD_INPUT;
    count = p.chunk;
  }

  // Stage (Probe: linear_probing_ht.cpp:45-49 / chaining_ht.cpp:46-50): keys through sel -> LDS.
  // Thread (wave, lane) stages rows j = 4q + wave, i.e. exactly the rows its lane owns: act bit q.
  // Every load in flight first (round 2d: under `if (i < count)` each row group's sel and key loads
  // waited for the previous group's): clamped indexes, the results masked afterwards.
  constexpr int kQs = (int)(kMaxChunk / kBlock);
  uint32_t act = 0;
  uint32_t rv[kQs];
  int64_t kv[kQs];
#pragma unroll
  for (int q = 0; q < kQs; ++q) {
    const uint32_t i = tid + (uint32_t)q * kBlock;
    rv[q] = count ? phys_row(p, base, i < count ? i : 0u) : 0u;  // (no sel entry is read past the count)
  }
#pragma unroll
  for (int q = 0; q < kQs; ++q) kv[q] = p.keys[base + (rv[q] < phys ? rv[q] : 0u)];
#pragma unroll
  for (int q = 0; q < kQs; ++q) {
    const uint32_t i = tid + (uint32_t)q * kBlock;
    if (i >= nj * kWave) break;
    int64_t k = 0;
    if (i < count) {
      if (rv[q] < phys) {
        k = kv[q];
        act |= 1u << q;
      } else {
        flags |= CCJ_FLAG_BAD_INPUT;
      }
    }
    s_key[i] = k;
    s_mm[i] = 0u;
  }
  for (uint32_t q = tid; q < kMaxFastRounds * 32; q += kBlock) s_off[q] = 0u;
  const uint32_t nq = nj > wave ? (nj - wave + kChunkWaves - 1) / kChunkWaves : 0;

  // Walk.
  uint32_t lane_rounds = 0;
  const bool long_run = walk_rows<KIND, G>(p, s_key, s_mm, act, nq, wave, lane, [&](uint32_t, uint32_t r) {
    lane_rounds = r > lane_rounds ? r : lane_rounds;
  });

  // Block-wide round count and long-run flag.
  {
    const uint32_t wr = wave_max(lane_rounds);
    const bool wl = __ballot(long_run) != 0ull;
    if (lane == 0) {
      s_red[wave] = wr;
      s_red[kChunkWaves + wave] = wl ? 1u : 0u;
    }
  }
  __syncthreads();
  uint32_t rounds = 0, any_long = 0;
#pragma unroll
  for (int w = 0; w < kChunkWaves; ++w) {
    rounds = s_red[w] > rounds ? s_red[w] : rounds;
    any_long |= s_red[kChunkWaves + w];
  }

  uint64_t total = 0;
  if (any_long) {
    if (wave == 0) {
      uint32_t act_all = 0;
      for (uint32_t j = 0; j < nj; ++j) {
        const uint32_t i = j * kWave + lane;
        if (i < count && phys_row(p, base, i) < phys) act_all |= 1u << j;
      }
      rounds_generic<KIND>(p, c, base, nj, act_all, s_key, flags, total, rounds);
    }
  } else {
    // Count: matches per (round r, row group j); wave w takes the row groups it owns.
    for (uint32_t j = wave; j < nj; j += kChunkWaves) {
      const uint32_t m = s_mm[j * kWave + lane];
      for (uint32_t any = wave_or(m); any != 0u; any &= any - 1u) {
        const uint32_t r = (uint32_t)__builtin_ctz(any);
        const uint32_t n = (uint32_t)__popcll(__ballot((m >> r) & 1u));
        if (lane == 0) s_off[r * 32 + j] = n;
      }
    }
    __syncthreads();
    // Scan: exclusive prefix over (r, j) in round-major order, 16 entries per lane of wave 0.
    if (wave == 0) {
      uint32_t loc[16], sum = 0;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        loc[t] = s_off[lane * 16 + t];
        sum += loc[t];
      }
      uint32_t incl = wave_incl_scan(sum);
      uint32_t run = incl - sum;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        s_off[lane * 16 + t] = run;
        run += loc[t];
      }
      if (lane == kWave - 1) s_red[2 * kChunkWaves] = incl;
    }
    __syncthreads();
    total = s_red[2 * kChunkWaves];
    // Per-round counts (Next return values): differences of the round starts.
    if (p.out_round_counts) {
      for (uint32_t r = tid; r < rounds; r += kBlock) {
        const uint32_t a = s_off[r * 32], b = r + 1 < rounds ? s_off[(r + 1) * 32] : (uint32_t)total;
        if (r < p.max_rounds) p.out_round_counts[c * p.max_rounds + r] = b - a;
      }
      if (rounds > p.max_rounds) flags |= CCJ_FLAG_ROUND_OVERFLOW;
    }
    // Emit.
    const uint64_t obase = p.out_base ? p.out_base[c] : c * p.cap;
    // When the chunk's output fits kMaxChunk entries (no C5 extras, aligned region), it is assembled
    // in its final order in LDS — in s_mm (sel) and s_key (payload), free once every thread holds
    // its rows' masks, rows and keys in registers — and written with 16-byte stores instead of one
    // partly idle store pair per (round, row group) (the ordered probe's emit: 7.8 -> 4.3 ms).
    // (not with p.out_base: the pipeline packs chunk outputs back to back, so the last partial
    // 16-byte group would overwrite the next chunk's first entries)
    const bool img = total <= kMaxChunk && total <= p.cap && p.cap % 4 == 0 && !p.out_base && !p.out_pos &&
                     p.n_pay == 0;
    if (img) {
      constexpr int kG = (int)((kMaxChunk / kWave + kChunkWaves - 1) / kChunkWaves);  // groups per wave
      uint32_t m[kG], rr[kG];
      int64_t kk[kG];
#pragma unroll
      for (int g = 0; g < kG; ++g) {
        const uint32_t j = wave + (uint32_t)g * kChunkWaves;
        m[g] = j < nj ? s_mm[j * kWave + lane] : 0u;
        rr[g] = m[g] ? phys_row(p, base, j * kWave + lane) : 0u;
        kk[g] = j < nj ? s_key[j * kWave + lane] : 0;
      }
      __syncthreads();  // s_mm and s_key are read: from here on they hold the output image
      uint32_t *s_osel = s_mm;
      int64_t *s_opay = s_key;
#pragma unroll
      for (int g = 0; g < kG; ++g) {
        const uint32_t j = wave + (uint32_t)g * kChunkWaves;
        if (j >= nj) continue;
        for (uint32_t any = wave_or(m[g]); any != 0u; any &= any - 1u) {
          const uint32_t r = (uint32_t)__builtin_ctz(any);
          const bool bit = (m[g] >> r) & 1u;
          const uint64_t mb = __ballot(bit);
          if (bit) {
            const uint32_t o = s_off[r * 32 + j] + lane_prefix(mb);
            s_osel[o] = rr[g];
            s_opay[o] = kk[g];
          }
        }
      }
      __syncthreads();
      const uint32_t tot = (uint32_t)total;
      // a last partial group writes past the count inside the chunk's own cap region
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(p.out_sel + obase, (short)0, (int)(p.cap * 4), 0x00020000);
      for (uint32_t g = tid; g * 4 < tot; g += kBlock) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(&s_osel[4 * g]);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(16 * g), 0, 0);
      }
      if (p.out_payload) {
        const auto rp = __builtin_amdgcn_make_buffer_rsrc(p.out_payload + obase, (short)0, (int)(p.cap * 8), 0x00020000);
        for (uint32_t g = tid; g * 2 < tot; g += kBlock) {
          const u32x4 v = *reinterpret_cast<const u32x4 *>(&s_opay[2 * g]);
          __builtin_amdgcn_raw_buffer_store_b128(v, rp, (int)(16 * g), 0, 0);
        }
      }
    }
    for (uint32_t jb = wave; jb < nj && !img; jb += kChunkWaves * kEmitRows) {
      uint32_t m[kEmitRows], rr[kEmitRows];
#pragma unroll
      for (int g = 0; g < kEmitRows; ++g) {
        const uint32_t j = jb + g * kChunkWaves;
        m[g] = j < nj ? s_mm[j * kWave + lane] : 0u;
        rr[g] = m[g] ? phys_row(p, base, j * kWave + lane) : 0u;
      }
#pragma unroll
      for (int g = 0; g < kEmitRows; ++g) {
        const uint32_t j = jb + g * kChunkWaves;
        for (uint32_t any = wave_or(m[g]); any != 0u; any &= any - 1u) {
          const uint32_t r = (uint32_t)__builtin_ctz(any);
          const bool bit = (m[g] >> r) & 1u;
          const uint64_t mb = __ballot(bit);
          if (bit) {
            const uint64_t o = (uint64_t)s_off[r * 32 + j] + lane_prefix(mb);
            if (o < p.cap) {
              const int64_t k = s_key[j * kWave + lane];
              p.out_sel[obase + o] = rr[g];
              if (p.out_payload) p.out_payload[obase + o] = k;  // matched table value == probe key
              emit_extra<KIND>(p, obase, o, k, r);
            }
          }
        }
      }
    }
  }

  if (total > p.cap) flags |= CCJ_FLAG_CAP_OVERFLOW;
  if (tid == 0) {
    p.out_count[c] = (uint32_t)(total < p.cap ? total : p.cap);
    if (p.out_rounds) p.out_rounds[c] = rounds;
  }
  if (p.status) {
    const uint64_t any = __ballot(flags != 0u);
    if (any && flags) atomicOr(p.status, flags);
  }
}

// Walks of slot-partitioned input (ccj_probe_partitioned): the output order inside a chunk is
// free (L1/L2 parity), so there is no per-round bookkeeping; 256 threads per 2048-row chunk.
constexpr int kFlatThreads = 256;
constexpr int kFlatRows = kMaxChunk / kFlatThreads;  // 8
constexpr uint32_t kFlatStage = kMaxChunk;          // matches staged in LDS per chunk

// A chunk's live keys into LDS: every thread issues all of its kFlatRows loads before the first
// LDS write (a rolled loop waits out one memory latency per load).
__device__ __forceinline__ void stage_keys(int64_t *s_key, const int64_t *keys, uint32_t phys, uint32_t tid) {
  int64_t v[kFlatRows];
#pragma unroll
  for (int j = 0; j < kFlatRows; ++j) {
    const uint32_t i = tid + (uint32_t)j * kFlatThreads;
    v[j] = i < phys ? __builtin_nontemporal_load(keys + i) : 0;
  }
#pragma unroll
  for (int j = 0; j < kFlatRows; ++j) {
    const uint32_t i = tid + (uint32_t)j * kFlatThreads;
    if (i < phys) s_key[i] = v[j];
  }
}

// Live rows of the flat chunk starting at position `base`: all of them, or with the fixed-capacity
// split's layout the part of the chunk below its segment's fill level.
__device__ __forceinline__ uint32_t flat_phys(const ProbeParams &p, uint64_t base) {
  const uint64_t rem = p.n_rows - base;
  uint32_t phys = rem < p.chunk ? (uint32_t)rem : p.chunk;
  if (p.seg_count && p.ovf_base && base >= p.ovf_base) {  // the overflow area's chunks
    const uint64_t sub = p.ovf_sub ? (base - p.ovf_base) / p.ovf_sub : kOvfSubs;  // its sub-area
    uint64_t live = sub < kOvfSubs ? p.seg_count[ovf_cursor_index(p.seg_parts, (uint32_t)sub)] : 0u;
    live = live < p.ovf_sub ? live : p.ovf_sub;
    const uint64_t off = sub < kOvfSubs ? base - p.ovf_base - sub * p.ovf_sub : 0u;
    phys = live > off ? (live - off < phys ? (uint32_t)(live - off) : phys) : 0u;
  } else if (p.counts && !p.seg_count) {  // identity layout of a column with per-chunk live counts
    const uint32_t cn = p.counts[base / p.chunk];
    phys = cn < phys ? cn : phys;
  } else if (p.seg_count) {
    const uint64_t seg = base / p.seg_cap;
    const uint64_t off = base - seg * p.seg_cap;
    uint64_t live = p.seg_count[seg_cursor_index(p.seg_parts, (uint32_t)(seg & 7), (uint32_t)(seg >> 3))];
    live = live < p.seg_cap ? live : p.seg_cap;
    phys = live > off ? (live - off < phys ? (uint32_t)(live - off) : phys) : 0u;
  }
  return phys;
}

// Several small chunks per workgroup (chunk B a multiple of 64, B <= 512: the reference's default
// kBlockSize 256, base.h:42).  One chunk per workgroup would leave each lane a single row — one
// window load in flight and a workgroup's fixed cost per 256 rows; here 2048 / B chunks share the
// 256 threads, so every lane again walks 8 rows.  Row group j (64 rows) belongs to chunk
// j / (B / 64); the walk is probe_chunks', and counts, scan and emit are done per chunk, so each
// chunk's output is exactly probe_chunks' (L3).
template <int KIND, int G>
__global__ __launch_bounds__(kBlock) void probe_multi(ProbeParams p) {
  constexpr uint32_t kMaxSub = kMaxChunk / kWave;  // 32 chunks of 64 rows at most
  __shared__ int64_t s_key[kMaxChunk];
  __shared__ uint32_t s_mm[kMaxChunk];
  __shared__ uint32_t s_off[kMaxFastRounds * 32];  // (round r, row group j) -> count, then offset
  __shared__ uint32_t s_rounds[kMaxSub], s_total[kMaxSub], s_cnt[kMaxSub];
  __shared__ uint64_t s_base[kMaxSub];
  __shared__ uint32_t s_long;
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const uint32_t B = p.chunk, gpc = B / kWave, K = kMaxChunk / B;
  const uint64_t c0 = (uint64_t)blockIdx.x * K;
  const uint32_t nk = (uint32_t)(p.n_chunks - c0 < K ? p.n_chunks - c0 : K);  // chunks of this block
  uint32_t flags = 0;
  if (tid < kMaxSub) {
    s_rounds[tid] = 0;
    s_total[tid] = 0;
    uint64_t base = 0;
    uint32_t cnt = 0;
    if (tid < nk) {
      const uint64_t c = c0 + tid;
      base = p.chunk_base ? p.chunk_base[c] : c * B;
      const uint64_t rem = p.n_rows - base;
      const uint32_t phys = rem < B ? (uint32_t)rem : B;
      cnt = p.counts ? p.counts[c] : phys;
      if (cnt > B) {
        flags |= CCJ_FLAG_BAD_INPUT;
        cnt = B;
      }
    }
    s_base[tid] = base;
    s_cnt[tid] = cnt;
  }
  if (tid == 0) s_long = 0;
  for (uint32_t q = tid; q < kMaxFastRounds * 32; q += kBlock) s_off[q] = 0u;
  __syncthreads();

  // Stage: the row of group j, lane l is row (j - k*gpc)*64 + l of chunk k = j / gpc.
  uint32_t act = 0;
  for (uint32_t i = tid, q = 0; i < kMaxChunk; i += kBlock, ++q) {
    const uint32_t k = i / B, li = i - k * B;
    int64_t key = 0;
    if (k < nk && li < s_cnt[k]) {
      const uint64_t base = s_base[k];
      const uint64_t rem = p.n_rows - base;
      const uint32_t phys = rem < B ? (uint32_t)rem : B;
      const uint32_t r = phys_row(p, base, li);
      if (r < phys) {
        key = p.keys[base + r];
        act |= 1u << q;
      } else {
        flags |= CCJ_FLAG_BAD_INPUT;
      }
    }
    s_key[i] = key;
    s_mm[i] = 0u;
  }
  __syncthreads();
  const uint32_t nq = kMaxChunk / kWave / kChunkWaves;  // 8 row groups per wave

  // Walk (rounds per chunk through LDS max).
  const bool long_run = walk_rows<KIND, G>(p, s_key, s_mm, act, nq, wave, lane, [&](uint32_t row, uint32_t r) {
    if (r) atomicMax(&s_rounds[row / B], r);
  });
  if (__ballot(long_run) != 0ull && lane == 0) s_long = 1;
  __syncthreads();

  if (s_long) {
    // Rare: some run exceeds kMaxFastRounds; every chunk of the block takes the generic path.
    if (wave == 0) {
      for (uint32_t k = 0; k < nk; ++k) {
        const uint64_t c = c0 + k, base = s_base[k];
        const uint64_t rem = p.n_rows - base;
        const uint32_t phys = rem < B ? (uint32_t)rem : B;
        uint32_t act_k = 0;
        for (uint32_t j = 0; j < gpc; ++j) {
          const uint32_t i = j * kWave + lane;
          if (i < s_cnt[k] && phys_row(p, base, i) < phys) act_k |= 1u << j;
        }
        uint64_t total = 0;
        uint32_t rounds = 0;
        rounds_generic<KIND>(p, c, base, gpc, act_k, s_key + k * B, flags, total, rounds);
        if (total > p.cap) flags |= CCJ_FLAG_CAP_OVERFLOW;
        if (lane == 0) {
          p.out_count[c] = (uint32_t)(total < p.cap ? total : p.cap);
          if (p.out_rounds) p.out_rounds[c] = rounds;
        }
      }
    }
  } else {
    // Count: matches per (round r, row group j).
    for (uint32_t j = wave; j < kMaxChunk / kWave; j += kChunkWaves) {
      const uint32_t m = s_mm[j * kWave + lane];
      for (uint32_t any = wave_or(m); any != 0u; any &= any - 1u) {
        const uint32_t r = (uint32_t)__builtin_ctz(any);
        const uint32_t n = (uint32_t)__popcll(__ballot((m >> r) & 1u));
        if (lane == 0) s_off[r * 32 + j] = n;
      }
    }
    __syncthreads();
    // Scan per chunk, round-major: wave w takes chunks k = w, w+4, ...; lane r holds round r.
    for (uint32_t k = wave; k < nk; k += kChunkWaves) {
      uint32_t tk = 0;
      if (lane < kMaxFastRounds)
        for (uint32_t j = k * gpc; j < (k + 1) * gpc; ++j) tk += s_off[lane * 32 + j];
      const uint32_t incl = wave_incl_scan(tk);  // lanes >= kMaxFastRounds add 0
      if (lane < kMaxFastRounds) {
        uint32_t run = incl - tk;
        for (uint32_t j = k * gpc; j < (k + 1) * gpc; ++j) {
          const uint32_t n = s_off[lane * 32 + j];
          s_off[lane * 32 + j] = run;
          run += n;
        }
        const uint64_t c = c0 + k;
        const uint32_t rounds = s_rounds[k];
        if (p.out_round_counts && lane < rounds) {
          if (lane < p.max_rounds) p.out_round_counts[c * p.max_rounds + lane] = tk;  // Next return values
        }
        if (lane == kMaxFastRounds - 1) s_total[k] = incl;
      }
    }
    __syncthreads();
    // Emit: group j's matches of round r go to s_off[r][j] + ballot prefix in its chunk's output.
    for (uint32_t jb = wave; jb < kMaxChunk / kWave; jb += kChunkWaves * kEmitRows) {
      uint32_t m[kEmitRows], rr[kEmitRows];
#pragma unroll
      for (int g = 0; g < kEmitRows; ++g) {
        const uint32_t j = jb + g * kChunkWaves, k = j / gpc;
        m[g] = s_mm[j * kWave + lane];
        rr[g] = m[g] ? phys_row(p, s_base[k], (j - k * gpc) * kWave + lane) : 0u;
      }
#pragma unroll
      for (int g = 0; g < kEmitRows; ++g) {
        const uint32_t j = jb + g * kChunkWaves, k = j / gpc;
        const uint64_t c = c0 + k;
        const uint64_t obase = (k < nk && p.out_base) ? p.out_base[c] : c * p.cap;
        for (uint32_t any = wave_or(m[g]); any != 0u; any &= any - 1u) {
          const uint32_t r = (uint32_t)__builtin_ctz(any);
          const bool bit = (m[g] >> r) & 1u;
          const uint64_t mb = __ballot(bit);
          if (bit) {
            const uint64_t o = (uint64_t)s_off[r * 32 + j] + lane_prefix(mb);
            if (o < p.cap) {
              const int64_t key = s_key[j * kWave + lane];
              p.out_sel[obase + o] = rr[g];
              if (p.out_payload) p.out_payload[obase + o] = key;  // matched table value == probe key
              emit_extra<KIND>(p, obase, o, key, r);
            }
          }
        }
      }
    }
    if (tid < nk) {
      const uint64_t c = c0 + tid;
      const uint32_t total = s_total[tid];
      if (total > p.cap) flags |= CCJ_FLAG_CAP_OVERFLOW;
      if (p.out_round_counts && s_rounds[tid] > p.max_rounds) flags |= CCJ_FLAG_ROUND_OVERFLOW;
      p.out_count[c] = (uint32_t)(total < p.cap ? total : p.cap);
      if (p.out_rounds) p.out_rounds[c] = s_rounds[tid];
    }
  }
  if (p.status) {
    if (__ballot(flags != 0u) && flags) atomicOr(p.status, flags);
  }
}

template <int KIND>
hipError_t launch_kind(const ProbeParams &p, hipStream_t s) {
  // Chunks of <= 512 rows (the reference's default kBlockSize 256, base.h:42) share a workgroup.
  if (p.chunk % kWave == 0 && p.chunk <= 512 && !p.xcd_swizzle) {
    const uint64_t per = kMaxChunk / p.chunk;
    hipLaunchKernelGGL((probe_multi<KIND, kWalkRows>), dim3((unsigned)((p.n_chunks + per - 1) / per)), dim3(kBlock), 0,
                       s, p);
    return hipGetLastError();
  }
  // G = 2 cursors per lane (G = 4 / 6 / 8 measured 34.2 / 33.3 / 22.5 G tuples/s vs 35.3 at C2)
  hipLaunchKernelGGL((probe_chunks<KIND, kWalkRows>), dim3((unsigned)p.n_chunks), dim3(kBlock), 0, s, p);
  return hipGetLastError();
}

// linear_probing_ht.cpp:16-25: key t of the generator is (t / cf) * step.
__global__ void gen_reference_keys(int64_t *out, uint64_t first, uint64_t n, uint64_t cf, uint64_t step) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
    out[t] = (int64_t)(((first + t) / cf) * step);
}

__global__ void fill_i64(int64_t *p, uint64_t n, int64_t v) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
    p[t] = v;
}

// Parallel linear-probing insert (CCJ_LAYOUT_DEVICE): CAS into the first empty slot at or after
// h(k) & mask.  Occupied-slot set and per-cluster key sets equal the sequential build's.
__global__ void lp_insert(const int64_t *keys, uint64_t n, int64_t *slots, uint32_t *slot_row, uint32_t mask) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t k = keys[t];
    if (k == -1) continue;  // the reference "stores" -1 into an empty slot: a no-op
    uint32_t s = (uint32_t)murmurhash64((uint64_t)k) & mask;
    while (true) {
      const unsigned long long old =
          atomicCAS(reinterpret_cast<unsigned long long *>(slots + s), ~0ull, (unsigned long long)k);
      if (old == ~0ull) break;
      s = (s + 1u) & mask;
    }
    if (slot_row) slot_row[s] = (uint32_t)t;  // the slot now owned by build tuple t
  }
}

// Re-lays build payload rows (build order) out by table position: dst[pos][c] = src[row(pos)][c].
__global__ void scatter_payload(const int64_t *src, uint32_t n_cols, const uint32_t *row, uint64_t positions,
                                int64_t *dst) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < positions * n_cols;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t pos = t / n_cols, c = t - pos * n_cols;
    const uint32_t r = row[pos];
    dst[t] = r == kNoRow ? 0 : src[(uint64_t)r * n_cols + c];
  }
}

// Longest occupied run per 4096-slot segment: one wave per segment, 64 slots per step.
__global__ __launch_bounds__(256) void lp_runs(const int64_t *slots, uint64_t n_slots, uint32_t *stats) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t seg = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t n_seg = (n_slots + kRunSegment - 1) / kRunSegment;
  if (seg >= n_seg) return;
  const uint64_t b = seg * kRunSegment;
  uint32_t lead = 0, cur = 0, best = 0;
  bool in_lead = true;
  for (uint64_t s = 0; s < kRunSegment; s += 64) {
    const uint64_t i = b + s + lane;
    const bool occ = i < n_slots && slots[i] != -1;
    uint64_t m = __ballot(occ);
    if (i - lane >= n_slots) break;  // wave-uniform
    // the step's slots: 64, or fewer in a table of < 64 slots (the table's end is bit valid - 1)
    const uint32_t valid = n_slots - (b + s) < 64u ? (uint32_t)(n_slots - (b + s)) : 64u;
    const bool all = m == (valid == 64u ? ~0ull : (1ull << valid) - 1ull);
    // run continuing from the previous step
    const uint32_t lo = all ? valid : (uint32_t)__builtin_ctzll(~m);
    if (in_lead) {
      lead += lo;
      if (!all) in_lead = false;
    }
    if (all) {
      cur += valid;
    } else {
      cur += lo;
      best = cur > best ? cur : best;
      // longest run strictly inside the mask
      uint64_t x = m >> lo;
      uint32_t inner = 0;
      uint64_t y = x;
      while (y) {
        y &= y >> 1;
        ++inner;
      }
      best = inner > best ? inner : best;
      // trailing run: the occupied slots that end at the step's last slot (bit valid - 1; round 6:
      // bit 63 was taken as the table's end, so a run wrapping round a table of < 64 slots lost its
      // tail and max_rounds / max_dup came out short)
      const uint64_t top = m << (64u - valid);
      cur = top == 0 ? 0u : (uint32_t)__builtin_clzll(~top);
    }
    best = cur > best ? cur : best;
  }
  if (lane == 0) {
    stats[seg * 4 + 0] = lead;
    stats[seg * 4 + 1] = cur;
    stats[seg * 4 + 2] = best;
    stats[seg * 4 + 3] = in_lead ? 1u : 0u;
  }
}

// SplitMix64 stream (oracle/ccj_gen.h ccj_splitmix_at): output i of a generator seeded `seed`.
__device__ __forceinline__ uint64_t splitmix_at(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// C3 probe stream: the device twin of oracle/ccj_gen.h ccj_c3_key (same integer arithmetic).
__device__ __forceinline__ uint32_t bitlen64(uint64_t x) { return x ? 64u - (uint32_t)__clzll(x) : 0u; }

__device__ __forceinline__ uint64_t perm_n(uint64_t x, uint64_t n, uint64_t seed) {
  const uint32_t k = n > 1 ? bitlen64(n - 1) : 1u;
  const uint64_t mask = k >= 64 ? ~0ull : (1ull << k) - 1;
  do {
    x = (x * 0xd1342543de82ef95ull + (seed | 1ull)) & mask;
    x ^= x >> (k / 2 + 1);
  } while (x >= n);
  return x;
}

__global__ void gen_c3(int64_t *out, uint64_t n, uint64_t seed, uint64_t first, uint64_t n_build, uint64_t cf,
                       uint32_t hit_ppm, const uint32_t *zipf) {
  const uint64_t n_unique = n_build / cf + (n_build % cf != 0);
  const uint64_t step = n_unique ? n_build / n_unique : 1;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = first + t;
    const uint64_t z1 = splitmix_at(seed, 3 * i), z2 = splitmix_at(seed, 3 * i + 1);
    const uint64_t z3 = splitmix_at(seed, 3 * i + 2);
    int64_t key;
    if (z1 % 1000000ull < hit_ppm && n_unique) {  // Zipf s = 1 rank: bucket = top 16 bits of z2
      const uint32_t j = (uint32_t)(z2 >> (64 - kZipfBits));
      const uint64_t lo = zipf[j], hi = zipf[j + 1] > zipf[j] ? (uint64_t)zipf[j + 1] - 1 : lo;
      const uint64_t r = lo + (z2 & 0xffffffffull) % (hi - lo + 1);
      key = (int64_t)(perm_n(r - 1, n_unique, seed) * step);
    } else {
      key = (int64_t)(n_build + z3 % ((1ull << 62) - n_build));
    }
    out[t] = key;
  }
}

__global__ void gen_uniform(int64_t *out, uint64_t n, uint64_t seed, uint64_t first, uint64_t range) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
    out[t] = (int64_t)(splitmix_at(seed, first + t) % range);
}

// Work accounting (roofline).  acc[0] += table words the reference examines (LP: every slot from
// the home slot through the terminating empty, linear_probing_ht.cpp:72-110; chaining: every chain
// key, chaining_ht.cpp:82-124), acc[1] += matches.  FM (ccj_probe_cost_walk): also what a walk that
// ends a row at its first match examines (the throughput path's first_match walk, distinct-key
// tables) — acc[2] += words (LP: home through the match, or through the empty slot on a miss;
// chaining: chain keys through the match, or the whole chain), acc[3] += the aligned 32-byte windows
// those words lie in (LP: 4-slot windows; chaining: 2-key windows of the chain array after round 0,
// which the 8-byte bucket record's fingerprint / 16-byte record's first key serves).
template <int KIND, bool FM>
__global__ void probe_cost(const int64_t *table, const uint32_t *off, uint32_t mask, const int64_t *keys,
                           uint64_t n, unsigned long long *acc) {
  unsigned long long ex = 0, mt = 0, fw = 0, win = 0;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t k = keys[t];
    const uint32_t h = (uint32_t)murmurhash64((uint64_t)k) & mask;
    uint32_t first = 0;  // words examined through the first match (0: no match yet)
    if (KIND == CCJ_TABLE_LP) {
      uint32_t s = h, w = 0;
      while (true) {
        const int64_t v = table[s];
        ++ex;
        ++w;
        if (v == -1) break;
        if (v == k) {
          ++mt;
          if (!first) first = w;
        }
        s = (s + 1u) & mask;
      }
      if (FM) {
        const uint32_t L = first ? first : w;
        fw += L;
        win += ((h & 3u) + L - 1u) / 4u + 1u;  // aligned 4-slot windows from the home slot's
      }
    } else {
      const uint32_t lo = off[h], e = off[h + 1];
      for (uint32_t q = lo; q < e; ++q) {
        ++ex;
        if (table[q] == k) {
          ++mt;
          if (!first) first = q - lo + 1u;
        }
      }
      if (FM) {
        const uint32_t L = first ? first : e - lo;
        fw += L;
        // round 0 from the bucket record; later keys q in [lo + 1, lo + L) in aligned 2-key windows
        if (L > 1) win += ((lo + L - 1u) >> 1) - ((lo + 1u) >> 1) + 1u;
      }
    }
  }
  for (int d = 32; d > 0; d >>= 1) {
    ex += __shfl_xor(ex, d);
    mt += __shfl_xor(mt, d);
    if (FM) {
      fw += __shfl_xor(fw, d);
      win += __shfl_xor(win, d);
    }
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(acc, ex);
    atomicAdd(acc + 1, mt);
    if (FM) {
      atomicAdd(acc + 2, fw);
      atomicAdd(acc + 3, win);
    }
  }
}

// ccj_probe_visits: the values InOneNext writes into result column m+1 for every active row
// (linear_probing_ht.cpp:125-141, chaining_ht.cpp:148-163).  One thread per row; only the facade's
// one-chunk InOneNext calls it, so it is a plain walk.
template <int KIND>
__global__ void probe_visits(const int64_t *table, const uint32_t *off, uint32_t mask, const int64_t *keys,
                             const uint32_t *sel, uint32_t count, uint32_t max_rounds, int64_t *vals, uint32_t *len) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int64_t k = keys[sel ? sel[i] : i];
  const uint32_t h = (uint32_t)murmurhash64((uint64_t)k) & mask;
  int64_t *v = vals + (uint64_t)i * max_rounds;
  uint32_t r = 0;
  if (KIND == CCJ_TABLE_LP) {
    // active in round r while slot home + r is occupied (Probe :53-56, advance :136-140)
    for (uint32_t s = h; r < max_rounds; s = (s + 1u) & mask) {
      const int64_t x = table[s];
      if (x == -1) break;
      v[r++] = x;
    }
  } else {
    for (uint32_t q = off[h], e = off[h + 1]; q < e && r < max_rounds; ++q) v[r++] = table[q];
  }
  len[i] = r;
}

__device__ __forceinline__ uint64_t fmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// One wave per output chunk region; matches + L2 checksum (oracle/ccj_gen.h ccj_l2_term).
__global__ __launch_bounds__(256) void result_checksum(const uint32_t *count, const uint32_t *sel,
                                                       const int64_t *payload, uint64_t n_chunks, uint64_t cap,
                                                       uint32_t chunk, uint64_t row_base,
                                                       const uint64_t *row_map, unsigned long long *acc) {
  const uint32_t lane = threadIdx.x & 63u;
  unsigned long long m = 0, l2 = 0;
  for (uint64_t c = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < n_chunks; c += (uint64_t)gridDim.x * 4) {
    const uint32_t n = count[c];
    m += n;
    for (uint32_t j = lane; j < n; j += 64) {
      const uint64_t local = c * chunk + sel[c * cap + j];
      const uint64_t row = row_map ? row_map[local] : row_base + local;
      l2 += fmix64(row * 0x9e3779b97f4a7c15ULL + fmix64((uint64_t)payload[c * cap + j] + 1ULL));
    }
  }
  for (int d = 32; d > 0; d >>= 1) l2 += __shfl_xor(l2, d);
  if (lane == 0) {
    atomicAdd(acc, m);
    atomicAdd(acc + 1, l2);
  }
}

unsigned grid_for(uint64_t n, unsigned block) {
  uint64_t g = (n + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g == 0) g = 1;
  return (unsigned)g;
}

}  // namespace

// probe_win<R>: the LP walk of slot-partitioned input that also records every match's table
// position (C5: the payload gather reads the rows by position).  Two lanes per row, each loading
// 16 B of a 32-byte window that starts at the row's next unread slot (clamped to the table end and
// to the window's 128-byte line), R rows in flight per pair.  The step's matches are placed with a
// bit-sliced wave prefix (<= 5 ballots + mbcnt) and one LDS atomic per wave, staged in LDS with
// their positions and written out coalesced; a finished pair takes the chunk's next unwalked row
// from an LDS counter.
template <int R>
__device__ __forceinline__ void walk_chunk(const ProbeParams &p, uint64_t c, uint32_t &s_cnt, uint32_t &s_rounds,
                                           uint32_t &s_next, int64_t *s_key, uint16_t *s_sel, uint32_t *s_pos) {
  constexpr int LPR = 2, WS = 4, LINE = 16;  // lanes per row, window slots, slots per 128-B line
  constexpr bool ALIGN = false, POS = true;
  constexpr uint32_t kGroups = kFlatThreads / LPR;  // rows walked side by side
  constexpr int kSlotsPerLane = WS / LPR;
  constexpr int kLoads = kSlotsPerLane / 2;  // 16-byte pieces per lane and window
  static_assert(kLoads >= 1 && WS <= 16 && (LPR == 1 || LPR == 2), "window shape");
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1);
  const uint32_t sub = LPR == 1 ? 0u : (tid & 1u), grp = tid / LPR;
  const uint32_t last_start = p.mask - (uint32_t)(WS - 1);  // table size - WS (size >= 16)
  const uint64_t base = c * p.chunk;
  const uint32_t phys = flat_phys(p, base);
  const uint64_t obase = c * p.cap;
  stage_keys(s_key, p.keys + base, phys, tid);
  if (tid == 0) {
    s_cnt = 0;
    s_rounds = 0;
    s_next = kGroups * R;
  }
  __syncthreads();
  int64_t key[R];
  uint32_t row[R], cur[R], r0[R];
  uint32_t need = 0, lane_rounds = 0, overflow = 0;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    row[k] = (uint32_t)k * kGroups + grp;
    r0[k] = 0;
    key[k] = 0;
    cur[k] = 0;
    if (row[k] < phys) {
      key[k] = s_key[row[k]];
      cur[k] = (uint32_t)murmurhash64((uint64_t)key[k]) & p.mask;
      need |= 1u << k;
    }
  }
  while (__ballot(need != 0u) != 0ull) {
    int64_t v[R][kSlotsPerLane];
    uint32_t st[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      st[k] = ALIGN ? (cur[k] & ~(uint32_t)(WS - 1)) : (cur[k] < last_start ? cur[k] : last_start);
      if (!ALIGN && LINE) {  // keep the window inside one LINE-slot line: end it at the boundary
        const uint32_t lim = (st[k] & ~(uint32_t)(LINE - 1)) + (uint32_t)(LINE - WS);
        st[k] = st[k] < lim ? st[k] : lim;
      }
      if ((need >> k) & 1u) {
        const int64_t *w = p.table + st[k] + sub * kSlotsPerLane;
#pragma unroll
        for (int t = 0; t < kSlotsPerLane; t += 2) {
          if (CCJ_ABLATED(p.ablate, 2u)) {  // timing only: no table reads
            v[k][t] = t ? -1 : key[k];
            v[k][t + 1] = -1;
          } else if (ALIGN) {
            const longlong2 x = *reinterpret_cast<const longlong2 *>(w + t);
            v[k][t] = x.x;
            v[k][t + 1] = x.y;
          } else {  // 8-byte aligned pair of slots
            v[k][t] = w[t];
            v[k][t + 1] = w[t + 1];
          }
        }
      }
    }
    uint32_t hits[R], n = 0, done = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      uint32_t e = 0, m = 0;
#pragma unroll
      for (int t = 0; t < kSlotsPerLane; ++t) {
        const uint32_t b = sub * kSlotsPerLane + t;
        e |= ((v[k][t] == -1) ? 1u : 0u) << b;
        m |= ((v[k][t] == key[k]) ? 1u : 0u) << b;
      }
      if (LPR == 2) {  // the pair's halves of the window: swap with the partner lane (quad_perm 1,0,3,2)
        e |= (uint32_t)__builtin_amdgcn_mov_dpp((int)e, 0xB1, 0xF, 0xF, false);
        m |= (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0xB1, 0xF, 0xF, false);
      }
      hits[k] = 0;
      if ((need >> k) & 1u) {
        const uint32_t off = cur[k] - st[k];
        const uint32_t from = ~0u << off;
        e &= from;
        const uint32_t f = e ? (uint32_t)__builtin_ctz(e) : (uint32_t)WS;  // first empty slot: the run's end
        hits[k] = m & from & ((1u << f) - 1u);
        if (e) {
          const uint32_t r = r0[k] + f - off;  // occupied slots walked = the reference's rounds
          lane_rounds = r > lane_rounds ? r : lane_rounds;
          done |= 1u << k;
        } else {
          r0[k] += (uint32_t)WS - off;
          cur[k] = (st[k] + (uint32_t)WS) & p.mask;
        }
      }
      if (sub) hits[k] = 0;  // the pair's first lane emits
      n += (uint32_t)__builtin_popcount(hits[k]);
    }
    // Wave prefix of the step's matches, bit-sliced over ballots (n <= R * WS).
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int b = 0; (1 << b) <= R * WS; ++b) {
      const uint64_t bm = __ballot((n >> b) & 1u);
      pre += lane_prefix(bm) << b;
      tot += (uint32_t)__popcll(bm) << b;
    }
    if (tot) {
      uint32_t wb = 0;
      if (lane == 0) wb = atomicAdd(&s_cnt, tot);
      wb = (uint32_t)__builtin_amdgcn_readfirstlane((int)wb);
      if (n && !(CCJ_ABLATED(p.ablate, 1u))) {
        uint32_t o = wb + pre;
#pragma unroll
        for (int k = 0; k < R; ++k) {
          for (uint32_t hm = hits[k]; hm; hm &= hm - 1u, ++o) {
            if (o < kFlatStage) {
              s_sel[o] = (uint16_t)row[k];  // payload = s_key[row]: the matched table value == probe key
              if (POS) s_pos[o] = st[k] + (uint32_t)__builtin_ctz(hm);
            } else if (o < p.cap) {
              p.out_sel[obase + o] = row[k];
              if (p.out_payload) p.out_payload[obase + o] = key[k];
              if (POS) p.out_pos[obase + o] = st[k] + (uint32_t)__builtin_ctz(hm);
            } else {
              overflow = 1;
            }
          }
        }
      }
    }
    // Finished cursors take the chunk's next rows: one LDS atomic per wave and step.
    const uint32_t nd = sub ? 0u : (uint32_t)__builtin_popcount(done);
    uint32_t dpre = 0, dtot = 0;
#pragma unroll
    for (int b = 0; (1 << b) <= R; ++b) {
      const uint64_t bm = __ballot((nd >> b) & 1u);
      dpre += lane_prefix(bm) << b;
      dtot += (uint32_t)__popcll(bm) << b;
    }
    if (dtot) {
      uint32_t rb = 0;
      if (lane == 0) rb = atomicAdd(&s_next, dtot);
      rb = (uint32_t)__builtin_amdgcn_readfirstlane((int)rb) + dpre;
      if (LPR == 2) rb = (uint32_t)__builtin_amdgcn_mov_dpp((int)rb, 0xA0, 0xF, 0xF, false);  // quad_perm 0,0,2,2
#pragma unroll
      for (int k = 0; k < R; ++k) {
        if ((done >> k) & 1u) {
          need &= ~(1u << k);
          row[k] = rb++;
          r0[k] = 0;
          if (row[k] < phys) {
            key[k] = s_key[row[k]];
            cur[k] = (uint32_t)murmurhash64((uint64_t)key[k]) & p.mask;
            need |= 1u << k;
          }
        }
      }
    }
  }
  {
    const uint32_t wr = wave_max(lane_rounds);
    if (lane == 0) atomicMax(&s_rounds, wr);
  }
  __syncthreads();
  const uint32_t total = s_cnt;
  const uint32_t staged = total < kFlatStage ? total : kFlatStage;
  if (!(CCJ_ABLATED(p.ablate, 1u))) {
    // 16-byte stores (4 sel / 2 payload / 4 position entries per lane; round 2d) for the whole
    // groups when the chunk's region is 16-byte aligned (cap a multiple of 4), single entries else
    typedef long long i64x2 __attribute__((ext_vector_type(2)));
    const uint32_t lim = staged < p.cap ? staged : (uint32_t)p.cap;
    const uint32_t vec = p.cap % 4 == 0 ? (lim & ~3u) : 0u;  // entries written by the vector stores
    for (uint32_t g = tid; 4 * g < vec; g += kFlatThreads) {
      const u32x4 sv = {s_sel[4 * g], s_sel[4 * g + 1], s_sel[4 * g + 2], s_sel[4 * g + 3]};
      __builtin_nontemporal_store(sv, reinterpret_cast<u32x4 *>(p.out_sel + obase + 4 * g));
      if (POS) {
        const u32x4 pv = *reinterpret_cast<const u32x4 *>(&s_pos[4 * g]);
        __builtin_nontemporal_store(pv, reinterpret_cast<u32x4 *>(p.out_pos + obase + 4 * g));
      }
    }
    if (p.out_payload) {
      for (uint32_t g = tid; 2 * g < vec; g += kFlatThreads) {
        const i64x2 kv = {s_key[s_sel[2 * g]], s_key[s_sel[2 * g + 1]]};
        __builtin_nontemporal_store(kv, reinterpret_cast<i64x2 *>(p.out_payload + obase + 2 * g));
      }
    }
    for (uint32_t o = vec + tid; o < lim; o += kFlatThreads) {  // the rest, one entry per lane
      const uint32_t r = s_sel[o];
      __builtin_nontemporal_store(r, p.out_sel + obase + o);
      if (POS) __builtin_nontemporal_store(s_pos[o], p.out_pos + obase + o);
      if (p.out_payload) __builtin_nontemporal_store(s_key[r], p.out_payload + obase + o);
    }
  }
  if (tid == 0) {
    p.out_count[c] = total < p.cap ? total : (uint32_t)p.cap;
    if (p.out_rounds) p.out_rounds[c] = s_rounds;
  }
  if (p.status && (overflow || total > p.cap)) atomicOr(p.status, CCJ_FLAG_CAP_OVERFLOW);
}

template <int R>
__global__ __launch_bounds__(kFlatThreads) void probe_win(ProbeParams p) {
  __shared__ uint32_t s_cnt, s_rounds, s_next;
  __shared__ int64_t s_key[kMaxChunk];
  __shared__ uint16_t s_sel[kFlatStage];  // chunk rows fit 16 bits
  __shared__ __attribute__((aligned(16))) uint32_t s_pos[kFlatStage];  // every match's table position
  uint64_t c = blockIdx.x;
  if (p.xcd_swizzle) {
    const uint64_t n8 = (p.swz_chunks ? p.swz_chunks : p.n_chunks) & ~7ull;
    if (c < n8) c = (c & 7) * (n8 >> 3) + (c >> 3);
  }
  walk_chunk<R>(p, c, s_cnt, s_rounds, s_next, s_key, s_sel, s_pos);
}

// Chaining walk for bucket-partitioned input (probe_chain_win): one lane per row, R rows in
// flight, the chunk's rows handed out by an LDS counter as in probe_win.  Round 0 comes from the
// bucket record {start | len << 32, first key} (one 16-byte load); longer chains continue through
// aligned 2-key windows of the CSR key array.  After the bucket-range split both the records and
// the chains of a chunk's window (2^17 buckets) are L2-resident.  Rounds per row = chain length
// (chaining_ht.cpp:60-136 walks the whole chain); matches = chain entries equal to the key.
template <int R>
__global__ __launch_bounds__(kFlatThreads) void probe_chain_win(ProbeParams p) {
  __shared__ uint32_t s_cnt, s_rounds, s_next;
  __shared__ int64_t s_key[kMaxChunk];
  __shared__ uint32_t s_sel[kFlatStage];
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1);
  uint64_t c = blockIdx.x;
  if (p.xcd_swizzle) {
    const uint64_t n8 = (p.swz_chunks ? p.swz_chunks : p.n_chunks) & ~7ull;
    if (c < n8) c = (c & 7) * (n8 >> 3) + (c >> 3);
  }
  c += p.chunk0;  // (the filter walk's overflow-area pass: chunks from chunk0 on)
  const uint64_t base = c * p.chunk;
  const uint32_t phys = flat_phys(p, base);
  const uint64_t obase = c * p.cap;
  stage_keys(s_key, p.keys + base, phys, tid);
  if (tid == 0) {
    s_cnt = 0;
    s_rounds = 0;
    s_next = kFlatThreads * R;
  }
  __syncthreads();
  int64_t key[R];
  uint32_t row[R], cur[R], lim[R], kfp[R];
  uint32_t need = 0, fresh = 0, lane_rounds = 0, overflow = 0;  // fresh bit k: at the bucket record
  const bool rec8 = p.bucket8 != nullptr;
  auto start = [&](int k, uint32_t i) {
    row[k] = i;
    if (i < phys) {
      key[k] = s_key[i];
      const uint64_t h = murmurhash64((uint64_t)key[k]);
      cur[k] = (uint32_t)h & p.mask;
      kfp[k] = bucket_fp(h);
      need |= 1u << k;
      fresh |= 1u << k;
    }
  };
#pragma unroll
  for (int k = 0; k < R; ++k) {
    key[k] = 0;
    cur[k] = lim[k] = kfp[k] = 0;
    start(k, (uint32_t)k * kFlatThreads + tid);
  }
  while (__ballot(need != 0u) != 0ull) {
    longlong2 v[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {  // unconditional (an idle row reads bucket 0): no wait per load
      const bool nd = (need >> k) & 1u, fr = (fresh >> k) & 1u;
      const longlong2 *src = nd && !fr ? reinterpret_cast<const longlong2 *>(p.table + (cur[k] & ~1u))
                             : rec8    ? reinterpret_cast<const longlong2 *>(p.bucket8 + (nd ? cur[k] & ~1u : 0u))
                                       : p.bucket + (nd ? cur[k] : 0u);
      v[k] = *src;
    }
    uint32_t hits[R], n = 0, done = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      hits[k] = 0;
      if ((need >> k) & 1u) {
        if ((fresh >> k) & 1u) {
          fresh &= ~(1u << k);
          // 8-byte records come in aligned pairs: this bucket's is the half cur & 1
          const uint64_t r = rec8 ? (uint64_t)((cur[k] & 1u) ? v[k].y : v[k].x) : (uint64_t)v[k].x;
          const uint32_t st = (uint32_t)r, len = rec8 ? (uint32_t)(r >> 32) & 0xFFu : (uint32_t)(r >> 32);
          lane_rounds = len > lane_rounds ? len : lane_rounds;
          if (len == 0) {
            done |= 1u << k;  // empty bucket: not in the active set (chaining_ht.cpp:52-55)
          } else if (rec8) {
            // the first two chain keys are skipped without a read when their fingerprints differ;
            // the rest of the chain is read from the first node that can match
            cur[k] = rec8_first(r, kfp[k]);
            lim[k] = st + len;
            if (cur[k] >= lim[k]) done |= 1u << k;
          } else {
            hits[k] = v[k].y == key[k] ? 1u : 0u;  // round 0 from the record's first key
            cur[k] = st + 1;
            lim[k] = st + len;
            if (len == 1) done |= 1u << k;
          }
        } else {
          const uint32_t blk = cur[k] & ~1u;
          if (cur[k] == blk && v[k].x == key[k]) hits[k] |= 1u;      // entry blk (not yet walked)
          if (blk + 1 < lim[k] && v[k].y == key[k]) hits[k] |= 2u;  // entry blk + 1 (inside the chain)
          cur[k] = blk + 2;
          if (cur[k] >= lim[k]) done |= 1u << k;
        }
      }
      n += (uint32_t)__builtin_popcount(hits[k]);
    }
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int b = 0; (1 << b) <= 2 * R; ++b) {
      const uint64_t bm = __ballot((n >> b) & 1u);
      pre += lane_prefix(bm) << b;
      tot += (uint32_t)__popcll(bm) << b;
    }
    if (tot) {
      uint32_t wb = 0;
      if (lane == 0) wb = atomicAdd(&s_cnt, tot);
      wb = (uint32_t)__builtin_amdgcn_readfirstlane((int)wb);
      if (n && !(CCJ_ABLATED(p.ablate, 1u))) {
        uint32_t o = wb + pre;
#pragma unroll
        for (int k = 0; k < R; ++k) {
          for (uint32_t hm = hits[k]; hm; hm &= hm - 1u, ++o) {
            if (o < kFlatStage) {
              s_sel[o] = row[k];  // payload = s_key[row]: the matched chain key == probe key
            } else if (o < p.cap) {
              p.out_sel[obase + o] = row[k];
              if (p.out_payload) p.out_payload[obase + o] = key[k];
            } else {
              overflow = 1;
            }
          }
        }
      }
    }
    const uint32_t nd = (uint32_t)__builtin_popcount(done);
    uint32_t dpre = 0, dtot = 0;
#pragma unroll
    for (int b = 0; (1 << b) <= R; ++b) {
      const uint64_t bm = __ballot((nd >> b) & 1u);
      dpre += lane_prefix(bm) << b;
      dtot += (uint32_t)__popcll(bm) << b;
    }
    if (dtot) {
      uint32_t rb = 0;
      if (lane == 0) rb = atomicAdd(&s_next, dtot);
      rb = (uint32_t)__builtin_amdgcn_readfirstlane((int)rb) + dpre;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        if ((done >> k) & 1u) {
          need &= ~(1u << k);
          start(k, rb++);
        }
      }
    }
  }
  {
    const uint32_t wr = wave_max(lane_rounds);
    if (lane == 0) atomicMax(&s_rounds, wr);
  }
  __syncthreads();
  const uint32_t total = s_cnt;
  const uint32_t staged = total < kFlatStage ? total : kFlatStage;
  if (!(CCJ_ABLATED(p.ablate, 1u))) {
    for (uint32_t o = tid; o < staged && o < p.cap; o += kFlatThreads) {
      __builtin_nontemporal_store(s_sel[o], p.out_sel + obase + o);
      if (p.out_payload) __builtin_nontemporal_store(s_key[s_sel[o]], p.out_payload + obase + o);
    }
  }
  if (tid == 0) {
    p.out_count[c] = total < p.cap ? total : (uint32_t)p.cap;
    if (p.out_rounds) p.out_rounds[c] = s_rounds;
  }
  if (p.status && (overflow || total > p.cap)) atomicOr(p.status, CCJ_FLAG_CAP_OVERFLOW);
}

// probe_chain_filt: the chaining walk of the bucket-partitioned column with each partition's
// bucket filter in LDS (VERDICT r3 task 5).  At C3 90 % of the rows miss, yet
// probe_chain_win spends one L2 request per row on its bucket record (1.11 requests per row, bound
// by the CU's ~90 reads in flight).  The filter holds 2 bits per bucket (ccj_build.hip
// chain_filter): 0 = empty bucket, 1 / 2 = a one-key chain whose key has hash bit 40 = 0 / 1,
// 3 = a longer chain; 2^18 buckets of a partition are 64 KiB.  A row needs the L2 only when its
// code is 3 or equals 1 + its own hash bit 40 (C3: a miss passes with p ~ 0.09 + 0.30 / 2).
// Persistent: one 1024-thread workgroup per CU; XCD x walks partitions [x P / 8, (x + 1) P / 8) in
// order, all its workgroups on the same partition (its records and chains sit in the XCD's L2),
// each loading the partition's filter into LDS once.  Work unit = a quarter chunk (512 rows); a
// wave stages the unit's keys in registers, hashes and filters them, queues the passing rows (key,
// row) in its LDS queue, then reads their 8-byte bucket records (rec8_first skips nodes whose 12-bit
// fingerprint differs) and, where a node can still match, the 2-key windows of the chain.  Matches
// of a chunk are appended to its output region through out_count[c] (zeroed by the launcher) with
// one atomic per wave step: the order inside a chunk is free here (L1 / L2 parity), as in every
// partitioned walk.  Chunks of the overflow area (key skew) are walked by probe_chain_win.
// Both walks: 768 threads and two workgroups per CU (filter 64 KiB + 12 queues of 1.3 KiB each).
// The walk is issue-bound (r4 v3 profile: ~520 VALU instructions per 256-row unit and wave, a
// quarter of them 64-bit unit arithmetic), so v4 keeps the unit arithmetic scalar (wave index
// through readfirstlane, no 64-bit division), reads bucket records for the passing rows only
// (exec-masked), and walks chains on a packed queue: after the records, the unit's rows whose chain
// can still hold their key (~10 % at C3) move to the wave's LDS queue, one per lane, so a chain
// round is one 16-byte load and one compare per lane instead of four.
constexpr int kFiltThreads = 768, kFiltWordThreads = 768;
constexpr uint32_t kFiltUnit = 256;                  // rows per work unit (4 per lane)
constexpr uint32_t kFiltQ = 64;                      // queue entries per wave (more: extra passes)
constexpr uint32_t kFiltMaxWords = (1u << 18) / 16;  // 2 bits per bucket, windows <= 2^18 buckets
__device__ __forceinline__ uint32_t filt_code_of(uint64_t h) { return 1u + (uint32_t)((h >> 40) & 1u); }

template <bool WORDS>
struct FiltQueue {  // one wave's chain rows of a unit
  int64_t key[kFiltQ];
  uint32_t cur[kFiltQ], lim[kFiltQ];
  uint32_t st[WORDS ? kFiltQ : 1];  // the chain's first node (the round of a node)
  uint8_t row[kFiltQ];              // the row in the unit
};

// WORDS = false: matches appended to each chunk's output (the partitioned probe); WORDS = true: every
// row's Next-round word at its position (the ordered probe, chain_words' output: the filter gives an
// empty bucket's 0 rounds and a one-key chain's miss — 1 round, no match — without any read; a
// passing row whose fingerprints rule its chain out has the chain's length in rounds, no match).
// Chunk slots of the match walk (per workgroup, LDS): the workgroup takes whole chunks of the
// partition (k, k + K, ...), its waves take their units in order from an LDS counter, and a chunk's
// matches are counted in LDS — no device atomic per unit (that reply was a round trip in every
// unit's critical path) — the unit that completes a chunk writes its count.  Slot m % kFiltSlots
// serves the workgroup's m-th chunk; a wave whose unit belongs to a chunk more than kFiltSlots
// ahead of the oldest unfinished one waits for that slot (gen) — the oldest chunk never waits.
constexpr uint32_t kFiltSlots = 32;
struct FiltSlots {
  uint32_t next;                 // the workgroup's next unit
  uint32_t cnt[kFiltSlots];      // matches of the slot's chunk so far
  uint32_t done[kFiltSlots];     // its units finished
  uint32_t gen[kFiltSlots];      // the chunk ordinal allowed to use the slot
};

template <bool WORDS, int NT>
__device__ __forceinline__ void chain_filt_body(const ProbeParams &p, uint32_t *s_f, FiltQueue<WORDS> *s_q,
                                                FiltSlots *s_s) {
  constexpr uint32_t kJ = kFiltUnit / kWave;  // rows per lane and unit
  constexpr uint32_t kWaves = NT / kWave;
  static_assert(kJ % 2 == 0, "pairs of rows per lane");
  const uint32_t lane = threadIdx.x & (kWave - 1);
  // row jj of this lane inside the unit: rows 2L and 2L + 1 of each 128-row half, so the keys
  // arrive as 16-byte loads (probe_walk2's stage, round 5)
  auto urow = [&](int jj) { return (uint32_t)(jj >> 1) * 128u + 2u * lane + (uint32_t)(jj & 1); };
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  FiltQueue<WORDS> &q = s_q[wave];
  const uint32_t x = blockIdx.x & 7u, k0 = blockIdx.x >> 3, K = gridDim.x >> 3;
  const uint32_t P = p.seg_parts;
  const uint32_t chunk = p.chunk;
  const uint32_t spc = (uint32_t)(p.seg_cap / chunk);  // chunks per segment
  const uint32_t upc = chunk / kFiltUnit;              // units per chunk (chunk: a multiple of kFiltUnit)
  const uint32_t ups = spc * upc;                      // units per segment
  const uint32_t cpp = 8u * spc;                       // chunks per partition
  const bool cp2 = (chunk & (chunk - 1u)) == 0u;
  const uint32_t cl2 = (uint32_t)__builtin_ctz(chunk);
  const uint32_t wb = p.filt_wb;
  const uint32_t fwords = (1u << wb) / 16u;
  const uint32_t wmask = (1u << wb) - 1u;
  const bool rec8 = p.bucket8 != nullptr;
  const bool fm = WORDS ? p.w16 != 0u : p.first_match != 0u;  // distinct build keys
  const uint32_t stride = K * kWaves;
  auto take = [&]() {  // wave-uniform: the workgroup's next unit
    uint32_t j = 0;
    if (lane == 0) j = atomicAdd(&s_s->next, 1u);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)j);
  };
  for (uint32_t d = x * P / 8; d < (x + 1) * P / 8; ++d) {
    // The workgroup's place among the XCD's K workgroups rotates with the partition.  With a fixed
    // place, workgroup k took chunks k, k + K, ... of EVERY partition — the first cpp mod K
    // workgroups one chunk more each time — so the others ran ahead by a chunk per partition and the
    // XCD's workgroups spread over several partitions at once: their records and chains (3 MiB
    // each) then shared the XCD's 4 MiB L2 (round 4 profile: 37 % of record / chain reads missed).
    const uint32_t k = (k0 + d) % K;
    // match walk: the workgroup's units, in order — j = m * upc + kk is unit kk of its m-th chunk
    const uint32_t n_mine = k < cpp ? (cpp - k + K - 1) / K : 0u;  // the workgroup's chunks per partition
    const uint32_t nu = n_mine * upc;
    __syncthreads();  // the previous partition's filter and chunk slots are no longer used
    for (uint32_t w = threadIdx.x * 4; w < fwords; w += NT * 4)
      *reinterpret_cast<u32x4 *>(&s_f[w]) = *reinterpret_cast<const u32x4 *>(p.filt + (uint64_t)d * fwords + w);
    if (!WORDS) {
      if (threadIdx.x == 0) s_s->next = 0;
      if (threadIdx.x < kFiltSlots) {
        s_s->cnt[threadIdx.x] = 0;
        s_s->done[threadIdx.x] = 0;
        s_s->gen[threadIdx.x] = threadIdx.x;
      }
    }
    __syncthreads();
    // a unit (wave-uniform, scalar): chunk c, rows [u0, uend) of it (uend <= u0: nothing live), and
    // (match walk) the workgroup's chunk ordinal m.  Segment d * 8 + g holds seg_count[seg_cursor_index(P, g, d)] rows.
    auto unit_at = [&](uint32_t g, uint32_t ci, uint32_t kk, uint64_t &c, uint32_t &u0, uint32_t &uend) {
      c = (uint64_t)(d * 8u + g) * spc + ci;
      u0 = kk * kFiltUnit;
      const uint64_t fill = p.seg_count[g < 8u ? seg_cursor_index(P, g, d) : 0u];
      uint64_t live = g < 8u ? fill : 0u;
      live = live < p.seg_cap ? live : p.seg_cap;
      const uint64_t off = (uint64_t)ci * chunk;
      const uint32_t phys = live > off ? (live - off < chunk ? (uint32_t)(live - off) : chunk) : 0u;
      uend = phys <= u0 ? u0 : (phys - u0 < kFiltUnit ? phys : u0 + kFiltUnit);
    };
    // WORDS: the static order — a wave's units are u = g * ups + r = k + K * wave + stride * i,
    // (g, r) advanced without division
    auto advance = [&](uint32_t &g, uint32_t &r, uint32_t by) {
      r += by;
      while (g < 8u && r >= ups) {
        r -= ups;
        ++g;
      }
    };
    auto unit_static = [&](uint32_t g, uint32_t r, uint64_t &c, uint32_t &u0, uint32_t &uend) {
      const uint32_t pos = r * kFiltUnit;
      const uint32_t ci = cp2 ? pos >> cl2 : pos / chunk;
      unit_at(g, ci, r - ci * upc, c, u0, uend);
    };
    // match walk: unit j of the workgroup (valid: j < nu)
    auto unit_dyn = [&](uint32_t j, uint64_t &c, uint32_t &u0, uint32_t &uend, uint32_t &m) {
      const uint32_t jj = j < nu ? j : 0u;
      m = jj / upc;
      const uint32_t pc = k + K * m, g = pc / spc;
      unit_at(j < nu ? g : 8u, pc - g * spc, jj - m * upc, c, u0, uend);
    };
    auto load_keys = [&](uint64_t c, uint32_t u0, uint32_t uend, int64_t(&kk)[kJ]) {
      // (timing only, tuning build: 0x10000 = keys from chunk c & 63, L2-resident lines)
      const uint64_t kc = CCJ_ABLATED(p.ablate, 0x10000u) ? (c & 63u) : c;
      typedef long long i64x2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int j = 0; j < (int)kJ; j += 2) {
        // even; row i + 1 is inside the unit's 256 positions; chunk is a multiple of kFiltUnit, so
        // the pair is 16-byte aligned (chain_filt_applies)
        const uint32_t i = u0 + urow(j);
        const i64x2 v = __builtin_nontemporal_load(reinterpret_cast<const i64x2 *>(p.keys + kc * chunk + (i < uend ? i : u0)));
        kk[j] = v.x;
        kk[j + 1] = v.y;
      }
    };
    uint32_t g = 0, r = 0, j = 0, m = 0;
    uint64_t c = 0;
    uint32_t u0 = 0, uend = 0;
    bool more;
    if (WORDS) {
      advance(g, r, k + K * wave);
      unit_static(g, r, c, u0, uend);
      more = g < 8u;
    } else {
      j = take();
      unit_dyn(j, c, u0, uend, m);
      more = j < nu;
    }
    int64_t kk[kJ], kn[kJ];
    if (more) load_keys(c, u0, uend, kk);
    while (more) {
      // filter, then the passing rows' bucket records
      uint32_t pass = 0, kfp[kJ], bk[kJ];
#pragma unroll
      for (int jj = 0; jj < (int)kJ; ++jj) {
        const uint32_t i = u0 + urow(jj);
        const uint64_t h = murmurhash64((uint64_t)kk[jj]);
        const uint32_t bl = (uint32_t)h & wmask;
        const uint32_t code = (s_f[bl >> 4] >> ((bl & 15u) * 2u)) & 3u;
        const bool ps = (i < uend) & ((code == 3u) | (code == filt_code_of(h)));  // (no branches)
        pass |= (ps ? 1u : 0u) << jj;
        bk[jj] = (uint32_t)h & p.mask;
        // (timing only, tuning build: records and chains from the lower half / quarter of the
        // partition's buckets — a smaller L2 working set, wrong results)
        if (CCJ_ABLATED(p.ablate, 0x4000u)) bk[jj] &= ~(1u << (wb - 1u));
        if (CCJ_ABLATED(p.ablate, 0x8000u)) bk[jj] &= ~(3u << (wb - 2u));
        kfp[jj] = ps ? bucket_fp(h) : code;  // (a rejected row keeps its code: 0 empty, else a one-key chain)
      }
      uint64_t rec[kJ];
#pragma unroll
      for (int jj = 0; jj < (int)kJ; ++jj) {
        rec[jj] = 0;
        if ((pass >> jj) & 1u) rec[jj] = rec8 ? p.bucket8[bk[jj]] : (uint64_t)p.bucket[bk[jj]].x;
      }
      // the next unit's keys, in flight during this unit's record and chain round trips
      uint32_t gn = g, rn = r, jn = 0, mn = 0;
      uint64_t cn = 0;
      uint32_t u0n = 0, uendn = 0;
      bool moren;
      if (WORDS) {
        advance(gn, rn, stride);
        unit_static(gn, rn, cn, u0n, uendn);
        moren = gn < 8u;
      } else {
        jn = take();
        unit_dyn(jn, cn, u0n, uendn, mn);
        moren = jn < nu;
      }
      load_keys(moren ? cn : c, moren ? u0n : u0, moren ? uendn : uend, kn);
      // slot jj's chain range from its record: nodes [cur, lim) can still hold the key
      auto range = [&](int jj, uint32_t &st, uint32_t &cur, uint32_t &lim) {
        const bool ps = (pass >> jj) & 1u;
        st = (uint32_t)rec[jj];
        const uint32_t len = rec8 ? (uint32_t)(rec[jj] >> 32) & 0xFFu : (uint32_t)(rec[jj] >> 32);
        lim = ps ? st + len : 0u;
        cur = ps ? (rec8 ? rec8_first(rec[jj], kfp[jj]) : st) : 0u;
        // (timing only, tuning build: three rows in four read their record but walk no chain — the
        // hits of the 0x8000 ablation with the full record working set; wrong results)
        if (CCJ_ABLATED(p.ablate, 0x40000u) && (urow(jj) & 3u)) lim = cur;
      };
      // queue index of every chain row (slot-major); WORDS: the other rows' words now, coalesced
      uint64_t qm[kJ];  // wave-uniform: slot jj's chain rows, and the queue index of its first
      uint32_t qs[kJ], qn = 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the previous unit's queue reads are done
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int jj = 0; jj < (int)kJ; ++jj) {
        uint32_t st, cur, lim;
        range(jj, st, cur, lim);
        const bool act = cur < lim;
        const uint64_t bm = __ballot(act);
        const uint32_t qi = qn + lane_prefix(bm);
        qm[jj] = bm;
        qs[jj] = qn;
        qn += (uint32_t)__popcll(bm);
        if (act && qi < kFiltQ) {
          q.key[qi] = kk[jj];
          q.cur[qi] = cur;
          q.lim[qi] = lim;
          if (WORDS) q.st[WORDS ? qi : 0] = st;
          q.row[qi] = (uint8_t)urow(jj);
        }
        if (WORDS) {
          const uint32_t i = u0 + urow(jj);
          if (!act && i < uend) {
            const uint32_t len = lim - st;
            const uint32_t word = (pass >> jj) & 1u ? (len <= kMmRounds ? len << kMmRounds : kMmLong | len)
                                                    : (kfp[jj] == 0u ? 0u : 1u << kMmRounds);
            if (p.w16) __builtin_nontemporal_store(round_word16(word), (uint16_t *)p.out_w + c * chunk + i);
            else __builtin_nontemporal_store(word, p.out_w + c * chunk + i);
          }
        }
      }
      // match walk: this unit's chunk slot (a chunk kFiltSlots ahead of an unfinished one waits)
      const uint32_t slot = m % kFiltSlots;
      if (!WORDS && m >= kFiltSlots) {
        while ((uint32_t)__builtin_amdgcn_readfirstlane((int)__hip_atomic_load(&s_s->gen[slot], __ATOMIC_RELAXED,
                                                                              __HIP_MEMORY_SCOPE_WORKGROUP)) != m)
          __builtin_amdgcn_s_sleep(2);
      }
      for (uint32_t qb = 0; qb < qn; qb += kFiltQ) {
        if (qb) {  // a unit with more than kFiltQ chain rows: the next kFiltQ of them
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int jj = 0; jj < (int)kJ; ++jj) {
            const uint32_t qi = qs[jj] + lane_prefix(qm[jj]), e = qi - qb;
            if (((qm[jj] >> lane) & 1u) && qi >= qb && e < kFiltQ) {
              uint32_t st, cur, lim;
              range(jj, st, cur, lim);
              q.key[e] = kk[jj];
              q.cur[e] = cur;
              q.lim[e] = lim;
              if (WORDS) q.st[WORDS ? e : 0] = st;
              q.row[e] = (uint8_t)urow(jj);
            }
          }
        }
        // the queue written by other lanes of this wave is read below
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t ne = qn - qb < kFiltQ ? qn - qb : kFiltQ;
        const bool live = lane < ne;
        const int64_t key = q.key[lane];
        const uint32_t lim = live ? q.lim[lane] : 0u;
        const uint32_t st = WORDS ? q.st[WORDS ? lane : 0] : 0u;
        const uint32_t row = q.row[lane];
        uint32_t cur = live ? q.cur[lane] : 0u;
        uint32_t nh = 0, mm = 0;
        while (__ballot(cur < lim) != 0ull) {  // one 2-key window per chain row and round
          const longlong2 v = *reinterpret_cast<const longlong2 *>(p.table + (cur < lim ? cur & ~1u : 0u));
          if (cur < lim) {
            const uint32_t blk = cur & ~1u;
            const uint32_t r0 = blk - st;  // node blk's round (chaining_ht.cpp:88-99: one node per Next)
            if (cur == blk && v.x == key) {
              ++nh;
              if (WORDS && r0 < 32u) mm |= 1u << r0;
            }
            if (blk + 1u < lim && v.y == key) {
              ++nh;
              if (WORDS && r0 + 1u < 32u) mm |= 1u << (r0 + 1u);
            }
            // distinct build keys: a row's only match ends its walk (its word's rounds are the
            // chain's length from the record, and no later node can match)
            cur = fm && nh ? lim : blk + 2u;
          }
        }
        if (WORDS) {
          if (live) {
            const uint32_t len = lim - st;
            const uint32_t word =
                len <= kMmRounds ? (mm & ((1u << kMmRounds) - 1u)) | len << kMmRounds : kMmLong | len;
            const uint64_t at = c * chunk + u0 + row;
            if (p.w16) __builtin_nontemporal_store(round_word16(word), (uint16_t *)p.out_w + at);
            else __builtin_nontemporal_store(word, p.out_w + at);
          }
        } else {  // append the matches: their places from the chunk's LDS count (one LDS atomic per pass)
          const uint32_t incl = wave_incl_scan(nh);
          const uint32_t tot = (uint32_t)__shfl((int)incl, kWave - 1);
          if (tot) {
            uint32_t ob = 0;
            if (lane == 0) ob = atomicAdd(&s_s->cnt[slot], tot);
            ob = (uint32_t)__shfl((int)ob, 0) + incl - nh;
            bool over = false;
            const uint64_t obase = c * p.cap;
            for (uint32_t e = 0; e < nh; ++e, ++ob) {
              if (ob < p.cap) {  // (non-temporal: the partition's records and chains keep the L2)
                __builtin_nontemporal_store(u0 + row, p.out_sel + obase + ob);
                if (p.out_payload) __builtin_nontemporal_store(key, p.out_payload + obase + ob);
              } else {
                over = true;
              }
            }
            if (over && p.status) atomicOr(p.status, CCJ_FLAG_CAP_OVERFLOW);
          }
        }
      }
      if (!WORDS && lane == 0) {  // the unit is done; the chunk's last unit writes its count and frees the slot
        // (this wave's LDS adds to cnt completed before this one: LDS operations of a wave are in order)
        if (atomicAdd(&s_s->done[slot], 1u) == upc - 1u) {
          const uint32_t total = atomicAdd(&s_s->cnt[slot], 0u);
          p.out_count[c] = total < p.cap ? total : (uint32_t)p.cap;
          if (total > p.cap && p.status) atomicOr(p.status, CCJ_FLAG_CAP_OVERFLOW);
          s_s->cnt[slot] = 0;
          s_s->done[slot] = 0;
          __hip_atomic_store(&s_s->gen[slot], m + kFiltSlots, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
#pragma unroll
      for (int jj = 0; jj < (int)kJ; ++jj) kk[jj] = kn[jj];
      g = gn;
      r = rn;
      j = jn;
      m = mn;
      c = cn;
      u0 = u0n;
      uend = uendn;
      more = moren;
    }
  }
}

__global__ __launch_bounds__(kFiltThreads, 6) void probe_chain_filt(ProbeParams p) {
  __shared__ uint32_t s_f[kFiltMaxWords];  // the partition's filter (64 KiB)
  __shared__ FiltQueue<false> s_q[kFiltThreads / kWave];
  __shared__ FiltSlots s_s;
  chain_filt_body<false, kFiltThreads>(p, s_f, s_q, &s_s);
}
__global__ __launch_bounds__(kFiltWordThreads, 6) void chain_words_filt(ProbeParams p) {
  __shared__ uint32_t s_f[kFiltMaxWords];
  __shared__ FiltQueue<true> s_q[kFiltWordThreads / kWave];
  chain_filt_body<true, kFiltWordThreads>(p, s_f, s_q, nullptr);
}

// The filter walks apply to the fixed-capacity split's segments of >= 8 partitions of <= 2^18
// buckets (one XCD's range each), chunks a multiple of the work unit, no rounds asked for (partitioned
// probe); the overflow area's chunks (key skew) go to the per-chunk walks.
__device__ __host__ __forceinline__ bool chain_filt_applies(const ProbeParams &p, uint32_t unit) {
  const uint32_t P = p.seg_parts;
  return p.filt && p.seg_count && p.ovf_base && p.filt_wb <= 18 && p.filt_wb >= 4 && P >= 8 && P % 8 == 0 &&
         p.chunk % unit == 0 && p.seg_cap % p.chunk == 0;
}

// Ordered probe of a chaining table (ccj_probe_ordered), step 2: probe_chain_win's walk of the
// bucket-partitioned column, leaving each row's Next-round word at its position instead of emitting
// matches.  The reference walks a row's whole chain, one node per Next round
// (chaining_ht.cpp:60-80, :109-124), so the row's rounds are its chain length L and bit r of mm says
// chain node r equals the key (chaining_ht.cpp:88-99); an empty bucket's row has no rounds (:52-55).
// Word: mm | L << 26, or kMmLong | L for chains longer than 26 (the emit re-walks that chunk round
// by round); 16-bit words (p.w16) for distinct build keys.  The words are staged in LDS and
// written out coalesced.
template <int R>
__global__ __launch_bounds__(kFlatThreads) void chain_words(ProbeParams p) {
  __shared__ int64_t s_key[kMaxChunk];
  __shared__ uint32_t s_w[kMaxChunk];
  __shared__ uint32_t s_next;
  const uint32_t tid = threadIdx.x;
  uint64_t c = blockIdx.x;
  if (p.xcd_swizzle) {
    const uint64_t n8 = (p.swz_chunks ? p.swz_chunks : p.n_chunks) & ~7ull;
    if (c < n8) c = (c & 7) * (n8 >> 3) + (c >> 3);
  }
  c += p.chunk0;  // (the filter walk's overflow-area pass: chunks from chunk0 on)
  const uint64_t base = c * p.chunk;
  const uint32_t phys = flat_phys(p, base);
  stage_keys(s_key, p.keys + base, phys, tid);
  if (tid == 0) s_next = kFlatThreads * R;
  __syncthreads();
  int64_t key[R];
  uint32_t row[R], cur[R], lim[R], st0[R], kfp[R], mm[R];
  uint32_t need = 0, fresh = 0;
  const bool rec8 = p.bucket8 != nullptr;
  auto start = [&](int k, uint32_t i) {
    row[k] = i;
    mm[k] = 0;
    if (i < phys) {
      key[k] = s_key[i];
      const uint64_t h = murmurhash64((uint64_t)key[k]);
      cur[k] = (uint32_t)h & p.mask;
      kfp[k] = bucket_fp(h);
      need |= 1u << k;
      fresh |= 1u << k;
    }
  };
  auto word = [&](int k) {
    const uint32_t L = lim[k] - st0[k];
    s_w[row[k]] = L <= kMmRounds ? (mm[k] & ((1u << kMmRounds) - 1u)) | L << kMmRounds : kMmLong | L;
  };
#pragma unroll
  for (int k = 0; k < R; ++k) {
    key[k] = 0;
    cur[k] = lim[k] = st0[k] = kfp[k] = 0;
    start(k, (uint32_t)k * kFlatThreads + tid);
  }
  while (__ballot(need != 0u) != 0ull) {
    longlong2 v[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {  // unconditional (an idle row reads bucket 0): no wait per load
      const bool nd = (need >> k) & 1u, fr = (fresh >> k) & 1u;
      const longlong2 *src = nd && !fr ? reinterpret_cast<const longlong2 *>(p.table + (cur[k] & ~1u))
                             : rec8    ? reinterpret_cast<const longlong2 *>(p.bucket8 + (nd ? cur[k] & ~1u : 0u))
                                       : p.bucket + (nd ? cur[k] : 0u);
      v[k] = *src;
    }
    uint32_t done = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if ((need >> k) & 1u) {
        if ((fresh >> k) & 1u) {
          fresh &= ~(1u << k);
          const uint64_t r = rec8 ? (uint64_t)((cur[k] & 1u) ? v[k].y : v[k].x) : (uint64_t)v[k].x;
          const uint32_t st = (uint32_t)r, len = rec8 ? (uint32_t)(r >> 32) & 0xFFu : (uint32_t)(r >> 32);
          st0[k] = st;
          lim[k] = st + len;
          if (len == 0) {
            done |= 1u << k;  // empty bucket: no rounds
          } else if (rec8) {  // nodes 0 / 1 whose fingerprints differ: their rounds without a read
            cur[k] = rec8_first(r, kfp[k]);
            if (cur[k] >= lim[k]) done |= 1u << k;
          } else {
            mm[k] |= v[k].y == key[k] ? 1u : 0u;  // round 0 from the record's first key
            cur[k] = st + 1;
            if (len == 1) done |= 1u << k;
          }
        } else {
          const uint32_t blk = cur[k] & ~1u;
          const uint32_t r0 = blk - st0[k];  // chain node blk's round (node blk + 1: r0 + 1)
          if (cur[k] == blk && v[k].x == key[k] && r0 < 32u) mm[k] |= 1u << r0;
          if (blk + 1 < lim[k] && v[k].y == key[k] && r0 + 1 < 32u) mm[k] |= 1u << (r0 + 1);
          cur[k] = blk + 2;
          if (cur[k] >= lim[k]) done |= 1u << k;
        }
      }
    }
    const uint32_t nd = (uint32_t)__builtin_popcount(done);
    uint32_t dpre = 0, dtot = 0;
#pragma unroll
    for (int b = 0; (1 << b) <= R; ++b) {
      const uint64_t bm = __ballot((nd >> b) & 1u);
      dpre += lane_prefix(bm) << b;
      dtot += (uint32_t)__popcll(bm) << b;
    }
    if (dtot) {
      uint32_t rb = 0;
      if ((tid & (kWave - 1)) == 0) rb = atomicAdd(&s_next, dtot);
      rb = (uint32_t)__builtin_amdgcn_readfirstlane((int)rb) + dpre;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        if ((done >> k) & 1u) {
          need &= ~(1u << k);
          word(k);
          start(k, rb++);
        }
      }
    }
  }
  __syncthreads();
  for (uint32_t i = tid; i < phys; i += kFlatThreads) {  // the rows' words, coalesced at their positions
    if (p.w16) __builtin_nontemporal_store(round_word16(s_w[i]), (uint16_t *)p.out_w + base + i);
    else __builtin_nontemporal_store(s_w[i], p.out_w + base + i);
  }
}

// probe_walk: the LP walk of slot-partitioned input, one wave per 512-row quarter of a chunk,
// no per-step output bookkeeping.  Each wave stages its own rows' keys (and, with
// HOME, their home slots) in LDS; its lanes walk rows through 32-byte windows from the row's next
// unread slot (a window never crosses a 128-byte line: one L2 request); a finished row only
// leaves its match count in LDS and takes the wave's next row (a wave-uniform cursor, ballot
// prefix, no LDS atomic).  After the walk the wave reserves its output range with one LDS atomic
// and writes its rows' matches in row order, coalesced (payload = the probe key, sel = the row's
// position).  A lane pair walks a row, 16 B each (one DPP swap joins the halves), R rows per pair
// in flight.

template <bool HOME>
struct WalkShared {
  int64_t key[kMaxChunk];
  // HOME: the row's home slot, then its match count; else only the count (16 bits: a row's
  // matches are at most max_dup; 20 KB of LDS in all, 8 workgroups per CU)
  std::conditional_t<HOME, uint32_t, uint16_t> hc[kMaxChunk];
  uint32_t total, rounds;
};

__device__ __forceinline__ void wave_lds_sync() {
  // Rows move between lanes of one wave only: its LDS writes must land before other lanes read.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A pair of consecutive keys (rows i, i + 1, i even) for the walks' staging: one 16-byte load when
// the pair is 16-byte aligned (an even chunk: every chunk base of the partitioned workspace is),
// else two 8-byte loads (odd chunks; a16 is wave-uniform, so this is a scalar branch).  Row i + 1
// may lie past the chunk's live rows (the caller discards it): an aligned pair never leaves the
// 16-byte granule of row i, so it stays inside the key array's allocation.
typedef long long key_pair_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ key_pair_t load_key_pair(const int64_t *q, bool a16) {
  if (a16) return __builtin_nontemporal_load(reinterpret_cast<const key_pair_t *>(q));
  return key_pair_t{__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 1)};
}

template <uint32_t kWaveRows, bool HOME, typename SM>
__device__ __forceinline__ void walk_stage(const ProbeParams &p, SM &sm, uint64_t base, uint32_t w0,
                                           uint32_t wend, uint32_t lane) {
  // all loads in flight before the first LDS write; lane L loads rows 2L, 2L + 1 of each 128-row
  // block as one 16-byte load (half the load instructions; probe_walk2's stage, round 5)
  typedef long long i64x2 __attribute__((ext_vector_type(2)));
  constexpr int kH = (int)(kWaveRows / (2 * kWave));
  static_assert(kWaveRows % (2 * kWave) == 0, "pairs of rows per lane");
  i64x2 v[kH];
  const bool a16 = ((uintptr_t)(p.keys + base) & 15u) == 0u;
#pragma unroll
  for (int j = 0; j < kH; ++j) {
    const uint32_t i = w0 + (uint32_t)j * 2u * kWave + 2u * lane;
    v[j] = i < wend ? load_key_pair(p.keys + base + i, a16) : i64x2{0, 0};
    if (i + 1 >= wend) v[j].y = 0;
  }
#pragma unroll
  for (int j = 0; j < kH; ++j) {
    const uint32_t i = w0 + (uint32_t)j * 2u * kWave + 2u * lane;
    *reinterpret_cast<i64x2 *>(&sm.key[i]) = v[j];
    if (HOME) {
      typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
      const u32x2 hh = {(uint32_t)murmurhash64((uint64_t)v[j].x) & p.mask, (uint32_t)murmurhash64((uint64_t)v[j].y) & p.mask};
      *reinterpret_cast<u32x2 *>(&sm.hc[i]) = hh;
    }
  }
  wave_lds_sync();
}

// Emit the wave's rows [w0, wend): counts in sm.hc; returns 1 on output overflow.
template <uint32_t kWaveRows, typename SM>
__device__ __forceinline__ uint32_t walk_emit(const ProbeParams &p, SM &sm, uint64_t c, uint32_t w0,
                                              uint32_t wend, uint32_t lane) {
  wave_lds_sync();
  uint32_t lsum = 0;
#pragma unroll
  for (int j = 0; j < (int)(kWaveRows / kWave); ++j) {
    const uint32_t i = w0 + (uint32_t)j * kWave + lane;
    lsum += i < wend ? sm.hc[i] : 0u;
  }
  uint32_t wsum = lsum;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) wsum += (uint32_t)__shfl_xor((int)wsum, d);
  uint32_t ob = 0;
  if (lane == 0 && wsum) ob = atomicAdd(&sm.total, wsum);
  ob = (uint32_t)__builtin_amdgcn_readfirstlane((int)ob);
  const uint64_t obase = c * p.cap;
  uint32_t overflow = 0;
#pragma unroll 2
  for (int j = 0; j < (int)(kWaveRows / kWave); ++j) {
    const uint32_t i = w0 + (uint32_t)j * kWave + lane;
    const uint32_t n = i < wend ? sm.hc[i] : 0u;
    uint32_t pre, tot;
    if (!__ballot(n > 1u)) {  // every row 0 or 1 match: one ballot
      const uint64_t bm = __ballot(n != 0u);
      pre = lane_prefix(bm);
      tot = (uint32_t)__popcll(bm);
    } else {
      uint32_t incl = wave_incl_scan(n);
      pre = incl - n;
      tot = (uint32_t)__shfl((int)incl, kWave - 1);
    }
    if (n && !CCJ_ABLATED(p.ablate, 1u)) {
      const int64_t k = sm.key[i];
      for (uint32_t t = 0; t < n; ++t) {
        const uint64_t o = (uint64_t)ob + pre + t;
        if (o < p.cap) {
          __builtin_nontemporal_store(i, p.out_sel + obase + o);
          if (p.out_payload) __builtin_nontemporal_store(k, p.out_payload + obase + o);
        } else {
          overflow = 1;
        }
      }
    }
    ob += tot;
  }
  return overflow;
}

__device__ __forceinline__ uint64_t walk_chunk_index(const ProbeParams &p) {
  uint64_t c = blockIdx.x;
  if (p.xcd_swizzle) {
    const uint64_t n8 = (p.swz_chunks ? p.swz_chunks : p.n_chunks) & ~7ull;
    if (c < n8) c = (c & 7) * (n8 >> 3) + (c >> 3);
  }
  return c + p.chunk0;
}

template <typename SM>
__device__ __forceinline__ void walk_finish(const ProbeParams &p, SM &sm, uint64_t c, uint32_t lane,
                                            uint32_t lane_rounds, uint32_t overflow, unsigned long long t0,
                                            unsigned long long t1, unsigned long long t2, uint32_t steps) {
  if (p.out_rounds) {
    const uint32_t wr = wave_max(lane_rounds);
    if (lane == 0) atomicMax(&sm.rounds, wr);
  }
  unsigned long long t3;
  CCJ_STAMP(t3);
  if (p.stats && lane == 0) {
    atomicAdd(&p.stats[0], t1 - t0);
    atomicAdd(&p.stats[1], t2 - t1);
    atomicAdd(&p.stats[2], t3 - t2);
    atomicAdd(&p.stats[3], (unsigned long long)steps);
    atomicAdd(&p.stats[4], 1ull);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t total = sm.total;
    p.out_count[c] = total < p.cap ? total : (uint32_t)p.cap;
    if (p.out_rounds) p.out_rounds[c] = sm.rounds;
  }
  if (p.status && overflow) atomicOr(p.status, CCJ_FLAG_CAP_OVERFLOW);
}

// Workgroup emit (p.emit_pol != kEmitWave; needs HOME's u32 counts): when no row of the chunk has
// more than one match and the chunk fits its output, the chunk's matches are compacted in LDS in
// row order (keys in place in sm.key, row positions in sm.hc; every entry moves down, so one
// barrier between reading and writing suffices) and written from c * cap with 16-byte buffer
// stores of cache policy p.emit_pol: 4 sel or 2 payload entries per lane instead of one.
// Returns false (nothing written) when the per-wave emit must run instead.
// The compacted chunk (sel in sm.hc, payload in sm.key, tot entries) as 16-byte stores.  A last
// partial group writes past the count inside the chunk's own cap region (cap is a multiple of 4),
// which holds no data of the chunk's consumers.
template <int AUX, uint32_t kThreads, typename SM>
__device__ __forceinline__ void emit_wg_stores(const ProbeParams &p, SM &sm, uint64_t obase, uint32_t tot,
                                               bool pay) {
  const uint32_t tid = threadIdx.x;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(p.out_sel + obase, (short)0, (int)(p.cap * 4), 0x00020000);
  for (uint32_t q = tid; q * 4 < tot; q += kThreads) {
    const u32x4 v = *reinterpret_cast<const u32x4 *>(&sm.hc[4 * q]);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(16 * q), 0, AUX);
  }
  if (pay) {
    const auto rp = __builtin_amdgcn_make_buffer_rsrc(p.out_payload + obase, (short)0, (int)(p.cap * 8), 0x00020000);
    for (uint32_t q = tid; q * 2 < tot; q += kThreads) {
      const u32x4 v = *reinterpret_cast<const u32x4 *>(&sm.key[2 * q]);
      __builtin_amdgcn_raw_buffer_store_b128(v, rp, (int)(16 * q), 0, AUX);
    }
  }
}
template <uint32_t kWaveRows, int NW, typename SM>
__device__ __forceinline__ bool walk_emit_wg(const ProbeParams &p, SM &sm, uint64_t c, uint32_t w0,
                                             uint32_t wend, uint32_t lane, uint32_t wave, uint32_t *s_wtot,
                                             uint32_t phys) {
  constexpr int kJ = (int)(kWaveRows / kWave);
  uint32_t lsum = 0, multi = 0;
  uint32_t n[kJ];
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const uint32_t i = w0 + (uint32_t)j * kWave + lane;
    n[j] = i < wend ? sm.hc[i] : 0u;
    lsum += n[j];
    multi |= n[j] > 1u ? 1u : 0u;
  }
  const uint32_t wtot = (uint32_t)__shfl((int)wave_incl_scan(lsum), kWave - 1);
  const uint32_t wmulti = wave_or(multi);
  if (lane == 0) s_wtot[wave] = wtot | (wmulti ? 0x80000000u : 0u);
  __syncthreads();
  uint32_t base = 0, tot = 0, any_multi = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const uint32_t x = s_wtot[w];
    any_multi |= x >> 31;
    base += (uint32_t)w < wave ? (x & 0x7FFFFFFFu) : 0u;
    tot += x & 0x7FFFFFFFu;
  }
  if (any_multi || tot > p.cap) return false;
  const uint64_t obase = c * p.cap;
  // rows_in_sel (keys_in_out too): the split wrote every position's original row into out_sel
  // and its key into out_payload, so a chunk whose rows all matched once is complete as it is
  if (p.rows_in_sel && tot == phys) {
    if (threadIdx.x == 0) sm.total = tot;
    return true;
  }
  int64_t k[kJ];
  uint32_t t[kJ], rid[kJ];
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const uint32_t i = w0 + (uint32_t)j * kWave + lane;
    const uint64_t bm = __ballot(n[j] != 0u);
    t[j] = base + lane_prefix(bm);
    base += (uint32_t)__popcll(bm);
    k[j] = sm.key[i & (kMaxChunk - 1)];
    rid[j] = i;
    if (p.rows_in_sel && n[j]) rid[j] = p.out_sel[obase + i];  // the row the split stored there
  }
  __syncthreads();  // every key (and row) read before any entry moves down
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    if (n[j]) {
      sm.key[t[j]] = k[j];
      sm.hc[t[j]] = rid[j];
    }
  }
  __syncthreads();
  // keys_in_out and every row matched once: the payload column already holds the chunk's output
  // (the split wrote each key at its position); only sel is written
  const bool pay = p.out_payload && !(p.keys_in_out && tot == phys);
  switch (p.emit_pol) {  // the buffer stores' cache bits are an immediate
    case 2: emit_wg_stores<2, kWave * NW>(p, sm, obase, tot, pay); break;
    case 16: emit_wg_stores<16, kWave * NW>(p, sm, obase, tot, pay); break;
    case 18: emit_wg_stores<18, kWave * NW>(p, sm, obase, tot, pay); break;
    default: emit_wg_stores<0, kWave * NW>(p, sm, obase, tot, pay); break;
  }
  if (threadIdx.x == 0) sm.total = tot;
  return true;
}

// MM (the ordered probe, ccj_probe_ordered): instead of counts, each row leaves its Next-round
// word W = mm | L << 26 (bit r of mm: the row matches in round r; L: occupied slots walked = its
// rounds, the reference's Next calls for it; L > 26: bit 31 | L, the chunk re-walks round by
// round), written to p.out_w at the row's position; no emit.
// LN: lanes per row (2: 32-byte windows, 4: 64-byte windows; 16 bytes per lane either way).
template <int R, bool HOME, int NW = 4, bool MM = false, int LN = 2, bool DMA = false>
__global__ __launch_bounds__(kWave * NW) void probe_walk(ProbeParams p) {
  constexpr uint32_t kWaveRows = kMaxChunk / NW;  // rows per wave
  __shared__ WalkShared<HOME> sm;
  // DMA: the table windows land in LDS by LDS-DMA (global_load_lds_dwordx4, a per-lane source
  // address), one 1 KiB slot per (wave, row k): 16 bytes per lane at lane * 16
  __shared__ __attribute__((aligned(16))) int64_t s_win[DMA ? NW * R * 2 * kWave : 2];
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  constexpr uint32_t kWin = 2 * LN;  // slots per window
  constexpr uint32_t kRowsPer = kWave / LN;  // rows per wave instruction
  const uint32_t sub = lane & (LN - 1);
  unsigned long long t0, t1, t2;
  uint32_t steps = 0;
  CCJ_STAMP(t0);
  const uint64_t c = walk_chunk_index(p);
  const uint64_t base = c * p.chunk;
  const uint32_t phys = flat_phys(p, base);
  const uint32_t w0 = wave * kWaveRows;
  const uint32_t wend = phys > w0 ? (phys - w0 < kWaveRows ? phys : w0 + kWaveRows) : w0;  // wave's rows [w0, wend)
  if (tid == 0) {
    sm.total = 0;
    sm.rounds = 0;
  }
  walk_stage<kWaveRows, HOME>(p, sm, base, w0, wend, lane);
  CCJ_STAMP(t1);
  const uint32_t last_start = p.mask - (kWin - 1);  // table size - window (size >= 16)
  const uint32_t pair = lane / LN;
  int64_t key[R];
  uint32_t row[R], cur[R], cnt[R], r0[R];
  uint32_t need = 0, lane_rounds = 0;
  auto start = [&](int k, uint32_t i) {
    row[k] = i;
    cnt[k] = 0;
    r0[k] = 0;
    if (i < wend) {
      key[k] = sm.key[i];
      cur[k] = HOME ? sm.hc[i] : (uint32_t)murmurhash64((uint64_t)key[k]) & p.mask;
      need |= 1u << k;
    }
  };
#pragma unroll
  for (int k = 0; k < R; ++k) {
    key[k] = 0;
    cur[k] = 0;
    start(k, w0 + (uint32_t)k * kRowsPer + pair);
  }
  uint32_t next = w0 + (uint32_t)R * kRowsPer;  // wave-uniform: the wave's next unwalked row
  while (__ballot(need != 0u) != 0ull) {
    ++steps;
    int64_t v0[R], v1[R];
    uint32_t st[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      uint32_t s = cur[k] < last_start ? cur[k] : last_start;
      const uint32_t lim = (s & ~15u) + (16u - kWin);  // the window ends at its 128-byte line
      s = s < lim ? s : lim;
      st[k] = s;
      // Unconditional loads: a load under `if (need)` made the compiler wait for each row's load
      // before issuing the next (vmcnt(0) after every one: R dependent L2 round trips per step).
      // An idle row reads slot 0's line instead (one request per instruction at most), and its
      // values are never used.  Same box, C2 step: 12.28 / 12.58 ms against 12.79 / 12.58
      // predicated — the walk is bound by requests in flight per CU, not by one wave's chain.
      const uint32_t a = ((need >> k) & 1u) ? s + 2 * sub : 0u;
      if constexpr (DMA) {
        __builtin_amdgcn_global_load_lds(static_cast<const void *>(p.table + a),
                                         (__attribute__((address_space(3))) void *)&s_win[(wave * R + k) * 2 * kWave],
                                         16, 0, 0);
      } else if (CCJ_ABLATED(p.ablate, 2u)) {  // timing only: no table reads
        v0[k] = sub ? -1 : key[k];
        v1[k] = -1;
      } else {
        const longlong2 x = *reinterpret_cast<const longlong2 *>(p.table + a);
        v0[k] = x.x;
        v1[k] = x.y;
      }
    }
    if constexpr (DMA) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every window of the step has landed
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const longlong2 x = *reinterpret_cast<const longlong2 *>(&s_win[(wave * R + k) * 2 * kWave + 2 * lane]);
        v0[k] = x.x;
        v1[k] = x.y;
      }
    }
    uint32_t done = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      uint32_t e = ((v0[k] == -1) ? 1u : 0u) | ((v1[k] == -1) ? 2u : 0u);
      uint32_t m = ((v0[k] == key[k]) ? 1u : 0u) | ((v1[k] == key[k]) ? 2u : 0u);
      uint32_t em = (e | m << kWin) << (2 * sub);
      em |= (uint32_t)__builtin_amdgcn_mov_dpp((int)em, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
      if (LN == 4) em |= (uint32_t)__builtin_amdgcn_mov_dpp((int)em, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
      if ((need >> k) & 1u) {
        const uint32_t off = cur[k] - st[k];
        const uint32_t ee = (em & ((1u << kWin) - 1u)) >> off;
        const uint32_t f = (uint32_t)__builtin_ctz(ee | ((1u << kWin) >> off));  // run end (or window end) past cur
        const uint32_t hits = ((em >> kWin) >> off) & ((1u << f) - 1u);
        if (MM) cnt[k] |= r0[k] < kMmRounds ? hits << r0[k] : 0u;  // rounds >= 26 end as long rows
        else cnt[k] += (uint32_t)__builtin_popcount(hits);
        if (ee) {
          const uint32_t r = r0[k] + f;  // occupied slots walked = the reference's rounds
          lane_rounds = r > lane_rounds ? r : lane_rounds;
          if (MM) cnt[k] = r <= kMmRounds ? (cnt[k] & ((1u << kMmRounds) - 1u)) | r << kMmRounds : kMmLong | r;
          done |= 1u << k;
        } else {
          r0[k] += kWin - off;
          cur[k] = (st[k] + kWin) & p.mask;
        }
      }
    }
    // Finished rows leave their count and take the wave's next rows (pairs in lane order).
    const uint32_t nd = (uint32_t)__builtin_popcount(done);
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int b = 0; (1 << b) <= R; ++b) {
      const uint64_t bm = __ballot(((nd >> b) & 1u) && !sub);
      pre += lane_prefix(bm) << b;
      tot += (uint32_t)__popcll(bm) << b;
    }
    if (tot) {
      pre = (uint32_t)__builtin_amdgcn_mov_dpp((int)pre, LN == 4 ? 0x00 : 0xA0, 0xF, 0xF, false);  // the row's first lane's
      uint32_t rb = next + pre;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        if ((done >> k) & 1u) {
          need &= ~(1u << k);
          if (!sub) sm.hc[row[k]] = (std::remove_reference_t<decltype(sm.hc[0])>)cnt[k];
          start(k, rb++);
        }
      }
      next += tot;
    }
  }
  CCJ_STAMP(t2);
  if (MM) {  // the rows' round words, coalesced at their positions
    wave_lds_sync();
    if (p.w16 && kWaveRows == 8 * kWave && w0 + kWaveRows <= p.chunk && (p.chunk & 7u) == 0u) {
      // 8 words per lane in one 16-byte store (rows past wend write don't-care words inside the
      // chunk's own positions, which no run points at; a wave whose rows pass the chunk's end —
      // chunks under 2048 — stores word by word, and so does a chunk width that is not a
      // multiple of 8, whose chunks do not start 16-byte aligned)
      const uint32_t i0 = w0 + 8 * lane;
      uint32_t h[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        h[t] = (uint32_t)round_word16((uint32_t)sm.hc[i0 + 2 * t]) |
               (uint32_t)round_word16((uint32_t)sm.hc[i0 + 2 * t + 1]) << 16;
      const u32x4 v = {h[0], h[1], h[2], h[3]};
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>((uint16_t *)p.out_w + base + i0));
      return;
    }
#pragma unroll
    for (int j = 0; j < (int)(kWaveRows / kWave); ++j) {
      const uint32_t i = w0 + (uint32_t)j * kWave + lane;
      if (i < wend) {
        if (p.w16) __builtin_nontemporal_store(round_word16((uint32_t)sm.hc[i]), (uint16_t *)p.out_w + base + i);
        else __builtin_nontemporal_store((uint32_t)sm.hc[i], p.out_w + base + i);
      }
    }
    return;
  }
  if constexpr (HOME) {
    if (p.emit_pol != kEmitWave || p.rows_in_sel) {  // (rows_in_sel: only the workgroup emit maps rows)
      __shared__ uint32_t s_wtot[NW];
      wave_lds_sync();
      if (walk_emit_wg<kWaveRows, NW>(p, sm, c, w0, wend, lane, wave, s_wtot, phys)) {
        walk_finish(p, sm, c, lane, lane_rounds, 0u, t0, t1, t2, steps);
        return;
      }
    }
  }
  const uint32_t overflow = walk_emit<kWaveRows>(p, sm, c, w0, wend, lane);
  walk_finish(p, sm, c, lane, lane_rounds, overflow, t0, t1, t2, steps);
}

// probe_walk1<NB, MM>: probe_walk's walk with ONE lane per row and the table windows brought in by
// LDS-DMA (global_load_lds_dwordx4, per-lane source address).  Round 3 measurements (tools/reqpath):
// random 32-byte windows from an L2-resident window reach ~490 G/s chip-wide by LDS-DMA against
// ~255 G/s as vector loads; probe_walk's lane pairs (3.4 VALU wave-instructions per row) and its
// wait for every window of a step (vmcnt(0)) left it at 7.7 ms either way.  Here each wave keeps NB
// batches of 64 rows in flight in a ring of LDS slots: per batch, two DMA instructions (lane 2p + h
// loads half h of batch entry 2p + k's window, k = the instruction) put entry e's 32-byte window at
// slot + (e & 1) * 1024 + (e >> 1) * 32; the
// wave waits for the OLDEST batch only (vmcnt(2 * (NB - 1))), checks it one row per lane, and
// refills it — rows whose run continues keep their lane, finished rows are replaced from the wave's
// cursor — so the memory pipeline stays full while a batch is checked.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// One LDS-DMA wave-instruction: lane L's 16 bytes at `g` land at LDS byte lds + 16 * L.  Issued as
// inline asm so that the compiler, which cannot tell which ring slot a DMA writes, does not wait for
// every DMA in flight (vmcnt(0)) before each LDS read of the ring: the caller waits itself
// (wait_vmcnt), and no compiler-tracked vector-memory operation may be in flight across these.
// M0 is saved and restored: the compiler treats M0 as reserved and does not honour a clobber of it.
__device__ __forceinline__ void dma16(const void *g, uint32_t lds) {
  uint32_t saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(saved)
               : "v"(g), "s"(lds)
               : "memory");
}
constexpr uint32_t kRingSlot = 2 * 1024;  // one batch: 64 windows of 32 B, two DMA halves
// The walks move each row's window start to the two lanes that DMA its halves with DPP quad-perms
// (a0: lanes 2q and 2q + 1 get lane 2q's address, a1: lane 2q + 1's), and clamp the result into the
// table so that a DMA can never leave it.  The clamp alone would turn a DPP that read a switched-off
// lane (round 3: a structurised loop did) into silently wrong windows, so the tuning build checks
// every move against the partner lanes' addresses fetched by ds_bpermute and raises
// CCJ_FLAG_INTERNAL in args->status on a mismatch (tests/test_probe_gpu.py runs the walks there).
__device__ __forceinline__ void dpp_check(const ProbeParams &p, uint32_t a, uint32_t a0, uint32_t a1, uint32_t lane) {
#ifdef CCJ_TUNING
  const uint32_t e0 = (uint32_t)__shfl((int)a, (int)(lane & ~1u));
  const uint32_t e1 = (uint32_t)__shfl((int)a, (int)(lane | 1u));
  if ((a0 != e0 || a1 != e1) && p.status) atomicOr(p.status, CCJ_FLAG_INTERNAL);
#else
  (void)p, (void)a, (void)a0, (void)a1, (void)lane;
#endif
}
// Window prefetch (p.pf_dist): chunk c (its XCD's order, partitioned layout) touches the table lines
// of slice (c + pf_dist) mod K of partition (c + pf_dist) / K, K = chunks per partition, so that
// the next window is in L2 before its first chunk starts.  One LDS-DMA of wave 0 into `lds` (1 KiB
// of the chunk's home-slot array, written by the stage only after its loads — and with them this
// older DMA — have landed).
__device__ __forceinline__ void walk_prefetch(const ProbeParams &p, uint64_t c, uint32_t lane, uint32_t lds) {
  const uint64_t cl = c - p.chunk0;
  if (cl >= p.swz_chunks || p.seg_parts == 0) return;
  const uint64_t K = 8 * (p.seg_cap / p.chunk);
  const uint64_t t = cl + p.pf_dist;
  const uint64_t d2 = t / K;
  if (d2 >= p.seg_parts) return;
  const uint64_t wl = ((uint64_t)p.mask + 1) / p.seg_parts / 16;  // 128-byte lines per window
  const uint64_t first = d2 * wl + (t % K) * wl / K;
  const uint64_t last = ((uint64_t)p.mask + 1) / 16 - 1;
  uint64_t line = first + (lane < p.pf_lines ? lane : 0u);
  line = line < last ? line : last;
  const uint32_t m0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds);
  dma16(p.table + line * 16, m0);
}
// probe_walk1's LDS: the chunk's keys and home slots / counts, and the wave's DMA ring, which the
// emit's scratch (total, rounds, per-wave sums) overlaps once every wave's walk is over: 32 KiB at
// NB = 1 (5 workgroups per CU), 40 KiB at NB = 2 (4 per CU)
template <int NB, int NW>
struct Walk1Shared {
  int64_t key[kMaxChunk];
  uint32_t hc[kMaxChunk];
  union {
    __attribute__((aligned(16))) char ring[NW * NB * kRingSlot];
    struct {
      uint32_t total, rounds, wtot[NW];
    };
  };
};
// probe_walk1<POS>'s emit (CCJ_PART_ROWS with positions, distinct keys, cap == chunk): the split
// already wrote every position's original row (out_sel) and key (out_payload), and sm.hc holds
// matched | slot per row.  A chunk whose rows all matched writes only its positions, in place; a
// chunk with a miss (none at C5) writes its slots at their compacted output places directly and
// compacts rows (sm.hc) and keys (sm.key) in LDS, written with 16-byte stores.
template <uint32_t kWaveRows, int NW, typename SM>
__device__ __forceinline__ void walk_emit_pos(const ProbeParams &p, SM &sm, uint64_t c,
                                              uint32_t w0, uint32_t wend, uint32_t lane, uint32_t wave,
                                              uint32_t *s_wtot, uint32_t phys) {
  constexpr int kJ = (int)(kWaveRows / kWave);
  uint32_t lsum = 0;
  uint32_t h[kJ];
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const uint32_t i = w0 + (uint32_t)j * kWave + lane;
    h[j] = i < wend ? sm.hc[i] : 0u;
    lsum += h[j] >> 31;
  }
  const uint32_t wtot = (uint32_t)__shfl((int)wave_incl_scan(lsum), kWave - 1);
  if (lane == 0) s_wtot[wave] = wtot;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    base += (uint32_t)w < wave ? s_wtot[w] : 0u;
    tot += s_wtot[w];
  }
  const uint64_t obase = c * p.cap;
  if (tot == phys) {  // every row matched once: positions at the rows' own output slots
    if (kJ == 8 && wend == w0 + kWaveRows && (p.cap & 3u) == 0u) {
      const uint32_t i0 = w0 + 8 * lane;  // 8 consecutive rows per lane: two 16-byte stores
      const u32x4 m = {0x7FFFFFFFu, 0x7FFFFFFFu, 0x7FFFFFFFu, 0x7FFFFFFFu};
      const u32x4 v0 = *reinterpret_cast<const u32x4 *>(&sm.hc[i0]) & m;
      const u32x4 v1 = *reinterpret_cast<const u32x4 *>(&sm.hc[i0 + 4]) & m;
      __builtin_nontemporal_store(v0, reinterpret_cast<u32x4 *>(p.out_pos + obase + i0));
      __builtin_nontemporal_store(v1, reinterpret_cast<u32x4 *>(p.out_pos + obase + i0 + 4));
    } else {
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        const uint32_t i = w0 + (uint32_t)j * kWave + lane;
        if (i < wend) __builtin_nontemporal_store(h[j] & 0x7FFFFFFFu, p.out_pos + obase + i);
      }
    }
    if (threadIdx.x == 0) sm.total = tot;
    return;
  }
  int64_t k[kJ];
  uint32_t t[kJ], rid[kJ];
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const uint32_t i = w0 + (uint32_t)j * kWave + lane;
    const bool hit = (h[j] >> 31) != 0u;
    const uint64_t bm = __ballot(hit);
    t[j] = base + lane_prefix(bm);
    base += (uint32_t)__popcll(bm);
    k[j] = sm.key[i & (kMaxChunk - 1)];
    rid[j] = hit ? p.out_sel[obase + i] : 0u;  // the row the split stored there
    if (hit) __builtin_nontemporal_store(h[j] & 0x7FFFFFFFu, p.out_pos + obase + t[j]);
  }
  __syncthreads();  // every key and row read before any entry moves down
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    if (h[j] >> 31) {
      sm.key[t[j]] = k[j];
      sm.hc[t[j]] = rid[j];
    }
  }
  __syncthreads();
  emit_wg_stores<2, kWave * NW>(p, sm, obase, tot, true);
  if (threadIdx.x == 0) sm.total = tot;
}
// walk_emit_pos with p.out_sub (C5, round 6): every chunk's matches written in order of their slot's
// sub-range b = (slot >> sub_shift) & 7 (then row order), so the payload gather can take one 4 MiB
// slab of payload rows per XCD at a time (launch_gather_payload).  The output order inside a chunk
// is free on the partitioned path (L1 / L2), so this is a permutation of what walk_emit_pos writes:
// the rows the split stored at the chunk's output slots, the keys staged in LDS and the slots are
// placed in LDS in (sub-range, wave, row group, lane) order — ranks from 8 ballots per row group, a
// per-wave running count per sub-range, the waves' counts through LDS — and written with 16-byte
// stores (sel, payload, pos: 16 B per match instead of the 4 B of positions alone); out_sub[c * 8 + b]
// = where sub-range b starts.  LDS: the idle DMA ring holds the per-wave counts, then the slots.
// The rows the split stored at a chunk's output slots, in walk_emit_pos_sub's mapping (row
// w0 + 64 j + lane): loaded while the walk runs, so the emit does not wait on them.
template <int kJ>
__device__ __forceinline__ void load_emit_rows(const ProbeParams &p, uint64_t c, uint32_t w0, uint32_t wend,
                                               uint32_t lane, uint32_t (&rid)[kJ]) {
  const uint32_t *sel_c = p.out_sel + c * p.cap;  // (a uniform base: 32-bit lane offsets)
#pragma unroll
  for (int j = 0; j < kJ; ++j) {  // (a dead row reads slot 0; streamed: non-temporal, as the keys)
    const uint32_t i = w0 + (uint32_t)j * kWave + lane;
    rid[j] = __builtin_nontemporal_load(sel_c + (i < wend ? i : 0u));
  }
}
template <uint32_t kWaveRows, int NW, typename SM>
__device__ __forceinline__ void walk_emit_pos_sub(const ProbeParams &p, SM &sm, uint64_t c, uint32_t w0,
                                                  uint32_t wend, uint32_t lane, uint32_t wave,
                                                  const uint32_t (&rid)[kWaveRows / kWave]) {
  constexpr int kJ = (int)(kWaveRows / kWave);
  constexpr uint32_t kSubs = 8;
  static_assert(sizeof(sm.ring) >= kMaxChunk * 4, "the ring holds the chunk's slots");
  const uint64_t obase = c * p.cap;
  const uint64_t lt = (1ull << lane) - 1ull;
  // LDS beside the slots' first half: per wave and sub-range a running count, then the offsets and
  // the chunk's total
  uint32_t *s_cnt = reinterpret_cast<uint32_t *>(sm.ring + kMaxChunk * 2);  // [NW][8]
  uint32_t *s_off = s_cnt + NW * kSubs;                                     // [NW][8], then the total
  if (lane < kSubs) s_cnt[wave * kSubs + lane] = 0;
  uint32_t h[kJ], rk[kJ];  // rk: sub-range | rank inside the wave's sub-range << 3
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const uint32_t i = w0 + (uint32_t)j * kWave + lane;
    h[j] = i < wend ? sm.hc[i] : 0u;
    const bool hit = (h[j] >> 31) != 0u;
    const uint32_t b = ((h[j] & 0x7FFFFFFFu) >> p.sub_shift) & (kSubs - 1u);
    // the lanes of this row group with the same sub-range (3 ballots on its bits) and their order
    uint64_t peers = __ballot(hit);
#pragma unroll
    for (uint32_t bit = 0; bit < 3; ++bit) {
      const uint64_t on = __ballot((b >> bit) & 1u);
      peers &= ((b >> bit) & 1u) ? on : ~on;
    }
    const uint32_t before = (uint32_t)__popcll(peers & lt);
    const uint32_t cur = hit ? s_cnt[wave * kSubs + b] : 0u;  // every lane reads before the group's first writes
    rk[j] = b | (cur + before) << 3;
    __builtin_amdgcn_wave_barrier();
    if (hit && before == 0) s_cnt[wave * kSubs + b] = cur + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  if (threadIdx.x < kWave) {  // wave 0: offset of (wave w, sub-range b) — sub-range major, wave minor —
    // as an exclusive scan over lanes x = b * NW + w (x < 32) of the counts
    const uint32_t x = lane, b = x / NW, w = x % NW;
    const uint32_t v = x < NW * kSubs ? s_cnt[w * kSubs + b] : 0u;
    const uint32_t incl = wave_incl_scan(v);
    if (x < NW * kSubs) {
      s_off[w * kSubs + b] = incl - v;
      if (w == 0) p.out_sub[c * kSubs + b] = incl - v;  // where sub-range b starts in the chunk
    }
    if (x == NW * kSubs - 1) s_off[NW * kSubs] = incl;  // the chunk's matches
  }
  __syncthreads();
  const uint32_t tot = s_off[NW * kSubs];
  // two placements, so that fewer values are live at once (the walk's registers set its occupancy):
  // rows (sm.hc, whose reads all happened before the barrier above) and slots (the ring, once its
  // counts are read), then the keys (in place in sm.key)
#pragma unroll
  for (int j = 0; j < kJ; ++j) {  // each match's place, with the hit in bit 31
    rk[j] = (s_off[wave * kSubs + (rk[j] & 7u)] + (rk[j] >> 3)) | (h[j] & 0x80000000u);
    if (rk[j] >> 31) sm.hc[rk[j] & 0x7FFFFFFFu] = rid[j];
  }
  __syncthreads();  // the counts and offsets (in the ring) are read: the ring takes the slots
  uint32_t *s_pos = reinterpret_cast<uint32_t *>(sm.ring);
#pragma unroll
  for (int j = 0; j < kJ; ++j)
    if (rk[j] >> 31) s_pos[rk[j] & 0x7FFFFFFFu] = h[j] & 0x7FFFFFFFu;
  __syncthreads();
  emit_wg_stores<2, kWave * NW>(p, sm, obase, tot, false);  // sel
  const auto rq = __builtin_amdgcn_make_buffer_rsrc(p.out_pos + obase, (short)0, (int)(p.cap * 4), 0x00020000);
  for (uint32_t q = threadIdx.x; q * 4 < tot; q += kWave * NW) {
    const u32x4 v = *reinterpret_cast<const u32x4 *>(&s_pos[4 * q]);
    __builtin_amdgcn_raw_buffer_store_b128(v, rq, (int)(16 * q), 0, 2);
  }
  int64_t k[kJ];
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const uint32_t i = w0 + (uint32_t)j * kWave + lane;
    k[j] = sm.key[i & (kMaxChunk - 1)];
  }
  __syncthreads();  // every key is read before any moves
#pragma unroll
  for (int j = 0; j < kJ; ++j)
    if (rk[j] >> 31) sm.key[rk[j] & 0x7FFFFFFFu] = k[j];
  __syncthreads();
  {  // payload (the keys), 16-byte stores
    const auto rp = __builtin_amdgcn_make_buffer_rsrc(p.out_payload + obase, (short)0, (int)(p.cap * 8), 0x00020000);
    for (uint32_t q = threadIdx.x; q * 2 < tot; q += kWave * NW) {
      const u32x4 v = *reinterpret_cast<const u32x4 *>(&sm.key[2 * q]);
      __builtin_amdgcn_raw_buffer_store_b128(v, rp, (int)(16 * q), 0, 2);
    }
  }
  __syncthreads();  // the ring's slots are stored: its first words take the emit's total again
  if (threadIdx.x == 0) sm.total = tot;
}
// The ordered walks' output (MM): every row's round word at its position, coalesced (16-bit words,
// 8 per lane as one 16-byte store, for full 512-row waves of chunks that are multiples of 8).
template <uint32_t kWaveRows, typename SM>
__device__ __forceinline__ void walk_words_out(const ProbeParams &p, SM &sm, uint64_t base, uint32_t w0,
                                               uint32_t wend, uint32_t lane) {
  if (p.w16 && kWaveRows == 8 * kWave && w0 + kWaveRows <= p.chunk && (p.chunk & 7u) == 0u) {
    const uint32_t i0 = w0 + 8 * lane;
    uint32_t h[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      h[t] = (uint32_t)round_word16(sm.hc[i0 + 2 * t]) | (uint32_t)round_word16(sm.hc[i0 + 2 * t + 1]) << 16;
    const u32x4 v = {h[0], h[1], h[2], h[3]};
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>((uint16_t *)p.out_w + base + i0));
    return;
  }
#pragma unroll
  for (int j = 0; j < (int)(kWaveRows / kWave); ++j) {
    const uint32_t i = w0 + (uint32_t)j * kWave + lane;
    if (i < wend) {
      if (p.w16) __builtin_nontemporal_store(round_word16(sm.hc[i]), (uint16_t *)p.out_w + base + i);
      else __builtin_nontemporal_store(sm.hc[i], p.out_w + base + i);
    }
  }
}
// A row's round word (MM): the rounds it matched in (bits < kMmRounds) and its run's length r, or
// kMmLong | r for runs longer than kMmRounds
__device__ __forceinline__ uint32_t mm_word(uint32_t mask, uint32_t r) {
  return r <= kMmRounds ? (mask & ((1u << kMmRounds) - 1u)) | r << kMmRounds : kMmLong | r;
}

template <int NB, bool MM = false, bool POS = false, int NW = 4>
__global__ __launch_bounds__(kWave * NW) void probe_walk1(ProbeParams p) {
  constexpr uint32_t kWaveRows = kMaxChunk / NW;  // rows per wave
  __shared__ Walk1Shared<NB, NW> sm;
  char *const s_ring = sm.ring;
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  unsigned long long t0, t1, t2;
  uint32_t steps = 0;
  CCJ_STAMP(t0);
  const uint64_t c = walk_chunk_index(p);
  const uint64_t base = c * p.chunk;
  const uint32_t phys = flat_phys(p, base);
  const uint32_t w0 = wave * kWaveRows;
  const uint32_t wend = phys > w0 ? (phys - w0 < kWaveRows ? phys : w0 + kWaveRows) : w0;  // wave's rows [w0, wend)
  if (p.pf_dist && wave == 0) walk_prefetch(p, c, lane, (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)sm.hc);
  if (CCJ_ABLATED(p.ablate, 0x400u)) {  // (tuning: touch the keys of the chunk kp_dist later on this XCD)
    const uint64_t c2 = c + p.kp_dist;
    const uint64_t per = p.n_chunks / 8;
    if (per && c2 < p.n_chunks && c2 / per == c / per) {
      const uint32_t m0 = (uint32_t)__builtin_amdgcn_readfirstlane(
          (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)&sm.hc[w0]);
      dma16(p.keys + c2 * p.chunk + w0 + (lane & 31u) * 16u, m0);
    }
  }
  // (timing only, tuning build: 0x100 stages the keys of chunk c & 63 — L2-resident key lines)
  walk_stage<kWaveRows, true>(p, sm, CCJ_ABLATED(p.ablate, 0x100u) ? (c & 63u) * p.chunk : base, w0, wend, lane);
  CCJ_STAMP(t1);
  char *ring = s_ring + wave * NB * kRingSlot;
  // the ring's LDS byte address, wave-uniform (M0 of the DMAs)
  const uint32_t ring_lds = (uint32_t)__builtin_amdgcn_readfirstlane(
      (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)ring);
  const uint32_t last_start = p.mask - (kWin - 1);  // table size - window (size >= 16)
  const uint32_t half = (lane & 1u) * 2u;            // slots of the half this lane's DMA loads
  // this lane's row in ring slot b: key, row, next unread slot, window start, rounds walked, matches
  int64_t key[NB];
  uint32_t row[NB], cur[NB], st[NB], r0[NB], cnt[NB];
  uint32_t mpos[NB];  // POS: the row's matched slot (distinct keys: at most one)
  uint32_t live = 0, lane_rounds = 0;
  uint32_t next = w0;  // wave-uniform: the wave's next unwalked row
  auto take = [&](int b, bool want) {  // lanes with `want` take the wave's next rows, in lane order
    const uint64_t bm = __ballot(want);
    const uint32_t i = next + lane_prefix(bm);
    next += (uint32_t)__popcll(bm);
    if (want) {
      row[b] = i;
      r0[b] = 0;
      cnt[b] = 0;
      if (POS) mpos[b] = 0;
      if (i < wend) {
        key[b] = sm.key[i];
        cur[b] = sm.hc[i];
        live |= 1u << b;
      }
    }
  };
  auto issue = [&](int b) {
    uint32_t a = 0;  // an idle entry loads slot 0's line (every DMA is issued: fixed vmcnt depth)
    if ((live >> b) & 1u) {
      uint32_t s = cur[b] < last_start ? cur[b] : last_start;
      const uint32_t lim = (s & ~15u) + (16u - kWin);  // the window ends at its 128-byte line
      s = s < lim ? s : lim;
      st[b] = s;
      a = s;
    }
    if (CCJ_ABLATED(p.ablate, 0x200u)) a &= 0x1FFFu;  // (timing only: windows from the first 64 KiB)
    uint32_t a0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)a, 0xA0, 0xF, 0xF, false);  // quad_perm 0,0,2,2
    uint32_t a1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)a, 0xF5, 0xF, 0xF, false);  // quad_perm 1,1,3,3
    dpp_check(p, a, a0, a1, lane);
    a0 = a0 < last_start ? a0 : last_start;  // (a guard, as in probe_walk2: the DMA stays in the table)
    a1 = a1 < last_start ? a1 : last_start;
    const uint32_t slot = ring_lds + (uint32_t)b * kRingSlot;
    dma16(p.table + a0 + half, slot);
    dma16(p.table + a1 + half, slot + 1024u);
  };
  auto check = [&](int b) {
    const char *w = ring + b * kRingSlot + (lane & 1u) * 1024 + (lane >> 1) * 32;
    const longlong2 x0 = *reinterpret_cast<const longlong2 *>(w);
    const longlong2 x1 = *reinterpret_cast<const longlong2 *>(w + 16);
    if ((live >> b) & 1u) {
      const int64_t k = key[b];
      const uint32_t e = (x0.x == -1 ? 1u : 0u) | (x0.y == -1 ? 2u : 0u) | (x1.x == -1 ? 4u : 0u) | (x1.y == -1 ? 8u : 0u);
      const uint32_t m = (x0.x == k ? 1u : 0u) | (x0.y == k ? 2u : 0u) | (x1.x == k ? 4u : 0u) | (x1.y == k ? 8u : 0u);
      const uint32_t off = cur[b] - st[b];
      const uint32_t ee = e >> off;
      const uint32_t f = (uint32_t)__builtin_ctz(ee | ((1u << kWin) >> off));  // run end (or window end) past cur
      const uint32_t hits = (m >> off) & ((1u << f) - 1u);
      if (MM) cnt[b] |= r0[b] < kMmRounds ? hits << r0[b] : 0u;  // rounds >= 26 end as long rows
      else cnt[b] += (uint32_t)__builtin_popcount(hits);
      if (POS && hits) mpos[b] = cur[b] + (uint32_t)__builtin_ctz(hits);
      // p.first_match (distinct build keys, no rounds asked for): a row's only possible match
      // ends its walk — the rest of its run cannot hold its key again
      if (ee || (!MM && p.first_match && hits)) {
        const uint32_t r = r0[b] + f;  // occupied slots walked = the reference's rounds (run end)
        lane_rounds = r > lane_rounds ? r : lane_rounds;
        if (MM) cnt[b] = mm_word(cnt[b], r);
        if (CCJ_ABLATED(p.ablate, 0x200u)) cnt[b] = 1;  // (timing only: the emit path of the real data)
        // POS (tables of <= 2^31 slots): bit 31 = matched, the low bits its slot
        sm.hc[row[b]] = POS ? (cnt[b] ? mpos[b] | 0x80000000u : 0u) : cnt[b];
        live &= ~(1u << b);
      } else {
        r0[b] += kWin - off;
        cur[b] = (st[b] + kWin) & p.mask;
      }
    }
  };
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    key[b] = 0;
    row[b] = cur[b] = st[b] = r0[b] = cnt[b] = mpos[b] = 0;
    take(b, true);
    issue(b);
  }
  for (bool more = true; more;) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      ++steps;
      wait_vmcnt<2 * (NB - 1)>();  // batch b (the oldest) has landed
      check(b);
      take(b, ((live >> b) & 1u) == 0u);
      if (__ballot(live != 0u) == 0ull) {  // every slot empty and no rows left
        more = false;
        break;
      }
      issue(b);
    }
  }
  wait_vmcnt<0>();
  CCJ_STAMP(t2);
  __syncthreads();  // every wave's ring is idle: the emit's scratch may overlap it
  if (tid == 0) {
    sm.total = 0;
    sm.rounds = 0;
  }
  __syncthreads();
  if (MM) {  // the rows' round words, coalesced at their positions (probe_walk's MM tail)
    walk_words_out<kWaveRows>(p, sm, base, w0, wend, lane);
    return;
  }
  if (POS) {  // CCJ_PART_ROWS with match positions (C5): sel and payload are the split's
    if (p.out_sub) {
      uint32_t rid[kWaveRows / kWave];
      load_emit_rows(p, c, w0, wend, lane, rid);
      walk_emit_pos_sub<kWaveRows, NW>(p, sm, c, w0, wend, lane, wave, rid);
    } else {
      walk_emit_pos<kWaveRows, NW>(p, sm, c, w0, wend, lane, wave, sm.wtot, phys);
    }
    walk_finish(p, sm, c, lane, lane_rounds, 0u, t0, t1, t2, steps);
    return;
  }
  if (p.emit_pol != kEmitWave || p.rows_in_sel) {  // (rows_in_sel: only the workgroup emit maps rows)
    if (walk_emit_wg<kWaveRows, NW>(p, sm, c, w0, wend, lane, wave, sm.wtot, phys)) {
      walk_finish(p, sm, c, lane, lane_rounds, 0u, t0, t1, t2, steps);
      return;
    }
  }
  const uint32_t overflow = walk_emit<kWaveRows>(p, sm, c, w0, wend, lane);
  walk_finish(p, sm, c, lane, lane_rounds, overflow, t0, t1, t2, steps);
}

// probe_walk2<POS>: probe_walk1 for tables of distinct keys with no rounds asked for
// (p.first_match), where a row's walk ends at its match and 98.7 % of C2's rows end in their first
// 32-byte window.  Phase A gives every row its first window with a fixed assignment — lane L of
// wave w walks row w0 + 64 j + L in step j — so the row's key and home slot stay in the registers
// the stage loaded and hashed them into: no refill ballot, no LDS reads of the row before its
// DMA, about half of probe_walk1's instructions per batch.  A row whose run continues past that
// window (no match yet, no empty slot) leaves its next slot in sm.hc and a bit in its lane's mask;
// phase B walks those rows lane by lane (a lane takes its next continuing row as soon as one
// finishes).  Same outputs as probe_walk1 (counts 0 / 1, or matched | slot for POS) in sm.hc,
// then the same emits.
// The stage's key loads as buffer loads of cache policy AUX (tuning build: CCJ_KEY_AUX A/B of how
// the streamed key lines share the L2 with the table window).
#ifdef CCJ_TUNING
template <int AUX, int KJ>
__device__ __forceinline__ void stage_keys_aux(const int64_t *keys, uint32_t phys, uint32_t w0, uint32_t wend,
                                               uint32_t lane, int64_t (&k)[KJ]) {
  // the descriptor spans the chunk's live rows only: a load past them returns 0 (no access)
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int64_t *>(keys), (short)0, (int)(phys * 8), 0x00020000);
#pragma unroll
  for (int j = 0; j < KJ; ++j) {  // probe_walk2's row mapping: lane L holds rows 2L, 2L + 1 of each 128-row block
    const uint32_t i = w0 + (uint32_t)(j >> 1) * 128u + 2u * lane + (uint32_t)(j & 1);
    k[j] = (int64_t)__builtin_amdgcn_raw_buffer_load_b64(rs, (int)(i * 8), 0, AUX);
  }
#pragma unroll
  for (int j = 0; j < KJ; ++j)
    if (w0 + (uint32_t)(j >> 1) * 128u + 2u * lane + (uint32_t)(j & 1) >= wend) k[j] = 0;
}
#endif
// (Round 5: an MM form for the ordered route — every row walking its whole run, phase A's
// continuing rows keeping their first window's hits — measured slower than probe_walk1<MM>: 7.75
// against 7.49 ms, same box; the ~16 % of rows that go on are walked lane by lane in phase B.)
template <bool POS, int NB = 1>
__global__ __launch_bounds__(kWave * 4, POS && NB == 1 ? 5 : 1) void probe_walk2(ProbeParams p) {
  constexpr int NW = 4;
  constexpr uint32_t kWaveRows = kMaxChunk / NW;      // rows per wave
  constexpr int kJ = (int)(kWaveRows / kWave);         // row groups (phase-A steps) per wave
  __shared__ Walk1Shared<NB, NW> sm;
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  unsigned long long t0, t1, t2;
  uint32_t steps = 0;
  CCJ_STAMP(t0);
  const uint64_t c = walk_chunk_index(p);
  const uint64_t base = c * p.chunk;
  const uint32_t phys = flat_phys(p, base);
  const uint32_t w0 = wave * kWaveRows;
  const uint32_t wend = phys > w0 ? (phys - w0 < kWaveRows ? phys : w0 + kWaveRows) : w0;  // wave's rows [w0, wend)
  // stage: keys (all loads in flight first) and home slots stay in registers; the keys also go to
  // LDS for phase B and the emit's compaction.  Lane L holds rows 2L and 2L + 1 of each 128-row
  // block (row_of(j)), so its keys arrive as 16-byte loads: half the load instructions of one
  // key per lane and row (round 5, tools/overlap_emu.hip: the walk's pattern 6.11 -> 5.86-5.98 ms).
  auto row_of = [&](int j) { return w0 + (uint32_t)(j >> 1) * 128u + 2u * lane + (uint32_t)(j & 1); };
  int64_t k[kJ];
  uint32_t h[kJ];
#ifdef CCJ_TUNING
  if (p.key_aux == 0u) {
#endif
    typedef long long i64x2 __attribute__((ext_vector_type(2)));
    const bool a16 = ((uintptr_t)(p.keys + base) & 15u) == 0u;
#pragma unroll
    for (int j = 0; j < kJ; j += 2) {
      const uint32_t i = row_of(j);  // even: the pair (i, i + 1) lies inside the wave's 512 rows
      const i64x2 v = i < wend ? load_key_pair(p.keys + base + i, a16) : i64x2{0, 0};
      k[j] = v.x;
      k[j + 1] = i + 1 < wend ? v.y : 0;
    }
#ifdef CCJ_TUNING
  } else {  // (tuning build only: p.key_aux = 1 + the buffer loads' cache-policy bits)
    switch (p.key_aux - 1u) {
      case 1: stage_keys_aux<1>(p.keys + base, phys, w0, wend, lane, k); break;
      case 2: stage_keys_aux<2>(p.keys + base, phys, w0, wend, lane, k); break;
      case 3: stage_keys_aux<3>(p.keys + base, phys, w0, wend, lane, k); break;
      case 16: stage_keys_aux<16>(p.keys + base, phys, w0, wend, lane, k); break;
      case 17: stage_keys_aux<17>(p.keys + base, phys, w0, wend, lane, k); break;
      case 18: stage_keys_aux<18>(p.keys + base, phys, w0, wend, lane, k); break;
      case 19: stage_keys_aux<19>(p.keys + base, phys, w0, wend, lane, k); break;
      default: stage_keys_aux<0>(p.keys + base, phys, w0, wend, lane, k); break;
    }
  }
#endif
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    sm.key[row_of(j)] = k[j];
    h[j] = (uint32_t)murmurhash64((uint64_t)k[j]) & p.mask;
  }
  // slab order (C5): the rows the split stored at the outputs arrive while the chunk is walked
  uint32_t rid_e[kJ];
  if (POS && p.out_sub) load_emit_rows(p, c, w0, wend, lane, rid_e);
  CCJ_STAMP(t1);
  char *ring = sm.ring + wave * NB * kRingSlot;
  const uint32_t ring_lds = (uint32_t)__builtin_amdgcn_readfirstlane(
      (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)ring);
  const char *win = ring + (lane & 1u) * 1024 + (lane >> 1) * 32;  // this lane's window, once landed
  const uint32_t last_start = p.mask - (kWin - 1);  // table size - window (size >= 16)
  const uint32_t half = (lane & 1u) * 2u;
  // the window [s, s + kWin) that holds slot `cur` (never past the table's end or its 128-byte line)
  auto start = [&](uint32_t cur) {
    uint32_t s = cur < last_start ? cur : last_start;
    const uint32_t lim = (s & ~15u) + (16u - kWin);
    return s < lim ? s : lim;
  };
  // Every lane issues (an idle one loads slot 0's line), and with all lanes active: the DPP moves
  // read the pair's other lane, so a lane switched off here would hand its partner a stale address.
  // The callers keep these in uniform control flow (phase B's loop exits on a ballot, like
  // probe_walk1's; a `while (__ballot(...))` form was structurised into a nested loop whose lanes
  // left one by one — the DMAs then ran with lanes off and read wild addresses).
  auto issue = [&](uint32_t a, uint32_t slot) {
    uint32_t a0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)a, 0xA0, 0xF, 0xF, false);  // quad_perm 0,0,2,2
    uint32_t a1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)a, 0xF5, 0xF, 0xF, false);  // quad_perm 1,1,3,3
    dpp_check(p, a, a0, a1, lane);  // (tuning build: the DPP gave the partner lanes' own addresses)
    a0 = a0 < last_start ? a0 : last_start;  // (a guard: whatever a DPP returns, the DMA stays in the table)
    a1 = a1 < last_start ? a1 : last_start;
    dma16(p.table + a0 + half, ring_lds + slot * kRingSlot);
    dma16(p.table + a1 + half, ring_lds + slot * kRingSlot + 1024u);
  };
  // the landed window against key kk from slot cur (window start s): hits (bits from cur) and
  // whether the run ends inside the window
  auto look = [&](int64_t kk, uint32_t cur, uint32_t s, uint32_t &hits, uint32_t slot) {
    const longlong2 x0 = *reinterpret_cast<const longlong2 *>(win + slot * kRingSlot);
    const longlong2 x1 = *reinterpret_cast<const longlong2 *>(win + slot * kRingSlot + 16);
    const uint32_t e = (x0.x == -1 ? 1u : 0u) | (x0.y == -1 ? 2u : 0u) | (x1.x == -1 ? 4u : 0u) | (x1.y == -1 ? 8u : 0u);
    const uint32_t m = (x0.x == kk ? 1u : 0u) | (x0.y == kk ? 2u : 0u) | (x1.x == kk ? 4u : 0u) | (x1.y == kk ? 8u : 0u);
    const uint32_t off = cur - s;
    const uint32_t ee = e >> off;
    const uint32_t f = (uint32_t)__builtin_ctz(ee | ((1u << kWin) >> off));  // run end (or window end) past cur
    hits = (m >> off) & ((1u << f) - 1u);
    return ee != 0u || hits != 0u;
  };
  auto result = [&](uint32_t cur, uint32_t hits) {
    return POS ? (hits ? (cur + (uint32_t)__builtin_ctz(hits)) | 0x80000000u : 0u) : (hits ? 1u : 0u);
  };

  // phase A: every row's first window (NB = 2: step j + 1's windows are fetched while step j's
  // are checked)
  uint32_t cont = 0;
  uint32_t sa[kJ];
#pragma unroll
  for (int j = 0; j < kJ; ++j) sa[j] = start(h[j]);
  if (NB > 1) issue(w0 < wend ? sa[0] : 0u, 0u);
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    ++steps;
    const uint32_t i = row_of(j);
    const bool valid = i < wend;
    const uint32_t s = sa[j];
    if (NB > 1) {
      if (j + 1 < kJ) {
        issue(row_of(j + 1) < wend ? sa[j + 1] : 0u, (uint32_t)(j + 1) & 1u);
        wait_vmcnt<2>();  // step j's two DMAs have landed (step j + 1's are in flight)
      } else {
        wait_vmcnt<0>();
      }
    } else {
      issue(valid ? s : 0u, 0u);
      wait_vmcnt<0>();
    }
    if (valid) {
      uint32_t hits;
      if (look(k[j], h[j], s, hits, NB > 1 ? (uint32_t)j & 1u : 0u)) {
        sm.hc[i] = result(h[j], hits);
      } else {
        sm.hc[i] = (s + kWin) & p.mask;  // the next unread slot
        cont |= 1u << j;
      }
    }
  }
  // phase B: the rows whose run went on, each lane its own, one window per step
  if (__ballot(cont != 0u)) {
    bool have = false;
    uint32_t bi = 0, bcur = 0, bst = 0;
    int64_t bkey = 0;
    auto take = [&]() {
      if (!have && cont) {
        const int j = __builtin_ctz(cont);
        cont &= cont - 1u;
        bi = row_of(j);
        bkey = sm.key[bi];
        bcur = sm.hc[bi];
        have = true;
      }
    };
    take();
    bst = start(bcur);
    issue(have ? bst : 0u, 0u);
    for (bool more = true; more;) {
      ++steps;
      wait_vmcnt<0>();
      if (have) {
        uint32_t hits;
        if (look(bkey, bcur, bst, hits, 0u)) {
          sm.hc[bi] = result(bcur, hits);
          have = false;
        } else {
          bcur = (bst + kWin) & p.mask;
        }
      }
      take();
      if (__ballot(have) == 0ull) {  // every lane's rows done
        more = false;
        break;
      }
      bst = start(bcur);
      issue(have ? bst : 0u, 0u);
    }
  }
  CCJ_STAMP(t2);
  __syncthreads();  // every wave's ring is idle: the emit's scratch may overlap it
  if (tid == 0) {
    sm.total = 0;
    sm.rounds = 0;
  }
  __syncthreads();
  if (POS) {
    if (p.out_sub) walk_emit_pos_sub<kWaveRows, NW>(p, sm, c, w0, wend, lane, wave, rid_e);
    else walk_emit_pos<kWaveRows, NW>(p, sm, c, w0, wend, lane, wave, sm.wtot, phys);
    walk_finish(p, sm, c, lane, 0u, 0u, t0, t1, t2, steps);
    return;
  }
  if (p.emit_pol != kEmitWave || p.rows_in_sel) {
    if (walk_emit_wg<kWaveRows, NW>(p, sm, c, w0, wend, lane, wave, sm.wtot, phys)) {
      walk_finish(p, sm, c, lane, 0u, 0u, t0, t1, t2, steps);
      return;
    }
  }
  const uint32_t overflow = walk_emit<kWaveRows>(p, sm, c, w0, wend, lane);
  walk_finish(p, sm, c, lane, 0u, overflow, t0, t1, t2, steps);
}

// Ordered probe, step 4 (emit_ordered): one chunk per 256-thread workgroup, the reference's
// per-Next stream from its rows' round words (p.in_w: mm | rounds << 26, or kMmLong | rounds).
// Thread (wave, lane) owns rows q*256 + tid (q < 8), i.e. row group j = 4q + wave, lane `lane`:
// its keys and words stay in registers, and the count / scan / emit phases are probe_chunks'
// (per (round, row group) ballots, a round-major exclusive scan, ballot-prefix stores), so the
// output is exactly ccj_probe's.  A chunk with a row of more than 26 rounds re-walks round by
// round (rounds_generic).  LDS: s_off (4 KB) plus the staged output (s_osel 8 KB + s_opay 16 KB),
// about 28 KB per workgroup: 5 workgroups per CU (round 2d: 8 before the output was staged).
template <int KIND>
__global__ __launch_bounds__(kBlock) void emit_ordered(ProbeParams p) {
  constexpr int kQ = kMaxChunk / kBlock;  // 8 rows per thread
  __shared__ uint32_t s_off[kMaxFastRounds * 32];
  __shared__ uint32_t s_red[3 * kChunkWaves];
  // the chunk's output in its final (round-major) order, written out with whole 16-byte stores
  __shared__ __attribute__((aligned(16))) uint32_t s_osel[kMaxChunk];
  __shared__ __attribute__((aligned(16))) int64_t s_opay[kMaxChunk];
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const uint64_t c = blockIdx.x;
  const uint64_t base = c * p.chunk;
  const uint64_t rem = p.n_rows - base;
  const uint32_t phys = rem < p.chunk ? (uint32_t)rem : p.chunk;
  const uint32_t nj = (p.chunk + kWave - 1) / kWave;
  uint32_t count = p.counts ? p.counts[c] : phys;
  uint32_t flags = 0;
  if (count > phys) {
    flags |= CCJ_FLAG_BAD_INPUT;
    count = phys;
  }
  int64_t key[kQ];
  uint32_t w[kQ];
#pragma unroll
  for (int q = 0; q < kQ; ++q) {  // every load in flight first: unconditional (row 0 past the
    // count), since a load under `if` made the compiler wait for each before the next
    const uint32_t i = (uint32_t)q * kBlock + tid;
    key[q] = __builtin_nontemporal_load(p.keys + base + (i < count ? i : 0u));
  }
  if (p.w16) {  // (the width branch outside the loads: one inside made each load wait for its use)
    uint16_t h[kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const uint32_t i = (uint32_t)q * kBlock + tid;
      h[q] = __builtin_nontemporal_load((const uint16_t *)p.in_w + base + (i < count ? i : 0u));
    }
#pragma unroll
    for (int q = 0; q < kQ; ++q) w[q] = round_word32(h[q]);
  } else {
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const uint32_t i = (uint32_t)q * kBlock + tid;
      w[q] = __builtin_nontemporal_load(p.in_w + base + (i < count ? i : 0u));
    }
  }
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    if ((uint32_t)q * kBlock + tid >= count) {
      key[q] = 0;
      w[q] = 0;
    }
  }
  for (uint32_t q = tid; q < kMaxFastRounds * 32; q += kBlock) s_off[q] = 0u;
  uint32_t lane_rounds = 0;
  bool long_run = false;
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    const uint32_t r = w[q] & kMmLong ? w[q] & ~kMmLong : w[q] >> kMmRounds;
    long_run |= (w[q] & kMmLong) != 0u;
    lane_rounds = r > lane_rounds ? r : lane_rounds;
    w[q] &= (1u << kMmRounds) - 1u;  // from here on: the row's match rounds (mm)
  }
  {
    const uint32_t wr = wave_max(lane_rounds);
    const bool wl = __ballot(long_run) != 0ull;
    if (lane == 0) {
      s_red[wave] = wr;
      s_red[kChunkWaves + wave] = wl ? 1u : 0u;
    }
  }
  __syncthreads();
  uint32_t rounds = 0, any_long = 0;
#pragma unroll
  for (int v = 0; v < kChunkWaves; ++v) {
    rounds = s_red[v] > rounds ? s_red[v] : rounds;
    any_long |= s_red[kChunkWaves + v];
  }
  uint64_t total = 0;
  const uint64_t obase = c * p.cap;
  if (any_long) {  // (rare) round by round, the chunk's keys read again from the column: no 16 KB
    // key image in LDS on the common path (8 workgroups per CU instead of 7; same box, ordered step
    // 22.45 / 22.49 / 22.47 ms against 22.45 / 22.49 / 22.50 with it: the emit is not occupancy-bound)
    if (wave == 0) {
      uint32_t act_all = 0;
      for (uint32_t j = 0; j < nj; ++j)
        if (j * kWave + lane < count) act_all |= 1u << j;
      rounds_generic<KIND>(p, c, base, nj, act_all, p.keys + base, flags, total, rounds);
    }
  } else {
    // Count: matches per (round r, row group j = 4q + wave).
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const uint32_t j = (uint32_t)q * kChunkWaves + wave;
      if (j < nj) {
        for (uint32_t any = wave_or(w[q]); any != 0u; any &= any - 1u) {
          const uint32_t r = (uint32_t)__builtin_ctz(any);
          const uint32_t n = (uint32_t)__popcll(__ballot((w[q] >> r) & 1u));
          if (lane == 0) s_off[r * 32 + j] = n;
        }
      }
    }
    __syncthreads();
    if (wave == 0) {  // exclusive prefix over (r, j) in round-major order, 16 entries per lane
      uint32_t loc[16], sum = 0;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        loc[t] = s_off[lane * 16 + t];
        sum += loc[t];
      }
      uint32_t incl = wave_incl_scan(sum);
      uint32_t run = incl - sum;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        s_off[lane * 16 + t] = run;
        run += loc[t];
      }
      if (lane == kWave - 1) s_red[2 * kChunkWaves] = incl;
    }
    __syncthreads();
    total = s_red[2 * kChunkWaves];
    if (p.out_round_counts) {  // Next return values: differences of the round starts
      for (uint32_t r = tid; r < rounds; r += kBlock) {
        const uint32_t a = s_off[r * 32], b = r + 1 < rounds ? s_off[(r + 1) * 32] : (uint32_t)total;
        if (r < p.max_rounds) p.out_round_counts[c * p.max_rounds + r] = b - a;
      }
      if (rounds > p.max_rounds) flags |= CCJ_FLAG_ROUND_OVERFLOW;
    }
    // Emit: group j's matches of round r go to s_off[r][j] + their ballot prefix — into the LDS
    // image of the chunk's output when it fits (every chunk of a distinct-key table), then out with
    // 16-byte stores (per (round, group) stores left most lanes of each store instruction idle);
    // otherwise straight to memory.
    const bool img = total <= kMaxChunk && total <= p.cap && p.cap % 4 == 0 && !p.out_base && !CCJ_ABLATED(p.ablate, 1u);
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const uint32_t j = (uint32_t)q * kChunkWaves + wave;
      const uint32_t i = (uint32_t)q * kBlock + tid;
      if (j < nj) {
        for (uint32_t any = wave_or(w[q]); any != 0u; any &= any - 1u) {
          const uint32_t r = (uint32_t)__builtin_ctz(any);
          const bool bit = (w[q] >> r) & 1u;
          const uint64_t mb = __ballot(bit);
          if (bit && !CCJ_ABLATED(p.ablate, 1u)) {
            const uint64_t o = (uint64_t)s_off[r * 32 + j] + lane_prefix(mb);
            if (img) {
              s_osel[o] = i;
              s_opay[o] = key[q];
            } else if (o < p.cap) {
              __builtin_nontemporal_store(i, p.out_sel + obase + o);
              if (p.out_payload) __builtin_nontemporal_store(key[q], p.out_payload + obase + o);
            }
          }
        }
      }
    }
    if (img) {
      __syncthreads();
      const uint32_t tot = (uint32_t)total;
      // a last partial group writes past the count inside the chunk's own cap region (no consumer
      // reads there); the buffer records stop every store at the cap
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(p.out_sel + obase, (short)0, (int)(p.cap * 4), 0x00020000);
      for (uint32_t g = tid; g * 4 < tot; g += kBlock) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(&s_osel[4 * g]);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(16 * g), 0, 2);
      }
      if (p.out_payload) {
        const auto rp = __builtin_amdgcn_make_buffer_rsrc(p.out_payload + obase, (short)0, (int)(p.cap * 8), 0x00020000);
        for (uint32_t g = tid; g * 2 < tot; g += kBlock) {
          const u32x4 v = *reinterpret_cast<const u32x4 *>(&s_opay[2 * g]);
          __builtin_amdgcn_raw_buffer_store_b128(v, rp, (int)(16 * g), 0, 2);
        }
      }
    }
  }
  if (total > p.cap) flags |= CCJ_FLAG_CAP_OVERFLOW;
  if (tid == 0) {
    p.out_count[c] = (uint32_t)(total < p.cap ? total : p.cap);
    if (p.out_rounds) p.out_rounds[c] = rounds;
  }
  if (p.status) {
    const uint64_t any = __ballot(flags != 0u);
    if (any && flags) atomicOr(p.status, flags);
  }
}

// Ordered probe, step 3: the round words of one split tile back into row order.  The split
// recorded where each (tile, partition) run went (runs / ovf_runs); the tile's runs are numbered
// consecutively (an exclusive scan of their lengths) — the order of the split's tile image — every
// thread takes entries j = tid, tid + 1024, ..., finds j's partition by a binary search over the
// scan, and drops the word into an LDS image of the tile at the row the split recorded for image
// entry j (row_loc[t0 + j], 16 bits: the row inside its tile, written by the split in image order,
// so these reads are whole lines; round 4 — before, the rows sat beside the words at the runs'
// positions and both were read from partial lines); the image is written out whole.  Rows that were
// not live stay 0.
// C2: 4.6 ms, 22.5 GiB of DRAM traffic (the runs' partial lines: ~2x the 8 B read per row) =
// 5.2 TB/s.  One binary search per thread over kPer consecutive entries (each load instruction then
// spans ~kPer * 64 entries) measured 13.6 ms; tiles read in the split's XCD order 4.66 ms.
constexpr int kUnsplitThreads = 1024;
// Threads of the unsplit's workgroup when the partitions fit (one per thread in the runs' scan): 512
// (32 KiB of LDS, four tiles in flight per CU instead of two) against 1024, same box, interleaved:
// unsplit + emit 7.55 → 6.82 ms at C2 ordered (20.26 → 19.53 ms per step), 6.53-6.56 → 5.81-5.84 ms
// at C3 ordered (profiles/r4_ab_r4ak_unsplit_nt.log); 256 threads leave C2 / C3's 512 partitions
// to the 1024-thread form.
#ifndef CCJ_UNSPLIT_NT
#define CCJ_UNSPLIT_NT 512
#endif
constexpr uint32_t kUnsplitMaxTile = 13u * kUnsplitThreads;  // the split's largest tile (13 keys per thread)

template <typename W, int NT>
__global__ __launch_bounds__(NT) void unsplit_words(const uint2 *runs, const uint32_t *ovf_runs,
                                                                 const uint16_t *row_loc, const W *w_pos,
                                                                 W *w_row, uint64_t n, uint32_t parts,
                                                                 uint32_t tile, uint32_t *status) {
  __shared__ __attribute__((aligned(16))) W s_img[kUnsplitMaxTile];
  __shared__ uint32_t s_loc[NT + 1];
  __shared__ uint2 s_run[NT];
  __shared__ uint32_t s_wsum[NT / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint64_t t = blockIdx.x, t0 = t * tile;
  const uint32_t tn = (uint32_t)(n - t0 < tile ? n - t0 : tile);
  for (uint32_t i = tid; i < tn; i += NT) s_img[i] = 0;
  const uint2 r = tid < parts ? runs[t * parts + tid] : make_uint2(0u, 0u);
  const uint32_t len = (r.y & 0xFFFFu) + (r.y >> 16);
  uint32_t incl = wave_incl_scan(len);
  if (lane == 63) s_wsum[wave] = incl;
  __syncthreads();
  uint32_t wpre = 0;
  for (uint32_t w = 0; w < wave; ++w) wpre += s_wsum[w];
  if (tid < parts) {
    s_loc[tid] = wpre + incl - len;
    s_run[tid] = r;
  }
  if (tid == parts - 1) s_loc[parts] = wpre + incl;
  __syncthreads();
  const uint32_t total = s_loc[parts];
  bool bad = false;
  // kU entries per thread per pass, all their loads in flight together (a load under `if`, or one
  // waiting on the previous entry's, made each entry two dependent round trips)
  constexpr uint32_t kU = 4;
  for (uint32_t j0 = tid; j0 < total; j0 += kU * NT) {
    uint64_t pos[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      uint32_t j = j0 + u * NT;
      j = j < total ? j : total - 1;  // (a repeat of the last entry: the same word to the same row)
      uint32_t lo = 0, hi = parts;    // the last d with s_loc[d] <= j
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_loc[mid] <= j) lo = mid;
        else hi = mid;
      }
      const uint32_t o = j - s_loc[lo];
      const uint2 rr = s_run[lo];
      const uint32_t lim = rr.y & 0xFFFFu;
      pos[u] = o < lim ? (uint64_t)rr.x + o : (uint64_t)ovf_runs[t * parts + lo] + (o - lim);
    }
    uint32_t rm[kU];
    W wv[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint32_t j = j0 + u * NT;
      rm[u] = row_loc[t0 + (j < total ? j : total - 1)];  // image order: consecutive, whole lines
      wv[u] = w_pos[pos[u]];
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      if (rm[u] < tn) s_img[rm[u]] = wv[u];
      else bad = true;
    }
  }
  if (bad && status) atomicOr(status, CCJ_FLAG_BAD_INPUT);
  __syncthreads();
  // 16-byte stores where the tile's rows start 16-byte aligned (round 2d), single words for the rest
  constexpr uint32_t kPer16 = 16 / sizeof(W);
  const uint32_t vec = ((t0 * sizeof(W)) % 16 == 0) ? tn / kPer16 * kPer16 : 0u;
  for (uint32_t g = tid; g * kPer16 < vec; g += NT)
    __builtin_nontemporal_store(*reinterpret_cast<const u32x4 *>(&s_img[g * kPer16]),
                                reinterpret_cast<u32x4 *>(w_row + t0 + g * kPer16));
  for (uint32_t i = vec + tid; i < tn; i += NT) __builtin_nontemporal_store(s_img[i], w_row + t0 + i);
}

hipError_t launch_probe_flat(int kind, const ProbeParams &p, hipStream_t s) {
  if (p.n_chunks == 0) return hipSuccess;
  const dim3 g((unsigned)p.n_chunks), b(kFlatThreads);
  const uint64_t size = (uint64_t)p.mask + 1;
  if (kind != CCJ_TABLE_LP) {
    if (!p.bucket) return hipErrorInvalidValue;  // every chaining table carries bucket records
    // the LDS bucket filter walk (probe_chain_filt) for the fixed-capacity split's segments, when the
    // table has a filter, the partitions are at most 2^18 buckets and there are >= 8 of them (one
    // XCD's range each), the chunk is a multiple of 256 rows and no rounds are asked for; the
    // overflow area's chunks (key skew) go to probe_chain_win
    if (chain_filt_applies(p, kFiltUnit) && !p.out_rounds && ccj_tune_int("CCJ_CHAIN_FILT", 1)) {
      hipError_t e = hipMemsetAsync(p.out_count, 0, p.n_chunks * sizeof(uint32_t), s);
      if (e != hipSuccess) return e;
      // two 64 KiB workgroups per CU
      const uint32_t grid = std::max<uint32_t>(8u, 2 * stream_cus(s) / 8 * 8);
      hipLaunchKernelGGL(probe_chain_filt, dim3(grid), dim3(kFiltThreads), 0, s, p);
      ProbeParams q = p;  // the overflow area's chunks, in plain order
      q.chunk0 = p.ovf_base / p.chunk;
      q.xcd_swizzle = 0;
      if (p.n_chunks > q.chunk0)
        hipLaunchKernelGGL((probe_chain_win<3>), dim3((unsigned)(p.n_chunks - q.chunk0)), b, 0, s, q);
      return hipGetLastError();
    }
    hipLaunchKernelGGL((probe_chain_win<3>), g, b, 0, s, p);
    return hipGetLastError();
  }
  if (size < 16) return launch_probe(kind, p, s);  // a table of < 16 slots is one identity window
  // At C2 (DESIGN §3.2, r2 sweeps): probe_walk 9.4 ms against 9.9-10.1 for probe_win's per-step
  // output placement; R = 2 / 3 / 4 / 6 rows per pair 9.65 / 9.4 / 9.7 / 10.9 ms; home slots
  // staged in LDS 9.4 vs hashed at row start 9.6 ms; 8 waves x 256 rows per chunk 10.0 ms; one
  // lane per row with two 16-B loads (twice the L2 requests) 11.0-12.3 ms; a rolling load
  // pipeline (each slot re-issued as soon as it is consumed, vmcnt(R - 1) waits) 10.4-10.5 ms;
  // write-through (sc1) or plain output stores 10.2 ms vs non-temporal.
  const bool walk2 = p.first_match && ccj_tune_int("CCJ_WALK2", 1);
  if (p.out_pos && p.rows_in_sel) {
    // C5 under CCJ_PART_ROWS (distinct keys, tables of <= 2^31 slots): the split wrote rows and keys,
    // the walk leaves each row's matched slot at its output slot
    if (walk2 && ccj_tune_int("CCJ_WALK2_POS_NB", 1) == 2) hipLaunchKernelGGL((probe_walk2<true, 2>), g, b, 0, s, p);
    else if (walk2) hipLaunchKernelGGL((probe_walk2<true>), g, b, 0, s, p);
    else hipLaunchKernelGGL((probe_walk1<1, false, true>), g, b, 0, s, p);
  } else if (p.out_pos) {
    hipLaunchKernelGGL((probe_win<3>), g, b, 0, s, p);  // C5: match positions too
  } else {
    // 64-byte windows (4 lanes per row: 1.109 instead of 1.169 window reads per row in a host
    // simulation of the C2 table) measured slower, same box: 13.42 / 14.35 ms per C2 step against
    // 13.24 / 13.22 (half the rows per load instruction); tuning build only (CCJ_WALK_LANES=4)
    if (ccj_tune_int("CCJ_WALK_LANES", 2) == 4)
      hipLaunchKernelGGL((probe_walk<3, true, 4, false, 4>), g, b, 0, s, p);
    else if (ccj_tune_int("CCJ_WALK_DMA", 2) == 0)
      hipLaunchKernelGGL((probe_walk<3, true>), g, b, 0, s, p);
    else if (ccj_tune_int("CCJ_WALK_DMA", 2) == 1)
      hipLaunchKernelGGL((probe_walk<3, true, 4, false, 2, true>), g, b, 0, s, p);
    // probe_walk1: one batch of 64 rows in flight per wave (NB = 1) 12.07-12.09 ms per C2 step,
    // NB = 2 / 3 / 4 12.23 / 12.40 / 14.27 (fewer workgroups per CU; profiles/r3_ab.md)
    else if (ccj_tune_int("CCJ_WALK_NB", 1) == 2)
      hipLaunchKernelGGL((probe_walk1<2>), g, b, 0, s, p);
    else if (ccj_tune_int("CCJ_WALK_NB", 1) == 3)
      hipLaunchKernelGGL((probe_walk1<3>), g, b, 0, s, p);
    // distinct keys, no rounds: fixed first windows (step j + 1's fetched while step j's are
    // checked: 40 KiB, 4 workgroups per CU), then the rows that go on.  Same box, C2 step:
    // 11.34 / 11.36 ms against 11.47 / 11.39 with one window batch in flight (5 workgroups per CU)
    else if (walk2 && ccj_tune_int("CCJ_WALK2_NB", 2) == 1)
      hipLaunchKernelGGL((probe_walk2<false, 1>), g, b, 0, s, p);
    else if (walk2)
      hipLaunchKernelGGL((probe_walk2<false, 2>), g, b, 0, s, p);
    else if (ccj_tune_int("CCJ_WALK_NW", 4) == 8)  // 8 waves x 256 rows: 40 KiB, 4 workgroups = 32 waves per CU
      hipLaunchKernelGGL((probe_walk1<1, false, false, 8>), g, dim3(kWave * 8), 0, s, p);
    else
      hipLaunchKernelGGL((probe_walk1<1>), g, b, 0, s, p);
  }
  return hipGetLastError();
}

namespace {
// Wide-payload materialisation (C5) after the probe: every match's table position -> its
// position-major payload row (one 64-byte line for 8 columns), written column by column.  Run as
// its own pass so each thread keeps two rows' loads in flight instead of the probe's emit phase
// waiting on one dependent row per match.
struct GatherParams {
  const uint32_t *count, *pos;
  const uint64_t *out_base;
  uint64_t cap;
  const int64_t *pay;
  uint32_t stride;
  int64_t *cols[CCJ_MAX_PAYLOAD_COLS];
  uint32_t shift;  // timing only (tuning build, CCJ_GATHER_SHIFT): row = position >> shift
  uint32_t mask;   // timing only (tuning build, CCJ_GATHER_MASK): row = (position >> shift) & mask
  uint32_t ablate; // timing only (tuning build, CCJ_GATHER_ABLATE): 1 = no column stores
  // slab order (gather_payload_cols_sub): the walk's sub-range starts per chunk, the partitions'
  // chunk ranges (parts x cpp chunks, then the overflow area's), chunk groups per (partition, slab)
  const uint32_t *sub;
  uint32_t parts, groups;
  uint64_t cpp, main_chunks, n_main_items;
};

template <int NP, bool VEC>
__global__ __launch_bounds__(256) void gather_payload(GatherParams g) {
  const uint64_t c = blockIdx.x;
  const uint64_t ob = g.out_base ? g.out_base[c] : c * g.cap;
  const uint32_t n = g.count[c];
  for (uint32_t j0 = threadIdx.x; j0 < n; j0 += 512) {
    int64_t v[2][NP];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t j = j0 + u * 256;
      if (j < n) {
        const int64_t *row = g.pay + (uint64_t)g.pos[ob + j] * g.stride;
        if (VEC) {
#pragma unroll
          for (int q = 0; q + 1 < NP; q += 2) {
            const longlong2 x = *reinterpret_cast<const longlong2 *>(row + q);
            v[u][q] = x.x;
            v[u][q + 1] = x.y;
          }
          if (NP & 1) v[u][NP - 1] = row[NP - 1];
        } else {
#pragma unroll
          for (int q = 0; q < NP; ++q) v[u][q] = row[q];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t j = j0 + u * 256;
      if (j < n) {
#pragma unroll
        for (int q = 0; q < NP; ++q) __builtin_nontemporal_store(v[u][q], g.cols[q] + ob + j);
      }
    }
  }
}

// 8 columns, 64-byte rows: four lanes share a row, each loading 16 bytes of it, so one wave
// instruction fetches 16 whole rows (one request per row instead of four); lane q then writes
// columns 2q and 2q+1 of its row (16 consecutive rows per column per instruction).
template <int U>
__global__ __launch_bounds__(256) void gather_payload_quad(GatherParams g) {
  __shared__ int64_t *s_cols[CCJ_MAX_PAYLOAD_COLS];
  if (threadIdx.x < CCJ_MAX_PAYLOAD_COLS) s_cols[threadIdx.x] = g.cols[threadIdx.x];
  __syncthreads();
  const uint64_t c = blockIdx.x;
  const uint64_t ob = g.out_base ? g.out_base[c] : c * g.cap;
  const uint32_t n = g.count[c];
  const uint32_t q = threadIdx.x & 3u, r0 = threadIdx.x >> 2;  // 64 rows per block step
  int64_t *c0 = s_cols[2 * q], *c1 = s_cols[2 * q + 1];
  for (uint32_t base = 0; base < n; base += 64 * U) {
    // the U positions, then the U rows: each phase's loads in flight together (loads under `if`
    // made the compiler wait for every position and row before the next)
    uint32_t ps[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t j = base + u * 64 + r0;
      ps[u] = g.pos[ob + (j < n ? j : 0u)];
    }
    __builtin_amdgcn_sched_barrier(0);  // every position load issued before the first row load
    longlong2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = reinterpret_cast<const longlong2 *>(g.pay + (uint64_t)((ps[u] >> g.shift) & g.mask) * g.stride)[q];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t j = base + u * 64 + r0;
      if (j < n && (!CCJ_ABLATED(g.ablate, 1u) || (v[u].x ^ v[u].y) == 0x5A5A5A5A5A5A5A5All)) {
        __builtin_nontemporal_store(v[u].x, c0 + ob + j);
        __builtin_nontemporal_store(v[u].y, c1 + ob + j);
      }
    }
  }
}

// 8 columns, the stores transposed through LDS: per step of 64 x U rows the quads load rows as in
// gather_payload_quad and drop them into a column-major LDS tile (8 x 64U int64; U = 8: 32 KiB);
// each wave then stores 1 KiB of ONE column per instruction (16 bytes = two rows per lane) instead
// of four columns' 128-byte pieces of 8 bytes per lane.  The stores alone (rows from one line,
// timing only) take 14.0 ms per C5 step against the quad form's 19.2; the row reads alone 15.1
// against 17.1 (profiles/r5_ab_gather_cols.log).  The column pointers come from the kernel
// arguments (the store pass's column is its unrolled index), so the LDS tile is the workgroup's
// only LDS — 32 KiB, five workgroups per CU instead of four with a pointer table beside it: same
// box, gather 26.7-27.2 (four) -> 25.2-25.6 ms (profiles/r5_ab_gather_cols_5wg.log).
template <int U>
__global__ __launch_bounds__(256) void gather_payload_cols(GatherParams g) {
  constexpr uint32_t kStep = 64 * U;  // rows per step
  typedef long long i64x2 __attribute__((ext_vector_type(2)));
  static_assert(kStep / 2 % 64 == 0, "a wave's 64 store pieces lie in one column");
  __shared__ int64_t s_t[8][kStep];  // U = 8: exactly 32 KiB, five workgroups per CU
  const uint64_t c = blockIdx.x;
  const uint64_t ob = g.out_base ? g.out_base[c] : c * g.cap;
  const uint32_t n = g.count[c];
  const uint32_t q = threadIdx.x & 3u, r0 = threadIdx.x >> 2;
  // software pipeline: step i's tile is stored while step i + 1's rows and step i + 2's positions
  // are in flight (loads issued before the stores, so no wait on a load drains them)
  // positions: each lane loads its own (U / 4 loads of 64 distinct positions per wave) and the
  // quads take theirs by ds_bpermute — 4x fewer position-load instructions than a load per quad
  // lane: same box, 3 x interleaved, gather 25.55-25.58 -> 25.37-25.39 ms (profiles/r5_ab_gather_pos.log)
  static_assert(U % 4 == 0, "U / 4 position loads per lane");
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t pl[U / 4];
  i64x2 v[U];
  auto load_pos = [&](uint32_t b) {
#pragma unroll
    for (int h = 0; h < U / 4; ++h) {  // row (4h + lane / 16) * 64 + 16 wave + lane % 16 of the step
      const uint32_t j = b + (uint32_t)(4 * h + (lane >> 4)) * 64u + wave * 16u + (lane & 15u);
      pl[h] = g.pos[ob + (j < n ? j : 0u)];
    }
  };
  auto load_rows = [&]() {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t pu = (uint32_t)__shfl((int)pl[u / 4], (int)(((u & 3) << 4) | (lane >> 2)));
      v[u] = reinterpret_cast<const i64x2 *>(g.pay + (uint64_t)((pu >> g.shift) & g.mask) * g.stride)[q];
    }
  };
  if (n == 0) return;
  load_pos(0);
  load_rows();
  if (kStep < n) load_pos(kStep);
  for (uint32_t base = 0; base < n; base += kStep) {
    __syncthreads();  // the previous tile is stored
    // the tile's rows XOR-swizzled by 8 x (column / 2): the four quad lanes' columns (2q, 2q + 1) sit
    // 4 KiB apart, i.e. on the same banks, so without it every 8-byte write is a 4-way conflict
    // (60 % of the LDS cycles, profiles/r5u3_c5_units.json); same box, gather 25.39 / 26.87 / 26.83 ->
    // 25.33 / 25.33 / 25.33 ms (profiles/r5_ab_gather_swizzle.log)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s_t[2 * q][(u * 64 + r0) ^ (8u * q)] = v[u].x;
      s_t[2 * q + 1][(u * 64 + r0) ^ (8u * q)] = v[u].y;
    }
    __syncthreads();
    if (base + kStep < n) load_rows();
    if (base + 2 * kStep < n) load_pos(base + 2 * kStep);
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t rows = n - base < kStep ? n - base : kStep;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      // 8 columns x kStep rows = 4U 16-byte pieces per thread; a wave's 64 lanes: 1 KiB of one column
      // piece k * 256 + tid: column (k * 256 + tid) / (kStep / 2) — k itself at U = 8 — rows pr, pr + 1
      const uint32_t idx = (uint32_t)k * 256u + threadIdx.x;
      const uint32_t col = kStep / 2 == 256 ? (uint32_t)k : (uint32_t)__builtin_amdgcn_readfirstlane((int)(idx / (kStep / 2)));
      const uint32_t pr = (idx % (kStep / 2)) * 2u;
      const i64x2 x = *reinterpret_cast<const i64x2 *>(&s_t[col][pr ^ (8u * (col >> 1))]);
      int64_t *cp = g.cols[0];
#pragma unroll
      for (int cc = 1; cc < 8; ++cc) cp = col == (uint32_t)cc ? g.cols[cc] : cp;  // (wave-uniform select)
      int64_t *dst = cp + ob + base + pr;
      if (CCJ_ABLATED(g.ablate, 1u) && (x.x ^ x.y) != 0x5A5A5A5A5A5A5A5All) continue;
      if (pr + 1 < rows) __builtin_nontemporal_store(x, reinterpret_cast<i64x2 *>(dst));
      else if (pr < rows) __builtin_nontemporal_store((int64_t)x.x, dst);
    }
  }
}

// gather_payload_cols in slab order (round 6, with the walk's sub-range order, walk_emit_pos_sub):
// workgroup b takes, for XCD x = b & 7 (the hardware deals workgroups to the XCDs in turn),
// partition d of x's range, sub-range s and a group of G of d's chunks, the piece of each chunk
// whose matches fall in sub-range s — so an XCD's workgroups work through one slab of 2^sub_shift
// slots (4 MiB of payload rows at C5, ~1.8 MiB of them touched) at a time and its rows stay in that
// XCD's L2 instead of being fetched from the fabric once per match (the slab walk of the whole
// 32 MiB partition slice did: 1.62x the rows' bytes read).  The pieces, widened to even bounds so
// the transposed column stores stay 16-byte pairs (a boundary row is written twice, with the same
// values), are concatenated into the 512-row steps of gather_payload_cols; a step row finds its
// piece among G wave-uniform bounds.  The overflow area's chunks follow, one whole chunk each.
template <int U, int G>
__global__ __launch_bounds__(256, 5) void gather_payload_cols_sub(GatherParams g) {
  constexpr uint32_t kStep = 64 * U;
  typedef long long i64x2 __attribute__((ext_vector_type(2)));
  static_assert(kStep / 2 == 256 && G <= 64, "one column per store step (U = 8)");
  __shared__ int64_t s_t[8][kStep];  // 32 KiB, five workgroups per CU (as gather_payload_cols)
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t q = threadIdx.x & 3u, r0 = threadIdx.x >> 2;
  uint64_t c0, nch;
  uint32_t s = 0;
  bool whole;
  if ((uint64_t)blockIdx.x < g.n_main_items) {
    const uint64_t x = blockIdx.x & 7u, i = blockIdx.x >> 3;
    const uint64_t per_part = 8ull * g.groups;
    const uint64_t d = x * (g.parts / 8u) + i / per_part;
    s = (uint32_t)((i / g.groups) % 8u);
    c0 = d * g.cpp + (i % g.groups) * (uint64_t)G;
    const uint64_t cend = (d + 1) * g.cpp;
    nch = cend - c0 < (uint64_t)G ? cend - c0 : (uint64_t)G;
    whole = false;
  } else {
    c0 = g.main_chunks + ((uint64_t)blockIdx.x - g.n_main_items);
    nch = 1;
    whole = true;
  }
  // lane p < nch: chunk c0 + p's piece [a, e), widened to even bounds
  uint32_t pa = 0, pl_ = 0;
  if (lane < nch) {
    const uint64_t cc = c0 + lane;
    const uint32_t n = g.count[cc];
    uint32_t a = whole ? 0u : g.sub[cc * 8 + s];
    uint32_t e = (whole || s == 7u) ? n : g.sub[cc * 8 + s + 1];
    a &= ~1u;
    e = (e + 1u) & ~1u;
    e = e < n ? e : n;
    pa = a;
    pl_ = e > a ? e - a : 0u;
  }
  const uint32_t vl = (pl_ + 1u) & ~1u;  // the piece's rows in the step list (even)
  uint32_t incl = vl;
#pragma unroll
  for (uint32_t dd = 1; dd < (uint32_t)G; dd <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)incl, dd);
    if (lane >= dd) incl += t;
  }
  // the pieces' bounds stay in lanes 0 .. G - 1 (a piece is found by comparing against the G
  // uniform starts, its fields fetched by ds_bpermute: select chains over per-piece arrays became
  // a scratch lookup table)
  const uint32_t vst_l = incl - vl;
  const uint64_t ob_l = (c0 + (uint64_t)lane) * g.cap + pa;
  uint32_t vst[G];
#pragma unroll
  for (int pp = 0; pp < G; ++pp) vst[pp] = (uint32_t)__builtin_amdgcn_readlane((int)vst_l, pp);
  const uint32_t V = (uint32_t)__builtin_amdgcn_readlane((int)incl, G - 1);  // rows in the step list
  if (V == 0) return;
  // a valid position index for the list's dead rows: the first live piece's
  const uint64_t live_mask = __ballot(lane < (uint32_t)G && pl_ != 0u);
  const int first = (int)__builtin_ctzll(live_mask | (1ull << (G - 1)));
  const uint64_t fb = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ob_l, first) |
                      (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ob_l >> 32), first) << 32;
  // step-list row vr -> its piece, offset in it, its length and output base
  auto locate = [&](uint32_t vr, uint32_t &off, uint32_t &len, uint64_t &base) {
    uint32_t pc = 0;
#pragma unroll
    for (int pp = 1; pp < G; ++pp) pc += vr >= vst[pp] ? 1u : 0u;
    off = vr - (uint32_t)__shfl((int)vst_l, (int)pc);
    len = (uint32_t)__shfl((int)pl_, (int)pc);
    base = (uint64_t)(uint32_t)__shfl((int)(uint32_t)ob_l, (int)pc) |
           (uint64_t)(uint32_t)__shfl((int)(uint32_t)(ob_l >> 32), (int)pc) << 32;
  };
  uint32_t pl[U / 4];
  i64x2 v[U];
  auto load_pos = [&](uint32_t b) {
#pragma unroll
    for (int h = 0; h < U / 4; ++h) {  // row (4h + lane / 16) * 64 + 16 wave + lane % 16 of the step
      const uint32_t j = b + (uint32_t)(4 * h + (lane >> 4)) * 64u + wave * 16u + (lane & 15u);
      uint32_t off, len;
      uint64_t base;
      locate(j, off, len, base);
      pl[h] = g.pos[j < V && off < len ? base + off : fb];
    }
  };
  auto load_rows = [&]() {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t pu = (uint32_t)__shfl((int)pl[u / 4], (int)(((u & 3) << 4) | (lane >> 2)));
      v[u] = reinterpret_cast<const i64x2 *>(g.pay + (uint64_t)((pu >> g.shift) & g.mask) * g.stride)[q];
    }
  };
  load_pos(0);
  load_rows();
  if (kStep < V) load_pos(kStep);
  for (uint32_t base = 0; base < V; base += kStep) {
    __syncthreads();  // the previous tile is stored
#pragma unroll
    for (int u = 0; u < U; ++u) {  // (the XOR swizzle of gather_payload_cols)
      s_t[2 * q][(u * 64 + r0) ^ (8u * q)] = v[u].x;
      s_t[2 * q + 1][(u * 64 + r0) ^ (8u * q)] = v[u].y;
    }
    __syncthreads();
    if (base + kStep < V) load_rows();
    if (base + 2 * kStep < V) load_pos(base + 2 * kStep);
    __builtin_amdgcn_sched_barrier(0);
    // this thread's rows pr, pr + 1 of the step, the same in every column: their place once
    const uint32_t pr = threadIdx.x * 2u;
    uint32_t off, len;
    uint64_t ob0;
    locate(base + pr, off, len, ob0);
    const bool live = base + pr < V && off < len, pair = off + 1 < len;
    const uint64_t at = ob0 + off;
#pragma unroll
    for (int k = 0; k < U; ++k) {  // column k
      const i64x2 x = *reinterpret_cast<const i64x2 *>(&s_t[k][pr ^ (8u * ((uint32_t)k >> 1))]);
      if (!live) continue;
      if (CCJ_ABLATED(g.ablate, 1u) && (x.x ^ x.y) != 0x5A5A5A5A5A5A5A5All) continue;
      int64_t *dst = g.cols[k] + at;
      if (pair) __builtin_nontemporal_store(x, reinterpret_cast<i64x2 *>(dst));
      else __builtin_nontemporal_store((int64_t)x.x, dst);
    }
  }
}

thread_local const char *t_gather_kernel = "";

template <int NP>
hipError_t launch_gather_np(const GatherParams &g, uint64_t n_chunks, hipStream_t s) {
  const bool vec = (g.stride % 2 == 0) && ((uintptr_t)g.pay % 16 == 0);
  // 8 columns: 2 / 4 / 8 rows in flight per lane group 26.9 ms each at C5, the walk's XCD order
  // 27.0, plain instead of non-temporal stores 27.8-28.9 (profiles/r1g_*)
  // (row pieces by LDS-DMA instead: 42.2-42.5 ms per C5 step against 42.2-42.3, round 3)
  // 8 columns: the transposed stores (gather_payload_cols<8>: C5 gather 26.7-27.0 -> 25.2-25.6 ms,
  // 256-row steps 26.9-28.4, 1024-row steps 27.0, profiles/r5_ab_gather_cols*.log) where every
  // column's rows are 16-byte aligned (no packed pipeline outputs: out_base == nullptr, cap even,
  // columns 16-byte aligned); the tuning build's CCJ_GATHER_T=0 runs the quad form for A/B
  bool cols16 = NP == 8 && (g.out_base == nullptr && g.cap % 2 == 0);
  for (int q = 0; q < NP; ++q) cols16 = cols16 && (uintptr_t)g.cols[q] % 16 == 0;
  if (NP == 8 && vec && cols16 && ccj_tune_int("CCJ_GATHER_T", 1)) {
#ifdef CCJ_TUNING
    // (tuning build: 256-row steps, 16 KiB tiles; 384-row steps measured 26.6 ms before the per-lane
    // position loads, which need U a multiple of 4)
    if (ccj_tune_int("CCJ_GATHER_U", 8) == 4)
      hipLaunchKernelGGL(gather_payload_cols<4>, dim3((unsigned)n_chunks), dim3(256), 0, s, g);
    else
#endif
    hipLaunchKernelGGL(gather_payload_cols<8>, dim3((unsigned)n_chunks), dim3(256), 0, s, g);
    t_gather_kernel = "gather_payload_cols<8> (stores transposed through LDS)";
  } else if (NP == 8 && vec) {
    hipLaunchKernelGGL((gather_payload_quad<4>), dim3((unsigned)n_chunks), dim3(256), 0, s, g);
    t_gather_kernel = "gather_payload_quad<4> (16-byte row pieces, column-unaligned fallback)";
  } else if (vec) {
    hipLaunchKernelGGL((gather_payload<NP, true>), dim3((unsigned)n_chunks), dim3(256), 0, s, g);
    t_gather_kernel = "gather_payload<NP, vec> (16-byte row loads)";
  } else {
    hipLaunchKernelGGL((gather_payload<NP, false>), dim3((unsigned)n_chunks), dim3(256), 0, s, g);
    t_gather_kernel = "gather_payload<NP, scalar> (8-byte loads)";
  }
  return hipGetLastError();
}
}  // namespace

const char *last_gather_kernel() { return t_gather_kernel; }

hipError_t launch_gather_payload(const ProbeParams &p, const uint32_t *pos, hipStream_t s, uint32_t parts,
                                 uint64_t cpp) {
  GatherParams g{};
  g.count = p.out_count;
  g.pos = pos;
  g.out_base = p.out_base;
  g.cap = p.cap;
  g.pay = p.pay;
  g.stride = p.pay_stride;
  for (uint32_t q = 0; q < p.n_pay; ++q) g.cols[q] = p.out_cols[q];
  g.shift = (uint32_t)ccj_tune_int("CCJ_GATHER_SHIFT", 0);
  g.mask = (uint32_t)ccj_tune_int("CCJ_GATHER_MASK", -1);
  g.ablate = (uint32_t)ccj_tune_int("CCJ_GATHER_ABLATE", 0);
  if (p.out_sub) {  // the walk wrote each chunk in sub-range order: the slab-order gather (8 columns)
    constexpr int kG = 8;
    bool ok = p.n_pay == 8 && parts >= 8 && parts % 8 == 0 && cpp && p.out_base == nullptr && p.cap % 2 == 0 &&
              g.stride % 2 == 0 && (uintptr_t)g.pay % 16 == 0 && (uint64_t)parts * cpp <= p.n_chunks;
    for (int q = 0; q < 8; ++q) ok = ok && (uintptr_t)g.cols[q] % 16 == 0;
    if (!ok) return hipErrorInvalidValue;  // (the caller asks for sub-range order only where this holds)
    g.sub = p.out_sub;
    g.parts = parts;
    g.cpp = cpp;
    g.groups = (uint32_t)((cpp + kG - 1) / kG);
    g.main_chunks = (uint64_t)parts * cpp;
    g.n_main_items = (uint64_t)parts * 8u * g.groups;
    const uint64_t grid = g.n_main_items + (p.n_chunks - g.main_chunks);
#ifdef CCJ_TUNING
    if (ccj_tune_int("CCJ_GATHER_G", kG) == 16) {  // (tuning: 16 chunks per workgroup)
      g.groups = (uint32_t)((cpp + 15) / 16);
      g.n_main_items = (uint64_t)parts * 8u * g.groups;
      const uint64_t grid16 = g.n_main_items + (p.n_chunks - g.main_chunks);
      hipLaunchKernelGGL((gather_payload_cols_sub<8, 16>), dim3((unsigned)grid16), dim3(256), 0, s, g);
      t_gather_kernel = "gather_payload_cols_sub<8> (slab order, 16 chunks per workgroup)";
      return hipGetLastError();
    }
#endif
    hipLaunchKernelGGL((gather_payload_cols_sub<8, kG>), dim3((unsigned)grid), dim3(256), 0, s, g);
    t_gather_kernel = "gather_payload_cols_sub<8> (slab order: one 4 MiB payload slab per XCD at a time)";
    return hipGetLastError();
  }
  switch (p.n_pay) {
    case 1: return launch_gather_np<1>(g, p.n_chunks, s);
    case 2: return launch_gather_np<2>(g, p.n_chunks, s);
    case 3: return launch_gather_np<3>(g, p.n_chunks, s);
    case 4: return launch_gather_np<4>(g, p.n_chunks, s);
    case 5: return launch_gather_np<5>(g, p.n_chunks, s);
    case 6: return launch_gather_np<6>(g, p.n_chunks, s);
    case 7: return launch_gather_np<7>(g, p.n_chunks, s);
    case 8: return launch_gather_np<8>(g, p.n_chunks, s);
    default: return hipSuccess;
  }
}

hipError_t launch_ordered_walk(int kind, const ProbeParams &p, hipStream_t s) {
  if (p.n_chunks == 0) return hipSuccess;
  if (kind == CCJ_TABLE_CHAIN) {
    if (!p.bucket) return hipErrorInvalidValue;  // every chaining table carries bucket records
    if (chain_filt_applies(p, kFiltUnit) && ccj_tune_int("CCJ_CHAIN_FILT", 1)) {  // the bucket filter in LDS
      const uint32_t grid = std::max<uint32_t>(8u, 2 * stream_cus(s) / 8 * 8);  // two workgroups per CU
      hipLaunchKernelGGL(chain_words_filt, dim3(grid), dim3(kFiltWordThreads), 0, s, p);
      ProbeParams q = p;  // the overflow area's chunks, in plain order
      q.chunk0 = p.ovf_base / p.chunk;
      q.xcd_swizzle = 0;
      if (p.n_chunks > q.chunk0)
        hipLaunchKernelGGL((chain_words<3>), dim3((unsigned)(p.n_chunks - q.chunk0)), dim3(kFlatThreads), 0, s, q);
      return hipGetLastError();
    }
    hipLaunchKernelGGL((chain_words<3>), dim3((unsigned)p.n_chunks), dim3(kFlatThreads), 0, s, p);
  } else if (ccj_tune_int("CCJ_OWALK", 1) == 1)
    hipLaunchKernelGGL((probe_walk1<1, true>), dim3((unsigned)p.n_chunks), dim3(kFlatThreads), 0, s, p);
  else
    hipLaunchKernelGGL((probe_walk<3, true, 4, true>), dim3((unsigned)p.n_chunks), dim3(kFlatThreads), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_unsplit_words(const uint2 *runs, const uint32_t *ovf_runs, const uint16_t *row_loc,
                                const void *w_pos, void *w_row, uint64_t n, uint32_t parts, uint32_t tile,
                                uint32_t *status, hipStream_t s, bool w16) {
  if (n == 0) return hipSuccess;
  if (tile > kUnsplitMaxTile || parts > (uint32_t)kUnsplitThreads) return hipErrorInvalidValue;
  const uint64_t n_tiles = (n + tile - 1) / tile;
  const dim3 grid((unsigned)n_tiles);
  if (parts <= (uint32_t)CCJ_UNSPLIT_NT) {  // one partition per thread in the runs' scan
    constexpr int NT = CCJ_UNSPLIT_NT;
    if (w16)
      hipLaunchKernelGGL((unsplit_words<uint16_t, NT>), grid, dim3(NT), 0, s, runs, ovf_runs, row_loc,
                         (const uint16_t *)w_pos, (uint16_t *)w_row, n, parts, tile, status);
    else
      hipLaunchKernelGGL((unsplit_words<uint32_t, NT>), grid, dim3(NT), 0, s, runs, ovf_runs, row_loc,
                         (const uint32_t *)w_pos, (uint32_t *)w_row, n, parts, tile, status);
    return hipGetLastError();
  }
  if (w16)
    hipLaunchKernelGGL((unsplit_words<uint16_t, kUnsplitThreads>), grid, dim3(kUnsplitThreads), 0, s, runs, ovf_runs,
                       row_loc, (const uint16_t *)w_pos, (uint16_t *)w_row, n, parts, tile, status);
  else
    hipLaunchKernelGGL((unsplit_words<uint32_t, kUnsplitThreads>), grid, dim3(kUnsplitThreads), 0, s, runs, ovf_runs,
                       row_loc, (const uint32_t *)w_pos, (uint32_t *)w_row, n, parts, tile, status);
  return hipGetLastError();
}

hipError_t launch_ordered_emit(int kind, const ProbeParams &p, hipStream_t s) {
  if (p.n_chunks == 0) return hipSuccess;
  if (kind == CCJ_TABLE_CHAIN)
    hipLaunchKernelGGL(emit_ordered<CCJ_TABLE_CHAIN>, dim3((unsigned)p.n_chunks), dim3(kBlock), 0, s, p);
  else
    hipLaunchKernelGGL(emit_ordered<CCJ_TABLE_LP>, dim3((unsigned)p.n_chunks), dim3(kBlock), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_probe(int kind, const ProbeParams &p, hipStream_t s) {
  if (p.n_chunks == 0) return hipSuccess;
  return kind == CCJ_TABLE_LP ? launch_kind<CCJ_TABLE_LP>(p, s) : launch_kind<CCJ_TABLE_CHAIN>(p, s);
}

hipError_t launch_gen_reference_keys(int64_t *out, uint64_t first, uint64_t n, uint64_t n_total, uint64_t cf,
                                     hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t num_unique = n_total / cf + (n_total % cf != 0);
  const uint64_t step = n_total / num_unique;
  hipLaunchKernelGGL(gen_reference_keys, dim3(grid_for(n, 256)), dim3(256), 0, s, out, first, n, cf, step);
  return hipGetLastError();
}

__global__ void iota_u32(uint32_t *p, uint64_t n) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x)
    p[t] = (uint32_t)t;
}

hipError_t launch_iota_u32(uint32_t *p, uint64_t n, hipStream_t s) {
  hipLaunchKernelGGL(iota_u32, dim3(grid_for(n, 256)), dim3(256), 0, s, p, n);
  return hipGetLastError();
}

// Device-to-device copy for the measured HBM copy ceiling ("report a measured
// STREAM-copy ceiling on the box"): one 16-byte non-temporal load and store per thread, one
// workgroup per 4 KiB (no grid-stride loop).  tools/copybench.hip on the box (4 GiB, read + write
// bytes / time; profiles/r4_copybench.log): this form 6.59 TB/s; plain loads / stores 6.29;
// grid-stride persistent grids (8-32 workgroups per CU, 1-8 loads in flight per thread) 4.9-5.7 —
// round 3's copy16 was one of those (5.16).
__global__ __launch_bounds__(256) void copy16(const u32x4 *src, u32x4 *dst, uint64_t n16) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

hipError_t launch_copy16(const void *src, void *dst, uint64_t n16, hipStream_t s) {
  if (n16 == 0) return hipSuccess;
  const uint64_t grid = (n16 + 255) / 256;
  if (grid > 0xFFFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(copy16, dim3((unsigned)grid), dim3(256), 0, s, (const u32x4 *)src, (u32x4 *)dst, n16);
  return hipGetLastError();
}

hipError_t launch_fill(int64_t *p, uint64_t n, int64_t v, hipStream_t s) {
  hipLaunchKernelGGL(fill_i64, dim3(grid_for(n, 256)), dim3(256), 0, s, p, n, v);
  return hipGetLastError();
}

hipError_t launch_lp_insert(const int64_t *keys, uint64_t n, int64_t *slots, uint32_t *slot_row, uint32_t mask,
                            hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(lp_insert, dim3(grid_for(n, 256)), dim3(256), 0, s, keys, n, slots, slot_row, mask);
  return hipGetLastError();
}

hipError_t launch_scatter_payload(const int64_t *src, uint32_t n_cols, const uint32_t *row, uint64_t positions,
                                  int64_t *dst, hipStream_t s) {
  if (positions == 0 || n_cols == 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_payload, dim3(grid_for(positions * n_cols, 256)), dim3(256), 0, s, src, n_cols, row,
                     positions, dst);
  return hipGetLastError();
}

hipError_t launch_gen_c3(int64_t *out, uint64_t n, uint64_t seed, uint64_t first_row, uint64_t n_build, uint64_t cf,
                         uint32_t hit_ppm, const uint32_t *zipf, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(gen_c3, dim3(grid_for(n, 256)), dim3(256), 0, s, out, n, seed, first_row, n_build, cf, hit_ppm,
                     zipf);
  return hipGetLastError();
}

hipError_t launch_gen_uniform(int64_t *out, uint64_t n, uint64_t seed, uint64_t first_row, uint64_t range,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(gen_uniform, dim3(grid_for(n, 256)), dim3(256), 0, s, out, n, seed, first_row, range);
  return hipGetLastError();
}

hipError_t launch_probe_cost(int kind, const int64_t *table, const uint32_t *off, uint32_t mask,
                             const int64_t *keys, uint64_t n, unsigned long long *acc, hipStream_t s, bool walk) {
  if (n == 0) return hipSuccess;
  const dim3 g(grid_for(n, 256)), b(256);
  if (kind == CCJ_TABLE_LP) {
    if (walk) hipLaunchKernelGGL((probe_cost<CCJ_TABLE_LP, true>), g, b, 0, s, table, off, mask, keys, n, acc);
    else hipLaunchKernelGGL((probe_cost<CCJ_TABLE_LP, false>), g, b, 0, s, table, off, mask, keys, n, acc);
  } else {
    if (walk) hipLaunchKernelGGL((probe_cost<CCJ_TABLE_CHAIN, true>), g, b, 0, s, table, off, mask, keys, n, acc);
    else hipLaunchKernelGGL((probe_cost<CCJ_TABLE_CHAIN, false>), g, b, 0, s, table, off, mask, keys, n, acc);
  }
  return hipGetLastError();
}

hipError_t launch_probe_visits(int kind, const int64_t *table, const uint32_t *off, uint32_t mask,
                               const int64_t *keys, const uint32_t *sel, uint32_t count, uint32_t max_rounds,
                               int64_t *vals, uint32_t *len, hipStream_t s) {
  if (count == 0) return hipSuccess;
  const dim3 g((count + 255) / 256), b(256);
  if (kind == CCJ_TABLE_LP)
    hipLaunchKernelGGL(probe_visits<CCJ_TABLE_LP>, g, b, 0, s, table, off, mask, keys, sel, count, max_rounds, vals, len);
  else
    hipLaunchKernelGGL(probe_visits<CCJ_TABLE_CHAIN>, g, b, 0, s, table, off, mask, keys, sel, count, max_rounds, vals, len);
  return hipGetLastError();
}

hipError_t launch_result_checksum(const uint32_t *count, const uint32_t *sel, const int64_t *payload,
                                  uint64_t n_chunks, uint64_t cap, uint32_t chunk, uint64_t row_base,
                                  const uint64_t *row_map, unsigned long long *acc, hipStream_t s) {
  if (n_chunks == 0) return hipSuccess;
  hipLaunchKernelGGL(result_checksum, dim3(grid_for(n_chunks, 4)), dim3(256), 0, s, count, sel, payload, n_chunks,
                     cap, chunk, row_base, row_map, acc);
  return hipGetLastError();
}

namespace {
// Largest multiplicity of one key in an LP slot array: all copies of a key share a home slot and
// so sit in one run; the first copy counts the equal keys from itself to the run's end.
__global__ void lp_max_dup(const int64_t *slots, uint64_t n_slots, uint32_t max_run, uint32_t *out) {
  uint32_t best = 0;
  const uint64_t mask = n_slots - 1;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_slots;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t k = slots[i];
    if (k == -1) continue;
    uint32_t c = 1;
    for (uint32_t t = 1; t <= max_run; ++t) {
      const int64_t v = slots[(i + t) & mask];
      if (v == -1) break;
      c += v == k;
    }
    best = c > best ? c : best;
  }
  for (int d = 32; d > 0; d >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)best, d);
    best = o > best ? o : best;
  }
  if ((threadIdx.x & 63u) == 0 && best) atomicMax(out, best);
}
}  // namespace

hipError_t launch_lp_max_dup(const int64_t *slots, uint64_t n_slots, uint32_t max_run, uint32_t *out, hipStream_t s) {
  hipError_t e = hipMemsetAsync(out, 0, sizeof(uint32_t), s);
  if (e != hipSuccess || n_slots == 0) return e;
  const uint64_t want = (n_slots + 255) / 256;
  hipLaunchKernelGGL(lp_max_dup, dim3((unsigned)(want < 8192 ? want : 8192)), dim3(256), 0, s, slots, n_slots,
                     max_run, out);
  return hipGetLastError();
}

hipError_t launch_lp_runs(const int64_t *slots, uint64_t n_slots, uint32_t *seg_stats, hipStream_t s) {
  const uint64_t n_seg = (n_slots + kRunSegment - 1) / kRunSegment;
  hipLaunchKernelGGL(lp_runs, dim3((unsigned)((n_seg + 3) / 4)), dim3(256), 0, s, slots, n_slots, seg_stats);
  return hipGetLastError();
}

}  // namespace ccj
