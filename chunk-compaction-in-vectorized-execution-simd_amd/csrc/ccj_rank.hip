// ccj_rank.hip — the rank walk: the LP walk of slot-partitioned input with each partition's table
// window resolved in LDS (the north star's "LDS-staged bucket windows for linear probing").
//
// The reference walks slots_[h], slots_[h+1], ... until an empty slot (linear_probing_ht.cpp:72-80,
// :100-110), so a probe row's candidates are exactly the occupied slots of the run starting at its
// home slot h, in slot order.  That run is a property of the table's occupancy alone.  With the
// table's window index (built once with the table, untimed like the build, main.cpp:62-68):
//   occ[w]   bit b = slot 64w + b occupied            (size / 8 bytes)
//   pre[b]   occupied slots before slot 128b          (size / 32 bytes)
//   ckeys[i] the i-th occupied slot's key, slot order (n_keys x 8 bytes: 1/4 of the slot array at C2)
// a row's run is L = (first zero bit of occ at or after h) - h occupied slots, and its candidate
// keys are ckeys[rank(h) .. rank(h) + L), rank(h) = pre[h >> 7] + popcount(occ below h in its
// 128-slot block).  A window of 2^19 slots needs 64 KiB of occ + 16 KiB of pre: the workgroup holds the whole window's
// index in LDS, so the run boundaries cost no memory request, and the key reads go to a 1 MiB
// slice of ckeys (the slot window itself is 4 MiB, the whole of an XCD's L2) — one request per row
// for runs of up to 4 keys in one 128-byte line.
//
// probe_rank: one persistent 768-thread workgroup per CU.  The workgroups on XCD x (blockIdx % 8)
// take partitions [x P/8, (x+1) P/8) one after another; for each, the workgroup loads the window's
// index into LDS and its 12 waves take 512-row blocks of the partition's 8 segments from a
// per-partition counter (the next block is claimed while the current one is walked).  A wave
// stages its block's keys with their (rank, L) in LDS, then walks it with probe_walk's lane-pair
// engine (16 B per lane, R rows per pair, a wave-uniform row cursor) over ckeys.  Rows whose run
// reaches the window's end continue on the slot array (rare).  Per block it leaves a 512-bit hit
// mask and the hit count; rank_finish turns them into the chunk's count and compacts (in place)
// the chunks where a row missed.  Tables of distinct keys only (max_dup 1: a row matches at most
// once), with the partitioned keys in out_payload (cap == chunk).
#include <hip/hip_runtime.h>

#include <cstdio>

#include "ccj_internal.h"
#include "ccj_tuning.h"

namespace ccj {
namespace {

// Shape (round-2 sweep at C2, step ms with the split: waves x block rows x R): 12 x 512 x 6 14.8,
// 12 x 512 x 8 15.6, 16 x 256 x 4 15.7, 16 x 256 x 6 16.3, 12 x 512 x 4 17.2, 8 x 512 x 3 19.3.
#ifndef CCJ_RANK_WAVES
#define CCJ_RANK_WAVES 12
#define CCJ_RANK_BLOCK 512
#endif
constexpr uint32_t kRankWaves = CCJ_RANK_WAVES;  // 768 threads: one workgroup per CU (152 KiB of LDS)
constexpr uint32_t kRankBlock = CCJ_RANK_BLOCK;  // rows per wave block (8 per lane)
constexpr uint32_t kRankMaxWords = 8192;     // occ words of a 2^19-slot window
constexpr uint32_t kRankSlow = 8191u;        // run reaches the window's end: walk the slot array
constexpr uint32_t kRankRelBits = 19;        // staged row: rank in the window (19 bits) | L << 19
#ifndef CCJ_RANK_R
#define CCJ_RANK_R 6
#endif
constexpr int kRankR = CCJ_RANK_R;           // rows per lane pair in flight

struct RankParams {
  const int64_t *keys;     // partitioned column
  const int64_t *table;    // slot array (rows whose run leaves the window)
  const uint64_t *occ;
  const uint32_t *pre;
  const int64_t *ckeys;
  uint32_t mask, wbits, parts;
  uint64_t seg_cap;
  const uint32_t *seg_count;  // the split's cursors: seg_count[seg_cursor_index(parts, g, d)]
  uint32_t *ctr;              // per-partition block counters (zeroed before the launch)
  uint64_t *hit_words;        // 8 per 512-row block of the segment area
  uint32_t *blk_hits;         // per block
  unsigned long long *stats;  // tuning build only (CCJ_STATS): rows, slow rows, walk loads, blocks
};

__device__ __forceinline__ uint32_t rk_lane_prefix(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ void rk_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct RankShared {
  uint64_t occ[kRankMaxWords];
  uint32_t pre[kRankMaxWords / 2];
  int64_t key[kRankWaves][kRankBlock];
  // rank - the window's first rank (19 bits) | run length in keys (or kRankSlow) << 19; after the
  // walk: the row's matches (slow rows keep kRankSlow << 19)
  uint32_t info[kRankWaves][kRankBlock];
  uint32_t nblk[9];  // cumulative blocks of the partition's 8 segments
  uint32_t live[8];  // live rows of the partition's 8 segments
};

// Stage block rows [0, m) at q0: keys, rank of the home slot, occupied run length in the window.
__device__ __forceinline__ void rank_stage(const RankParams &q, RankShared &sm, uint32_t wave, uint64_t q0,
                                           uint32_t m, uint32_t lane, uint64_t win0, uint32_t words) {
  constexpr int kJ = (int)(kRankBlock / kWave);
  int64_t v[kJ];
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const uint32_t i = (uint32_t)j * kWave + lane;
    v[j] = i < m ? __builtin_nontemporal_load(q.keys + q0 + i) : 0;
  }
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const uint32_t i = (uint32_t)j * kWave + lane;
    if (i >= m) continue;
    const uint64_t o = (uint64_t)((uint32_t)murmurhash64((uint64_t)v[j]) & q.mask) - win0;
    uint32_t r = 0, L = kRankSlow;
    if (o < ((uint64_t)words << 6)) {  // (always, for rows the split put in this partition)
      const uint32_t w = (uint32_t)(o >> 6), b = (uint32_t)(o & 63);
      const ulonglong2 pr = *reinterpret_cast<const ulonglong2 *>(&sm.occ[w & ~1u]);  // the 128-slot block
      const uint64_t x = (w & 1u) ? pr.y : pr.x;
      r = sm.pre[w >> 1] - sm.pre[0] + ((w & 1u) ? (uint32_t)__popcll(pr.x) : 0u) +
          (uint32_t)__popcll(x & ((1ull << b) - 1ull));
      const uint64_t y = ~x >> b;
      if (y) {
        L = (uint32_t)__builtin_ctzll(y);
      } else {  // the run continues past this word
        L = 64u - b;
        uint32_t ww = w + 1;
        for (; ww < words; ++ww) {
          const uint64_t z = ~sm.occ[ww];
          if (z) {
            L += (uint32_t)__builtin_ctzll(z);
            break;
          }
          L += 64u;
        }
        if (ww >= words || L >= kRankSlow) L = kRankSlow;  // leaves the window
      }
    }
    sm.key[wave][i] = v[j];
    sm.info[wave][i] = r | L << kRankRelBits;
  }
  rk_wave_sync();
}

// probe_walk's lane-pair engine over ckeys: each row's L candidates from its rank, 4-key windows
// that never cross a 128-byte line (one L2 request), the lane pair's halves joined by one DPP swap.
// A finished row leaves its match count in sm.info (slow rows keep kRankSlow << 19).
__device__ __forceinline__ void rank_walk(const RankParams &q, RankShared &sm, uint32_t wave, uint32_t m,
                                          uint32_t lane) {
  const uint32_t sub = lane & 1u, pair = lane >> 1;
  int64_t key[kRankR];
  uint32_t row[kRankR], r[kRankR], rem[kRankR], cnt[kRankR];
  uint32_t need = 0, slow = 0;
  const uint32_t rank0 = sm.pre[0];  // the window's first rank
  auto start = [&](int k, uint32_t i) {
    row[k] = i;
    cnt[k] = 0;
    rem[k] = 0;
    if (i < m) {
      key[k] = sm.key[wave][i];
      const uint32_t inf = sm.info[wave][i];
      r[k] = rank0 + (inf & ((1u << kRankRelBits) - 1u));
      const uint32_t L = inf >> kRankRelBits;
      if (L == kRankSlow) slow |= 1u << k;
      else rem[k] = L;
      need |= 1u << k;
    }
  };
#pragma unroll
  for (int k = 0; k < kRankR; ++k) {
    key[k] = 0;
    r[k] = 0;
    start(k, (uint32_t)k * (kWave / 2) + pair);
  }
  uint32_t next = (uint32_t)kRankR * (kWave / 2);  // wave-uniform: the next unwalked row
  while (__ballot(need != 0u) != 0ull) {
    int64_t v0[kRankR], v1[kRankR];
    uint32_t st[kRankR];
#pragma unroll
    for (int k = 0; k < kRankR; ++k) {
      uint32_t s = r[k];
      const uint32_t lim = (s & ~15u) + 12u;  // the 4-key window ends at its 128-byte line
      s = s < lim ? s : lim;
      st[k] = s;
      // unconditional (a predicated load makes the compiler wait for it before the next row's):
      // an idle row reads the window's first line, never used
      const longlong2 x = *reinterpret_cast<const longlong2 *>(q.ckeys + (((need >> k) & 1u) && rem[k] ? s + 2 * sub : rank0));
      v0[k] = x.x;
      v1[k] = x.y;
    }
#ifdef CCJ_TUNING
    if (q.stats) {
      uint32_t nl = 0;
#pragma unroll
      for (int k = 0; k < kRankR; ++k) nl += (uint32_t)__popcll(__ballot(!sub && ((need >> k) & 1u) && rem[k]));
      if (lane == 0) atomicAdd(&q.stats[2], (unsigned long long)nl);
    }
#endif
    uint32_t done = 0;
#pragma unroll
    for (int k = 0; k < kRankR; ++k) {
      uint32_t mm = (((v0[k] == key[k]) ? 1u : 0u) | ((v1[k] == key[k]) ? 2u : 0u)) << (2 * sub);
      mm |= (uint32_t)__builtin_amdgcn_mov_dpp((int)mm, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
      if ((need >> k) & 1u) {
        if (rem[k] == 0) {
          done |= 1u << k;  // home slot empty (a miss without a read) or a slow row
        } else {
          const uint32_t off = r[k] - st[k];
          const uint32_t nv = 4u - off < rem[k] ? 4u - off : rem[k];
          cnt[k] += (uint32_t)__builtin_popcount((mm >> off) & ((1u << nv) - 1u));
          rem[k] -= nv;
          r[k] += nv;
          if (rem[k] == 0) done |= 1u << k;
        }
      }
    }
    const uint32_t nd = (uint32_t)__builtin_popcount(done);
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int b = 0; (1 << b) <= kRankR; ++b) {
      const uint64_t bm = __ballot(((nd >> b) & 1u) && !sub);
      pre += rk_lane_prefix(bm) << b;
      tot += (uint32_t)__popcll(bm) << b;
    }
    if (tot) {
      pre = (uint32_t)__builtin_amdgcn_mov_dpp((int)pre, 0xA0, 0xF, 0xF, false);  // the pair's even lane's
      uint32_t rb = next + pre;
#pragma unroll
      for (int k = 0; k < kRankR; ++k) {
        if ((done >> k) & 1u) {
          need &= ~(1u << k);
          if (!sub && !((slow >> k) & 1u)) sm.info[wave][row[k]] = cnt[k];
          slow &= ~(1u << k);
          start(k, rb++);
        }
      }
      next += tot;
    }
  }
  rk_wave_sync();
}

__global__ __launch_bounds__(kWave * kRankWaves) void probe_rank(RankParams q) {
  __shared__ RankShared sm;
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const uint32_t grp = blockIdx.x & 7u;
  const uint32_t d_lo = (uint32_t)((uint64_t)q.parts * grp / 8), d_hi = (uint32_t)((uint64_t)q.parts * (grp + 1) / 8);
  const uint32_t words = 1u << (q.wbits - 6);
  for (uint32_t d = d_lo; d < d_hi; ++d) {
    __syncthreads();  // the previous window's walkers are done with the LDS index
    for (uint32_t i = tid; i < words; i += kWave * kRankWaves) {
      sm.occ[i] = q.occ[(uint64_t)d * words + i];
      if (i < words / 2) sm.pre[i] = q.pre[(uint64_t)d * (words / 2) + i];
    }
    if (tid == 0) {
      uint32_t acc = 0;
      sm.nblk[0] = 0;
      for (uint32_t g = 0; g < 8; ++g) {
        uint64_t live = q.seg_count[seg_cursor_index(q.parts, g, d)];
        live = live < q.seg_cap ? live : q.seg_cap;
        sm.live[g] = (uint32_t)live;
        acc += (uint32_t)((live + kRankBlock - 1) / kRankBlock);
        sm.nblk[g + 1] = acc;
      }
    }
    __syncthreads();
    const uint32_t total = sm.nblk[8];
    const uint64_t win0 = (uint64_t)d << q.wbits;
    uint32_t claim = 0;
    if (lane == 0) claim = atomicAdd(&q.ctr[d], 1u);
    uint32_t b = (uint32_t)__builtin_amdgcn_readfirstlane((int)claim);
    while (b < total) {
      if (lane == 0) claim = atomicAdd(&q.ctr[d], 1u);  // the next block, claimed under this one's walk
      uint32_t g = 0;
#pragma unroll
      for (uint32_t x = 1; x < 8; ++x) g += b >= sm.nblk[x] ? 1u : 0u;
      const uint32_t k = b - sm.nblk[g];
      const uint64_t seg = (uint64_t)d * 8 + g;
      const uint64_t live = sm.live[g];
      const uint64_t off = (uint64_t)k * kRankBlock;
      const uint32_t m = live - off < kRankBlock ? (uint32_t)(live - off) : kRankBlock;
      const uint64_t q0 = seg * q.seg_cap + off;
      rank_stage(q, sm, wave, q0, m, lane, win0, words);
#ifdef CCJ_TUNING
      if (q.stats) {
        uint32_t ns = 0;
        for (uint32_t i = lane; i < m; i += kWave) ns += (sm.info[wave][i] >> kRankRelBits) == kRankSlow ? 1u : 0u;
        for (int dd = 32; dd > 0; dd >>= 1) ns += (uint32_t)__shfl_xor((int)ns, dd);
        if (lane == 0) {
          atomicAdd(&q.stats[0], (unsigned long long)m);
          atomicAdd(&q.stats[1], (unsigned long long)ns);
          atomicAdd(&q.stats[3], 1ull);
        }
      }
#endif
      rank_walk(q, sm, wave, m, lane);
      // rows whose run leaves the window: the slot array from the home slot (reference order)
#pragma unroll
      for (int j = 0; j < (int)(kRankBlock / kWave); ++j) {
        const uint32_t i = (uint32_t)j * kWave + lane;
        if (i < m && (sm.info[wave][i] >> kRankRelBits) == kRankSlow) {
          const int64_t kk = sm.key[wave][i];
          uint32_t s = (uint32_t)murmurhash64((uint64_t)kk) & q.mask, c = 0;
          for (uint64_t n = 0; n <= q.mask; ++n) {
            const int64_t v = q.table[s];
            if (v == -1) break;
            c += v == kk ? 1u : 0u;
            s = (s + 1) & q.mask;
          }
          sm.info[wave][i] = c;
        }
      }
      rk_wave_sync();
      uint64_t word = 0;
      uint32_t hits = 0;
#pragma unroll
      for (int j = 0; j < (int)(kRankBlock / kWave); ++j) {
        const uint32_t i = (uint32_t)j * kWave + lane;
        const uint64_t bm = __ballot(i < m && sm.info[wave][i] != 0);
        word = lane == (uint32_t)j ? bm : word;
        hits += (uint32_t)__popcll(bm);
      }
      const uint64_t blk = q0 / kRankBlock;
      if (lane < kRankBlock / kWave) q.hit_words[blk * (kRankBlock / kWave) + lane] = word;
      if (lane == 0) q.blk_hits[blk] = hits;
      rk_wave_sync();  // the block's LDS rows are read before the next block's stage
      b = (uint32_t)__builtin_amdgcn_readfirstlane((int)claim);
    }
  }
}

// rank_finish: one wave per chunk of the segment area.  count = the chunk's blocks' hits; a chunk
// where a row missed is compacted in place in row order (sel: the split's original rows with
// rows_in_sel, else the row's position in the chunk; payload: the key the split left there);
// without rows_in_sel a full chunk's sel is the identity.
struct FinishParams {
  const uint32_t *seg_count;
  uint32_t parts;
  uint64_t seg_cap;
  uint32_t chunk;
  uint64_t n_chunks;
  const uint64_t *hit_words;
  const uint32_t *blk_hits;
  uint32_t *out_count;
  uint32_t *out_sel;
  int64_t *out_payload;
  uint32_t rows_in_sel;
};

__global__ __launch_bounds__(256) void rank_finish(FinishParams f) {
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint64_t c = (uint64_t)blockIdx.x * 4 + threadIdx.x / kWave;
  if (c >= f.n_chunks) return;
  const uint64_t base = c * f.chunk;
  const uint64_t seg = base / f.seg_cap;
  const uint64_t soff = base - seg * f.seg_cap;
  uint64_t live = f.seg_count[seg_cursor_index(f.parts, (uint32_t)(seg & 7), (uint32_t)(seg >> 3))];
  live = live < f.seg_cap ? live : f.seg_cap;
  const uint32_t phys = live > soff ? (live - soff < f.chunk ? (uint32_t)(live - soff) : f.chunk) : 0u;
  const uint64_t blk0 = base / kRankBlock;
  const uint32_t nb = (phys + kRankBlock - 1) / kRankBlock;
  uint32_t count = 0;
  for (uint32_t b = 0; b < nb; ++b) count += f.blk_hits[blk0 + b];
  if (lane == 0) f.out_count[c] = count;
  if (count == phys) {
    if (!f.rows_in_sel)
      for (uint32_t i = lane; i < phys; i += kWave) __builtin_nontemporal_store(i, f.out_sel + base + i);
    return;
  }
  uint32_t t = 0;
  for (uint32_t j = 0; j * kWave < phys; ++j) {
    const uint32_t i = j * kWave + lane;
    const uint64_t word = f.hit_words[blk0 * (kRankBlock / kWave) + j];
    const bool hit = i < phys && ((word >> lane) & 1ull);
    uint32_t sv = i;
    int64_t pv = 0;
    if (hit) {
      pv = f.out_payload[base + i];
      if (f.rows_in_sel) sv = f.out_sel[base + i];
    }
    const uint64_t bm = __ballot(hit);
    const uint64_t o = base + t + rk_lane_prefix(bm);  // <= base + i: every entry moves down
    if (hit) {
      f.out_payload[o] = pv;
      f.out_sel[o] = sv;
    }
    t += (uint32_t)__popcll(bm);
  }
}

__global__ void rank_occ(const int64_t *slots, uint64_t n_slots, uint64_t *occ, uint32_t *cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t bm = __ballot(i < n_slots && slots[i] != -1);
  if ((threadIdx.x & (kWave - 1)) == 0 && i < n_slots) {
    occ[i >> 6] = bm;
    cnt[i >> 6] = (uint32_t)__popcll(bm);
  }
}

__global__ void rank_compact_keys(const int64_t *slots, uint64_t n_slots, const uint64_t *occ, const uint32_t *pre,
                                  int64_t *ckeys) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_slots) return;
  const int64_t v = slots[i];
  if (v == -1) return;
  const uint64_t w = i >> 6;
  ckeys[pre[w >> 1] + ((w & 1) ? __popcll(occ[w - 1]) : 0) + __popcll(occ[w] & ((1ull << (i & 63)) - 1ull))] = v;
}

}  // namespace

bool rank_walk_fits(uint32_t window_bits) { return window_bits >= 7 && window_bits <= 19; }

hipError_t launch_rank_index(const int64_t *slots, uint64_t n_slots, uint64_t *occ, uint32_t *pre, uint32_t *cnt,
                             hipStream_t s) {
  if (n_slots % 64) return hipErrorInvalidValue;
  const unsigned g = (unsigned)((n_slots + 255) / 256);
  hipLaunchKernelGGL(rank_occ, dim3(g), dim3(256), 0, s, slots, n_slots, occ, cnt);
  hipError_t e = hipGetLastError();
  if (e) return e;
  // pre = exclusive scan of the 128-slot blocks' counts (on the host: a build-time step)
  if (n_slots % 128) return hipErrorInvalidValue;
  const uint64_t words = n_slots / 64;
  uint32_t *h = nullptr;
  e = hipHostMalloc((void **)&h, words * 4);
  if (e) return e;
  e = hipMemcpyAsync(h, cnt, words * 4, hipMemcpyDeviceToHost, s);
  if (!e) e = hipStreamSynchronize(s);
  if (!e) {
    uint32_t acc = 0;
    for (uint64_t b = 0; b < words / 2; ++b) {
      const uint32_t x = h[2 * b] + h[2 * b + 1];
      h[b] = acc;
      acc += x;
    }
    e = hipMemcpyAsync(pre, h, words / 2 * 4, hipMemcpyHostToDevice, s);
    if (!e) e = hipStreamSynchronize(s);
  }
  (void)hipHostFree(h);
  return e;
}

hipError_t launch_rank_compact_keys(const int64_t *slots, uint64_t n_slots, const uint64_t *occ, const uint32_t *pre,
                                    int64_t *ckeys, hipStream_t s) {
  const unsigned g = (unsigned)((n_slots + 255) / 256);
  hipLaunchKernelGGL(rank_compact_keys, dim3(g), dim3(256), 0, s, slots, n_slots, occ, pre, ckeys);
  return hipGetLastError();
}

size_t rank_workspace(uint64_t positions, uint32_t parts) {
  const uint64_t blocks = (positions + kRankBlock - 1) / kRankBlock;
  auto a = [](uint64_t b) { return (b + 255) & ~255ull; };
  return a(blocks * 64) + a(blocks * 4) + a((uint64_t)parts * 4);
}

// p: the walk's parameters after the split (seg_count, seg_parts, seg_cap, ovf_base, keys ==
// out_payload); the segment area's chunks take probe_rank + rank_finish, the overflow area's
// probe_walk.
hipError_t launch_probe_rank(const ProbeParams &p, const RankIndex &ix, void *ws, hipStream_t s) {
  static const unsigned cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return (unsigned)(n >= 8 ? n / 8 * 8 : 8);
  }();
  const uint64_t seg_positions = p.ovf_base;
  const uint64_t blocks = (seg_positions + kRankBlock - 1) / kRankBlock;
  auto a = [](uint64_t b) { return (b + 255) & ~255ull; };
  RankParams q{};
  q.keys = p.keys;
  q.table = p.table;
  q.occ = ix.occ;
  q.pre = ix.pre;
  q.ckeys = ix.ckeys;
  q.mask = p.mask;
  q.wbits = ix.wbits;
  q.parts = p.seg_parts;
  q.seg_cap = p.seg_cap;
  q.seg_count = p.seg_count;
  q.hit_words = (uint64_t *)ws;
  q.blk_hits = (uint32_t *)((char *)ws + a(blocks * 64));
  q.ctr = (uint32_t *)((char *)ws + a(blocks * 64) + a(blocks * 4));
  hipError_t e = hipMemsetAsync(q.ctr, 0, (size_t)q.parts * 4, s);
  if (e) return e;
#ifdef CCJ_TUNING
  static unsigned long long *stats = nullptr;
  if (ccj_tune_env("CCJ_STATS")) {
    if (!stats && (e = hipMalloc((void **)&stats, 8 * sizeof(unsigned long long)))) return e;
    if ((e = hipMemsetAsync(stats, 0, 8 * sizeof(unsigned long long), s))) return e;
    q.stats = stats;
  }
#endif
  hipLaunchKernelGGL(probe_rank, dim3(cus), dim3(kWave * kRankWaves), 0, s, q);
  if ((e = hipGetLastError())) return e;
#ifdef CCJ_TUNING
  if (q.stats) {
    unsigned long long h[8];
    if ((e = hipMemcpyAsync(h, q.stats, sizeof(h), hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s))) return e;
    fprintf(stderr, "[rank stats] rows %llu slow %llu walk loads %llu (%.3f per row) blocks %llu\n", h[0], h[1], h[2],
            h[0] ? (double)h[2] / (double)h[0] : 0.0, h[3]);
  }
#endif
  FinishParams f{};
  f.seg_count = p.seg_count;
  f.parts = p.seg_parts;
  f.seg_cap = p.seg_cap;
  f.chunk = p.chunk;
  f.n_chunks = seg_positions / p.chunk;
  f.hit_words = q.hit_words;
  f.blk_hits = q.blk_hits;
  f.out_count = p.out_count;
  f.out_sel = p.out_sel;
  f.out_payload = p.out_payload;
  f.rows_in_sel = p.rows_in_sel;
  if (f.n_chunks) {
    hipLaunchKernelGGL(rank_finish, dim3((unsigned)((f.n_chunks + 3) / 4)), dim3(256), 0, s, f);
    if ((e = hipGetLastError())) return e;
  }
  if (p.n_chunks > f.n_chunks) {  // the overflow area: rows of any partition, the slot-array walk
    ProbeParams o = p;
    o.chunk0 = f.n_chunks;
    o.n_chunks = p.n_chunks - f.n_chunks;
    o.xcd_swizzle = 0;
    o.swz_chunks = 0;
    return launch_probe_flat(CCJ_TABLE_LP, o, s);
  }
  return hipSuccess;
}

}  // namespace ccj
