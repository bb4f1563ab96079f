// proto_scatter.hip — timing prototype: one-pass slot-range split of a probe column into
// 2^PBITS partitions x 8 XCD groups of fixed capacity (atomic reservation per tile), against the
// two-pass exact split.  Not part of the library; tools/ scratch for design decisions.
//   hipcc -O3 --offload-arch=gfx950 -I../include -I../chunk-compaction-in-vectorized-execution-simd_amd/csrc proto_scatter.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ccj_internal.h"

using ccj::murmurhash64;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_) {                                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void gen(int64_t *k, uint64_t n, uint64_t range) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t z = i * 0x9E3779B97F4A7C15ull + 42;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  k[i] = (int64_t)(z % range);
}

template <int NT, int PER, int PBITS>
__global__ __launch_bounds__(NT) void scatter1(const int64_t *keys, uint64_t n, uint32_t shift, uint64_t n_tiles,
                                               uint32_t *cur, uint64_t cap, int64_t *out_k, uint32_t *out_r,
                                               uint32_t *status) {
  constexpr int T = NT * PER, P = 1 << PBITS, DPT = P / NT > 0 ? P / NT : 1;
  __shared__ int64_t s_k[T];
  __shared__ uint32_t s_r[T];
  __shared__ uint16_t s_d[T];
  __shared__ uint32_t s_hist[P], s_loc[P], s_lim[P];
  __shared__ uint64_t s_dst[P];
  __shared__ uint32_t s_wsum[NT / 64];
  uint64_t tile = blockIdx.x;
  const uint32_t g = blockIdx.x & 7;
  const uint64_t n8 = n_tiles & ~7ull;
  if (tile < n8) tile = (tile & 7) * (n8 >> 3) + (tile >> 3);
  const uint64_t t0 = tile * T;
  const uint32_t tn = (uint32_t)(n - t0 < (uint64_t)T ? n - t0 : T);
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < P; i += NT) s_hist[i] = 0;
  int64_t kk[PER];
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const uint32_t li = it * NT + tid;
    kk[it] = li < tn ? __builtin_nontemporal_load(keys + t0 + li) : 0;
  }
  __syncthreads();
  uint32_t dd[PER], rk[PER];
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const uint32_t li = it * NT + tid;
    dd[it] = (uint32_t)(murmurhash64((uint64_t)kk[it]) >> shift) & (P - 1);
    if (li < tn) rk[it] = atomicAdd(&s_hist[dd[it]], 1u);
  }
  __syncthreads();
  // exclusive scan of s_hist: thread owns DPT consecutive digits
  uint32_t loc[DPT], sum = 0;
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const uint32_t d = tid * DPT + j;
    loc[j] = sum;
    sum += d < P ? s_hist[d] : 0;
  }
  uint32_t incl = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o);
    if (lane >= (uint32_t)o) incl += v;
  }
  if (lane == 63) s_wsum[wave] = incl;
  __syncthreads();
  uint32_t wpre = 0;
  for (uint32_t w = 0; w < wave; ++w) wpre += s_wsum[w];
  const uint32_t excl = wpre + incl - sum;
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const uint32_t d = tid * DPT + j;
    if (d < P) {
      const uint32_t h = s_hist[d];
      s_loc[d] = excl + loc[j];
      uint64_t b = 0;
      uint32_t lim = 0;
      if (h) {
        const uint64_t seg = (uint64_t)d * 8 + g;
        const uint32_t r = atomicAdd(&cur[seg], h);
        b = seg * cap + r;
        lim = r >= cap ? 0u : (uint32_t)(cap - r < h ? cap - r : h);
        if (lim < h) atomicOr(status, 1u);
      }
      s_dst[d] = b;
      s_lim[d] = lim;
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const uint32_t li = it * NT + tid;
    if (li < tn) {
      const uint32_t pos = s_loc[dd[it]] + rk[it];
      s_k[pos] = kk[it];
      s_r[pos] = (uint32_t)(t0 + li);
      s_d[pos] = (uint16_t)dd[it];
    }
  }
  __syncthreads();
  for (uint32_t q = tid; q < tn; q += NT) {
    const uint32_t d = s_d[q];
    const uint32_t o = q - s_loc[d];
    if (o < s_lim[d]) {
      const uint64_t dest = s_dst[d] + o;
      out_k[dest] = s_k[q];
      out_r[dest] = s_r[q];
    }
  }
}

// Persistent form: block b serves XCD group g = b & 7 and walks that group's tiles j, j + bpg, ...;
// the next tile's keys are loaded into registers while the current tile is written out, and the
// reservation atomics fly while the LDS image is built.  WRITE = false: ablation without stores.
template <int NT, int PER, int PBITS, bool WRITE>
__global__ __launch_bounds__(NT) void scatter2(const int64_t *keys, uint64_t n, uint32_t shift, uint64_t n_tiles,
                                               uint32_t *cur, uint64_t cap, int64_t *out_k, uint32_t *out_r,
                                               uint32_t *status, uint32_t bpg) {
  constexpr int T = NT * PER, P = 1 << PBITS, DPT = P / NT > 0 ? P / NT : 1;
  __shared__ int64_t s_k[T];
  __shared__ uint16_t s_i[T];
  __shared__ uint32_t s_hist[P], s_loc[P], s_lim[P];
  __shared__ uint64_t s_dst[P];
  __shared__ uint32_t s_wsum[NT / 64];
  const uint32_t g = blockIdx.x & 7, j = blockIdx.x >> 3;
  const uint64_t per_g = n_tiles / 8;
  const uint64_t tend = (g + 1) * per_g;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint64_t tile = g * per_g + j;
  int64_t kk[PER];
  auto load = [&](uint64_t t) {
    const uint64_t t0 = t * T;
    const uint32_t tn = (uint32_t)(n - t0 < (uint64_t)T ? n - t0 : T);
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const uint32_t li = it * NT + tid;
      kk[it] = li < tn ? __builtin_nontemporal_load(keys + t0 + li) : 0;
    }
  };
  if (tile < tend) load(tile);
  for (; tile < tend; tile += bpg) {
    const uint64_t t0 = tile * T;
    const uint32_t tn = (uint32_t)(n - t0 < (uint64_t)T ? n - t0 : T);
    for (int i = tid; i < P; i += NT) s_hist[i] = 0;
    __syncthreads();
    uint32_t dd[PER], rk[PER];
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const uint32_t li = it * NT + tid;
      dd[it] = (uint32_t)(murmurhash64((uint64_t)kk[it]) >> shift) & (P - 1);
      if (li < tn) rk[it] = atomicAdd(&s_hist[dd[it]], 1u);
    }
    __syncthreads();
    uint32_t loc[DPT], hh[DPT], sum = 0;
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      const uint32_t d = tid * DPT + q;
      hh[q] = d < P ? s_hist[d] : 0;
      loc[q] = sum;
      sum += hh[q];
    }
    uint32_t incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o);
      if (lane >= (uint32_t)o) incl += v;
    }
    if (lane == 63) s_wsum[wave] = incl;
    uint32_t res[DPT], rh[DPT];
#pragma unroll
    for (int q = 0; q < DPT; ++q) {  // reservations fly while the image is built; lanes take
      const uint32_t d = q * NT + tid;  // consecutive digits of the group-major cursor array
      rh[q] = d < P ? s_hist[d] : 0u;
      res[q] = rh[q] ? atomicAdd(&cur[(uint64_t)g * P + d], rh[q]) : 0u;
    }
    __syncthreads();
    uint32_t wpre = 0;
    for (uint32_t w = 0; w < wave; ++w) wpre += s_wsum[w];
    const uint32_t excl = wpre + incl - sum;
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      const uint32_t d = tid * DPT + q;
      if (d < P) s_loc[d] = excl + loc[q];
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const uint32_t li = it * NT + tid;
      if (li < tn) {
        const uint32_t pos = s_loc[dd[it]] + rk[it];
        s_k[pos] = kk[it];
        s_i[pos] = (uint16_t)li;
      }
    }
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      const uint32_t d = q * NT + tid;
      if (d < P) {
        const uint64_t seg = (uint64_t)d * 8 + g;
        const uint32_t r = res[q], h = rh[q];
        s_dst[d] = seg * cap + r;
        const uint32_t lim = r >= cap ? 0u : (uint32_t)(cap - r < h ? cap - r : h);
        s_lim[d] = lim;
        if (lim < h) atomicOr(status, 1u);
      }
    }
    __syncthreads();
    if (tile + bpg < tend) load(tile + bpg);
    for (uint32_t q = tid; q < tn; q += NT) {
      const int64_t k = s_k[q];
      const uint32_t d = (uint32_t)(murmurhash64((uint64_t)k) >> shift) & (P - 1);
      const uint32_t o = q - s_loc[d];
      if (WRITE && o < s_lim[d]) {
        const uint64_t dest = s_dst[d] + o;
        out_k[dest] = k;
        out_r[dest] = (uint32_t)(t0 + s_i[q]);
      }
    }
    __syncthreads();
  }
}

__global__ void check(const uint32_t *cur, uint32_t segs, uint64_t *tot) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < segs) atomicAdd((unsigned long long *)tot, (unsigned long long)cur[i]);
}

template <int NT, int PER, int PBITS>
void run(const char *name, const int64_t *keys, uint64_t n, uint32_t shift, uint32_t *cur, uint64_t cap,
         int64_t *ok, uint32_t *orow, uint32_t *st, int reps) {
  constexpr uint64_t T = NT * PER;
  const uint64_t n_tiles = (n + T - 1) / T;
  const uint32_t segs = (1u << PBITS) * 8;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e9, tot_ms = 0;
  for (int r = 0; r < reps + 1; ++r) {
    CK(hipMemsetAsync(cur, 0, segs * 4, 0));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((scatter1<NT, PER, PBITS>), dim3(n_tiles), dim3(NT), 0, 0, keys, n, shift, n_tiles, cur, cap, ok,
                       orow, st);
    CK(hipGetLastError());
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r) {
      best = ms < best ? ms : best;
      tot_ms += ms;
    }
  }
  uint64_t *dt;
  CK(hipMalloc(&dt, 8));
  CK(hipMemset(dt, 0, 8));
  hipLaunchKernelGGL(check, dim3((segs + 255) / 256), dim3(256), 0, 0, cur, segs, dt);
  uint64_t tot = 0;
  uint32_t s = 0;
  CK(hipMemcpy(&tot, dt, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&s, st, 4, hipMemcpyDeviceToHost));
  printf("%-14s tile %5llu parts %5u: best %.3f ms avg %.3f ms (%.2f TB/s at 20 B/key) rows %llu overflow %u\n", name,
         (unsigned long long)T, 1u << PBITS, best, tot_ms / reps, n * 20.0 / (best * 1e-3) / 1e12,
         (unsigned long long)tot, s);
  CK(hipFree(dt));
}

template <int NT, int PER, int PBITS, bool WRITE>
void run2(const char *name, const int64_t *keys, uint64_t n, uint32_t shift, uint32_t *cur, uint64_t cap,
          int64_t *ok, uint32_t *orow, uint32_t *st, int reps, uint32_t blocks) {
  constexpr uint64_t T = NT * PER;
  const uint64_t n_tiles = (n + T - 1) / T;
  const uint32_t segs = (1u << PBITS) * 8;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e9, tot_ms = 0;
  for (int r = 0; r < reps + 1; ++r) {
    CK(hipMemsetAsync(cur, 0, segs * 4, 0));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((scatter2<NT, PER, PBITS, WRITE>), dim3(blocks), dim3(NT), 0, 0, keys, n, shift, n_tiles, cur,
                       cap, ok, orow, st, blocks / 8);
    CK(hipGetLastError());
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r) {
      best = ms < best ? ms : best;
      tot_ms += ms;
    }
  }
  uint64_t *dt;
  CK(hipMalloc(&dt, 8));
  CK(hipMemset(dt, 0, 8));
  hipLaunchKernelGGL(check, dim3((segs + 255) / 256), dim3(256), 0, 0, cur, segs, dt);
  uint64_t tot = 0;
  uint32_t s = 0;
  CK(hipMemcpy(&tot, dt, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&s, st, 4, hipMemcpyDeviceToHost));
  printf("%-14s tile %5llu parts %5u blocks %4u: best %.3f ms avg %.3f ms (%.2f TB/s at 20 B/key) rows %llu overflow %u\n",
         name, (unsigned long long)T, 1u << PBITS, blocks, best, tot_ms / reps, n * 20.0 / (best * 1e-3) / 1e12,
         (unsigned long long)tot, s);
  CK(hipFree(dt));
}

int main(int argc, char **argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 30);
  const uint32_t sbits = 28;  // 2^28-slot table (C2)
  int64_t *keys, *ok;
  uint32_t *orow, *cur, *st;
  CK(hipMalloc(&keys, n * 8));
  hipLaunchKernelGGL(gen, dim3((n + 255) / 256), dim3(256), 0, 0, keys, n, 1ull << 26);
  const uint64_t npos = n + n / 8 + (1ull << 27);  // >= segs * cap for every shape below
  CK(hipMalloc(&ok, 8 * npos));
  CK(hipMalloc(&orow, 4 * npos));
  CK(hipMalloc(&cur, 2048 * 8 * 4));
  CK(hipMalloc(&st, 4));
  CK(hipMemset(st, 0, 4));
  auto capf = [&](int pbits) {
    const uint64_t m = n >> (pbits + 3);
    return ((m + m / 16 + 4096 + 2047) / 2048) * 2048;
  };
  const int reps = 5;
  // partition p = slot >> 18 = (h & (2^28-1)) >> 18: shift 18, 10 bits
  run2<1024, 8, 10, true>("persist", keys, n, 18, cur, capf(10), ok, orow, st, reps, 256);
  run2<1024, 8, 10, false>("persist-nowr", keys, n, 18, cur, capf(10), ok, orow, st, reps, 256);
  run2<512, 16, 10, true>("persist", keys, n, 18, cur, capf(10), ok, orow, st, reps, 256);
  run2<512, 16, 10, false>("persist-nowr", keys, n, 18, cur, capf(10), ok, orow, st, reps, 256);
  run2<512, 8, 10, true>("persist", keys, n, 18, cur, capf(10), ok, orow, st, reps, 512);
  run2<512, 8, 10, false>("persist-nowr", keys, n, 18, cur, capf(10), ok, orow, st, reps, 512);
  run2<1024, 12, 10, true>("persist", keys, n, 18, cur, capf(10), ok, orow, st, reps, 256);
  (void)sbits;
  return 0;
}
