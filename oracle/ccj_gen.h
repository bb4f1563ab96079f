/* ccj_gen.h — fully specified synthetic-input generators shared by the oracle, the
 * reference driver and the tests.  TEST INFRASTRUCTURE (see oracle/README.md): the product
 * library carries its own device copy of the same generators in csrc/ccj_kernels.hip.
 *
 * Nothing here exists in the reference; the reference's main.cpp draws probe keys with
 * std::mt19937(2) + std::uniform_int_distribution<int>(0, n) (main.cpp:43,53), whose algorithm
 * is implementation-defined.  We restate the libstdc++-11 algorithm (Lemire's nearly
 * divisionless method, bits/uniform_int_dist.h:245-268,311-316) so main.cpp-shaped fixtures can
 * be regenerated bit-for-bit, and we add a counter-based SplitMix64 stream for every other
 * config so any element can be produced independently on host or device.
 */
#ifndef CCJ_GEN_H
#define CCJ_GEN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* SplitMix64 finaliser (Steele, Lea, Flood 2014). */
static inline uint64_t ccj_fmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

#define CCJ_GOLDEN_GAMMA 0x9e3779b97f4a7c15ULL

/* i-th output of a SplitMix64 generator whose initial state is `seed`. */
static inline uint64_t ccj_splitmix_at(uint64_t seed, uint64_t i) {
  return ccj_fmix64(seed + (i + 1) * CCJ_GOLDEN_GAMMA);
}

/* Uniform probe key in [0, range): the i-th key of the stream (seed, range). */
static inline int64_t ccj_uniform_key(uint64_t seed, uint64_t i, uint64_t range) {
  return (int64_t)(ccj_splitmix_at(seed, i) % range);
}

/* ---- C3 probe stream: Zipf-skewed hits, ~hit_ppm/1e6 match rate ---- */
static inline uint32_t ccj_bitlen(uint64_t x) { return x ? 64u - (uint32_t)__builtin_clzll(x) : 0u; }

/* A fixed bijection on [0, n) (n >= 1): an odd multiply + add + xor-shift on the enclosing
 * power-of-two range, cycle-walked back into [0, n). */
static inline uint64_t ccj_perm(uint64_t x, uint64_t n, uint64_t seed) {
  const uint32_t k = n > 1 ? ccj_bitlen(n - 1) : 1u;
  const uint64_t mask = k >= 64 ? ~0ULL : (1ULL << k) - 1;
  do {
    x = (x * 0xd1342543de82ef95ULL + (seed | 1ULL)) & mask;
    x ^= x >> (k / 2 + 1);
  } while (x >= n);
  return x;
}

/* Zipf s = 1 over ranks 1..n ("Zipf s=1.0 over 2^26 ranks") as a 2^16-bucket
 * inverse CDF: T[j] = the smallest rank r whose CDF H_r / H_n exceeds j / 2^16, T[2^16] = n + 1
 * (T has 2^16 + 1 entries; n < 2^32).  A draw takes bucket j from the top 16 bits of a random word
 * and a rank uniform over the bucket's ranks [T[j], max(T[j], T[j+1] - 1)]: rank 1 alone holds
 * 1 / H_n of the buckets (5.4 % at n = 2^26), and where a bucket spans several ranks their 1 / r
 * weights differ by at most the bucket's width / r (< 0.03 % at n = 2^26).  Plain IEEE double
 * sums and products of exactly-representable operands, so every compiler builds the same table;
 * the device generator (csrc/ccj_api.hip) builds it the same way. */
#define CCJ_ZIPF_BITS 16
#define CCJ_ZIPF_BUCKETS (1u << CCJ_ZIPF_BITS)
static inline void ccj_zipf_table(uint64_t n, uint32_t *T) {
  double hn = 0.0;
  for (uint64_t r = 1; r <= n; ++r) hn += 1.0 / (double)r;
  uint32_t j = 0;
  double h = 0.0;
  for (uint64_t r = 1; r <= n && j < CCJ_ZIPF_BUCKETS; ++r) {
    h += 1.0 / (double)r;
    while (j < CCJ_ZIPF_BUCKETS && h * (double)CCJ_ZIPF_BUCKETS > (double)j * hn) T[j++] = (uint32_t)r;
  }
  while (j < CCJ_ZIPF_BUCKETS) T[j++] = (uint32_t)(n ? n : 1);
  T[CCJ_ZIPF_BUCKETS] = (uint32_t)(n + 1);
}

/* Zipf rank in [1, n] from random word z and table T (ccj_zipf_table). */
static inline uint64_t ccj_zipf_rank(const uint32_t *T, uint64_t z) {
  const uint32_t j = (uint32_t)(z >> (64 - CCJ_ZIPF_BITS));
  const uint64_t lo = T[j], hi = T[j + 1] > T[j] ? (uint64_t)T[j + 1] - 1 : lo;
  return lo + (z & 0xffffffffULL) % (hi - lo + 1);
}

/* Row i of the C3 stream over the reference generator's build side (n_build, cf): with
 * probability hit_ppm / 1e6 a build key whose rank r in [1, n_unique] is Zipf (s = 1) distributed
 * (zipf = ccj_zipf_table(n_unique)), mapped through ccj_perm so the popular keys spread over the
 * table; otherwise a key in [n_build, 2^62), which is never a build key (every build key is
 * < n_build, linear_probing_ht.cpp:16-25). */
static inline int64_t ccj_c3_key(const uint32_t *zipf, uint64_t seed, uint64_t i, uint64_t n_build, uint64_t cf,
                                 uint32_t hit_ppm) {
  const uint64_t z1 = ccj_splitmix_at(seed, 3 * i), z2 = ccj_splitmix_at(seed, 3 * i + 1);
  const uint64_t z3 = ccj_splitmix_at(seed, 3 * i + 2);
  const uint64_t n_unique = n_build / cf + (n_build % cf != 0);
  if (z1 % 1000000ULL < hit_ppm && n_unique) {
    const uint64_t step = n_build / n_unique;
    const uint64_t r = ccj_zipf_rank(zipf, z2);
    return (int64_t)(ccj_perm(r - 1, n_unique, seed) * step);
  }
  return (int64_t)(n_build + z3 % ((1ULL << 62) - n_build));
}

/* ---- mt19937 / mt19937_64 (Matsumoto & Nishimura), std:: parameterisation ---- */
typedef struct { uint32_t mt[624]; int idx; } ccj_mt19937;
typedef struct { uint64_t mt[312]; int idx; } ccj_mt19937_64;

static inline void ccj_mt19937_seed(ccj_mt19937 *g, uint32_t s) {
  g->mt[0] = s;
  for (int i = 1; i < 624; ++i) g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
  g->idx = 624;
}
static inline uint32_t ccj_mt19937_next(ccj_mt19937 *g) {
  if (g->idx >= 624) {
    for (int i = 0; i < 624; ++i) {
      uint32_t y = (g->mt[i] & 0x80000000u) | (g->mt[(i + 1) % 624] & 0x7fffffffu);
      uint32_t v = g->mt[(i + 397) % 624] ^ (y >> 1);
      if (y & 1u) v ^= 0x9908b0dfu;
      g->mt[i] = v;
    }
    g->idx = 0;
  }
  uint32_t y = g->mt[g->idx++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
static inline void ccj_mt19937_64_seed(ccj_mt19937_64 *g, uint64_t s) {
  g->mt[0] = s;
  for (int i = 1; i < 312; ++i)
    g->mt[i] = 6364136223846793005ULL * (g->mt[i - 1] ^ (g->mt[i - 1] >> 62)) + (uint64_t)i;
  g->idx = 312;
}
static inline uint64_t ccj_mt19937_64_next(ccj_mt19937_64 *g) {
  if (g->idx >= 312) {
    for (int i = 0; i < 312; ++i) {
      uint64_t y = (g->mt[i] & 0xFFFFFFFF80000000ULL) | (g->mt[(i + 1) % 312] & 0x7FFFFFFFULL);
      uint64_t v = g->mt[(i + 156) % 312] ^ (y >> 1);
      if (y & 1ULL) v ^= 0xB5026F5AA96619E9ULL;
      g->mt[i] = v;
    }
    g->idx = 0;
  }
  uint64_t x = g->mt[g->idx++];
  x ^= (x >> 29) & 0x5555555555555555ULL;
  x ^= (x << 17) & 0x71D67FFFEDA60000ULL;
  x ^= (x << 37) & 0xFFF7EEE000000000ULL;
  x ^= x >> 43;
  return x;
}

/* std::uniform_int_distribution<int>(0, b)(mt19937) as implemented by libstdc++ 11
 * (bits/uniform_int_dist.h:311-316 -> _S_nd<uint64_t>, :245-268): 32-bit engine, downscale. */
static inline int32_t ccj_uniform_int_0_b(ccj_mt19937 *g, int32_t b) {
  uint32_t range = (uint32_t)b + 1u; /* __uerange */
  uint64_t product = (uint64_t)ccj_mt19937_next(g) * (uint64_t)range;
  uint32_t low = (uint32_t)product;
  if (low < range) {
    uint32_t threshold = (uint32_t)(-range) % range;
    while (low < threshold) {
      product = (uint64_t)ccj_mt19937_next(g) * (uint64_t)range;
      low = (uint32_t)product;
    }
  }
  return (int32_t)(product >> 32);
}

/* ---- result checksums (defined here, used identically by oracle, driver, tests, bench) ----
 * L2 (order-insensitive): sum over matches of ccj_l2_term(global probe row, payload) mod 2^64.
 * L3 (order-sensitive):   h = ccj_l3_fold(h, row, payload) over the emission order, h0 = CCJ_L3_SEED.
 * SURVEY chk: sum of payload * 1315423911 + chunk-local physical row. */
static inline uint64_t ccj_l2_term(uint64_t row, int64_t payload) {
  return ccj_fmix64(row * CCJ_GOLDEN_GAMMA + ccj_fmix64((uint64_t)payload + 1ULL));
}
#define CCJ_L3_SEED 0x243F6A8885A308D3ULL
static inline uint64_t ccj_l3_fold(uint64_t h, uint64_t row, int64_t payload) {
  return ccj_fmix64(ccj_fmix64(h ^ row) ^ (uint64_t)payload);
}

#ifdef __cplusplus
}
#endif
#endif
