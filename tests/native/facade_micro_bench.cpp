// facade_micro_bench.cpp — TEST INFRASTRUCTURE (built by tests/test_known_answers_gpu.py).  The
// reference's variant micro-bench (simd_micro_bench.cpp:75-361) on the C++ operator facade
// (host/ccj_operators.h): kLHSTuples = 2^27 probe keys rand() & (kRHSTuples * kHitFreq - 1)
// (:78-79), kBlockSize = 256 << scale, kRHSTuples = 128 << scale (:62-63), one table per variant,
// and for every block Probe / SIMDProbe then Next / InOneNext / SIMDNext / SIMDInOneNext until
// HasNext() is false, summing the returned counts into #tuples (:92-116 and its 7 siblings).
//   facade_micro_bench <scale> <hit_frequency> <chunk_factor> [parallel]
// Prints "#tuples <table> <variant> <n> <seconds>" per variant (the reference prints
// "#tuples: 134217728" for all 8 at scale 0, hit frequency 1, chunk factor 1).
// parallel = 1 runs the 8 variants in 8 host threads (each its own table and HIP stream); each
// prints a progress line to stderr every 2^16 blocks.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "ccj_operators.h"

using namespace simd_compaction_amd;

static const size_t kLHSTuples = size_t(1024) << 17;  // base.h:44

template <typename Table>
static void Run(const char *tname, const std::string &variant, const std::vector<int64_t> &keys, size_t n_rhs,
                size_t cf) {
  const auto t0 = std::chrono::steady_clock::now();
  Table ht(n_rhs, cf);
  std::vector<uint32_t> sel_vector(kBlockSize);
  for (uint32_t i = 0; i < kBlockSize; ++i) sel_vector[i] = i;
  DataChunk input(vector<AttributeType>{AttributeType::INTEGER});
  DataChunk output(vector<AttributeType>{AttributeType::INTEGER, AttributeType::INTEGER, AttributeType::INTEGER});
  Vector keys_block(AttributeType::INTEGER);
  const bool simd = variant.rfind("simd", 0) == 0;
  uint64_t n_tuples = 0;
  size_t blocks = 0;
  for (size_t k = 0; k < kLHSTuples; k += kBlockSize, ++blocks) {
    const size_t n_filling = std::min(kBlockSize, kLHSTuples - k);
    for (size_t i = 0; i < n_filling; ++i) keys_block.GetValue(i) = keys[k + i];
    input.data_[0] = keys_block;
    input.count_ = n_filling;
    auto ss = simd ? ht.SIMDProbe(keys_block, n_filling, sel_vector) : ht.Probe(keys_block, n_filling, sel_vector);
    while (ss.HasNext()) {
      if (variant == "next") n_tuples += ss.Next(keys_block, input, output);
      else if (variant == "inone") n_tuples += ss.InOneNext(keys_block, input, output);
      else if (variant == "simdnext") n_tuples += ss.SIMDNext(keys_block, input, output);
      else n_tuples += ss.SIMDInOneNext(keys_block, input, output);
    }
    if ((blocks & 0xFFFF) == 0xFFFF) fprintf(stderr, "[%s %s] %zu blocks\n", tname, variant.c_str(), blocks + 1);
  }
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("#tuples %s %s %llu %.2f\n", tname, variant.c_str(), (unsigned long long)n_tuples, s);
  fflush(stdout);
}

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s scale hit_frequency chunk_factor [parallel]\n", argv[0]);
    return 2;
  }
  const size_t scale = std::stoul(argv[1]), hit = std::stoul(argv[2]), cf = std::stoul(argv[3]);
  const bool parallel = argc > 4 && std::stoi(argv[4]) != 0;
  kBlockSize = size_t(256) << scale;
  const size_t n_rhs = size_t(128) << scale;
  std::vector<int64_t> keys(kLHSTuples);
  for (size_t i = 0; i < kLHSTuples; ++i) keys[i] = rand() & (int64_t)(n_rhs * hit - 1);  // :78-79
  try {
    InitDevice(0);
    const char *variants[4] = {"simdnext", "next", "simdinone", "inone"};  // the reference's print order
    std::vector<std::thread> th;
    for (int kind = 0; kind < 2; ++kind)
      for (const char *v : variants) {
        auto job = [=, &keys]() {
          try {
            if (kind == 0) Run<HashTable>("chain", v, keys, n_rhs, cf);
            else Run<LPHashTable>("lp", v, keys, n_rhs, cf);
          } catch (const std::exception &e) {
            fprintf(stderr, "error: %s\n", e.what());
            std::exit(1);
          }
        };
        if (parallel) th.emplace_back(job);
        else job();
      }
    for (auto &t : th) t.join();
  } catch (const std::exception &e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  return 0;
}
