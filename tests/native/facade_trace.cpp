// facade_trace.cpp — TEST INFRASTRUCTURE (built by tests/test_facade_gpu.py).  Drives the C++
// operator facade (host/ccj_operators.h) exactly as the reference's callers drive the reference
// (simd_micro_bench.cpp:92-106: Probe, then Next until HasNext() is false) and prints every Next
// result, for comparison with the per-Next traces recorded from the reference itself
// (tests/golden/trace_*).
//   facade_trace <lp|chain> <next|inone|simdnext|simdinone> B n_build cf n_probe range seed selmode
// Output: "N <chunk> <rc>" per Next call, then "M <sel> <payload>" per result row, then "P <fold>"
// of result column m+1 over all kBlockSize physical rows.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../oracle/ccj_gen.h"
#include "ccj_operators.h"

using namespace simd_compaction_amd;

// Per-chunk selection vector of the trace cases (oracle/ref_driver.cpp MakeSel): 0 identity,
// 1 a filtered ascending subset, 2 reversed.
static size_t MakeSel(int mode, size_t chunk_id, size_t n_phys, vector<uint32_t> &sel) {
  size_t n = 0;
  for (size_t i = 0; i < n_phys; ++i) {
    if (mode == 0) sel[n++] = (uint32_t)i;
    else if (mode == 1) {
      if ((ccj_fmix64(chunk_id * 1000003ULL + i + 7) & 3ULL) != 0) sel[n++] = (uint32_t)i;
    } else sel[n++] = (uint32_t)(n_phys - 1 - i);
  }
  return n;
}

template <typename Table>
static void Run(Table &ht, const std::string &variant, size_t n_probe, uint64_t range, uint64_t seed, int selmode) {
  vector<AttributeType> in_types{AttributeType::INTEGER};
  vector<AttributeType> out_types{AttributeType::INTEGER, AttributeType::INTEGER, AttributeType::INTEGER};
  DataChunk input(in_types), output(out_types);
  vector<uint32_t> sel(kBlockSize);
  size_t chunk_id = 0;
  for (size_t start = 0; start < n_probe; start += kBlockSize, ++chunk_id) {
    const size_t n_phys = std::min(kBlockSize, n_probe - start);
    Vector &col = input.data_[0];
    for (size_t i = 0; i < n_phys; ++i) col.GetValue(i) = ccj_uniform_key(seed, start + i, range);
    const size_t count = MakeSel(selmode, chunk_id, n_phys, sel);
    input.count_ = count;
    input.selection_vector_ = sel;
    const bool simd = variant.rfind("simd", 0) == 0;
    auto ss = simd ? ht.SIMDProbe(col, count, input.selection_vector_) : ht.Probe(col, count, input.selection_vector_);
    while (ss.HasNext()) {
      if (variant == "next") ss.Next(col, input, output);
      else if (variant == "inone") ss.InOneNext(col, input, output);
      else if (variant == "simdnext") ss.SIMDNext(col, input, output);
      else ss.SIMDInOneNext(col, input, output);
      printf("N %zu %zu\n", chunk_id, output.count_);
      for (size_t i = 0; i < output.count_; ++i) {
        const uint32_t s = output.selection_vector_[i];
        printf("M %u %lld\n", s, (long long)output.data_[2].GetValue(s));
      }
      // column m+1 over every physical row (InOneNext's writes to unmatched active rows included)
      uint64_t h = CCJ_L3_SEED;
      for (size_t s = 0; s < kBlockSize; ++s) h = ccj_l3_fold(h, s, output.data_[2].GetValue(s));
      printf("P %llu\n", (unsigned long long)h);
    }
  }
}

int main(int argc, char **argv) {
  if (argc != 10) {
    fprintf(stderr, "usage: facade_trace <lp|chain> <variant> B n_build cf n_probe range seed selmode\n");
    return 2;
  }
  try {
    InitDevice(0);
    kBlockSize = strtoull(argv[3], nullptr, 10);
    const size_t n_build = strtoull(argv[4], nullptr, 10), cf = strtoull(argv[5], nullptr, 10);
    const size_t n_probe = strtoull(argv[6], nullptr, 10);
    const uint64_t range = strtoull(argv[7], nullptr, 10), seed = strtoull(argv[8], nullptr, 10);
    const int selmode = atoi(argv[9]);
    if (!strcmp(argv[1], "lp")) {
      LPHashTable ht(n_build, cf);
      Run(ht, argv[2], n_probe, range, seed, selmode);
    } else {
      HashTable ht(n_build, cf);
      Run(ht, argv[2], n_probe, range, seed, selmode);
    }
  } catch (const std::exception &e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  return 0;
}
