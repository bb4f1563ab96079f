// ref_driver.cpp — drives the REFERENCE implementation to produce golden vectors.
//
// TEST INFRASTRUCTURE ONLY.  This file is ours; it is compiled together with the reference's own
// sources *where they lie* under /root/reference (base.cpp, linear_probing_ht.cpp,
// chaining_ht.cpp, compactor.cpp, data_collection.cpp) by oracle/Makefile into oracle/_ref/,
// which is git-ignored.  Nothing of the reference is copied into this repository.
//
// It exercises the reference operator surface exactly as its callers do:
//   probe loop      simd_micro_bench.cpp:92-106 (Probe/SIMDProbe, while HasNext: Next variant)
//   pipeline        main.cpp:41-55 (data gen), :62-68 (tables), :79-102 (chunk loop),
//                   :119-170 ExecutePipeline, :172-191 FlushPipelineCache
// and prints per-Next traces / counts / checksums that tests/golden/make_golden.py stores.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "base.h"
#include "chaining_ht.h"
#include "compactor.h"
#include "data_collection.h"
#include "linear_probing_ht.h"

#include "ccj_gen.h"

using namespace simd_compaction;

namespace {

enum Variant { kNext = 0, kInOne = 1, kSimdNext = 2, kSimdInOne = 3 };

Variant ParseVariant(const char *s) {
  if (!strcmp(s, "next")) return kNext;
  if (!strcmp(s, "inone")) return kInOne;
  if (!strcmp(s, "simdnext")) return kSimdNext;
  if (!strcmp(s, "simdinone")) return kSimdInOne;
  fprintf(stderr, "bad variant %s\n", s);
  exit(2);
}

// Per-chunk selection vector modes (ours): 0 identity, 1 filtered subset (ascending),
// 2 reversed order.  Physical rows [0, n_phys) of the chunk always hold keys.
size_t MakeSel(int mode, size_t chunk_id, size_t n_phys, std::vector<uint32_t> &sel) {
  size_t n = 0;
  for (size_t i = 0; i < n_phys; ++i) {
    if (mode == 0) sel[n++] = (uint32_t)i;
    else if (mode == 1) {
      if ((ccj_fmix64(chunk_id * 1000003ULL + i + 7) & 3ULL) != 0) sel[n++] = (uint32_t)i;
    } else sel[n++] = (uint32_t)(n_phys - 1 - i);
  }
  return n;
}

struct Sink {
  bool trace = false;
  uint64_t matches = 0, l2 = 0, l3 = CCJ_L3_SEED, survey_chk = 0, nexts = 0, empty_nexts = 0;
  void Emit(size_t chunk_id, size_t round, DataChunk &result, size_t m) {
    size_t rc = result.count_;
    ++nexts;
    if (rc == 0) ++empty_nexts;
    if (trace) printf("N %zu %zu %zu", chunk_id, round, rc);
    for (size_t i = 0; i < rc; ++i) {
      uint32_t s = result.selection_vector_[i];
      int64_t p = result.data_[m + 1].GetValue(s);
      uint64_t row = (uint64_t)chunk_id * kBlockSize + s;
      matches++;
      l2 += ccj_l2_term(row, p);
      l3 = ccj_l3_fold(l3, row, p);
      survey_chk += (uint64_t)p * 1315423911ULL + s;
      if (trace) printf(" %u:%lld", s, (long long)p);
    }
    if (trace) printf("\n");
    if (trace) {
      // result column m+1 over all kBlockSize physical rows: InOneNext also writes unmatched
      // active rows (linear_probing_ht.cpp:133, chaining_ht.cpp:156), visible here only
      uint64_t h = CCJ_L3_SEED;
      for (size_t s = 0; s < kBlockSize; ++s) h = ccj_l3_fold(h, s, result.data_[m + 1].GetValue(s));
      printf("P %llu\n", (unsigned long long)h);
    }
  }
};

// Probe stream: key generator 0 = SplitMix64(seed) % range, 1 = mt19937_64(seed) % range
// (the SURVEY §4 driver).
template <typename Table>
void RunProbe(Table &ht, Variant v, size_t n_probe, uint64_t range, uint64_t seed, int gen, int selmode,
              Sink &sink) {
  std::vector<AttributeType> in_types{AttributeType::INTEGER};
  std::vector<AttributeType> out_types{AttributeType::INTEGER, AttributeType::INTEGER, AttributeType::INTEGER};
  DataChunk input(in_types);
  DataChunk output(out_types);
  std::vector<uint32_t> sel(kBlockSize);
  ccj_mt19937_64 mt;
  ccj_mt19937_64_seed(&mt, seed);
  size_t chunk_id = 0;
  for (size_t start = 0; start < n_probe; start += kBlockSize, ++chunk_id) {
    size_t n_phys = std::min(kBlockSize, n_probe - start);
    Vector &col = input.data_[0];
    for (size_t i = 0; i < n_phys; ++i) {
      uint64_t gi = start + i;
      col.GetValue(i) = gen == 0 ? ccj_uniform_key(seed, gi, range) : (int64_t)(ccj_mt19937_64_next(&mt) % range);
    }
    size_t count = MakeSel(selmode, chunk_id, n_phys, sel);
    input.count_ = count;
    input.selection_vector_ = sel;
    if (sink.trace) {
      printf("C %zu %zu", chunk_id, count);
      for (size_t i = 0; i < count; ++i) printf(" %u", sel[i]);
      printf("\n");
    }
    bool simd_probe = (v == kSimdNext || v == kSimdInOne);
    auto ss = simd_probe ? ht.SIMDProbe(col, count, input.selection_vector_) : ht.Probe(col, count, input.selection_vector_);
    size_t round = 0;
    while (ss.HasNext()) {
      switch (v) {
        case kNext: ss.Next(col, input, output); break;
        case kInOne: ss.InOneNext(col, input, output); break;
        case kSimdNext: ss.SIMDNext(col, input, output); break;
        default: ss.SIMDInOneNext(col, input, output); break;
      }
      sink.Emit(chunk_id, round++, output, 1);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// main.cpp-shaped pipeline (our replica of main.cpp:119-191 over the reference classes).
// compact: 0 = no compaction, 1 = the shipped NaiveCompactor (compactor.cpp:5-41, carries the
// aliasing defect of SURVEY §A.3), 2 = the same algorithm with a fresh temp chunk (the commented
// fix at compactor.cpp:36), implemented here.
struct FixedCompactor {
  explicit FixedCompactor(std::vector<AttributeType> &types)
      : types_(types), cached_(std::make_unique<DataChunk>(types)), temp_(std::make_unique<DataChunk>(types)) {}
  void Compact(std::unique_ptr<DataChunk> &chunk) {
    if (chunk->count_ == kBlockSize) return;
    if (chunk->count_ <= kBlockSize - cached_->count_) {
      cached_->Append(*chunk, chunk->count_);
      chunk->Reset();
      return;
    }
    size_t n_move = kBlockSize - cached_->count_;
    cached_->Append(*chunk, n_move);
    temp_->Append(*chunk, chunk->count_ - n_move, n_move);
    chunk.swap(cached_);
    cached_.swap(temp_);
    temp_ = std::make_unique<DataChunk>(types_);
  }
  void Flush(std::unique_ptr<DataChunk> &chunk) { chunk = std::move(cached_); }
  std::vector<AttributeType> types_;
  std::unique_ptr<DataChunk> cached_, temp_;
};

struct Pipe {
  int compact = 0;
  std::vector<std::unique_ptr<HashTable>> hts;
  std::vector<std::unique_ptr<LPHashTable>> lps;
  bool use_lp = false;
  std::vector<std::unique_ptr<DataChunk>> inter;
  std::vector<std::unique_ptr<NaiveCompactor>> naive;
  std::vector<std::unique_ptr<FixedCompactor>> fixed;
  uint64_t n_out = 0, l2 = 0;
  size_t ncols_out = 0;
  bool count_only = false;  // timing runs: main.cpp's ResultCollector without flag_collect_tuples
  std::vector<std::vector<int64_t>> head;

  void Sink(DataChunk &c) {
    if (count_only) {
      n_out += c.count_;
      return;
    }
    for (size_t i = 0; i < c.count_; ++i) {
      uint32_t s = c.selection_vector_[i];
      // order-insensitive tuple checksum over every column of the final result
      uint64_t t = 0x51ED27ULL;
      std::vector<int64_t> tup;
      for (size_t k = 0; k < c.data_.size(); ++k) {
        int64_t v = c.data_[k].GetValue(s);
        t = ccj_fmix64(t ^ (uint64_t)v) + k;
        tup.push_back(v);
      }
      l2 += ccj_fmix64(t);
      if (head.size() < 8) head.push_back(tup);
      ++n_out;
    }
  }

  template <typename SS>
  void Drive(SS &ss, DataChunk &input, size_t level) {
    auto &key = input.data_[level];
    auto &result = inter[level];
    while (ss.HasNext()) {
      ss.Next(key, input, *result);
      if (compact == 1) {
        naive[level]->Compact(result);
        if (result->count_ == 0) continue;
      } else if (compact == 2) {
        fixed[level]->Compact(result);
        if (result->count_ == 0) continue;
      }
      Exec(*result, level + 1);
    }
  }

  void Exec(DataChunk &input, size_t level) {
    size_t joins = use_lp ? lps.size() : hts.size();
    if (level == joins) {
      Sink(input);
      return;
    }
    if (use_lp) {
      auto ss = lps[level]->Probe(input.data_[level], input.count_, input.selection_vector_);
      Drive(ss, input, level);
    } else {
      auto ss = hts[level]->Probe(input.data_[level], input.count_, input.selection_vector_);
      Drive(ss, input, level);
    }
  }

  void Flush(size_t level) {
    size_t joins = use_lp ? lps.size() : hts.size();
    if (level == joins) return;
    auto &result = inter[level];
    if (compact == 1) naive[level]->Flush(result);
    else fixed[level]->Flush(result);
    Exec(*result, level + 1);
    Flush(level + 1);
  }
};

int RunPipeline(size_t joins, size_t cf, size_t lhs, size_t rhs, int compact, bool use_lp, bool count_only) {
  kJoins = joins;
  ccj_mt19937 gen;
  ccj_mt19937_seed(&gen, 2);  // main.cpp:43 std::mt19937 gen(2)
  std::vector<AttributeType> types;
  for (size_t i = 0; i < joins; ++i) types.push_back(AttributeType::INTEGER);
  DataCollection table(types);
  std::vector<Attribute> tuple(joins);
  for (size_t i = 0; i < lhs; ++i) {
    for (size_t j = 0; j < joins; ++j) tuple[j] = (size_t)ccj_uniform_int_0_b(&gen, (int32_t)rhs);
    table.AppendTuple(tuple);
  }
  Pipe p;
  p.count_only = count_only;
  p.compact = compact;
  p.use_lp = use_lp;
  p.inter.resize(joins);
  for (size_t i = 0; i < joins; ++i) {
    if (use_lp) p.lps.push_back(std::make_unique<LPHashTable>(rhs, cf));
    else p.hts.push_back(std::make_unique<HashTable>(rhs, cf));
    types.push_back(AttributeType::INTEGER);
    types.push_back(AttributeType::INTEGER);
    p.inter[i] = std::make_unique<DataChunk>(types);
    p.naive.push_back(std::make_unique<NaiveCompactor>(types));
    p.fixed.push_back(std::make_unique<FixedCompactor>(types));
  }
  size_t start = 0, end;
  double secs = 0;  // main.cpp:92-101: only ExecutePipeline and the final flush are timed
  do {
    end = std::min(start + kBlockSize, lhs);
    DataChunk chunk = table.FetchChunk(start, end);
    start = end;
    auto t0 = std::chrono::steady_clock::now();
    p.Exec(chunk, 0);
    secs += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  } while (end < lhs);
  auto t0 = std::chrono::steady_clock::now();
  if (compact) p.Flush(0);
  secs += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("PIPE n_out %llu l2 %llu\n", (unsigned long long)p.n_out, (unsigned long long)p.l2);
  printf("TIME seconds %.6f\n", secs);
  for (auto &t : p.head) {
    printf("ROW");
    for (auto v : t) printf(" %lld", (long long)v);
    printf("\n");
  }
  return 0;
}

// Timed probe loop of simd_micro_bench.cpp:92-106 shape over a pre-generated key column (the
// key generation and the per-chunk column fill stand in for DataCollection::FetchChunk and are
// untimed, as in main.cpp:88-94): Probe + while (HasNext) Next, counting matches only.
template <typename Table>
void BenchProbe(Table &ht, Variant v, size_t n_probe, uint64_t range, uint64_t seed, bool c3, size_t n_build,
                size_t cf) {
  std::vector<int64_t> keys(n_probe);
  std::vector<uint32_t> zipf(CCJ_ZIPF_BUCKETS + 1);
  if (c3) ccj_zipf_table(n_build / cf + (n_build % cf != 0), zipf.data());
  for (size_t i = 0; i < n_probe; ++i)
    keys[i] = c3 ? ccj_c3_key(zipf.data(), seed, i, n_build, cf, 100000) : ccj_uniform_key(seed, i, range);
  std::vector<AttributeType> in_types{AttributeType::INTEGER};
  std::vector<AttributeType> out_types{AttributeType::INTEGER, AttributeType::INTEGER, AttributeType::INTEGER};
  DataChunk input(in_types);
  DataChunk output(out_types);
  uint64_t matches = 0;
  double secs = 0;
  for (size_t start = 0; start < n_probe; start += kBlockSize) {
    const size_t n = std::min(kBlockSize, n_probe - start);
    Vector &col = input.data_[0];
    for (size_t i = 0; i < n; ++i) col.GetValue(i) = keys[start + i];
    input.Reset();
    input.count_ = n;
    auto t0 = std::chrono::steady_clock::now();
    const bool simd_probe = (v == kSimdNext || v == kSimdInOne);
    auto ss = simd_probe ? ht.SIMDProbe(col, n, input.selection_vector_) : ht.Probe(col, n, input.selection_vector_);
    while (ss.HasNext()) {
      switch (v) {
        case kNext: ss.Next(col, input, output); break;
        case kInOne: ss.InOneNext(col, input, output); break;
        case kSimdNext: ss.SIMDNext(col, input, output); break;
        default: ss.SIMDInOneNext(col, input, output); break;
      }
      matches += output.count_;
    }
    secs += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  printf("BENCH matches %llu seconds %.6f tuples_per_s %.1f\n", (unsigned long long)matches, secs,
         secs > 0 ? n_probe / secs : 0.0);
}

void Usage() {
  fprintf(stderr,
          "ref_driver probe <lp|chain> <next|inone|simdnext|simdinone> B n_build cf n_probe range seed gen selmode trace\n"
          "ref_driver pipeline <lp|chain> B joins cf lhs rhs compact [count_only]\n"
          "ref_driver bench <lp|chain> <next|inone|simdnext|simdinone> B n_build cf n_probe range seed [c3]\n");
  exit(2);
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 2) Usage();
  std::string cmd = argv[1];
  if (cmd == "probe") {
    if (argc != 13) Usage();
    bool lp = !strcmp(argv[2], "lp");
    Variant v = ParseVariant(argv[3]);
    kBlockSize = strtoull(argv[4], nullptr, 10);
    size_t n_build = strtoull(argv[5], nullptr, 10);
    size_t cf = strtoull(argv[6], nullptr, 10);
    size_t n_probe = strtoull(argv[7], nullptr, 10);
    uint64_t range = strtoull(argv[8], nullptr, 10);
    uint64_t seed = strtoull(argv[9], nullptr, 10);
    int gen = atoi(argv[10]);
    int selmode = atoi(argv[11]);
    Sink sink;
    sink.trace = atoi(argv[12]) != 0;
    if (lp) {
      LPHashTable ht(n_build, cf);
      RunProbe(ht, v, n_probe, range, seed, gen, selmode, sink);
    } else {
      HashTable ht(n_build, cf);
      RunProbe(ht, v, n_probe, range, seed, gen, selmode, sink);
    }
    printf("SUM matches %llu l2 %llu l3 %llu survey_chk %llu nexts %llu empty_nexts %llu\n",
           (unsigned long long)sink.matches, (unsigned long long)sink.l2, (unsigned long long)sink.l3,
           (unsigned long long)sink.survey_chk, (unsigned long long)sink.nexts,
           (unsigned long long)sink.empty_nexts);
    return 0;
  }
  if (cmd == "pipeline") {
    if (argc != 9 && argc != 10) Usage();
    bool lp = !strcmp(argv[2], "lp");
    kBlockSize = strtoull(argv[3], nullptr, 10);
    return RunPipeline(strtoull(argv[4], nullptr, 10), strtoull(argv[5], nullptr, 10),
                       strtoull(argv[6], nullptr, 10), strtoull(argv[7], nullptr, 10), atoi(argv[8]), lp,
                       argc > 9 && atoi(argv[9]) != 0);
  }
  if (cmd == "bench") {
    if (argc != 10 && argc != 11) Usage();
    const bool c3 = argc == 11 && !strcmp(argv[10], "c3");  // ccj_gen.h C3 stream instead of uniform
    const bool lp = !strcmp(argv[2], "lp");
    const Variant v = ParseVariant(argv[3]);
    kBlockSize = strtoull(argv[4], nullptr, 10);
    const size_t n_build = strtoull(argv[5], nullptr, 10), cf = strtoull(argv[6], nullptr, 10);
    const size_t n_probe = strtoull(argv[7], nullptr, 10);
    const uint64_t range = strtoull(argv[8], nullptr, 10), seed = strtoull(argv[9], nullptr, 10);
    if (lp) {
      LPHashTable ht(n_build, cf);
      BenchProbe(ht, v, n_probe, range, seed, c3, n_build, cf);
    } else {
      HashTable ht(n_build, cf);
      BenchProbe(ht, v, n_probe, range, seed, c3, n_build, cf);
    }
    return 0;
  }
  Usage();
}
