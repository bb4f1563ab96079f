// pipeline_main.cpp — the reference's pipeline driver (main.cpp) on the MI355X operators.
//
//   ccj_pipeline --join-num 3 --chunk-factor 5 --lhs-size 200000 --rhs-size 20000
//                [--table chain|lp] [--compact none|full] [--block-size 256] [--device 0]
//
// Same data generation (main.cpp:41-55: std::mt19937(2), uniform_int_distribution<int>(0, rhs)),
// same depth-first ExecutePipeline / FlushPipelineCache recursion (main.cpp:119-191), with every
// Probe/Next on the GPU through ccj_operators.h.  Prints the result count, an order-insensitive
// checksum over every column of every result tuple (the same formula as oracle/ref_driver.cpp's
// pipeline sink) and the first 8 result rows, plus the timed pipeline latency (main.cpp:92-94).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>

#include "ccj_operators.h"

using namespace simd_compaction_amd;

namespace {

inline uint64_t fmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

struct Sink {
  uint64_t n = 0, l2 = 0;
  vector<vector<int64_t>> head;
  void Consume(DataChunk &c) {  // DataCollection::AppendChunk's view of a chunk (data_collection.cpp:10-21)
    for (size_t i = 0; i < c.count_; ++i) {
      const uint32_t s = c.selection_vector_[i];
      uint64_t t = 0x51ED27ULL;
      vector<int64_t> tup;
      for (size_t k = 0; k < c.data_.size(); ++k) {
        const int64_t v = c.data_[k].GetValue(s);
        t = fmix64(t ^ (uint64_t)v) + k;
        tup.push_back(v);
      }
      l2 += fmix64(t);
      if (head.size() < 8) head.push_back(tup);
      ++n;
    }
  }
};

struct PipelineState {  // main.cpp:14-20
  bool lp = false, compact = false;
  vector<unique_ptr<HashTable>> hts;
  vector<unique_ptr<LPHashTable>> lps;
  vector<unique_ptr<DataChunk>> intermediates;
  vector<unique_ptr<Compactor>> compactors;
  Sink sink;
  size_t joins() const { return lp ? lps.size() : hts.size(); }
};

void ExecutePipeline(DataChunk &input, PipelineState &st, size_t level);

template <typename SS>
void Drive(SS &ss, DataChunk &input, PipelineState &st, size_t level) {
  auto &join_key = input.data_[level];
  auto &result = st.intermediates[level];
  while (ss.HasNext()) {
    ss.Next(join_key, input, *result);
    if (st.compact) {
      st.compactors[level]->Compact(result);  // main.cpp:153-157
      if (result->count_ == 0) continue;
    }
    ExecutePipeline(*result, st, level + 1);
  }
}

void ExecutePipeline(DataChunk &input, PipelineState &st, size_t level) {  // main.cpp:119-170
  if (level == st.joins()) {
    st.sink.Consume(input);
    return;
  }
  if (st.lp) {
    auto ss = st.lps[level]->Probe(input.data_[level], input.count_, input.selection_vector_);
    Drive(ss, input, st, level);
  } else {
    auto ss = st.hts[level]->Probe(input.data_[level], input.count_, input.selection_vector_);
    Drive(ss, input, st, level);
  }
}

void FlushPipelineCache(PipelineState &st, size_t level) {  // main.cpp:172-191
  if (level == st.joins()) return;
  auto &result = st.intermediates[level];
  st.compactors[level]->Flush(result);
  ExecutePipeline(*result, st, level + 1);
  FlushPipelineCache(st, level + 1);
}

}  // namespace

int main(int argc, char **argv) {
  size_t joins = 3, cf = 1, lhs = 20000000, rhs = 2000000;
  int device = 0;
  PipelineState st;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string a = argv[i], v = argv[i + 1];
    if (a == "--join-num") joins = std::stoul(v);
    else if (a == "--chunk-factor") cf = std::stoul(v);
    else if (a == "--lhs-size") lhs = std::stoul(v);
    else if (a == "--rhs-size") rhs = std::stoul(v);
    else if (a == "--table") st.lp = v == "lp";
    else if (a == "--compact") st.compact = v == "full";
    else if (a == "--block-size") kBlockSize = std::stoul(v);
    else if (a == "--device") device = std::stoi(v);
    else {
      fprintf(stderr, "unknown option %s\n", a.c_str());
      return 2;
    }
  }
  try {
    InitDevice(device);
    std::mt19937 gen(2);  // main.cpp:43
    std::uniform_int_distribution<> dist(0, (int)rhs);
    vector<AttributeType> types(joins, AttributeType::INTEGER);
    vector<vector<Attribute>> table(lhs, vector<Attribute>(joins));  // DataCollection (row store)
    for (size_t i = 0; i < lhs; ++i)
      for (size_t j = 0; j < joins; ++j) table[i][j] = (Attribute)(size_t)dist(gen);
    for (size_t i = 0; i < joins; ++i) {  // main.cpp:62-68
      if (st.lp) st.lps.push_back(std::make_unique<LPHashTable>(rhs, cf));
      else st.hts.push_back(std::make_unique<HashTable>(rhs, cf));
      types.push_back(AttributeType::INTEGER);
      types.push_back(AttributeType::INTEGER);
      st.intermediates.push_back(std::make_unique<DataChunk>(types));
      st.compactors.push_back(std::make_unique<Compactor>(types));
    }
    vector<AttributeType> in_types(joins, AttributeType::INTEGER);
    double latency = 0;
    size_t start = 0, end;
    do {  // main.cpp:79-102
      end = std::min(start + kBlockSize, lhs);
      DataChunk chunk(in_types);  // DataCollection::FetchChunk (data_collection.cpp:23-27), untimed
      for (size_t i = start; i < end; ++i) chunk.AppendTuple(table[i]);
      start = end;
      auto t0 = std::chrono::steady_clock::now();
      ExecutePipeline(chunk, st, 0);
      latency += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } while (end < lhs);
    if (st.compact) {
      auto t0 = std::chrono::steady_clock::now();
      FlushPipelineCache(st, 0);
      latency += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    printf("PIPE n_out %llu l2 %llu\n", (unsigned long long)st.sink.n, (unsigned long long)st.sink.l2);
    for (auto &t : st.sink.head) {
      printf("ROW");
      for (auto v : t) printf(" %lld", (long long)v);
      printf("\n");
    }
    fprintf(stderr, "[Total Time]: %.4fs\n", latency);
  } catch (const std::exception &e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  return 0;
}
