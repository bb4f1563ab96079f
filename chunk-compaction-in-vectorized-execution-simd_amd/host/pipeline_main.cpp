// pipeline_main.cpp — the reference's pipeline driver (main.cpp) on the MI355X operators.
//
//   ccj_pipeline --join-num 3 --chunk-factor 5 --lhs-size 200000 --rhs-size 20000
//                [--table chain|lp] [--compact none|full] [--block-size 256] [--device 0]
//                [--engine facade|batched] [--dump FILE] [--repeat N]
//                [--compact dynamic] [--thresholds T0,T1,...]
//
// --engine facade (default) runs the reference's own recursion on the per-chunk operator facade;
// --engine batched runs the same pipeline through ccj_pipeline_run (include/ccj.h): each join
// probes all of its input chunks in one launch, with device concatenation / compaction between
// joins.  --dump writes every result tuple (int64, row-major, all columns) for order checks.
// Batched engine only: --thresholds gives each join's compactor a pass-through threshold
// (results of >= T rows pass through, smaller ones are compacted; the BinaryCompactor idea of
// setting.h:20-22), and --compact dynamic lets the UCB tuner (ccj_tuner.h, the DynamicCompactor
// of setting.h:23-25 + negative_feedback.hpp) pick every join's threshold per run.
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

#include <hip/hip_runtime.h>

#include "ccj_operators.h"
#include "ccj_tuner.h"

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
  FILE *dump = nullptr;
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
      if (dump) fwrite(tup.data(), sizeof(int64_t), tup.size(), dump);
      if (head.size() < 8) head.push_back(tup);
      ++n;
    }
  }
};

struct PipelineState {  // main.cpp:14-20
  bool lp = false, compact = false, dynamic = false;
  vector<uint32_t> thresholds;
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

void HipCheck(hipError_t e, const char *what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void CcjCheck(int rc, const char *what) {
  if (rc != CCJ_OK) throw std::runtime_error(std::string(what) + ": " + ccj_last_error());
}

// The same pipeline through ccj_pipeline_run: returns the timed latency of the last repetition.
double RunBatched(PipelineState &st, const vector<vector<Attribute>> &table, size_t joins, size_t repeat) {
  const size_t n = table.size();
  vector<const ccj_table *> th;
  for (size_t l = 0; l < joins; ++l) th.push_back(st.lp ? st.lps[l]->handle() : st.hts[l]->handle());
  vector<int64_t *> d_cols(joins, nullptr);
  vector<int64_t> col(n);
  for (size_t j = 0; j < joins; ++j) {  // DataCollection -> device columns (untimed, like FetchChunk)
    for (size_t i = 0; i < n; ++i) col[i] = table[i][j];
    HipCheck(hipMalloc(&d_cols[j], std::max<size_t>(n, 1) * 8), "alloc");
    HipCheck(hipMemcpy(d_cols[j], col.data(), n * 8, hipMemcpyHostToDevice), "upload");
  }
  ccj_pipeline *pl = nullptr;
  CcjCheck(ccj_pipeline_create(th.data(), (uint32_t)joins, (uint32_t)kBlockSize,
                               st.compact ? CCJ_COMPACT_FULL : CCJ_COMPACT_NONE, &pl),
           "ccj_pipeline_create");
  ccj_pipeline_result res{};
  double latency = 0;
  if (!st.thresholds.empty()) {
    if (st.thresholds.size() != joins) throw std::runtime_error("--thresholds needs one value per join");
    CcjCheck(ccj_pipeline_set_thresholds(pl, st.thresholds.data()), "ccj_pipeline_set_thresholds");
  }
  CompactTuner tuner(joins, (uint32_t)kBlockSize);
  vector<size_t> arm(joins, 0);
  vector<uint32_t> thr(joins, 0);
  fprintf(stderr, "TIMES");
  for (size_t r = 0; r < std::max<size_t>(repeat, 1); ++r) {
    if (st.dynamic) {  // main.cpp:133-142: one threshold per compactor, chosen before the run
      for (size_t l = 0; l < joins; ++l) {
        arm[l] = tuner.SelectArm(l);
        thr[l] = tuner.Threshold(arm[l]);
      }
      CcjCheck(ccj_pipeline_set_thresholds(pl, thr.data()), "ccj_pipeline_set_thresholds");
    }
    HipCheck(hipDeviceSynchronize(), "sync");
    auto t0 = std::chrono::steady_clock::now();
    CcjCheck(ccj_pipeline_run(pl, (const int64_t *const *)d_cols.data(), n, nullptr, &res), "ccj_pipeline_run");
    HipCheck(hipDeviceSynchronize(), "sync");
    latency = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr, " %.6f", latency);
    if (st.dynamic) {  // main.cpp:161-167: reward = speed of join l and everything it feeds
      double tail_ms = 0;
      for (size_t l = joins; l-- > 0;) {
        tail_ms += res.level_ms[l];
        if (tail_ms > 0) tuner.UpdateArm(l, arm[l], (double)res.rows_in[l] / (tail_ms * 1e6));
      }
    }
  }
  fprintf(stderr, "\n");
  if (st.dynamic) {
    for (size_t l = 0; l < joins; ++l) {
      fprintf(stderr, "TUNER join %zu", l);
      for (size_t a = 0; a < tuner.thresholds().size(); ++a)
        fprintf(stderr, " thr=%u:sel=%zu:est=%.4f", tuner.thresholds()[a], tuner.bandit(l).Selections(a),
                tuner.bandit(l).Estimate(a));
      fprintf(stderr, "\n");
    }
  }
  for (size_t l = 0; l < joins; ++l)
    fprintf(stderr, "[join %zu] chunks_in %llu rows_in %llu rows_out %llu ms %.4f\n", l,
            (unsigned long long)res.chunks_in[l], (unsigned long long)res.rows_in[l],
            (unsigned long long)res.rows_out[l], res.level_ms[l]);
  uint64_t *d_acc = nullptr, acc[2] = {0, 0};
  HipCheck(hipMalloc(&d_acc, 16), "alloc");
  HipCheck(hipMemset(d_acc, 0, 16), "memset");
  CcjCheck(ccj_pipeline_checksum(&res, (uint32_t)joins, d_acc, nullptr), "ccj_pipeline_checksum");
  HipCheck(hipMemcpy(acc, d_acc, 16, hipMemcpyDeviceToHost), "download");
  st.sink.n = acc[0];
  st.sink.l2 = acc[1];
  // Head rows / dump: download the result columns in the sink's column order.
  const size_t m = st.sink.dump ? res.n_out : std::min<uint64_t>(res.n_out, 8);
  vector<vector<int64_t>> c(2 * joins, vector<int64_t>(m));
  for (size_t j = 0; j < joins && m; ++j) {
    HipCheck(hipMemcpy(c[j].data(), res.cols[j], m * 8, hipMemcpyDeviceToHost), "download");
    HipCheck(hipMemcpy(c[joins + j].data(), res.payload[j], m * 8, hipMemcpyDeviceToHost), "download");
  }
  for (size_t i = 0; i < m; ++i) {
    vector<int64_t> tup;
    for (size_t j = 0; j < joins; ++j) tup.push_back(c[j][i]);
    for (size_t l = 0; l < joins; ++l) {
      tup.push_back(0);
      tup.push_back(c[joins + l][i]);
    }
    if (st.sink.dump) fwrite(tup.data(), sizeof(int64_t), tup.size(), st.sink.dump);
    if (st.sink.head.size() < 8) st.sink.head.push_back(tup);
  }
  ccj_pipeline_free(pl);
  (void)hipFree(d_acc);
  for (auto *p : d_cols) (void)hipFree(p);
  return latency;
}

}  // namespace

int main(int argc, char **argv) {
  size_t joins = 3, cf = 1, lhs = 20000000, rhs = 2000000;
  int device = 0;
  size_t repeat = 1;
  std::string engine = "facade", dump;
  PipelineState st;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string a = argv[i], v = argv[i + 1];
    if (a == "--join-num") joins = std::stoul(v);
    else if (a == "--chunk-factor") cf = std::stoul(v);
    else if (a == "--lhs-size") lhs = std::stoul(v);
    else if (a == "--rhs-size") rhs = std::stoul(v);
    else if (a == "--table") st.lp = v == "lp";
    else if (a == "--compact") {
      st.compact = v == "full" || v == "dynamic";
      st.dynamic = v == "dynamic";
    } else if (a == "--thresholds") {
      for (size_t p = 0; p < v.size();) {
        const size_t q = v.find(',', p);
        st.thresholds.push_back((uint32_t)std::stoul(v.substr(p, q == std::string::npos ? q : q - p)));
        p = q == std::string::npos ? v.size() : q + 1;
      }
    }
    else if (a == "--block-size") kBlockSize = std::stoul(v);
    else if (a == "--device") device = std::stoi(v);
    else if (a == "--engine") engine = v;
    else if (a == "--dump") dump = v;
    else if (a == "--repeat") repeat = std::stoul(v);
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
    if (!dump.empty() && !(st.sink.dump = fopen(dump.c_str(), "wb"))) throw std::runtime_error("cannot open " + dump);
    vector<AttributeType> in_types(joins, AttributeType::INTEGER);
    double latency = 0;
    if (engine != "batched" && (st.dynamic || !st.thresholds.empty()))
      throw std::runtime_error("threshold / dynamic compaction runs on --engine batched");
    if (engine == "batched") {
      latency = RunBatched(st, table, joins, repeat);
    } else {
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
    }
    if (st.sink.dump) fclose(st.sink.dump);
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
