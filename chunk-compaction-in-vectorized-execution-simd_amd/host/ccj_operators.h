// ccj_operators.h — the reference's C++ operator surface for the probe path, on top of the
// MI355X engine's C ABI (include/ccj.h).  Same class and method names, argument meaning and
// return values as the reference (namespace simd_compaction → simd_compaction_amd):
//
//   Vector, DataChunk             base.h:59-100, base.cpp:5-47
//   LPHashTable / LPScanStructure linear_probing_ht.h:24-71
//   HashTable / ScanStructure     chaining_ht.h:29-101
//   NaiveCompactor / Compactor    compactor.h:14-29, setting.h:17-29
//
// Probe() runs the whole Probe + Next-loop of one chunk on the GPU in one ccj_probe launch; the
// returned scan structure then hands out the reference's Next() results one by one (LP: one per
// probe round, possibly empty; chaining Next: rounds without matches merged, chaining_ht.cpp:82-107).
// Differences from the reference, all deliberate:
//  - SIMD* variants are the scalar ones (the reference's variants agree result for result).
//    InOneNext / SIMDInOneNext also replay the reference's writes of the visited slot / chain key
//    into result column m+1 for every active row, matched or not (linear_probing_ht.cpp:133,
//    chaining_ht.cpp:156): the values come from one ccj_probe_visits launch on the first such call.
//  - NaiveCompactor allocates a fresh temp chunk (the commented compactor.cpp:36), removing the
//    aliasing defect of SURVEY §A.3.
//  - Errors from the engine throw simd_compaction_amd::EngineError (the reference only asserts).
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "ccj.h"

namespace simd_compaction_amd {

using std::shared_ptr;
using std::unique_ptr;
using std::vector;

inline size_t kBlockSize = 256;  // base.h:42 (the reference's default; BASELINE uses 2048)

using Attribute = int64_t;
using Key = int64_t;
enum class AttributeType : uint8_t { INTEGER = 0, INVALID = 3 };

struct EngineError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Vector {
 public:
  AttributeType type_;
  shared_ptr<vector<Attribute>> data_;
  Vector() : Vector(AttributeType::INTEGER) {}
  explicit Vector(AttributeType type) : type_(type), data_(std::make_shared<vector<Attribute>>(kBlockSize)) {}
  void Reference(Vector &other) { data_ = other.data_; }
  Attribute &GetValue(size_t idx) { return (*data_)[idx]; }
  Attribute *Data() { return data_->data(); }
  Attribute &operator[](size_t idx) { return (*data_)[idx]; }
};

class DataChunk {
 public:
  size_t count_;
  vector<Vector> data_;
  vector<AttributeType> types_;
  vector<uint32_t> selection_vector_;

  explicit DataChunk(const vector<AttributeType> &types);
  // dense gather of `num` selected rows starting at selection index `offset` (base.cpp:15-27)
  void Append(DataChunk &chunk, size_t num, size_t offset = 0);
  void AppendTuple(vector<Attribute> &tuple);
  // share `other`'s columns and compose selection vectors (base.cpp:37-47)
  void Slice(DataChunk &other, vector<uint32_t> &selection_vector, size_t count);
  void Reset();
};

// Device-side result of one chunk's probe (all rounds), shared by both scan structures.
struct ChunkProbeResult {
  vector<uint32_t> round_counts;  // matches per round (Next call)
  vector<uint32_t> sel;           // result selection vector entries, round-major
  vector<int64_t> payload;        // matched table value per entry
};

class DeviceTable;  // RAII wrapper of ccj_table + per-chunk probe buffers

// What the InOneNext variants need beyond the matches: the chunk's probe rows (copied at Probe
// time) and, fetched on first use, the table value each active row visits per round.
struct ChunkVisits {
  DeviceTable *table = nullptr;
  vector<int64_t> keys;  // the probe column (kBlockSize rows)
  vector<uint32_t> sel;  // Probe's sel_vec[0, count)
  bool loaded = false;
  uint32_t stride = 0;   // rounds per row in vals
  vector<int64_t> vals;  // [row][round]
  vector<uint32_t> len;  // rounds each row stays active
  // result column m+1 at the physical row of every row active in `round` := its visited value
  void Scribble(size_t round, DataChunk &input, DataChunk &result);
};

class LPScanStructure {
 public:
  size_t Next(Vector &join_key, DataChunk &input, DataChunk &result);
  size_t InOneNext(Vector &join_key, DataChunk &input, DataChunk &result);  // :117-146
  size_t SIMDNext(Vector &join_key, DataChunk &input, DataChunk &result) { return Next(join_key, input, result); }
  size_t SIMDInOneNext(Vector &join_key, DataChunk &input, DataChunk &result) {
    return InOneNext(join_key, input, result);
  }
  bool HasNext() const { return round_ < res_.round_counts.size(); }

 private:
  friend class LPHashTable;
  LPScanStructure(ChunkProbeResult res, ChunkVisits v) : res_(std::move(res)), visits_(std::move(v)) {}
  ChunkProbeResult res_;
  ChunkVisits visits_;
  size_t round_ = 0, pos_ = 0;
};

class LPHashTable {
 public:
  LPHashTable(size_t n_rhs_tuples, size_t chunk_factor);  // linear_probing_ht.cpp:4-37
  ~LPHashTable();
  LPScanStructure Probe(Vector &join_key, size_t count, vector<uint32_t> &sel_vec);
  LPScanStructure SIMDProbe(Vector &join_key, size_t count, vector<uint32_t> &sel_vec) {
    return Probe(join_key, count, sel_vec);
  }
  const ccj_table *handle() const;

 private:
  unique_ptr<DeviceTable> t_;
};

class ScanStructure {
 public:
  size_t Next(Vector &join_key, DataChunk &input, DataChunk &result);       // merged rounds
  size_t InOneNext(Vector &join_key, DataChunk &input, DataChunk &result);  // one round per call
  size_t SIMDNext(Vector &join_key, DataChunk &input, DataChunk &result, bool = true) {
    return Next(join_key, input, result);
  }
  size_t SIMDInOneNext(Vector &join_key, DataChunk &input, DataChunk &result, bool = false) {
    return InOneNext(join_key, input, result);
  }
  bool HasNext() const { return round_ < res_.round_counts.size(); }

 private:
  friend class HashTable;
  ScanStructure(ChunkProbeResult res, ChunkVisits v) : res_(std::move(res)), visits_(std::move(v)) {}
  size_t EmitRound(DataChunk &input, DataChunk &result);
  ChunkProbeResult res_;
  ChunkVisits visits_;
  size_t round_ = 0, pos_ = 0;
};

class HashTable {
 public:
  HashTable(size_t n_rhs_tuples, size_t chunk_factor);  // chaining_ht.cpp:4-36
  ~HashTable();
  ScanStructure Probe(Vector &join_key, size_t count, vector<uint32_t> &sel_vec);
  ScanStructure SIMDProbe(Vector &join_key, size_t count, vector<uint32_t> &sel_vec) {
    return Probe(join_key, count, sel_vec);
  }
  const ccj_table *handle() const;

 private:
  unique_ptr<DeviceTable> t_;
};

class NaiveCompactor {
 public:
  explicit NaiveCompactor(vector<AttributeType> &types)
      : types_(types), cached_chunk_(std::make_unique<DataChunk>(types)),
        temp_chunk_(std::make_unique<DataChunk>(types)) {}
  void Compact(unique_ptr<DataChunk> &chunk);  // compactor.cpp:5-41 (with the :36 fix)
  void Flush(unique_ptr<DataChunk> &chunk) { chunk = std::move(cached_chunk_); }  // compactor.h:23

 private:
  vector<AttributeType> types_;
  unique_ptr<DataChunk> cached_chunk_;
  unique_ptr<DataChunk> temp_chunk_;
};

using Compactor = NaiveCompactor;  // setting.h:17-19 / :26-28

// Initialises the engine on `device` (throws EngineError without a gfx950 device).
void InitDevice(int device = 0);

}  // namespace simd_compaction_amd
