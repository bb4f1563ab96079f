// ccj_operators.cpp — reference operator surface over the ccj C ABI (see ccj_operators.h).
#include <cstring>

#include "ccj_operators.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

namespace simd_compaction_amd {

namespace {

void check(int rc, const char *what) {
  if (rc != CCJ_OK) throw EngineError(std::string(what) + ": " + ccj_last_error());
}

void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw EngineError(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

void InitDevice(int device) { check(ccj_device_init(device), "ccj_device_init"); }

// ---------------------------------------------------------------------------------------------
DataChunk::DataChunk(const vector<AttributeType> &types)
    : count_(0), types_(types), selection_vector_(kBlockSize) {
  for (auto t : types) data_.emplace_back(t);
  for (size_t i = 0; i < kBlockSize; ++i) selection_vector_[i] = (uint32_t)i;
}

void DataChunk::Append(DataChunk &chunk, size_t num, size_t offset) {
  if (types_.size() != chunk.types_.size() || count_ + num > kBlockSize)
    throw EngineError("DataChunk::Append: column mismatch or overflow");  // base.cpp:16-17 asserts
  for (size_t c = 0; c < types_.size(); ++c) {
    auto &dst = *data_[c].data_;
    auto &src = *chunk.data_[c].data_;
    for (size_t j = 0; j < num; ++j) dst[count_ + j] = src[chunk.selection_vector_[j + offset]];
  }
  count_ += num;
}

void DataChunk::AppendTuple(vector<Attribute> &tuple) {
  for (size_t c = 0; c < types_.size(); ++c) data_[c].GetValue(count_) = tuple[c];
  ++count_;
}

void DataChunk::Slice(DataChunk &other, vector<uint32_t> &sel, size_t count) {
  count_ = count;
  for (size_t c = 0; c < other.data_.size(); ++c) data_[c].Reference(other.data_[c]);
  for (size_t i = 0; i < count; ++i) selection_vector_[i] = other.selection_vector_[sel[i]];
}

void DataChunk::Reset() {  // base.h:96-99
  count_ = 0;
  for (size_t i = 0; i < kBlockSize; ++i) selection_vector_[i] = (uint32_t)i;
}

// ---------------------------------------------------------------------------------------------
// One ccj_table plus the device buffers of a single-chunk probe (the compatibility path: one
// launch per Probe call; batched callers use ccj_probe directly).
class DeviceTable {
 public:
  DeviceTable(int kind, size_t n, size_t cf) {
    check(ccj_table_build_reference(kind, n, cf, CCJ_LAYOUT_REFERENCE, nullptr, &t_), "ccj_table_build_reference");
    check(ccj_table_get_info(t_, &info_), "ccj_table_get_info");
    hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
  }
  ~DeviceTable() {
    Release();
    ccj_table_free(t_);
    (void)hipStreamDestroy(stream_);
  }

  // Probe + every Next round of one chunk: the whole ScanStructure lifetime in one launch.  One
  // pinned staging buffer mirrors one device buffer: [keys | sel | count | out header (zeroed) |
  // round counts | out sel | payload]; one upload of the input + header, one launch, one download
  // of the outputs, one synchronisation.
  ChunkProbeResult Run(Vector &join_key, size_t count, const vector<uint32_t> &sel) {
    Ensure();
    const size_t n = kBlockSize;
    if (count > n || sel.size() < count) throw EngineError("Probe: count exceeds kBlockSize / sel");
    char *h = h_buf_;
    std::memcpy(h + off_keys_, join_key.Data(), n * sizeof(int64_t));
    if (count) std::memcpy(h + off_sel_, sel.data(), count * 4);
    *reinterpret_cast<uint32_t *>(h + off_cnt_) = (uint32_t)count;
    std::memset(h + off_hdr_, 0, 16);  // out count, rounds, status
    hip_check(hipMemcpyAsync(d_buf_, h, off_hdr_ + 16, hipMemcpyHostToDevice, stream_), "H2D");
    char *d = d_buf_;
    ccj_probe_args a{};
    a.keys = reinterpret_cast<const int64_t *>(d + off_keys_);
    a.sel = reinterpret_cast<const uint32_t *>(d + off_sel_);
    a.counts = reinterpret_cast<const uint32_t *>(d + off_cnt_);
    a.n_rows = n;
    a.chunk = (uint32_t)n;
    a.max_rounds = max_rounds_;
    a.cap = cap_;
    a.out_count = reinterpret_cast<uint32_t *>(d + off_hdr_);
    a.out_rounds = reinterpret_cast<uint32_t *>(d + off_hdr_ + 4);
    a.status = reinterpret_cast<uint32_t *>(d + off_hdr_ + 8);
    a.out_round_counts = reinterpret_cast<uint32_t *>(d + off_rc_);
    a.out_sel = reinterpret_cast<uint32_t *>(d + off_osel_);
    a.out_payload = reinterpret_cast<int64_t *>(d + off_pay_);
    check(ccj_probe(t_, &a, stream_), "ccj_probe");
    hip_check(hipMemcpyAsync(h + off_hdr_, d + off_hdr_, end_ - off_hdr_, hipMemcpyDeviceToHost, stream_), "D2H");
    hip_check(hipStreamSynchronize(stream_), "sync");
    const uint32_t *hdr = reinterpret_cast<const uint32_t *>(h + off_hdr_);
    if (hdr[2]) throw EngineError("ccj_probe raised status flags " + std::to_string(hdr[2]));
    ChunkProbeResult r;
    const uint32_t nm = hdr[0], nr = hdr[1] < max_rounds_ ? hdr[1] : max_rounds_;
    const uint32_t *rc = reinterpret_cast<const uint32_t *>(h + off_rc_);
    const uint32_t *os = reinterpret_cast<const uint32_t *>(h + off_osel_);
    const int64_t *op = reinterpret_cast<const int64_t *>(h + off_pay_);
    r.round_counts.assign(rc, rc + nr);
    r.sel.assign(os, os + nm);
    r.payload.assign(op, op + nm);
    return r;
  }
  const ccj_table *handle() const { return t_; }

  // ccj_probe_visits for one chunk: v.vals / v.len (the InOneNext side writes).  One pinned staging
  // buffer mirrors one device buffer: [keys | sel | len | vals].
  void Visits(ChunkVisits &v) {
    Ensure();
    const uint32_t count = (uint32_t)v.sel.size(), mr = max_rounds_;
    v.stride = mr;
    v.vals.assign((size_t)count * mr, 0);
    v.len.assign(count, 0);
    if (count) {
      if (count > kBlockSize || v.keys.size() != kBlockSize) throw EngineError("InOneNext: chunk exceeds kBlockSize");
      char *h = h_vis_, *d = d_vis_;
      std::memcpy(h, v.keys.data(), v.keys.size() * 8);
      std::memcpy(h + vis_sel_, v.sel.data(), count * 4);
      hip_check(hipMemcpyAsync(d, h, vis_len_, hipMemcpyHostToDevice, stream_), "H2D");
      check(ccj_probe_visits(t_, reinterpret_cast<const int64_t *>(d), reinterpret_cast<const uint32_t *>(d + vis_sel_),
                             count, mr, reinterpret_cast<int64_t *>(d + vis_vals_), reinterpret_cast<uint32_t *>(d + vis_len_),
                             stream_),
            "ccj_probe_visits");
      hip_check(hipMemcpyAsync(h + vis_len_, d + vis_len_, vis_end_ - vis_len_, hipMemcpyDeviceToHost, stream_), "D2H");
      hip_check(hipStreamSynchronize(stream_), "sync");
      std::memcpy(v.len.data(), h + vis_len_, count * 4);
      std::memcpy(v.vals.data(), h + vis_vals_, v.vals.size() * 8);
    }
    v.loaded = true;
  }

 private:
  static size_t Align(size_t x) { return (x + 15) & ~(size_t)15; }
  void Ensure() {
    if (sized_for_ == kBlockSize) return;
    Release();
    const size_t n = kBlockSize;
    cap_ = n * std::max<uint64_t>(1, info_.max_dup);
    max_rounds_ = info_.max_rounds + 1;
    off_keys_ = 0;
    off_sel_ = Align(n * 8);
    off_cnt_ = Align(off_sel_ + n * 4);
    off_hdr_ = Align(off_cnt_ + 4);
    off_rc_ = off_hdr_ + 16;
    off_osel_ = Align(off_rc_ + (size_t)max_rounds_ * 4);
    off_pay_ = Align(off_osel_ + cap_ * 4);
    end_ = off_pay_ + cap_ * 8;
    hip_check(hipMalloc(&d_buf_, end_), "hipMalloc");
    hip_check(hipHostMalloc(&h_buf_, end_, hipHostMallocDefault), "hipHostMalloc");
    vis_sel_ = Align(n * 8);
    vis_len_ = Align(vis_sel_ + n * 4);
    vis_vals_ = Align(vis_len_ + n * 4);
    vis_end_ = vis_vals_ + n * (size_t)max_rounds_ * 8;
    hip_check(hipMalloc(&d_vis_, vis_end_), "hipMalloc");
    hip_check(hipHostMalloc(&h_vis_, vis_end_, hipHostMallocDefault), "hipHostMalloc");
    sized_for_ = n;
  }
  void Release() {
    if (d_buf_) (void)hipFree(d_buf_);
    if (h_buf_) (void)hipHostFree(h_buf_);
    if (d_vis_) (void)hipFree(d_vis_);
    if (h_vis_) (void)hipHostFree(h_vis_);
    d_buf_ = h_buf_ = d_vis_ = h_vis_ = nullptr;
    sized_for_ = 0;
  }

  ccj_table *t_ = nullptr;
  ccj_table_info info_{};
  hipStream_t stream_{};
  size_t sized_for_ = 0;
  uint64_t cap_ = 0;
  uint32_t max_rounds_ = 0;
  size_t off_keys_ = 0, off_sel_ = 0, off_cnt_ = 0, off_hdr_ = 0, off_rc_ = 0, off_osel_ = 0, off_pay_ = 0, end_ = 0;
  char *d_buf_ = nullptr, *h_buf_ = nullptr;
  size_t vis_sel_ = 0, vis_len_ = 0, vis_vals_ = 0, vis_end_ = 0;  // ccj_probe_visits staging
  char *d_vis_ = nullptr, *h_vis_ = nullptr;
};

// Fills `result` with one Next result: Slice (base.cpp:37-47) + payload column m+1 at the selected
// physical rows (linear_probing_ht.cpp:85-94, chaining_ht.cpp:69-76).
static void Materialise(const ChunkProbeResult &res, size_t pos, size_t rc, DataChunk &input, DataChunk &result) {
  result.count_ = rc;
  for (size_t c = 0; c < input.data_.size(); ++c) result.data_[c].Reference(input.data_[c]);
  auto &pay = result.data_[input.data_.size() + 1];
  for (size_t i = 0; i < rc; ++i) {
    result.selection_vector_[i] = res.sel[pos + i];
    pay.GetValue(res.sel[pos + i]) = res.payload[pos + i];
  }
}

void ChunkVisits::Scribble(size_t round, DataChunk &input, DataChunk &result) {
  if (!loaded) table->Visits(*this);
  auto &col = result.data_[input.data_.size() + 1];
  // active rows in slot_sel_vector_ order (ascending row), so a later row wins a shared position
  for (size_t i = 0; i < sel.size(); ++i)
    if (round < len[i]) col.GetValue(sel[i]) = vals[i * stride + round];
}

static ChunkVisits MakeVisits(DeviceTable *t, Vector &join_key, size_t count, const vector<uint32_t> &sel) {
  ChunkVisits v;
  v.table = t;
  v.keys.assign(join_key.Data(), join_key.Data() + kBlockSize);
  v.sel.assign(sel.begin(), sel.begin() + count);
  return v;
}

// ---------------------------------------------------------------------------------------------
LPHashTable::LPHashTable(size_t n, size_t cf) : t_(new DeviceTable(CCJ_TABLE_LP, n, cf)) {}
LPHashTable::~LPHashTable() = default;
const ccj_table *LPHashTable::handle() const { return t_->handle(); }

LPScanStructure LPHashTable::Probe(Vector &join_key, size_t count, vector<uint32_t> &sel_vec) {
  return LPScanStructure(t_->Run(join_key, count, sel_vec), MakeVisits(t_.get(), join_key, count, sel_vec));
}

size_t LPScanStructure::Next(Vector &, DataChunk &input, DataChunk &result) {
  result.Reset();
  if (!HasNext()) return 0;
  const size_t rc = res_.round_counts[round_++];
  Materialise(res_, pos_, rc, input, result);  // LP Next slices even an empty result (:85)
  pos_ += rc;
  return rc;
}

size_t LPScanStructure::InOneNext(Vector &, DataChunk &input, DataChunk &result) {
  result.Reset();
  if (!HasNext()) return 0;
  visits_.Scribble(round_, input, result);  // :133, before the slice of :144
  const size_t rc = res_.round_counts[round_++];
  Materialise(res_, pos_, rc, input, result);
  pos_ += rc;
  return rc;
}

HashTable::HashTable(size_t n, size_t cf) : t_(new DeviceTable(CCJ_TABLE_CHAIN, n, cf)) {}
HashTable::~HashTable() = default;
const ccj_table *HashTable::handle() const { return t_->handle(); }

ScanStructure HashTable::Probe(Vector &join_key, size_t count, vector<uint32_t> &sel_vec) {
  return ScanStructure(t_->Run(join_key, count, sel_vec), MakeVisits(t_.get(), join_key, count, sel_vec));
}

size_t ScanStructure::EmitRound(DataChunk &input, DataChunk &result) {
  const size_t rc = res_.round_counts[round_++];
  if (rc > 0) Materialise(res_, pos_, rc, input, result);  // chaining slices only on a match (:67-76)
  pos_ += rc;
  return rc;
}

// chaining_ht.cpp:60-80 + ScanInnerJoin :82-107: repeat rounds until one matches or all ran out.
size_t ScanStructure::Next(Vector &, DataChunk &input, DataChunk &result) {
  result.Reset();
  while (HasNext()) {
    const size_t rc = EmitRound(input, result);
    if (rc > 0) return rc;
  }
  return 0;
}

// chaining_ht.cpp:138-173: exactly one round per call.
size_t ScanStructure::InOneNext(Vector &, DataChunk &input, DataChunk &result) {
  result.Reset();
  if (!HasNext()) return 0;
  visits_.Scribble(round_, input, result);  // :156, before the slice of :168
  const size_t rc = EmitRound(input, result);
  result.count_ = rc;
  return rc;
}

// ---------------------------------------------------------------------------------------------
void NaiveCompactor::Compact(unique_ptr<DataChunk> &chunk) {
  if (chunk->count_ == kBlockSize) return;  // compactor.cpp:6
  if (chunk->count_ <= kBlockSize - cached_chunk_->count_) {
    cached_chunk_->Append(*chunk, chunk->count_);
    chunk->Reset();
    return;
  }
  const size_t n_move = kBlockSize - cached_chunk_->count_;
  cached_chunk_->Append(*chunk, n_move);
  temp_chunk_->Append(*chunk, chunk->count_ - n_move, n_move);
  chunk.swap(cached_chunk_);
  cached_chunk_.swap(temp_chunk_);
  temp_chunk_ = std::make_unique<DataChunk>(types_);  // never recycle a chunk whose columns may be shared
}

}  // namespace simd_compaction_amd
