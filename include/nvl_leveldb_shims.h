// include/nvl_leveldb_shims.h -- C++ call-site shims of SURVEY.md §8f on top
// of include/nvl_framing.h: the reference's log::Reader / log::Writer and
// TableBuilder's block trailers with every CRC of a file computed in one GPU
// batch.  Header-only, C++11, no LevelDB headers needed: the classes keep the
// reference's method names and semantics, and INTEGRATION.md shows the
// adapters (Slice, Status, SequentialFile, WritableFile) for a LevelDB tree.
//
//   nvl::shims::LogReader   db/log_reader.h:20-120, db/log_reader.cc:17-281
//   nvl::shims::LogWriter   db/log_writer.h:18-47, db/log_writer.cc:17-109
//   nvl::shims::TableFile   TableBuilder::WriteRawBlock table/table_builder.cc:175-193
//                           + the checks of ReadBlock table/format.cc:65-98
//   nvl::shims::BatchingWritableFile  the WritableFile adapter around a table's file
//   nvl::shims::TableReader Table::Open + Table::BlockReader table/table.cc:38-82,163-215,
//                           checks batched per readahead window
#ifndef NVL_LEVELDB_SHIMS_H_
#define NVL_LEVELDB_SHIMS_H_

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#include <string>
#include <vector>

#include "nvl_framing.h"

namespace nvl {
namespace shims {

// ---------------------------------------------------------------------------
// The input of a streaming LogReader: leveldb::SequentialFile's contract
// (include/leveldb/env.h, SequentialFile::Read/Skip).  Read fills up to n
// bytes at buf and returns how many it read; a short read means the end of
// the file.  On failure it sets *error to the Status text (e.g. "IO error:
// ...") and returns the bytes it did read before the failure.
class LogSource {
 public:
  virtual ~LogSource() {}
  virtual size_t Read(size_t n, char* buf, std::string* error) = 0;
  virtual bool Skip(uint64_t n, std::string* error) = 0;
};

// log::Reader.  Two inputs:
//   * an image held in memory (the whole file, or its part from block offset
//     0): the first ReadRecord scans it once -- every physical record's
//     checksum in one batch;
//   * a LogSource read in windows of `window_blocks` kBlockSize pieces (the
//     reference reads one piece at a time, log_reader.cc:199-218): each
//     window's checksums go in one batch, so a file larger than memory, or
//     one still being written, is read as the reference reads it.
// The record-level state machine of log_reader.cc:62-175 then replays the
// scan.  Corruption reports carry the reference's byte counts and reason
// strings; a failed read is reported as the reference's ReportDrop(kBlockSize,
// status) (:205-211), through Reporter::Drop.
class LogReader {
 public:
  // log_reader.h:22-30 (the reason is the text of the Status::Corruption).
  class Reporter {
   public:
    virtual ~Reporter() {}
    virtual void Corruption(size_t bytes, const char* reason) = 0;
    // A drop whose Status is not a Corruption (a failed read or skip of a
    // streaming source): `status` is its full text.
    virtual void Drop(size_t bytes, const char* status) { Corruption(bytes, status); }
  };

  // log_reader.h:32-44.  `file` must stay live while the reader is used;
  // `flags`: 0 = the size policy (nvl_framing_uses_gpu), NVL_FRAMING_HOST / NVL_FRAMING_GPU force an engine.
  LogReader(const char* file, uint64_t file_len, Reporter* reporter, bool checksum, uint64_t initial_offset,
            uint32_t flags = 0)
      : file_(file),
        file_len_(file_len),
        src_(nullptr),
        window_blocks_(0),
        reporter_(reporter),
        checksum_(checksum),
        flags_(flags),
        initial_offset_(initial_offset),
        resyncing_(initial_offset > 0) {}

  // Streaming: `src` is positioned at file offset 0 and must outlive the
  // reader; each refill reads window_blocks * kBlockSize bytes.
  LogReader(LogSource* src, Reporter* reporter, bool checksum, uint64_t initial_offset, uint32_t flags = 0,
            size_t window_blocks = 16)
      : file_(nullptr),
        file_len_(0),
        src_(src),
        window_blocks_(window_blocks ? window_blocks : 1),
        reporter_(reporter),
        checksum_(checksum),
        flags_(flags),
        initial_offset_(initial_offset),
        resyncing_(initial_offset > 0) {}

  // log_reader.h:46-52.  False at the end of the input, or when the batch
  // scan failed (status() != NVL_CRC32C_OK; nothing is returned then).
  bool ReadRecord(const char** data, size_t* size, std::string* scratch) {
    if (!scanned_) Scan();
    scratch->clear();
    *data = "";
    *size = 0;
    if (status_ != NVL_CRC32C_OK || skip_failed_) return false;
    bool in_fragmented_record = false;
    uint64_t prospective_record_offset = 0;
    const char* frag = "";
    size_t frag_n = 0;
    while (true) {
      const unsigned record_type = ReadPhysicalRecord(&frag, &frag_n);
      const uint64_t physical_record_offset = pos_ - kHeader - frag_n;
      if (resyncing_) {  // log_reader.cc:86-95
        if (record_type == kMiddleType) {
          continue;
        } else if (record_type == kLastType) {
          resyncing_ = false;
          continue;
        } else {
          resyncing_ = false;
        }
      }
      switch (record_type) {
        case kFullType:
          if (in_fragmented_record) {
            if (scratch->empty()) in_fragmented_record = false;
            else ReportCorruption(scratch->size(), "partial record without end(1)");
          }
          prospective_record_offset = physical_record_offset;
          scratch->clear();
          *data = frag;
          *size = frag_n;
          last_record_offset_ = prospective_record_offset;
          return true;
        case kFirstType:
          if (in_fragmented_record) {
            if (scratch->empty()) in_fragmented_record = false;
            else ReportCorruption(scratch->size(), "partial record without end(2)");
          }
          prospective_record_offset = physical_record_offset;
          scratch->assign(frag, frag_n);
          in_fragmented_record = true;
          break;
        case kMiddleType:
          if (!in_fragmented_record) ReportCorruption(frag_n, "missing start of fragmented record(1)");
          else scratch->append(frag, frag_n);
          break;
        case kLastType:
          if (!in_fragmented_record) {
            ReportCorruption(frag_n, "missing start of fragmented record(2)");
          } else {
            scratch->append(frag, frag_n);
            *data = scratch->data();
            *size = scratch->size();
            last_record_offset_ = prospective_record_offset;
            return true;
          }
          break;
        case kEof:
          if (in_fragmented_record) scratch->clear();
          return false;
        case kBadRecord:
          if (in_fragmented_record) {
            ReportCorruption(scratch->size(), "error in middle of record");
            in_fragmented_record = false;
            scratch->clear();
          }
          break;
        default: {
          char buf[40];
          snprintf(buf, sizeof(buf), "unknown record type %u", record_type);
          ReportCorruption(frag_n + (in_fragmented_record ? scratch->size() : 0), buf);
          in_fragmented_record = false;
          scratch->clear();
          break;
        }
      }
    }
  }

  // The same for any Slice type with Slice(const char*, size_t).
  template <class Slice>
  bool ReadRecord(Slice* record, std::string* scratch) {
    const char* d;
    size_t n;
    const bool ok = ReadRecord(&d, &n, scratch);
    *record = Slice(d, n);
    return ok;
  }

  // log_reader.h:54-58
  uint64_t LastRecordOffset() const { return last_record_offset_; }

  int status() const { return status_; }

 private:
  enum : unsigned { kZeroType = 0, kFullType = 1, kFirstType = 2, kMiddleType = 3, kLastType = 4 };
  enum : unsigned { kEof = kLastType + 1, kBadRecord = kLastType + 2 };  // log_reader.h:84-92
  static const uint64_t kBlock = NVL_LOG_BLOCK_SIZE;
  static const uint64_t kHeader = NVL_LOG_HEADER_SIZE;

  // SkipToInitialBlock (log_reader.cc:36-60), then the one batch scan (or,
  // streaming, the first window).
  void Scan() {
    scanned_ = true;
    uint64_t in_block = initial_offset_ % kBlock;
    uint64_t block_start = initial_offset_ - in_block;
    if (in_block > kBlock - 6) block_start += kBlock;  // don't search a block if we'd be in the trailer
    pos_ = block_start;
    next_ = 0;
    if (src_) {
      win_start_ = block_start;
      if (block_start > 0) {
        std::string err;
        if (!src_->Skip(block_start, &err)) {  // ReportDrop(block_start_location, skip_status), unsigned as there
          if (reporter_ != nullptr && pos_ - block_start >= initial_offset_) reporter_->Drop((size_t)block_start, err.c_str());
          skip_failed_ = true;
          return;
        }
      }
      NextWindow();
      return;
    }
    if (block_start >= file_len_) {  // skipped to (or past) the end: the first read finds nothing
      nvl_log_event eof = {block_start, block_start, 0u, 0u, NVL_LOG_EOF, 0u};
      events_.assign(1, eof);
      return;
    }
    const uint64_t n = file_len_ - block_start;
    size_t ne = 0;
    const size_t cap = (size_t)(n / kHeader + n / kBlock + 4);  // bound on the event count
    events_.resize(cap);
    status_ = nvl_log_scan(file_ + block_start, n, block_start, checksum_ ? 1 : 0, events_.data(), cap, &ne, flags_);
    events_.resize(status_ == NVL_CRC32C_OK ? ne : 0);
  }

  // Streaming: read the next window and scan it.  A full window is not the
  // end of the file (the reference's eof_ stays false after a full piece),
  // so its scan's closing EOF event is dropped and the next refill decides;
  // a short window ends the file.  A failed read: the whole pieces read
  // before it are scanned, then the drop of the failing piece is reported
  // and the reader is at its end (log_reader.cc:205-211).
  void NextWindow() {
    events_.clear();
    next_ = 0;
    if (src_eof_) {
      nvl_log_event eof = {win_start_, win_start_, 0u, 0u, NVL_LOG_EOF, 0u};
      events_.assign(1, eof);
      return;
    }
    const size_t want = (size_t)(window_blocks_ * kBlock);
    win_.resize(want);
    std::string err;
    const size_t got = src_->Read(want, &win_[0], &err);
    const bool failed = !err.empty();
    const uint64_t start = win_start_;
    // pieces the reference would parse: every whole one; the last, short one
    // too unless the read failed inside it
    const uint64_t parse = failed ? (uint64_t)got / kBlock * kBlock : (uint64_t)got;
    if (parse > 0) {
      const size_t cap = (size_t)(parse / kHeader + parse / kBlock + 4);
      events_.resize(cap);
      size_t ne = 0;
      status_ = nvl_log_scan(win_.data(), parse, start, checksum_ ? 1 : 0, events_.data(), cap, &ne, flags_);
      events_.resize(status_ == NVL_CRC32C_OK ? ne : 0);
      if (status_ != NVL_CRC32C_OK) return;
      if (!events_.empty() && events_.back().kind == NVL_LOG_EOF) events_.pop_back();
    }
    win_start_ = start + parse;
    win_parsed_ = parse;
    if (failed) {
      fail_end_ = start + got;  // end_of_buffer_offset_ after the failing Read
      fail_msg_ = err;
      src_eof_ = true;
      has_fail_ = true;
    } else if (got < want) {
      src_eof_ = true;
      // a short window: its scan's EOF (a truncated record at the end of
      // the file is not a corruption) ends the stream
      nvl_log_event eof = {start + got, start + got, 0u, 0u, NVL_LOG_EOF, 0u};
      events_.push_back(eof);
    }
  }

  // ReadPhysicalRecord (log_reader.cc:199-281) replayed from the scan.
  // pos_ mirrors end_of_buffer_offset_ - buffer_.size().
  unsigned ReadPhysicalRecord(const char** frag, size_t* frag_n) {
    while (src_ && next_ >= events_.size()) {
      if (status_ != NVL_CRC32C_OK) return kEof;
      if (has_fail_) {  // the failing piece: ReportDrop(kBlockSize, status), then the end
        has_fail_ = false;
        pos_ = fail_end_;
        if (reporter_ != nullptr && pos_ - kBlock >= initial_offset_) reporter_->Drop((size_t)kBlock, fail_msg_.c_str());
        nvl_log_event eof = {fail_end_, fail_end_, 0u, 0u, NVL_LOG_EOF, 0u};
        events_.assign(1, eof);
        next_ = 0;
        break;
      }
      NextWindow();
    }
    if (next_ >= events_.size()) return kEof;
    const nvl_log_event& e = events_[next_];
    switch (e.kind) {
      case NVL_LOG_RECORD:
        ++next_;
        pos_ = e.offset + kHeader + e.length;
        if (e.offset < initial_offset_) {  // started before initial_offset_ (:270-275)
          *frag = "";
          *frag_n = 0;
          return kBadRecord;
        }
        *frag = (src_ ? win_.data() + (e.offset - (win_start_ - win_parsed())) : file_ + e.offset) + kHeader;
        *frag_n = e.length;
        return e.type;
      case NVL_LOG_BAD_LENGTH:
        ++next_;
        pos_ = e.block_end;
        ReportCorruption(e.block_end - e.offset, "bad record length");
        return kBadRecord;
      case NVL_LOG_CHECKSUM:
        ++next_;
        pos_ = e.block_end;
        ReportCorruption(e.block_end - e.offset, "checksum mismatch");
        return kBadRecord;
      case NVL_LOG_ZERO:
        ++next_;
        pos_ = e.block_end;
        return kBadRecord;
      default:  // NVL_LOG_EOF: stays at the end
        pos_ = e.block_end;
        return kEof;
    }
  }

  // ReportCorruption / ReportDrop (log_reader.cc:181-190), unsigned arithmetic as there.
  void ReportCorruption(uint64_t bytes, const char* reason) {
    if (reporter_ != nullptr && pos_ - bytes >= initial_offset_) reporter_->Corruption((size_t)bytes, reason);
  }

  // bytes of win_ that the current events were scanned from
  uint64_t win_parsed() const { return win_parsed_; }

  const char* const file_;
  const uint64_t file_len_;
  LogSource* const src_;
  const size_t window_blocks_;
  Reporter* const reporter_;
  const bool checksum_;
  const uint32_t flags_;
  const uint64_t initial_offset_;
  bool resyncing_;
  bool scanned_ = false;
  int status_ = NVL_CRC32C_OK;
  std::vector<nvl_log_event> events_;
  size_t next_ = 0;
  uint64_t pos_ = 0;
  uint64_t last_record_offset_ = 0;
  // streaming state
  std::string win_;
  uint64_t win_start_ = 0;   // file offset just past the window parsed last
  uint64_t win_parsed_ = 0;  // bytes of it parsed
  bool src_eof_ = false, has_fail_ = false, skip_failed_ = false;
  uint64_t fail_end_ = 0;
  std::string fail_msg_;
};

// ---------------------------------------------------------------------------
// log::Writer that stages physical records (fragmentation and block trailers
// exactly as log_writer.cc:36-82) and seals all their headers in one batch
// when the bytes are taken.  Byte-identical output to the reference writer.
class LogWriter {
 public:
  // log_writer.h:22-30: a writer appending to a file of dest_length bytes.
  explicit LogWriter(uint64_t dest_length = 0) : block_offset_(dest_length % NVL_LOG_BLOCK_SIZE) {}

  // log_writer.cc:36-82.
  void AddRecord(const char* ptr, size_t left) {
    bool begin = true;
    do {
      const uint64_t leftover = kBlock - block_offset_;
      if (leftover < kHeader) {  // switch to a new block, zero-filling the trailer
        buf_.append((size_t)leftover, '\0');
        block_offset_ = 0;
      }
      const size_t avail = (size_t)(kBlock - block_offset_ - kHeader);
      const size_t fragment_length = left < avail ? left : avail;
      const bool end = left == fragment_length;
      const unsigned type = begin && end ? 1u : begin ? 2u : end ? 4u : 3u;  // Full, First, Last, Middle
      EmitPhysicalRecord(type, ptr, fragment_length);
      ptr += fragment_length;
      left -= fragment_length;
      begin = false;
    } while (left > 0);
  }

  // Seal every staged header (one batch) and move the bytes into *out.
  int Take(std::string* out, uint32_t flags = 0) {
    const int rc = nvl_log_seal(&buf_[0], buf_.size(), headers_.data(), headers_.size(), flags);
    if (rc != NVL_CRC32C_OK) return rc;
    out->append(buf_);
    buf_.clear();
    headers_.clear();
    return NVL_CRC32C_OK;
  }

  size_t pending_bytes() const { return buf_.size(); }
  size_t pending_records() const { return headers_.size(); }

 private:
  static const uint64_t kBlock = NVL_LOG_BLOCK_SIZE;
  static const uint64_t kHeader = NVL_LOG_HEADER_SIZE;

  // log_writer.cc:84-109 with the CRC left for Take().
  void EmitPhysicalRecord(unsigned t, const char* ptr, size_t n) {
    headers_.push_back(buf_.size());
    const char h[NVL_LOG_HEADER_SIZE] = {0, 0, 0, 0, (char)(n & 0xff), (char)(n >> 8), (char)t};
    buf_.append(h, kHeader);
    buf_.append(ptr, n);
    block_offset_ += kHeader + n;
  }

  uint64_t block_offset_;
  std::string buf_;
  std::vector<uint64_t> headers_;
};

// ---------------------------------------------------------------------------
// An SSTable being written: TableBuilder appends raw bytes and blocks here
// instead of to its WritableFile; block offsets never depend on CRC values
// (fixed 5-byte trailer), so the trailers are sealed in one batch when the
// image is complete (TableBuilder::Finish, table_builder.cc:199-253).
class TableFile {
 public:
  void Append(const char* data, size_t n) { image_.append(data, n); }

  // WriteRawBlock (table_builder.cc:175-193) with the CRC deferred: returns
  // the BlockHandle {offset, size}.
  nvl_block_handle AppendBlock(const char* contents, size_t n, uint8_t type) {
    nvl_block_handle h{image_.size(), n};
    image_.append(contents, n);
    const char trailer[NVL_BLOCK_TRAILER_SIZE] = {(char)type, 0, 0, 0, 0};
    image_.append(trailer, NVL_BLOCK_TRAILER_SIZE);
    blocks_.push_back(h);
    return h;
  }

  // All trailers in one batch; the image is then byte-identical to the
  // reference builder's file.
  int Seal(uint32_t flags = 0) {
    return nvl_sstable_seal_trailers(&image_[0], image_.size(), blocks_.data(), blocks_.size(), flags);
  }

  uint64_t size() const { return image_.size(); }
  const std::string& image() const { return image_; }
  const std::vector<nvl_block_handle>& blocks() const { return blocks_; }

 private:
  std::string image_;
  std::vector<nvl_block_handle> blocks_;
};

// ---------------------------------------------------------------------------
// The writer-side adapter a LevelDB tree drops in around a table's file
// (SURVEY.md §8f rank 1): TableBuilder writes into it through the ordinary
// leveldb::WritableFile interface; WriteRawBlock's two Appends per block --
// the contents, then the 5-byte trailer (table/table_builder.cc:175-193) --
// stage the block with a placeholder CRC, and every staged trailer is sealed
// (Mask(Value(block | type)), one GPU batch) when the staged bytes pass
// `seal_bytes`, at Sync() and at Close(), before the bytes reach `target`.
// Block offsets never depend on CRC values (fixed 5-byte trailer), so the
// file is byte-identical to the reference builder's.  Flush() is a hint
// TableBuilder gives after every data block (table_builder.cc:146): it seals
// nothing, so a table's blocks batch together.  The template takes the
// tree's own types: BatchingWritableFile<leveldb::WritableFile,
// leveldb::Slice, leveldb::Status>.
//
// With the stock WriteRawBlock the reference still computes a CRC per block
// and this adapter discards it; the two-line edit of INTEGRATION.md §5
// (skip the CRC when DefersBlockCrc(r->file)) leaves the CRCs to the batch
// alone.  DeferredBlockCrc is the marker that edit tests for.
class DeferredBlockCrc {
 public:
  virtual ~DeferredBlockCrc() {}
};

// True when `file` (a leveldb::WritableFile*) seals block trailers itself.
template <class F>
inline bool DefersBlockCrc(F* file) {
  return file != nullptr && dynamic_cast<DeferredBlockCrc*>(file) != nullptr;
}

template <class WritableFileT, class SliceT, class StatusT>
class BatchingWritableFile : public WritableFileT, public DeferredBlockCrc {
 public:
  // target: receives every sealed byte (not owned; Close() closes it).
  // flags: 0 = the size policy; NVL_FRAMING_HOST / NVL_FRAMING_GPU force the host CRC / the GPU.
  explicit BatchingWritableFile(WritableFileT* target, uint64_t seal_bytes = 64ull << 20, uint32_t flags = 0)
      : target_(target), seal_bytes_(seal_bytes), flags_(flags) {}

  StatusT Append(const SliceT& data) override {
    if (have_ && data.size() == NVL_BLOCK_TRAILER_SIZE) {  // the trailer of the pending block
      const char* t = data.data();
      computed_ += (t[1] | t[2] | t[3] | t[4]) != 0;  // a CRC the writer computed (discarded here)
      const nvl_block_handle h = tf_.AppendBlock(pending_.data(), pending_.size(), (uint8_t)t[0]);
      handles_.push_back(nvl_block_handle{written_ + h.offset, h.size});
      have_ = false;
      pending_.clear();
      return tf_.size() >= seal_bytes_ ? Drain() : StatusT::OK();
    }
    StageRaw();
    pending_.assign(data.data(), data.size());
    have_ = true;
    return StatusT::OK();
  }
  StatusT Flush() override { return StatusT::OK(); }
  StatusT Sync() override {
    StageRaw();
    StatusT s = Drain();
    return s.ok() ? target_->Sync() : s;
  }
  StatusT Close() override {
    StageRaw();
    StatusT s = Drain();
    return s.ok() ? target_->Close() : s;
  }

  size_t seals() const { return seals_; }                    // batches issued
  const std::string& staged() const { return tf_.image(); }  // (tests: the bytes before sealing)
  // every block staged so far, {offset in the file, size}, in write order
  const std::vector<nvl_block_handle>& handles() const { return handles_; }
  // trailers that arrived with a nonzero CRC: the writer computed one (the
  // stock WriteRawBlock); 0 with INTEGRATION.md §5's edit
  size_t computed_crcs() const { return computed_; }

 private:
  // a pending Append that no trailer followed (the footer): plain bytes
  void StageRaw() {
    if (have_) tf_.Append(pending_.data(), pending_.size());
    have_ = false;
    pending_.clear();
  }
  // seal the staged trailers (one batch) and hand the bytes to the target
  StatusT Drain() {
    if (tf_.size() == 0) return StatusT::OK();
    if (!tf_.blocks().empty()) {
      const int rc = tf_.Seal(flags_);
      ++seals_;
      if (rc != NVL_CRC32C_OK) return StatusT::IOError(SliceT("nvl_sstable_seal_trailers"), SliceT(nvl_crc32c_strerror(rc)));
    }
    StatusT s = target_->Append(SliceT(tf_.image().data(), tf_.image().size()));
    written_ += tf_.size();
    tf_ = TableFile();
    return s;
  }

  WritableFileT* target_;
  uint64_t seal_bytes_;
  uint32_t flags_;
  TableFile tf_;
  std::string pending_;
  bool have_ = false;
  size_t seals_ = 0;
  size_t computed_ = 0;
  uint64_t written_ = 0;
  std::vector<nvl_block_handle> handles_;
};

// ---------------------------------------------------------------------------
// The reader-side shim of SURVEY.md §8f rank 2: Table::Open (footer, index
// and metaindex, table/table.cc:38-82) and Table::BlockReader
// (table.cc:163-215, ReadBlock with verify_checksums) over a table image in
// memory (an mmap'd file, util/env_posix.cc:199-209), with the checks of the
// blocks an iterator touches batched per readahead window: the first read of
// data block i checks data blocks [i, i + window) -- those not yet checked --
// in one batch, as a compaction input scan (db/version_set.cc:1308,1329)
// walks them in index order.  Meta blocks (the filter) are checked at Open in
// one batch.  Verdicts are ReadBlock's (NVL_BLOCK_*); a block whose index
// value is not a handle reads as NVL_BLOCK_BAD_HANDLE, as BlockReader's
// "bad block handle".
class TableReader {
 public:
  TableReader(const char* file, uint64_t file_len, size_t window_blocks = 64, uint32_t flags = 0)
      : file_(file), len_(file_len), window_(window_blocks ? window_blocks : 1), flags_(flags) {}

  // *table_status = NVL_TABLE_*; the index/metaindex and meta blocks listed
  // and checked.  Returns the engine status.
  int Open(uint32_t* table_status) {
    size_t n = 0;
    uint64_t bad = 0;
    int rc = nvl_sstable_verify_table(file_, len_, nullptr, 0, &n, table_status, &bad, flags_);
    if (rc != NVL_CRC32C_OK) return rc;
    blocks_.resize(n);
    rc = nvl_sstable_verify_table(file_, len_, blocks_.data(), n, &n, table_status, &bad,
                                  flags_ | NVL_TABLE_LIST_ONLY);
    if (rc != NVL_CRC32C_OK) return rc;
    blocks_.resize(n);
    data_.clear();
    std::vector<size_t> meta;
    for (size_t i = 0; i < blocks_.size(); ++i) {
      if (blocks_[i].role == NVL_TBLOCK_DATA) data_.push_back(i);
      // (a metaindex value that is not a handle is listed as BAD_HANDLE with
      // offset = size = 0: nothing to read, as BlockReader's "bad block handle")
      if (blocks_[i].role == NVL_TBLOCK_META && blocks_[i].verdict == NVL_BLOCK_UNCHECKED) meta.push_back(i);
    }
    return Check(meta);
  }

  size_t num_data_blocks() const { return data_.size(); }

  // Data block i (index order): its handle and ReadBlock verdict; the block's
  // contents are file + h->offset, h->size bytes.
  int ReadDataBlock(size_t i, nvl_block_handle* h, uint32_t* verdict) {
    if (i >= data_.size()) return NVL_CRC32C_EINVAL;
    nvl_table_block& b = blocks_[data_[i]];
    if (b.verdict == NVL_BLOCK_UNCHECKED) {
      std::vector<size_t> win;
      for (size_t k = i; k < data_.size() && win.size() < window_; ++k)
        if (blocks_[data_[k]].verdict == NVL_BLOCK_UNCHECKED) win.push_back(data_[k]);
      const int rc = Check(win);
      if (rc != NVL_CRC32C_OK) return rc;
    }
    h->offset = b.offset;
    h->size = b.size;
    *verdict = b.verdict;
    return NVL_CRC32C_OK;
  }

  // every listed block (index, metaindex, meta, data), with the verdicts so far
  const std::vector<nvl_table_block>& blocks() const { return blocks_; }
  size_t batches() const { return batches_; }

 private:
  int Check(const std::vector<size_t>& which) {
    if (which.empty()) return NVL_CRC32C_OK;
    std::vector<nvl_block_handle> h(which.size());
    for (size_t k = 0; k < which.size(); ++k) h[k] = nvl_block_handle{blocks_[which[k]].offset, blocks_[which[k]].size};
    std::vector<uint8_t> v(which.size(), NVL_BLOCK_OK);
    const int rc = nvl_sstable_verify_blocks(file_, len_, h.data(), h.size(), v.data(), nullptr, flags_);
    ++batches_;
    if (rc != NVL_CRC32C_OK) return rc;
    for (size_t k = 0; k < which.size(); ++k) blocks_[which[k]].verdict = v[k];
    return NVL_CRC32C_OK;
  }

  const char* file_;
  uint64_t len_;
  size_t window_;
  uint32_t flags_;
  std::vector<nvl_table_block> blocks_;
  std::vector<size_t> data_;
  size_t batches_ = 0;
};

// ReadBlock's checks (format.cc:77-135) for every block of a table image in
// one batch; verdict[i] = NVL_BLOCK_*.  Returns the batch status.
inline int VerifyBlocks(const char* file, uint64_t file_len, const std::vector<nvl_block_handle>& blocks,
                        std::vector<uint8_t>* verdict, uint64_t* n_bad, uint32_t flags = 0) {
  verdict->assign(blocks.size(), NVL_BLOCK_OK);
  return nvl_sstable_verify_blocks(file, file_len, blocks.data(), blocks.size(), verdict->data(), n_bad, flags);
}

// Whole-table verification (Table::Open's footer and index read,
// table/table.cc:38-82, then ReadBlock with verify_checksums of every block
// the index and metaindex point at) in one batch: *table_status gets
// NVL_TABLE_*, blocks the listed blocks with their roles and verdicts.
inline int VerifyTable(const char* file, uint64_t file_len, std::vector<nvl_table_block>* blocks,
                       uint32_t* table_status, uint64_t* n_bad, uint32_t flags = 0) {
  size_t n = 0;
  int rc = nvl_sstable_verify_table(file, file_len, nullptr, 0, &n, table_status, n_bad, flags);
  if (rc != NVL_CRC32C_OK) return rc;
  blocks->resize(n);
  rc = nvl_sstable_verify_table(file, file_len, blocks->data(), n, &n, table_status, n_bad, flags);
  blocks->resize(rc == NVL_CRC32C_OK ? n : 0);
  return rc;
}

}  // namespace shims
}  // namespace nvl

#endif  // NVL_LEVELDB_SHIMS_H_
