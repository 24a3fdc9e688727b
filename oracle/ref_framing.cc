// oracle/ref_framing.cc -- C-ABI harness over the REFERENCE's own log and
// table-block code, for the framing shims' parity tests.
//
// TEST INFRASTRUCTURE ONLY.  This file holds no reference code: it includes
// reference headers from /root/reference and is linked (oracle/Makefile)
// against db/log_reader.cc, db/log_writer.cc, table/format.cc, table/block.cc,
// table/iterator.cc, util/comparator.cc,
// util/{crc32c,coding,status,env}.cc and port/port_posix_sse.cc compiled
// straight from /root/reference into oracle/_ref/libref_framing.so.  The
// in-memory file classes below implement the reference's public interfaces
// (leveldb/env.h) the way its own tests do (db/log_test.cc StringDest /
// StringSource); nothing in the reference is stubbed or replaced.
// Used by oracle/gen_golden.py (tests/golden/log_cases.json) and, where
// /root/reference exists, directly by tests/test_framing.py.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>

#include "db/log_reader.h"
#include "db/log_writer.h"
#include "leveldb/env.h"
#include "leveldb/options.h"
#include "leveldb/comparator.h"
#include "leveldb/iterator.h"
#include "table/block.h"
#include "table/format.h"
#include "util/crc32c.h"

namespace {

class StringSink : public leveldb::WritableFile {
 public:
  std::string contents;
  leveldb::Status Append(const leveldb::Slice& s) override {
    contents.append(s.data(), s.size());
    return leveldb::Status::OK();
  }
  leveldb::Status Close() override { return leveldb::Status::OK(); }
  leveldb::Status Flush() override { return leveldb::Status::OK(); }
  leveldb::Status Sync() override { return leveldb::Status::OK(); }
};

class StringSource : public leveldb::SequentialFile {
 public:
  StringSource(const char* d, size_t n) : contents_(d, n) {}
  leveldb::Status Read(size_t n, leveldb::Slice* result, char* scratch) override {
    if (n > contents_.size()) n = contents_.size();
    memcpy(scratch, contents_.data(), n);
    *result = leveldb::Slice(scratch, n);
    contents_.remove_prefix(n);
    return leveldb::Status::OK();
  }
  leveldb::Status Skip(uint64_t n) override {
    if (n > contents_.size()) {
      contents_.clear();
      return leveldb::Status::NotFound("in-memory file skipped past end");
    }
    contents_.remove_prefix(n);
    return leveldb::Status::OK();
  }

 private:
  leveldb::Slice contents_;
};

// StringSource whose read covering byte `fail_at` fails: it returns the bytes
// before fail_at and IOError (a disk error in the middle of a WAL).
class FailingSource : public leveldb::SequentialFile {
 public:
  FailingSource(const char* d, size_t n, uint64_t fail_at) : d_(d), n_(n), fail_at_(fail_at) {}
  leveldb::Status Read(size_t n, leveldb::Slice* result, char* scratch) override {
    if (n > n_ - pos_) n = n_ - pos_;
    if (fail_at_ >= pos_ && fail_at_ < pos_ + n) {
      const size_t m = (size_t)(fail_at_ - pos_);
      memcpy(scratch, d_ + pos_, m);
      *result = leveldb::Slice(scratch, m);
      pos_ += m;
      return leveldb::Status::IOError("injected read failure");
    }
    memcpy(scratch, d_ + pos_, n);
    *result = leveldb::Slice(scratch, n);
    pos_ += n;
    return leveldb::Status::OK();
  }
  leveldb::Status Skip(uint64_t n) override {
    if (n > n_ - pos_) {
      pos_ = n_;
      return leveldb::Status::NotFound("in-memory file skipped past end");
    }
    pos_ += n;
    return leveldb::Status::OK();
  }

 private:
  const char* d_;
  size_t n_;
  uint64_t fail_at_;
  size_t pos_ = 0;
};

class MemRandomAccess : public leveldb::RandomAccessFile {
 public:
  MemRandomAccess(const char* d, size_t n) : d_(d), n_(n) {}
  leveldb::Status Read(uint64_t offset, size_t n, leveldb::Slice* result, char* scratch) const override {
    if (offset > n_) {
      *result = leveldb::Slice();
      return leveldb::Status::IOError("offset past end");
    }
    if (n > n_ - offset) n = n_ - offset;
    memcpy(scratch, d_ + offset, n);
    *result = leveldb::Slice(scratch, n);
    return leveldb::Status::OK();
  }

 private:
  const char* d_;
  size_t n_;
};

class TraceReporter : public leveldb::log::Reader::Reporter {
 public:
  std::string* trace;
  void Corruption(size_t bytes, const leveldb::Status& status) override {
    char buf[64];
    snprintf(buf, sizeof(buf), "C %zu ", bytes);
    trace->append(buf);
    trace->append(status.ToString());
    trace->push_back('\n');
  }
};

int copy_out(const std::string& s, void* out, size_t cap, size_t* out_len) {
  *out_len = s.size();
  if (s.size() > cap) return -5;
  memcpy(out, s.data(), s.size());
  return 0;
}

}  // namespace

extern "C" {

// log::Writer (db/log_writer.cc) over n records (payloads concatenated, lens[i]
// bytes each), appending to a file of dest_length bytes; the new bytes go to out.
__attribute__((visibility("default")))
int ref_log_write(const uint8_t* payloads, const uint64_t* lens, size_t n, uint64_t dest_length, uint8_t* out,
                  size_t cap, size_t* out_len) {
  StringSink sink;
  leveldb::log::Writer w(&sink, dest_length);
  const char* p = reinterpret_cast<const char*>(payloads);
  for (size_t i = 0; i < n; ++i) {
    if (!w.AddRecord(leveldb::Slice(p, lens[i])).ok()) return -1;
    p += lens[i];
  }
  return copy_out(sink.contents, out, cap, out_len);
}

// log::Reader (db/log_reader.cc) over a log image.  Trace lines, in order:
//   "R <LastRecordOffset> <size> <crc32c of the record>"  per record returned
//   "C <bytes> <Status::ToString()>"                      per reported drop
//   "E"                                                   when ReadRecord returns false
__attribute__((visibility("default")))
int ref_log_read(const uint8_t* file, size_t len, int checksum, uint64_t initial_offset, char* trace, size_t cap,
                 size_t* trace_len) {
  StringSource src(reinterpret_cast<const char*>(file), len);
  std::string t;
  TraceReporter rep;
  rep.trace = &t;
  leveldb::log::Reader r(&src, &rep, checksum != 0, initial_offset);
  leveldb::Slice rec;
  std::string scratch;
  while (r.ReadRecord(&rec, &scratch)) {
    char buf[96];
    snprintf(buf, sizeof(buf), "R %llu %zu %u\n", (unsigned long long)r.LastRecordOffset(), rec.size(),
             leveldb::crc32c::Value(rec.data(), rec.size()));
    t.append(buf);
  }
  t.append("E\n");
  return copy_out(t, trace, cap, trace_len);
}

// The same over a FailingSource (fail_at >= len: no failure).
__attribute__((visibility("default")))
int ref_log_read_failing(const uint8_t* file, size_t len, int checksum, uint64_t initial_offset, uint64_t fail_at,
                         char* trace, size_t cap, size_t* trace_len) {
  FailingSource src(reinterpret_cast<const char*>(file), len, fail_at);
  std::string t;
  TraceReporter rep;
  rep.trace = &t;
  leveldb::log::Reader r(&src, &rep, checksum != 0, initial_offset);
  leveldb::Slice rec;
  std::string scratch;
  while (r.ReadRecord(&rec, &scratch)) {
    char buf[96];
    snprintf(buf, sizeof(buf), "R %llu %zu %u\n", (unsigned long long)r.LastRecordOffset(), rec.size(),
             leveldb::crc32c::Value(rec.data(), rec.size()));
    t.append(buf);
  }
  t.append("E\n");
  return copy_out(t, trace, cap, trace_len);
}

// ReadBlock (table/format.cc:65-98) with verify_checksums on one block of a
// table image.  Returns 0 and an empty message when the block reads, else 1
// and the Status text.
__attribute__((visibility("default")))
int ref_read_block(const uint8_t* file, size_t len, uint64_t offset, uint64_t size, char* msg, size_t cap) {
  MemRandomAccess f(reinterpret_cast<const char*>(file), len);
  leveldb::ReadOptions opt;
  opt.verify_checksums = true;
  leveldb::BlockHandle h;
  h.set_offset(offset);
  h.set_size(size);
  leveldb::BlockContents bc;
  const leveldb::Status s = leveldb::ReadBlock(&f, opt, h, &bc);
  if (s.ok() && bc.heap_allocated) delete[] bc.data.data();
  const std::string m = s.ok() ? std::string() : s.ToString();
  snprintf(msg, cap, "%s", m.c_str());
  return s.ok() ? 0 : 1;
}

// Whole-table verification with the reference's own pieces, in the order
// Table::Open (table/table.cc:38-82) and its two-level iterator use them:
// Footer::DecodeFrom, ReadBlock(index, verify_checksums), Block::Iter over the
// index (BytewiseComparator), BlockHandle::DecodeFrom of every value and
// ReadBlock of every data block; and the same over the metaindex block and
// every block its entries point at (ReadMeta, table.cc:84-110, reads the
// "filter." one).  Trace lines:
//   "T <Status::ToString()>"            footer / index failure (then nothing else)
//   "B <role> <offset> <size> <status>" per block (role: 0 index, 1 metaindex, 2 meta, 3 data;
//                                       status "OK", a ReadBlock status, or the DecodeFrom status)
//   "S <role> <status>"                 a non-OK block iterator status after the scan
__attribute__((visibility("default")))
int ref_table_scan(const uint8_t* file, size_t len, char* trace, size_t cap, size_t* trace_len) {
  using leveldb::Status;
  MemRandomAccess f(reinterpret_cast<const char*>(file), len);
  leveldb::ReadOptions opt;
  opt.verify_checksums = true;
  std::string t;
  char buf[160];
  auto line = [&](int role, const leveldb::BlockHandle& h, const Status& s) {
    snprintf(buf, sizeof(buf), "B %d %llu %llu ", role, (unsigned long long)h.offset(),
             (unsigned long long)h.size());
    t.append(buf);
    t.append(s.ok() ? std::string("OK") : s.ToString());
    t.push_back('\n');
  };
  if (len < leveldb::Footer::kEncodedLength) {
    t = "T " + Status::Corruption("file is too short to be an sstable").ToString() + "\n";
    return copy_out(t, trace, cap, trace_len);
  }
  leveldb::Slice footer_input(reinterpret_cast<const char*>(file) + len - leveldb::Footer::kEncodedLength,
                              leveldb::Footer::kEncodedLength);
  leveldb::Footer footer;
  Status s = footer.DecodeFrom(&footer_input);
  if (!s.ok()) {
    t = "T " + s.ToString() + "\n";
    return copy_out(t, trace, cap, trace_len);
  }
  // one block and, when it reads, the blocks its entries point at
  auto walk = [&](const leveldb::BlockHandle& bh, int role, int child_role) -> bool {
    leveldb::BlockContents bc;
    Status rs = leveldb::ReadBlock(&f, opt, bh, &bc);
    line(role, bh, rs);
    if (!rs.ok()) return false;
    {
      leveldb::Block block(bc);  // owns bc.data when heap_allocated
      leveldb::Iterator* it = block.NewIterator(leveldb::BytewiseComparator());
      for (it->SeekToFirst(); it->Valid(); it->Next()) {
        leveldb::BlockHandle h;
        leveldb::Slice v = it->value();
        Status hs = h.DecodeFrom(&v);
        if (!hs.ok()) {
          leveldb::BlockHandle z;
          z.set_offset(0);
          z.set_size(0);
          line(child_role, z, hs);
          continue;
        }
        leveldb::BlockContents c;
        // ReadBlock allocates size + 5 bytes before it reads; a handle larger
        // than the file cannot be read from it (the Read would come back short)
        Status cs = h.size() > len ? Status::Corruption("truncated block read") : leveldb::ReadBlock(&f, opt, h, &c);
        if (cs.ok() && c.heap_allocated) delete[] c.data.data();
        line(child_role, h, cs);
      }
      if (!it->status().ok()) {
        snprintf(buf, sizeof(buf), "S %d ", role);
        t.append(buf);
        t.append(it->status().ToString());
        t.push_back('\n');
      }
      delete it;
    }
    return true;
  };
  if (!walk(footer.index_handle(), 0, 3)) {
    return copy_out(t, trace, cap, trace_len);
  }
  walk(footer.metaindex_handle(), 1, 2);
  return copy_out(t, trace, cap, trace_len);
}

}  // extern "C"
