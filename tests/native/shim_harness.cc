// tests/native/shim_harness.cc -- extern "C" driver of the header-only shims
// (include/nvl_leveldb_shims.h) for tests/test_framing.py: the same call
// sequence and trace format as oracle/ref_framing.cc drives the reference's
// log::Writer / log::Reader with, so the two traces compare line for line.
// This is the binding a LevelDB test would add; it is test code, not product.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>

#include "nvl_leveldb_shims.h"

namespace {

struct TraceReporter : nvl::shims::LogReader::Reporter {
  std::string* trace;
  void Corruption(size_t bytes, const char* reason) override {
    char buf[64];
    snprintf(buf, sizeof(buf), "C %zu Corruption: ", bytes);
    trace->append(buf);
    trace->append(reason);
    trace->push_back('\n');
  }
  void Drop(size_t bytes, const char* status) override {
    char buf[64];
    snprintf(buf, sizeof(buf), "C %zu ", bytes);
    trace->append(buf);
    trace->append(status);
    trace->push_back('\n');
  }
};

// A LogSource over memory whose read covering byte fail_at fails (the bytes
// before it are returned), as oracle/ref_framing.cc's FailingSource.
struct MemSource : nvl::shims::LogSource {
  const char* d;
  size_t n;
  uint64_t fail_at;
  size_t pos = 0;
  size_t reads = 0;
  size_t Read(size_t want, char* buf, std::string* error) override {
    ++reads;
    if (want > n - pos) want = n - pos;
    if (fail_at >= pos && fail_at < pos + want) {
      const size_t m = (size_t)(fail_at - pos);
      memcpy(buf, d + pos, m);
      pos += m;
      *error = "IO error: injected read failure";
      return m;
    }
    memcpy(buf, d + pos, want);
    pos += want;
    return want;
  }
  bool Skip(uint64_t k, std::string* error) override {
    if (k > n - pos) {
      pos = n;
      *error = "NotFound: in-memory file skipped past end";
      return false;
    }
    pos += k;
    return true;
  }
};

int copy_out(const std::string& s, void* out, size_t cap, size_t* out_len) {
  *out_len = s.size();
  if (s.size() > cap) return NVL_CRC32C_ENOSPC;
  memcpy(out, s.data(), s.size());
  return NVL_CRC32C_OK;
}

}  // namespace

extern "C" {

// nvl::shims::LogWriter over n records (payloads concatenated), appending to a
// file of dest_length bytes; the sealed new bytes go to out.
__attribute__((visibility("default")))
int shim_log_write(const uint8_t* payloads, const uint64_t* lens, size_t n, uint64_t dest_length, uint32_t flags,
                   uint8_t* out, size_t cap, size_t* out_len) {
  nvl::shims::LogWriter w(dest_length);
  const char* p = reinterpret_cast<const char*>(payloads);
  for (size_t i = 0; i < n; ++i) {
    w.AddRecord(p, lens[i]);
    p += lens[i];
  }
  std::string img;
  const int rc = w.Take(&img, flags);
  if (rc != NVL_CRC32C_OK) return rc;
  return copy_out(img, out, cap, out_len);
}

// nvl::shims::LogReader over a log image; trace format of ref_log_read.
__attribute__((visibility("default")))
int shim_log_read(const uint8_t* file, size_t len, int checksum, uint64_t initial_offset, uint32_t flags,
                  char* trace, size_t cap, size_t* trace_len) {
  std::string t;
  TraceReporter rep;
  rep.trace = &t;
  nvl::shims::LogReader r(reinterpret_cast<const char*>(file), len, &rep, checksum != 0, initial_offset, flags);
  const char* d;
  size_t n;
  std::string scratch;
  while (r.ReadRecord(&d, &n, &scratch)) {
    char buf[96];
    snprintf(buf, sizeof(buf), "R %llu %zu %u\n", (unsigned long long)r.LastRecordOffset(), n,
             nvl_crc32c_value(d, n));
    t.append(buf);
  }
  if (r.status() != NVL_CRC32C_OK) return r.status();
  t.append("E\n");
  return copy_out(t, trace, cap, trace_len);
}

// The streaming LogReader over a MemSource read window_blocks pieces at a
// time; same trace, plus the number of source reads in *reads.
__attribute__((visibility("default")))
int shim_log_read_stream(const uint8_t* file, size_t len, int checksum, uint64_t initial_offset, uint32_t flags,
                         size_t window_blocks, uint64_t fail_at, char* trace, size_t cap, size_t* trace_len,
                         size_t* reads) {
  std::string t;
  TraceReporter rep;
  rep.trace = &t;
  MemSource src;
  src.d = reinterpret_cast<const char*>(file);
  src.n = len;
  src.fail_at = fail_at;
  nvl::shims::LogReader r(&src, &rep, checksum != 0, initial_offset, flags, window_blocks);
  const char* d;
  size_t n;
  std::string scratch;
  while (r.ReadRecord(&d, &n, &scratch)) {
    char buf[96];
    snprintf(buf, sizeof(buf), "R %llu %zu %u\n", (unsigned long long)r.LastRecordOffset(), n,
             nvl_crc32c_value(d, n));
    t.append(buf);
  }
  if (r.status() != NVL_CRC32C_OK) return r.status();
  t.append("E\n");
  *reads = src.reads;
  return copy_out(t, trace, cap, trace_len);
}

// nvl::shims::VerifyTable over a table image: "<status> <n_bad>" then one
// "<offset> <size> <role> <verdict>" line per listed block.
__attribute__((visibility("default")))
int shim_table_verify(const uint8_t* file, size_t len, uint32_t flags, char* trace, size_t cap, size_t* trace_len) {
  std::vector<nvl_table_block> blocks;
  uint32_t status = 0;
  uint64_t n_bad = 0;
  const int rc = nvl::shims::VerifyTable(reinterpret_cast<const char*>(file), len, &blocks, &status, &n_bad, flags);
  if (rc != NVL_CRC32C_OK) return rc;
  char buf[96];
  snprintf(buf, sizeof(buf), "%u %llu\n", status, (unsigned long long)n_bad);
  std::string t(buf);
  for (size_t i = 0; i < blocks.size(); ++i) {
    snprintf(buf, sizeof(buf), "%llu %llu %u %u\n", (unsigned long long)blocks[i].offset,
             (unsigned long long)blocks[i].size, blocks[i].role, blocks[i].verdict);
    t.append(buf);
  }
  return copy_out(t, trace, cap, trace_len);
}

// nvl::shims::TableReader: Open, then every data block read in index order
// (order 0) or backwards (order 1) with `window` blocks checked per batch;
// the trace has shim_table_verify's format (every listed block with its
// verdict after the reads) and *batches the verify batches issued.
int shim_table_read(const uint8_t* file, size_t len, size_t window, uint32_t flags, int order, char* trace, size_t cap,
                    size_t* trace_len, size_t* batches) {
  nvl::shims::TableReader tr(reinterpret_cast<const char*>(file), len, window, flags);
  uint32_t status = 0;
  int rc = tr.Open(&status);
  if (rc != NVL_CRC32C_OK) return rc;
  const size_t nd = tr.num_data_blocks();
  for (size_t k = 0; k < nd; ++k) {
    const size_t i = order ? nd - 1 - k : k;
    nvl_block_handle h;
    uint32_t v = 0;
    if ((rc = tr.ReadDataBlock(i, &h, &v)) != NVL_CRC32C_OK) return rc;
  }
  const std::vector<nvl_table_block>& blocks = tr.blocks();
  uint64_t n_bad = 0;
  for (size_t i = 0; i < blocks.size(); ++i) n_bad += blocks[i].verdict != NVL_BLOCK_OK;
  char buf[96];
  snprintf(buf, sizeof(buf), "%u %llu\n", status, (unsigned long long)n_bad);
  std::string t(buf);
  for (size_t i = 0; i < blocks.size(); ++i) {
    snprintf(buf, sizeof(buf), "%llu %llu %u %u\n", (unsigned long long)blocks[i].offset,
             (unsigned long long)blocks[i].size, blocks[i].role, blocks[i].verdict);
    t.append(buf);
  }
  *batches = tr.batches();
  return copy_out(t, trace, cap, trace_len);
}

}  // extern "C"
