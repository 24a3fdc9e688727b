// oracle/ref_table.cc -- TEST INFRASTRUCTURE ONLY (tests/test_table_builder.py).
//
// The reference's own TableBuilder (table/table_builder.cc:1-270, with
// block_builder.cc, filter_block.cc, format.cc, util/bloom.cc) compiled from
// /root/reference into oracle/_ref/libref_table.so by oracle/Makefile, at the
// reference's own optimisation level (its Makefile: OPT ?= -g2, i.e. -O0):
// Options::Options() reaches Env::Default() (util/options.cc:17), whose
// PosixEnv builds an NVM_Library (util/env_posix.cc:895-902); there
// NVM_Manager::write_zero (nvm_library/nvm_manager.h:123-129) is declared to
// return nvAddr and has no return statement -- undefined behaviour that GCC
// at -O2 compiles as unreachable code, which is the segfault SURVEY.md §4
// found; at -O0 the function returns normally.  No stand-in Env is used.
//
// ref_table_build drives one key/value sequence through TableBuilder into
//   via_shim = 0: an in-memory WritableFile (the reference's file), or
//   via_shim = 1: a WritableFile that routes every block through
//                 nvl::shims::TableFile -- contents appended, the 5-byte
//                 trailer replaced by the block type with a zero CRC -- and
//                 seals all trailers in one engine batch (nvl_sstable_seal_trailers).
// The two images must be byte-identical.  Nothing here is product code.
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "leveldb/comparator.h"
#include "leveldb/env.h"
#include "leveldb/filter_policy.h"
#include "leveldb/options.h"
#include "leveldb/table_builder.h"
#include "nvl_leveldb_shims.h"

namespace {

class StringSink : public leveldb::WritableFile {
 public:
  std::string data;
  leveldb::Status Append(const leveldb::Slice& d) override {
    data.append(d.data(), d.size());
    return leveldb::Status::OK();
  }
  leveldb::Status Close() override { return leveldb::Status::OK(); }
  leveldb::Status Flush() override { return leveldb::Status::OK(); }
  leveldb::Status Sync() override { return leveldb::Status::OK(); }
};

// TableBuilder::WriteRawBlock appends a block's contents, then its 5-byte
// trailer (table_builder.cc:175-193); Finish appends the 48-byte footer.
class SealSink : public leveldb::WritableFile {
 public:
  nvl::shims::TableFile tf;
  leveldb::Status Append(const leveldb::Slice& d) override {
    if (have_ && d.size() == NVL_BLOCK_TRAILER_SIZE) {  // the trailer of the pending block
      tf.AppendBlock(pending_.data(), pending_.size(), (uint8_t)d[0]);
      have_ = false;
      return leveldb::Status::OK();
    }
    Flush1();
    pending_.assign(d.data(), d.size());
    have_ = true;
    return leveldb::Status::OK();
  }
  void Flush1() {
    if (have_) tf.Append(pending_.data(), pending_.size());
    have_ = false;
  }
  leveldb::Status Close() override { return leveldb::Status::OK(); }
  leveldb::Status Flush() override { return leveldb::Status::OK(); }
  leveldb::Status Sync() override { return leveldb::Status::OK(); }

 private:
  std::string pending_;
  bool have_ = false;
};

}  // namespace

extern "C" {

// keys/values concatenated in kv (key i then value i); returns 0 or a status.
__attribute__((visibility("default")))
int ref_table_build(const uint8_t* kv, const uint64_t* klen, const uint64_t* vlen, size_t n, uint64_t block_size,
                    int restart_interval, int bloom_bits, int via_shim, uint32_t seal_flags, uint8_t* out, size_t cap,
                    size_t* out_len, uint64_t* handles, size_t hcap, size_t* nh) {
  leveldb::Options opt;
  opt.block_size = (size_t)block_size;
  opt.block_restart_interval = restart_interval;
  opt.compression = leveldb::kNoCompression;
  const leveldb::FilterPolicy* fp = bloom_bits > 0 ? leveldb::NewBloomFilterPolicy(bloom_bits) : nullptr;
  opt.filter_policy = fp;
  StringSink plain;
  SealSink seal;
  leveldb::WritableFile* f = via_shim ? static_cast<leveldb::WritableFile*>(&seal) : &plain;
  leveldb::TableBuilder tb(opt, f);
  const char* p = reinterpret_cast<const char*>(kv);
  for (size_t i = 0; i < n; ++i) {
    tb.Add(leveldb::Slice(p, klen[i]), leveldb::Slice(p + klen[i], vlen[i]));
    p += klen[i] + vlen[i];
  }
  const leveldb::Status s = tb.Finish();
  delete fp;
  if (!s.ok()) return 100;
  const std::string* img = &plain.data;
  *nh = 0;
  if (via_shim) {
    seal.Flush1();
    const int rc = seal.tf.Seal(seal_flags);
    if (rc != NVL_CRC32C_OK) return rc;
    img = &seal.tf.image();
    const std::vector<nvl_block_handle>& b = seal.tf.blocks();
    *nh = b.size();
    for (size_t k = 0; k < b.size() && 2 * k + 1 < hcap; ++k) {
      handles[2 * k] = b[k].offset;
      handles[2 * k + 1] = b[k].size;
    }
  }
  *out_len = img->size();
  if (img->size() > cap) return NVL_CRC32C_ENOSPC;
  memcpy(out, img->data(), img->size());
  return 0;
}

}  // extern "C"
