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
//   via_shim = 0: an in-memory WritableFile (the reference's file), or the
//   shipped adapter nvl::shims::BatchingWritableFile<leveldb::WritableFile,
//   leveldb::Slice, leveldb::Status> (include/nvl_leveldb_shims.h) around it:
//   via_shim = 1: trailers sealed in one engine batch at Close();
//   via_shim = 2: sealed every ~5000 staged bytes (many batches);
//   via_shim = 3: the adapter's staged bytes before any seal.
// *computed: the trailers that reached the adapter with a CRC TableBuilder
// computed itself (every block with the stock WriteRawBlock, none with the
// edit).
// Built twice by oracle/Makefile: libref_table.so with the reference's
// table_builder.cc as it is (WriteRawBlock computes a CRC the adapter
// discards) and libref_table_deferred.so with INTEGRATION.md §5's edit
// applied at build time by apply_deferred_crc.py (WriteRawBlock leaves the
// CRC to the file when nvl::shims::DefersBlockCrc(file)).  The images of
// modes 0-2 must be byte-identical.  Nothing here is product code.
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

typedef nvl::shims::BatchingWritableFile<leveldb::WritableFile, leveldb::Slice, leveldb::Status> BatchingFile;

}  // namespace

extern "C" {

// keys/values concatenated in kv (key i then value i); returns 0 or a status.
__attribute__((visibility("default")))
int ref_table_build(const uint8_t* kv, const uint64_t* klen, const uint64_t* vlen, size_t n, uint64_t block_size,
                    int restart_interval, int bloom_bits, int via_shim, uint32_t seal_flags, uint8_t* out, size_t cap,
                    size_t* out_len, uint64_t* handles, size_t hcap, size_t* nh, size_t* seals,
                    size_t* computed) {
  leveldb::Options opt;
  opt.block_size = (size_t)block_size;
  opt.block_restart_interval = restart_interval;
  opt.compression = leveldb::kNoCompression;
  const leveldb::FilterPolicy* fp = bloom_bits > 0 ? leveldb::NewBloomFilterPolicy(bloom_bits) : nullptr;
  opt.filter_policy = fp;
  StringSink plain;
  BatchingFile batch(&plain, via_shim == 2 ? 5000u : (via_shim == 3 ? ~0ull : 64ull << 20), seal_flags);
  leveldb::WritableFile* f = via_shim ? static_cast<leveldb::WritableFile*>(&batch) : &plain;
  leveldb::TableBuilder tb(opt, f);
  const char* p = reinterpret_cast<const char*>(kv);
  for (size_t i = 0; i < n; ++i) {
    tb.Add(leveldb::Slice(p, klen[i]), leveldb::Slice(p + klen[i], vlen[i]));
    p += klen[i] + vlen[i];
  }
  leveldb::Status s = tb.Finish();
  delete fp;
  if (!s.ok()) return 100;
  std::string staged;
  if (via_shim == 3) staged = batch.staged();  // (the footer is still pending: Finish's last Append)
  if (via_shim) s = f->Close();
  if (!s.ok()) return 101;
  const std::string* img = via_shim == 3 ? &staged : &plain.data;
  *seals = via_shim ? batch.seals() : 0;
  *computed = via_shim ? batch.computed_crcs() : 0;
  *nh = 0;
  if (via_shim) {
    const std::vector<nvl_block_handle>& b = batch.handles();
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
