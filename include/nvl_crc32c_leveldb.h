// include/nvl_crc32c_leveldb.h -- C++ mirror of the reference's
// util/crc32c.h (/root/reference/util/crc32c.h:11-43) on top of the C ABI in
// nvl_crc32c.h.  A LevelDB tree that includes this header (or whose
// util/crc32c.cc forwards to nvl_crc32c_extend) keeps every
// call site -- table/table_builder.cc:185-187, table/format.cc:91-92,
// db/log_writer.cc:18,95-96, db/log_reader.cc:255-256 -- unchanged.
//
// The batch helpers in leveldb::crc32c::batch are what the block-batching
// shims at those call sites use (host buffers in, CRCs out, one GPU launch).
#ifndef NVL_CRC32C_LEVELDB_H_
#define NVL_CRC32C_LEVELDB_H_

#include <stddef.h>
#include <stdint.h>

#include "nvl_crc32c.h"

namespace leveldb {
namespace crc32c {

// util/crc32c.h:17 -- crc32c of concat(A, data[0,n-1]) given init_crc = crc32c(A).
inline uint32_t Extend(uint32_t init_crc, const char* data, size_t n) {
  return nvl_crc32c_extend(init_crc, data, n);
}

// util/crc32c.h:20-22
inline uint32_t Value(const char* data, size_t n) { return Extend(0, data, n); }

// util/crc32c.h:24
static const uint32_t kMaskDelta = 0xa282ead8ul;

// util/crc32c.h:31-34
inline uint32_t Mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }

// util/crc32c.h:37-40
inline uint32_t Unmask(uint32_t masked_crc) {
  uint32_t rot = masked_crc - kMaskDelta;
  return ((rot >> 17) | (rot << 15));
}

namespace batch {

// out[i] = Extend(init ? init[i] : init_all, ptrs[i], lens[i]) (Mask()ed when
// `mask`), n buffers in host memory, one GPU batch.  Returns an
// NVL_CRC32C_* status; on a non-zero status `out` is untouched and the caller
// decides whether to recompute with Extend() (no hidden fallback).
inline int Extend(const char* const* ptrs, const uint64_t* lens, const uint32_t* init, uint32_t init_all,
                  uint32_t* out, size_t n, bool mask = false) {
  return nvl_crc32c_batch_host(reinterpret_cast<const void* const*>(ptrs), lens, init, init_all, out, n,
                               mask ? NVL_CRC32C_FLAG_MASK : 0u);
}

inline bool GpuAvailable() { return nvl_crc32c_gpu_accelerated() != 0; }

}  // namespace batch
}  // namespace crc32c
}  // namespace leveldb

#endif  // NVL_CRC32C_LEVELDB_H_
