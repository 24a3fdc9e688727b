// nvlevelz_amd/csrc/crc32c_framing_core.h -- the whole-table verification
// core shared by nvl_sstable_verify_table (host image, crc32c_framing.cpp)
// and nvl_sstable_verify_table_dev (device image, crc32c_framing_dev.cpp).
// Internal; not installed.
#ifndef NVL_CRC32C_FRAMING_CORE_H_
#define NVL_CRC32C_FRAMING_CORE_H_

#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "nvl_framing.h"

namespace nvl {

// Where a table's bytes are: read() copies structure bytes (footer, index
// and metaindex blocks with their trailers) to the host; verify() runs
// ReadBlock's checks for a list of handles in one batch.
struct TableSource {
  virtual ~TableSource() {}
  virtual int read(uint64_t off, uint64_t n, uint8_t* dst) = 0;
  virtual int verify(const std::vector<nvl_block_handle>& h, std::vector<uint8_t>* verdict) = 0;
};

// ReadBlock's "truncated block read" test (table/format.cc:82-85): the block
// and its 5-byte trailer lie inside the file.
inline bool block_in_file(const nvl_block_handle& h, uint64_t file_len) {
  return h.size <= file_len && h.offset <= file_len - h.size &&
         file_len - h.size - h.offset >= (uint64_t)NVL_BLOCK_TRAILER_SIZE;
}

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;  // table/format.h:77

// BlockHandle::DecodeFrom (table/format.cc:23-30); trailing bytes are allowed.
const uint8_t* decode_handle(const uint8_t* p, const uint8_t* limit, nvl_block_handle* h);

// The entries of a block as Block::Iter walks them from SeekToFirst
// (table/block.cc:17-37, 47-72, 219-246): one handle per entry value, an
// undecodable value recorded as a bad handle.  Returns NVL_TABLE_OK,
// NVL_TABLE_BAD_INDEX_BLOCK or NVL_TABLE_BAD_INDEX_ENTRY.
uint32_t block_handles(const uint8_t* data, uint64_t size, std::vector<nvl_block_handle>* out,
                       std::vector<uint8_t>* bad);

// ReadBlock's trailer checks (format.cc:88-135) on one block held on the
// host with its 5-byte trailer: b[0 .. size + 5).
uint8_t host_block_verdict(const uint8_t* b, uint64_t size);

// list_only: NVL_TABLE_LIST_ONLY (meta and data blocks listed unchecked, no batch)
int verify_table_core(TableSource& src, uint64_t file_len, nvl_table_block* blocks, size_t cap, size_t* n_blocks,
                      uint32_t* table_status, uint64_t* n_bad, bool list_only = false);

}  // namespace nvl

#endif  // NVL_CRC32C_FRAMING_CORE_H_
