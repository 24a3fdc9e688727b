// nvlevelz_amd/csrc/crc32c_framing.cpp -- the batched call-site shims of
// SURVEY.md §8f behind include/nvl_framing.h: SSTable block trailers
// (table/table_builder.cc:175-193 / table/format.cc:65-98) and log physical
// records (db/log_writer.cc:84-109 / db/log_reader.cc:199-281).  The framing
// logic is host code; every CRC of a call goes to the GPU in ONE batch
// (nvl_crc32c_batch_region_host) unless NVL_FRAMING_HOST asks for the host
// CRC explicitly.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "crc32c_framing_core.h"
#include "crc32c_internal.h"
#include "crc32c_math.h"
#include "nvl_framing.h"

// flags = 0 crossover (bytes checksummed per host-resident call), from
// profiles/r05_shim_latency.jsonl: with the AVX-512 folding
// host CRC the host wins at 32 MiB (0.84-1.08 vs 1.49-1.51 ms), the GPU at
// 128 MiB (3.26-3.66 vs 5.29-5.70 ms) -> 64 MiB; with the SSE4.2 host CRC
// (a CPU without VPCLMULQDQ, or NVL_CRC32C_HOST=sse) round 4 measured the
// crossover at ~17 MiB -> 16 MiB (chosen by the host tier).
#ifndef NVL_FRAMING_DEFAULT_GPU_MIN_BYTES
#define NVL_FRAMING_DEFAULT_GPU_MIN_BYTES (64ull << 20)
#endif
#ifndef NVL_FRAMING_DEFAULT_GPU_MIN_BYTES_SSE
#define NVL_FRAMING_DEFAULT_GPU_MIN_BYTES_SSE (16ull << 20)
#endif

namespace nvl {
namespace {

inline uint32_t load_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

inline void store_le32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
  p[3] = (uint8_t)(v >> 24);
}

// Host-resident batches smaller than this run on the calling thread's host
// CRC when flags = 0 (the measured crossover of the host tier in use,
// DESIGN.md §9).
uint64_t default_gpu_min_bytes() {
  return host_tier_id() >= 2 ? NVL_FRAMING_DEFAULT_GPU_MIN_BYTES : NVL_FRAMING_DEFAULT_GPU_MIN_BYTES_SSE;
}

uint64_t gpu_min_bytes() {
  static const uint64_t v = [] {
    const uint64_t d = default_gpu_min_bytes();
    const char* e = getenv("NVL_FRAMING_GPU_MIN_BYTES");
    if (!e || !*e) return d;
    char* end = nullptr;
    const unsigned long long x = strtoull(e, &end, 0);
    return (end && *end == '\0') ? (uint64_t)x : d;
  }();
  return v;
}

// 1 GPU, 0 host, NVL_CRC32C_EINVAL for contradictory flags.
int uses_gpu(uint64_t bytes, uint32_t flags) {
  if ((flags & NVL_FRAMING_HOST) && (flags & NVL_FRAMING_GPU)) return NVL_CRC32C_EINVAL;
  if (flags & NVL_FRAMING_HOST) return 0;
  if (flags & NVL_FRAMING_GPU) return 1;
  return bytes >= gpu_min_bytes() ? 1 : 0;
}

// crc[i] = Value(region[off[i] .. off[i]+len[i])): one GPU batch or the host
// CRC, by uses_gpu().
int value_many(const uint8_t* region, uint64_t region_len, const std::vector<uint64_t>& off,
               const std::vector<uint64_t>& len, std::vector<uint32_t>* crc, uint32_t flags) {
  const size_t n = off.size();
  crc->assign(n, 0u);
  uint64_t bytes = 0;
  for (size_t i = 0; i < n; ++i) bytes += len[i];
  const int g = uses_gpu(bytes, flags);
  if (g < 0) return g;
  if (n == 0) return NVL_CRC32C_OK;
  if (!g) {
    for (size_t i = 0; i < n; ++i) (*crc)[i] = host_extend(0, region + off[i], len[i]);
    return NVL_CRC32C_OK;
  }
  return nvl_crc32c_batch_region_host(region, region_len, off.data(), len.data(), nullptr, 0, crc->data(), n, 0);
}

constexpr uint64_t kLogBlock = NVL_LOG_BLOCK_SIZE;
constexpr uint64_t kLogHeader = NVL_LOG_HEADER_SIZE;

// One block's speculative parse: every candidate record is assumed to pass
// its checksum; the block's closing event (if any) is what the parse reached
// under that assumption.
struct BlockParse {
  uint64_t start, end;      // file offsets of the block bytes read
  size_t first, count;      // candidate records: cand[first .. first+count)
  nvl_log_event closing;    // BAD_LENGTH / ZERO / EOF, or kind = UINT32_MAX (none: trailer skipped)
};

}  // namespace

// ---- SSTable structure (whole-table verify; crc32c_framing_core.h) ---------

// GetVarint64Ptr / GetVarint32Ptr (util/coding.cc): at most 10 / 5 bytes, never past limit.
static const uint8_t* get_varint(const uint8_t* p, const uint8_t* limit, unsigned max_shift, uint64_t* v) {
  uint64_t r = 0;
  for (unsigned shift = 0; shift <= max_shift && p < limit; shift += 7) {
    const uint64_t b = *p++;
    if (b & 128) {
      r |= (b & 127) << shift;
    } else {
      *v = r | (b << shift);
      return p;
    }
  }
  return nullptr;
}

// BlockHandle::DecodeFrom (table/format.cc:23-30); trailing bytes are allowed.
const uint8_t* decode_handle(const uint8_t* p, const uint8_t* limit, nvl_block_handle* h) {
  p = get_varint(p, limit, 63, &h->offset);
  return p ? get_varint(p, limit, 63, &h->size) : nullptr;
}

// The entries of a block as Block::Iter walks them from SeekToFirst
// (table/block.cc:17-37, 47-72, 219-246): one handle per entry value, an
// undecodable value recorded as a bad handle.  Returns NVL_TABLE_OK,
// NVL_TABLE_BAD_INDEX_BLOCK or NVL_TABLE_BAD_INDEX_ENTRY (entries before the
// bad one are kept, as the iterator yields them).
uint32_t block_handles(const uint8_t* data, uint64_t size, std::vector<nvl_block_handle>* out,
                       std::vector<uint8_t>* bad) {
  if (size < 4) return NVL_TABLE_BAD_INDEX_BLOCK;  // Block::Block size_ = 0 -> "bad block contents"
  const uint64_t num_restarts = load_le32(data + size - 4);
  if (num_restarts > (size - 4) / 4) return NVL_TABLE_BAD_INDEX_BLOCK;
  if (num_restarts == 0) return NVL_TABLE_OK;  // NewEmptyIterator
  const uint64_t restarts = size - (1 + num_restarts) * 4;
  const uint8_t* limit = data + restarts;
  uint64_t cur = load_le32(data + restarts);  // SeekToRestartPoint(0): GetRestartPoint(0)
  uint64_t key_len = 0;
  while (cur < restarts) {
    const uint8_t* p = data + cur;
    uint64_t shared, non_shared, value_len;
    if (limit - p < 3) return NVL_TABLE_BAD_INDEX_ENTRY;
    if ((p[0] | p[1] | p[2]) < 128) {
      shared = p[0], non_shared = p[1], value_len = p[2];
      p += 3;
    } else if (!(p = get_varint(p, limit, 28, &shared)) || !(p = get_varint(p, limit, 28, &non_shared)) ||
               !(p = get_varint(p, limit, 28, &value_len))) {
      return NVL_TABLE_BAD_INDEX_ENTRY;
    }
    // GetVarint32PtrFallback (util/coding.cc:112-129) accumulates into a
    // uint32_t: a 5-byte varint's high bits are dropped, not rejected.
    shared = (uint32_t)shared;
    non_shared = (uint32_t)non_shared;
    value_len = (uint32_t)value_len;
    // block.cc:70 (a 64-bit sum: the reference's uint32_t sum could wrap and read past the block)
    if ((uint64_t)(limit - p) < non_shared + value_len || key_len < shared)
      return NVL_TABLE_BAD_INDEX_ENTRY;
    key_len = shared + non_shared;
    const uint8_t* value = p + non_shared;
    nvl_block_handle h{0, 0};
    const bool ok = decode_handle(value, value + value_len, &h) != nullptr;
    out->push_back(ok ? h : nvl_block_handle{0, 0});
    bad->push_back(!ok);
    cur = (uint64_t)(value + value_len - data);
  }
  return NVL_TABLE_OK;
}

}  // namespace nvl

using namespace nvl;

extern "C" {

uint64_t nvl_framing_gpu_min_bytes(void) { return nvl::gpu_min_bytes(); }

int nvl_framing_uses_gpu(uint64_t crc_bytes, uint32_t flags) { return nvl::uses_gpu(crc_bytes, flags); }


int nvl_sstable_seal_trailers(void* file, uint64_t file_len, const nvl_block_handle* blocks, size_t n,
                              uint32_t flags) {
  if (n == 0) return NVL_CRC32C_OK;
  if (!file || !blocks) return NVL_CRC32C_EINVAL;
  std::vector<uint64_t> off(n), len(n);
  for (size_t i = 0; i < n; ++i) {
    if (!block_in_file(blocks[i], file_len)) return NVL_CRC32C_EINVAL;
    off[i] = blocks[i].offset;
    len[i] = blocks[i].size + 1;  // block contents | type (table_builder.cc:185-186)
  }
  uint8_t* f = static_cast<uint8_t*>(file);
  std::vector<uint32_t> crc;
  const int rc = value_many(f, file_len, off, len, &crc, flags);
  if (rc != NVL_CRC32C_OK) return rc;
  for (size_t i = 0; i < n; ++i) store_le32(f + blocks[i].offset + blocks[i].size + 1, mask(crc[i]));  // :187
  return NVL_CRC32C_OK;
}

int nvl_sstable_verify_blocks(const void* file, uint64_t file_len, const nvl_block_handle* blocks, size_t n,
                              uint8_t* verdict, uint64_t* n_bad, uint32_t flags) {
  if (n_bad) *n_bad = 0;
  if (n == 0) return NVL_CRC32C_OK;
  if (!file || !blocks || !verdict) return NVL_CRC32C_EINVAL;
  const uint8_t* f = static_cast<const uint8_t*>(file);
  std::vector<uint64_t> off, len;
  std::vector<size_t> which;
  off.reserve(n);
  len.reserve(n);
  which.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    if (!block_in_file(blocks[i], file_len)) continue;  // "truncated block read" (format.cc:82-85)
    off.push_back(blocks[i].offset);
    len.push_back(blocks[i].size + 1);
    which.push_back(i);
  }
  std::vector<uint32_t> crc;
  const int rc = value_many(f, file_len, off, len, &crc, flags);
  if (rc != NVL_CRC32C_OK) return rc;
  for (size_t i = 0; i < n; ++i) verdict[i] = NVL_BLOCK_TRUNCATED;
  for (size_t k = 0; k < which.size(); ++k) {
    const nvl_block_handle& h = blocks[which[k]];
    const uint8_t* trailer = f + h.offset + h.size;
    uint8_t v = NVL_BLOCK_OK;
    if (crc[k] != unmask(load_le32(trailer + 1))) v = NVL_BLOCK_CHECKSUM_MISMATCH;  // format.cc:88-96
    else if (trailer[0] != 0 && trailer[0] != 1) v = NVL_BLOCK_BAD_TYPE;           // format.cc:98-135
    verdict[which[k]] = v;
  }
  if (n_bad) {
    uint64_t b = 0;
    for (size_t i = 0; i < n; ++i) b += verdict[i] != NVL_BLOCK_OK;
    *n_bad = b;
  }
  return NVL_CRC32C_OK;
}

int nvl_log_scan(const void* data, uint64_t len, uint64_t start, int checksum, nvl_log_event* events, size_t cap,
                 size_t* n_events, uint32_t flags) {
  if (n_events) *n_events = 0;
  if ((!data && len) || !n_events || (start % kLogBlock) != 0) return NVL_CRC32C_EINVAL;
  const uint8_t* d = static_cast<const uint8_t*>(data);

  // Pass 1: speculative parse of every block (ReadPhysicalRecord's header
  // checks, log_reader.cc:203-252), collecting candidate records.
  std::vector<BlockParse> blocks;
  std::vector<nvl_log_event> cand;
  std::vector<uint64_t> coff, clen;
  uint64_t b0 = 0;
  while (true) {
    // log::Reader reads kBlockSize at a time; a short read (incl. 0 bytes)
    // marks EOF (log_reader.cc:205-218).
    const uint64_t m = (len - b0) < kLogBlock ? (len - b0) : kLogBlock;
    const bool eof = m < kLogBlock;
    BlockParse bp{start + b0, start + b0 + m, cand.size(), 0, nvl_log_event{}};
    bp.closing.kind = UINT32_MAX;
    uint64_t pos = 0;
    while (true) {
      nvl_log_event e{start + b0 + pos, bp.end, 0u, 0u, 0u, 0u};
      if (m - pos < kLogHeader) {
        if (eof) {  // empty, or a truncated header at the end of the file: EOF, not a corruption
          e.kind = NVL_LOG_EOF;
          bp.closing = e;
        }
        break;  // otherwise the block trailer is skipped
      }
      const uint8_t* h = d + b0 + pos;
      const uint32_t length = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
      const uint32_t type = h[6];
      if (kLogHeader + length > m - pos) {
        e.kind = eof ? NVL_LOG_EOF : NVL_LOG_BAD_LENGTH;  // :234-244
        bp.closing = e;
        break;
      }
      if (type == 0 && length == 0) {  // :246-252
        e.kind = NVL_LOG_ZERO;
        bp.closing = e;
        break;
      }
      e.kind = NVL_LOG_RECORD;
      e.length = length;
      e.type = type;
      cand.push_back(e);
      coff.push_back(b0 + pos + 6);  // Value(header + 6, 1 + length): type | payload (:256-257)
      clen.push_back(1u + length);
      ++bp.count;
      pos += kLogHeader + length;
    }
    blocks.push_back(bp);
    if (eof) break;
    b0 += kLogBlock;
  }

  // Pass 2: every candidate's CRC in one batch.
  std::vector<uint32_t> crc;
  if (checksum) {
    const int rc = value_many(d, len, coff, clen, &crc, flags);
    if (rc != NVL_CRC32C_OK) return rc;
  }

  // Pass 3: replay in reader order; a block is cut at its first mismatch
  // (the rest of the buffer is dropped, log_reader.cc:258-266).
  size_t ne = 0;
  auto emit = [&](const nvl_log_event& e) {
    if (events && ne < cap) events[ne] = e;
    ++ne;
  };
  for (const BlockParse& bp : blocks) {
    bool cut = false;
    for (size_t k = bp.first; k < bp.first + bp.count; ++k) {
      const nvl_log_event& e = cand[k];
      if (checksum && crc[k] != unmask(load_le32(d + (e.offset - start)))) {
        nvl_log_event x = e;
        x.kind = NVL_LOG_CHECKSUM;
        x.length = 0;
        x.type = 0;
        emit(x);
        cut = true;
        break;
      }
      emit(e);
    }
    if (!cut && bp.closing.kind != UINT32_MAX) emit(bp.closing);
    const bool eof_block = bp.end - bp.start < kLogBlock;
    if (eof_block && (cut || bp.closing.kind != NVL_LOG_EOF)) {
      // a drop or zero record emptied the last buffer: the next read finds nothing
      nvl_log_event x{bp.end, bp.end, 0u, 0u, NVL_LOG_EOF, 0u};
      emit(x);
    }
  }
  *n_events = ne;
  if (events && ne > cap) return NVL_CRC32C_ENOSPC;
  return NVL_CRC32C_OK;
}

int nvl_log_seal(void* data, uint64_t len, const uint64_t* header_offsets, size_t n, uint32_t flags) {
  if (n == 0) return NVL_CRC32C_OK;
  if (!data || !header_offsets) return NVL_CRC32C_EINVAL;
  uint8_t* d = static_cast<uint8_t*>(data);
  std::vector<uint64_t> off(n), ln(n);
  for (size_t i = 0; i < n; ++i) {
    const uint64_t o = header_offsets[i];
    if (o > len || len - o < kLogHeader) return NVL_CRC32C_EINVAL;
    const uint64_t length = (uint64_t)d[o + 4] | ((uint64_t)d[o + 5] << 8);
    if (len - o - kLogHeader < length) return NVL_CRC32C_EINVAL;
    off[i] = o + 6;  // type | payload (log_writer.cc:93-94)
    ln[i] = 1 + length;
  }
  std::vector<uint32_t> crc;
  const int rc = value_many(d, len, off, ln, &crc, flags);
  if (rc != NVL_CRC32C_OK) return rc;
  for (size_t i = 0; i < n; ++i) store_le32(d + header_offsets[i], mask(crc[i]));  // :95-96
  return NVL_CRC32C_OK;
}

}  // extern "C"

namespace nvl {
namespace {

struct HostTable : TableSource {
  const uint8_t* f;
  uint64_t len;
  uint32_t flags;
  int read(uint64_t off, uint64_t n, uint8_t* dst) override {
    memcpy(dst, f + off, n);
    return NVL_CRC32C_OK;
  }
  int verify(const std::vector<nvl_block_handle>& h, std::vector<uint8_t>* verdict) override {
    verdict->assign(h.size(), NVL_BLOCK_OK);
    if (h.empty()) return NVL_CRC32C_OK;
    return nvl_sstable_verify_blocks(f, len, h.data(), h.size(), verdict->data(), nullptr, flags);
  }
};

}  // namespace

uint8_t host_block_verdict(const uint8_t* b, uint64_t size) {
  const uint32_t crc = host_extend(0, b, size + 1);
  if (crc != unmask(load_le32(b + size + 1))) return NVL_BLOCK_CHECKSUM_MISMATCH;
  if (b[size] != 0 && b[size] != 1) return NVL_BLOCK_BAD_TYPE;
  return NVL_BLOCK_OK;
}

// Table::Open (table/table.cc:38-82), then ReadBlock with verify_checksums of
// every block the index and metaindex point at.  The index and metaindex
// blocks are small: read to the host and checked there; every other block's
// check goes to the source's batch.
int verify_table_core(TableSource& src, uint64_t file_len, nvl_table_block* blocks, size_t cap, size_t* n_blocks,
                      uint32_t* table_status, uint64_t* n_bad, bool list_only) {
  *table_status = NVL_TABLE_OK;
  if (file_len < NVL_FOOTER_SIZE) {  // table.cc:44-46
    *table_status = NVL_TABLE_TOO_SHORT;
    return NVL_CRC32C_OK;
  }
  uint8_t footer[NVL_FOOTER_SIZE];
  int rc = src.read(file_len - NVL_FOOTER_SIZE, NVL_FOOTER_SIZE, footer);
  if (rc != NVL_CRC32C_OK) return rc;
  const uint64_t magic = (uint64_t)load_le32(footer + 40) | ((uint64_t)load_le32(footer + 44) << 32);
  if (magic != kTableMagic) {  // format.cc:43-51
    *table_status = NVL_TABLE_BAD_MAGIC;
    return NVL_CRC32C_OK;
  }
  nvl_block_handle meta_h, index_h;
  const uint8_t* fp = decode_handle(footer, footer + NVL_FOOTER_SIZE, &meta_h);  // format.cc:53-56
  if (!fp || !decode_handle(fp, footer + NVL_FOOTER_SIZE, &index_h)) {
    *table_status = NVL_TABLE_BAD_FOOTER;
    return NVL_CRC32C_OK;
  }
  // the two structure blocks with their trailers (verdict: truncated when
  // they do not fit the file, format.cc:82-85)
  std::vector<uint8_t> index_b, meta_b;
  uint8_t v_index = NVL_BLOCK_TRUNCATED, v_meta = NVL_BLOCK_TRUNCATED;
  if (block_in_file(index_h, file_len)) {
    index_b.resize(index_h.size + NVL_BLOCK_TRAILER_SIZE);
    if ((rc = src.read(index_h.offset, index_b.size(), index_b.data())) != NVL_CRC32C_OK) return rc;
    v_index = host_block_verdict(index_b.data(), index_h.size);
  }
  if (block_in_file(meta_h, file_len)) {
    meta_b.resize(meta_h.size + NVL_BLOCK_TRAILER_SIZE);
    if ((rc = src.read(meta_h.offset, meta_b.size(), meta_b.data())) != NVL_CRC32C_OK) return rc;
    v_meta = host_block_verdict(meta_b.data(), meta_h.size);
  }
  std::vector<nvl_block_handle> data_h, meta_blocks;
  std::vector<uint8_t> data_bad, meta_bad;
  uint32_t index_parse = NVL_TABLE_OK;
  if (v_index == NVL_BLOCK_OK && index_b[index_h.size] == 0)
    index_parse = block_handles(index_b.data(), index_h.size, &data_h, &data_bad);
  const bool meta_ok = v_meta == NVL_BLOCK_OK && meta_b[meta_h.size] == 0;
  if (meta_ok) block_handles(meta_b.data(), meta_h.size, &meta_blocks, &meta_bad);

  std::vector<nvl_table_block> out;
  auto emit = [&](const nvl_block_handle& h, uint32_t role, uint32_t v) {
    out.push_back(nvl_table_block{h.offset, h.size, role, v});
  };
  if (v_index != NVL_BLOCK_OK) {  // Table::Open fails on the index block (table.cc:58-66)
    emit(index_h, NVL_TBLOCK_INDEX, v_index);
    *table_status = NVL_TABLE_INDEX_UNREADABLE;
  } else if (index_b[index_h.size] != 0) {
    emit(index_h, NVL_TBLOCK_INDEX, v_index);
    *table_status = NVL_TABLE_COMPRESSED_INDEX;
  } else {
    const size_t cnt = 2 + meta_blocks.size() + data_h.size();
    if (!blocks) {  // size query: the list's length needs no batch
      *n_blocks = cnt;
      *table_status = index_parse;
      return NVL_CRC32C_OK;
    }
    // one batch: every meta and data block
    std::vector<nvl_block_handle> all;
    all.reserve(meta_blocks.size() + data_h.size());
    for (size_t i = 0; i < meta_blocks.size(); ++i) all.push_back(meta_blocks[i]);
    for (size_t i = 0; i < data_h.size(); ++i) all.push_back(data_h[i]);
    std::vector<uint8_t> verdict;
    if (list_only) verdict.assign(all.size(), (uint8_t)NVL_BLOCK_UNCHECKED);
    else if ((rc = src.verify(all, &verdict)) != NVL_CRC32C_OK) return rc;
    emit(index_h, NVL_TBLOCK_INDEX, v_index);
    emit(meta_h, NVL_TBLOCK_METAINDEX, v_meta);
    size_t k = 0;
    for (size_t i = 0; i < meta_blocks.size(); ++i, ++k)
      emit(meta_blocks[i], NVL_TBLOCK_META, meta_bad[i] ? NVL_BLOCK_BAD_HANDLE : verdict[k]);
    for (size_t i = 0; i < data_h.size(); ++i, ++k)
      emit(data_h[i], NVL_TBLOCK_DATA, data_bad[i] ? NVL_BLOCK_BAD_HANDLE : verdict[k]);
    *table_status = index_parse;
  }
  *n_blocks = out.size();
  if (n_bad) {
    uint64_t b = 0;
    for (const nvl_table_block& t : out) b += t.verdict != NVL_BLOCK_OK && t.verdict != NVL_BLOCK_UNCHECKED;
    *n_bad = b;
  }
  if (!blocks) return NVL_CRC32C_OK;
  if (out.size() > cap) return NVL_CRC32C_ENOSPC;
  if (!out.empty()) memcpy(blocks, out.data(), out.size() * sizeof(nvl_table_block));
  return NVL_CRC32C_OK;
}

}  // namespace nvl

extern "C" {

int nvl_sstable_verify_table(const void* file, uint64_t file_len, nvl_table_block* blocks, size_t cap,
                             size_t* n_blocks, uint32_t* table_status, uint64_t* n_bad, uint32_t flags) {
  if (n_blocks) *n_blocks = 0;
  if (n_bad) *n_bad = 0;
  if ((!file && file_len) || !n_blocks || !table_status) return NVL_CRC32C_EINVAL;
  nvl::HostTable src;
  src.f = static_cast<const uint8_t*>(file);
  src.len = file_len;
  src.flags = flags;
  return nvl::verify_table_core(src, file_len, blocks, cap, n_blocks, table_status, n_bad,
                                (flags & NVL_TABLE_LIST_ONLY) != 0);
}


}  // extern "C"
