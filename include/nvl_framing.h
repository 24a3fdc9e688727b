/*
 * include/nvl_framing.h -- C ABI of the batched call-site shims (SURVEY.md
 * §8f): the CRC32C framing of LevelDB's on-disk formats computed or checked
 * for many blocks / records in one GPU batch.  Part of libnvl_crc32c.so.
 *
 *   SSTable block trailer  table/format.h:84 (kBlockTrailerSize = 5), written by
 *                          TableBuilder::WriteRawBlock table/table_builder.cc:175-193,
 *                          checked by ReadBlock table/format.cc:65-98:
 *                          block[0..n) | type (1 B) | Mask(Value(block | type)) (LE32)
 *   Log physical record    db/log_format.h:14-31 (kBlockSize 32768, kHeaderSize 7),
 *                          written by log::Writer db/log_writer.cc:45-109,
 *                          parsed by log::Reader::ReadPhysicalRecord db/log_reader.cc:199-281:
 *                          Mask(Value(type | payload)) (LE32) | len (LE16) | type | payload
 *
 * Every entry point computes its CRCs on the GPU (one batch per call) unless
 * the caller passes NVL_FRAMING_HOST, which selects the host CRC
 * (nvl_crc32c_extend) explicitly -- for batches too small to pay for a
 * launch.  There is no implicit fallback: without a usable GPU the device
 * mode returns the NVL_CRC32C_* error and writes nothing.
 */
#ifndef NVL_FRAMING_H_
#define NVL_FRAMING_H_

#include <stddef.h>
#include <stdint.h>

#include "nvl_crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Engine of a host-resident call's CRC batch.  flags = 0 chooses by size:
 * batches of fewer than nvl_framing_gpu_min_bytes() checksummed bytes run on
 * the calling thread's host CRC (nvl_crc32c_extend), larger ones on the GPU
 * (one staging copy, H2D, one batch kernel, D2H) -- the crossover measured at
 * the fork's call-site sizes (profiles/r05_shim_latency.jsonl);
 * the environment variable NVL_FRAMING_GPU_MIN_BYTES overrides it.  The two
 * flags force an engine.  A GPU batch that fails returns its error; no call
 * ever falls back to the other engine.  (nvl_sstable_verify_table_dev's image
 * is in HBM already: always the GPU.) */
#define NVL_FRAMING_HOST 0x100u /* compute CRCs with the host CRC */
#define NVL_FRAMING_GPU 0x400u  /* compute CRCs on the GPU whatever the size */

/* The crossover in bytes (flags = 0: GPU at or above it). */
NVL_API uint64_t nvl_framing_gpu_min_bytes(void);
/* 1 if a host-resident batch of `crc_bytes` checksummed bytes runs on the GPU
 * under `flags`, 0 if on the host CRC, NVL_CRC32C_EINVAL for both flags. */
NVL_API int nvl_framing_uses_gpu(uint64_t crc_bytes, uint32_t flags);

/* ---- SSTable blocks ------------------------------------------------------ */

#define NVL_BLOCK_TRAILER_SIZE 5 /* table/format.h:84 */

/* BlockHandle (table/format.h:22-48): a block of `size` bytes at `offset`,
 * followed in the file by its 5-byte trailer. */
typedef struct nvl_block_handle {
  uint64_t offset;
  uint64_t size;
} nvl_block_handle;

/* per-block verdicts of nvl_sstable_verify_blocks, in ReadBlock's order of
 * checks (table/format.cc:77-135) */
#define NVL_BLOCK_OK 0
#define NVL_BLOCK_TRUNCATED 1         /* "truncated block read"      format.cc:82-85 */
#define NVL_BLOCK_CHECKSUM_MISMATCH 2 /* "block checksum mismatch"   format.cc:88-96 */
#define NVL_BLOCK_BAD_TYPE 3          /* "bad block type"            format.cc:133-135 */

/* Writer side (replaces the per-block crc32c::Value/Extend/Mask of
 * table_builder.cc:185-187).  For every handle, file[offset + size] already
 * holds the block type; writes EncodeFixed32(Mask(Value(file[offset ..
 * offset+size]))) -- the CRC of block | type -- at file[offset + size + 1].
 * Every block must lie inside [0, file_len). */
NVL_API int nvl_sstable_seal_trailers(void* file, uint64_t file_len, const nvl_block_handle* blocks, size_t n,
                                      uint32_t flags);

/* Reader side (the checksum and type checks of ReadBlock with
 * verify_checksums, format.cc:77-135, for n blocks at once).  verdict[i]
 * gets NVL_BLOCK_*; *n_bad (optional) the number of non-OK blocks.  A
 * compressed block (type 1, kSnappyCompression) verifies as OK here; its
 * decompression stays with the caller. */
NVL_API int nvl_sstable_verify_blocks(const void* file, uint64_t file_len, const nvl_block_handle* blocks, size_t n,
                                      uint8_t* verdict, uint64_t* n_bad, uint32_t flags);

/* ---- whole-table verification ------------------------------------------- */

#define NVL_FOOTER_SIZE 48 /* Footer::kEncodedLength, table/format.h:64-66 */

/* table-level outcome of nvl_sstable_verify_table, following Table::Open
 * (table/table.cc:38-82) and the index block's iterator (table/block.cc) */
#define NVL_TABLE_OK 0
#define NVL_TABLE_TOO_SHORT 1       /* "file is too short to be an sstable"  table.cc:44-46 */
#define NVL_TABLE_BAD_MAGIC 2       /* "not an sstable (bad magic number)"   format.cc:49-51 */
#define NVL_TABLE_BAD_FOOTER 3      /* "bad block handle" in the footer      format.cc:28-29,54-57 */
#define NVL_TABLE_INDEX_UNREADABLE 4 /* ReadBlock(index) failed: blocks[0] holds its verdict (table.cc:58-66) */
#define NVL_TABLE_BAD_INDEX_BLOCK 5 /* "bad block contents" (restart array does not fit, block.cc:26-37,256-259) */
#define NVL_TABLE_BAD_INDEX_ENTRY 6 /* "bad entry in block": the index scan stopped there (block.cc:218-245);
                                       the entries before it are listed and verified */
#define NVL_TABLE_COMPRESSED_INDEX 7 /* index block stored with kSnappyCompression: not parsed here */

/* roles of the blocks nvl_sstable_verify_table lists */
#define NVL_TBLOCK_INDEX 0
#define NVL_TBLOCK_METAINDEX 1
#define NVL_TBLOCK_META 2 /* a block a metaindex entry points at (e.g. "filter.<policy>", table.cc:99-108) */
#define NVL_TBLOCK_DATA 3

#define NVL_BLOCK_BAD_HANDLE 4 /* the index/metaindex value is not a BlockHandle: "bad block handle"
                                  (Table::BlockReader table/table.cc:160-165); offset = size = 0 */
#define NVL_BLOCK_UNCHECKED 5  /* NVL_TABLE_LIST_ONLY: listed, not yet checked */

#define NVL_TABLE_LIST_ONLY 0x200u /* nvl_sstable_verify_table flag: list the blocks (footer, index and
                                      metaindex read and checked on the host) without checking the meta
                                      and data blocks -- Table::Open without the reads of the blocks an
                                      iterator will touch; they get NVL_BLOCK_UNCHECKED */

typedef struct nvl_table_block {
  uint64_t offset;
  uint64_t size;
  uint32_t role;    /* NVL_TBLOCK_* */
  uint32_t verdict; /* NVL_BLOCK_* */
} nvl_table_block;

/* Verify every block of an SSTable image (an mmap'd table file, or its
 * bytes) with ReadBlock's checks (verify_checksums = true), in ONE batch:
 * footer -> index block -> every data block handle in index order, plus the
 * metaindex block and every block its entries point at.  The index and
 * metaindex blocks are parsed speculatively before their own CRCs are known
 * so all CRCs go to the GPU together; a block list is only reported from a
 * parse whose block passed.  Output order: index, metaindex, meta blocks (in
 * metaindex order; only when the metaindex verified), data blocks (only when
 * the index verified).  *table_status gets NVL_TABLE_*; *n_blocks the number
 * of blocks listed (at most `cap` written, NVL_CRC32C_ENOSPC if more);
 * *n_bad (optional) the listed blocks whose verdict is not OK.  `blocks` may
 * be NULL to query the list's length cheaply: only the footer, the index and
 * metaindex blocks are read and checked (host CRC, no batch); *n_blocks and
 * *table_status are then exact and *n_bad is left 0.  Compressed (type 1)
 * data/meta blocks verify as OK here, as in nvl_sstable_verify_blocks. */
/* With NVL_TABLE_LIST_ONLY in flags the meta and data blocks are listed
 * with NVL_BLOCK_UNCHECKED (no batch): the open of a batched table reader
 * (nvl::shims::TableReader) that checks them per readahead window with
 * nvl_sstable_verify_blocks.  *n_bad counts the blocks whose check failed. */
NVL_API int nvl_sstable_verify_table(const void* file, uint64_t file_len, nvl_table_block* blocks, size_t cap,
                                     size_t* n_blocks, uint32_t* table_status, uint64_t* n_bad, uint32_t flags);

/* The same for a table image already in device memory (HBM) on `stream`'s
 * device (a hipStream_t; NULL = the null stream): the footer, index and
 * metaindex blocks come back in small copies and are parsed on the host,
 * every other block is checked in place by one batch and a trailer-check
 * kernel, and only the verdicts return.  Same results as
 * nvl_sstable_verify_table on the same bytes; synchronous on `stream`. */
NVL_API int nvl_sstable_verify_table_dev(const void* file, uint64_t file_len, nvl_table_block* blocks, size_t cap,
                                         size_t* n_blocks, uint32_t* table_status, uint64_t* n_bad, void* stream);

/* ---- log files ----------------------------------------------------------- */

#define NVL_LOG_BLOCK_SIZE 32768 /* db/log_format.h:27 */
#define NVL_LOG_HEADER_SIZE 7    /* db/log_format.h:30 */

/* Outcome of one ReadPhysicalRecord step (db/log_reader.cc:199-281). */
#define NVL_LOG_RECORD 0       /* a physical record that passed its checks: payload at offset+7 */
#define NVL_LOG_BAD_LENGTH 1   /* header length runs past the block: rest of the block dropped,
                                  "bad record length" (log_reader.cc:234-244) */
#define NVL_LOG_CHECKSUM 2     /* CRC mismatch: rest of the block dropped, "checksum mismatch"
                                  (log_reader.cc:254-267) */
#define NVL_LOG_ZERO 3         /* zero type + zero length (preallocated space): rest of the block
                                  skipped without a report (log_reader.cc:246-252) */
#define NVL_LOG_EOF 4          /* end of input, incl. a truncated header or payload in the last
                                  block, which is not a corruption (log_reader.cc:213-244) */

typedef struct nvl_log_event {
  uint64_t offset;    /* file offset of the header (RECORD/BAD_LENGTH/CHECKSUM/ZERO) */
  uint64_t block_end; /* file offset just past the block the event belongs to */
  uint32_t length;    /* RECORD: payload bytes */
  uint32_t type;      /* RECORD: the stored type byte (any value; the record-level
                         state machine reports unknown types) */
  uint32_t kind;      /* NVL_LOG_* */
  uint32_t reserved;
} nvl_log_event;

/* Parse a log image the way log::Reader reads it (32 KiB blocks from
 * `start`, a multiple of kBlockSize; data[0] is file offset `start`) and
 * return the sequence of ReadPhysicalRecord outcomes up to and including the
 * final NVL_LOG_EOF.  `checksum` = 0 skips CRC verification (Reader's
 * checksum flag).  All candidate records' CRCs (Value(type | payload),
 * 1 + length bytes) are verified in one batch; a block's records after its
 * first failure are discarded exactly as the reference drops the block.
 * `events` may be NULL to query the count: *n_events gets the number of
 * events; at most `cap` are written; NVL_CRC32C_ENOSPC if cap is too small. */
NVL_API int nvl_log_scan(const void* data, uint64_t len, uint64_t start, int checksum, nvl_log_event* events,
                         size_t cap, size_t* n_events, uint32_t flags);

/* Writer side (replaces the per-fragment crc32c::Extend/Mask of
 * log_writer.cc:93-97): for each header offset, data[off+4..off+7) already
 * holds length and type; writes EncodeFixed32(Mask(Value(data[off+6 ..
 * off+7+length)))) at data[off].  One batch for all n records. */
NVL_API int nvl_log_seal(void* data, uint64_t len, const uint64_t* header_offsets, size_t n, uint32_t flags);

#ifdef __cplusplus
}
#endif

#endif /* NVL_FRAMING_H_ */
