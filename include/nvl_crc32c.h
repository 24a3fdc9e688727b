/*
 * include/nvl_crc32c.h -- C ABI of the MI355X-native CRC32C block-checksum
 * engine (libnvl_crc32c.so).
 *
 * Drop-in boundary: this ABI sits beneath the reference's util/crc32c.h
 * (/root/reference/util/crc32c.h:17-40) and replaces its backend seam
 * port::AcceleratedCRC32C (/root/reference/port/port_posix.h:169, contract
 * port/port_example.h:132-136, implementation port/port_posix_sse.cc:69-126).
 * Plain pointers and sizes only; no C++ or torch types.
 *
 * Semantics are bit-exact with leveldb::crc32c::Extend (util/crc32c.cc:299-347):
 * CRC32C, reflected polynomial 0x82F63B78, register pre/post inverted, with
 * Extend(crc, "", 0) == crc.
 *
 * Threading: every entry point is reentrant and thread-safe.  Device
 * entry points are asynchronous on the HIP stream passed in `stream`
 * (a hipStream_t; NULL = the null stream) and run on THAT stream's device
 * (the null stream: the caller's current device), whatever the calling
 * thread's current device is; inputs must stay valid and
 * unmodified and outputs must not be read until that stream is synchronised.
 * The host-resident entry points run on the caller's current device; one
 * thread may drive every device in turn (hipSetDevice between calls).  The
 * streams and staging memory a thread acquires for them are freed when the
 * thread exits, or by nvl_crc32c_shutdown.
 * The library owns only its lookup tables (one small copy per device,
 * created on first use or by nvl_crc32c_init) and, when the caller passes no
 * workspace, stream-ordered scratch allocated and freed on `stream`.
 *
 * Errors: the reference has no error channel (its accelerator signals
 * "unavailable" by returning 0, util/crc32c.cc:290-303).  Here every batch
 * entry point returns an int status (NVL_CRC32C_OK = 0, negative on error)
 * and writes nothing on argument errors.  There is NO silent CPU fallback in
 * the batch entry points: a caller that wants one calls nvl_crc32c_extend
 * itself on a non-zero status.
 */
#ifndef NVL_CRC32C_H_
#define NVL_CRC32C_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NVL_CRC32C_ABI_VERSION 1

#if defined(__GNUC__)
#define NVL_API __attribute__((visibility("default")))
#else
#define NVL_API
#endif

/* status codes */
#define NVL_CRC32C_OK 0
#define NVL_CRC32C_EINVAL (-1)     /* bad argument (NULL pointer, size overflow) */
#define NVL_CRC32C_EHIP (-2)       /* a HIP runtime call failed */
#define NVL_CRC32C_ENODEV (-3)     /* no HIP device / device index out of range */
#define NVL_CRC32C_ESELFTEST (-4)  /* GPU backend failed its known-answer probe */
#define NVL_CRC32C_ENOSPC (-5)     /* caller workspace smaller than required */

/* flags */
#define NVL_CRC32C_FLAG_MASK 0x1u  /* store crc32c::Mask(crc) (util/crc32c.h:31-34),
                                      i.e. the on-disk trailer/header value of
                                      table/table_builder.cc:187 and
                                      db/log_writer.cc:96 */
#define NVL_CRC32C_FLAG_REGION_SHAPED 0x2u  /* nvl_crc32c_region_dev only: the caller has checked
                                              that the batch is region-shaped (see there), so the
                                              call is the region kernel alone, one launch.  A
                                              batch that is not still gets correct results, by
                                              a slow per-buffer path. */

/* Longest buffer the region path takes: a batch holding a longer one runs
 * the batch path (it would be re-streamed and folded serially). */
#define NVL_CRC32C_REGION_MAX_LEN (128u << 10)

/* ---- lifecycle ---------------------------------------------------------- */

/* Build the lookup tables on `device` and run the known-answer probe
 * "TestCRCBuffer" -> 0xdcbc59fa on the GPU (mirrors CanAccelerateCRC32C,
 * util/crc32c.cc:290-297).  Optional: batch calls initialise lazily. */
NVL_API int nvl_crc32c_init(int device);

/* Release every device's tables.  No batch call may be in flight. */
NVL_API int nvl_crc32c_shutdown(void);

/* 1 if the GPU backend on the current device passed its probe, else 0. */
NVL_API int nvl_crc32c_gpu_accelerated(void);

/* Human-readable text for a status code. */
NVL_API const char* nvl_crc32c_strerror(int status);

/* ABI version (NVL_CRC32C_ABI_VERSION). */
NVL_API int nvl_crc32c_abi_version(void);

/* ---- single buffer, host memory (util/crc32c.h:17-40) -------------------- */
/* These replace the reference's host path one-for-one.  One buffer of a few
 * KiB is not worth a GPU round trip, so they run on the calling CPU thread
 * (SSE4.2 crc32 instruction when present, else slice-by-8).  They are the
 * reference API's per-call semantics, not a fallback of the batch calls. */

/* util/crc32c.h:17 leveldb::crc32c::Extend */
NVL_API uint32_t nvl_crc32c_extend(uint32_t init_crc, const void* data, size_t n);
/* util/crc32c.h:20-22 leveldb::crc32c::Value */
NVL_API uint32_t nvl_crc32c_value(const void* data, size_t n);
/* util/crc32c.h:31-34 leveldb::crc32c::Mask */
NVL_API uint32_t nvl_crc32c_mask(uint32_t crc);
/* util/crc32c.h:37-40 leveldb::crc32c::Unmask */
NVL_API uint32_t nvl_crc32c_unmask(uint32_t masked_crc);

/* Which host implementation the single-buffer calls use (chosen once, after
 * a known-answer self-test, like util/crc32c.cc:290-303): "avx512 vpclmulqdq
 * fold + sse4.2", "sse4.2 crc32q x3" or "slice-by-8".  The environment
 * variable NVL_CRC32C_HOST=sse|table caps the tier (tests). */
NVL_API const char* nvl_crc32c_host_impl(void);

/* ---- batched, device-resident (the hot path) ----------------------------- */

/* Fixed-stride batch: buffer i is the `len` bytes at base + i*stride (device
 * memory).  out[i] = Extend(init_i, buffer i, len) where init_i = init[i] if
 * `init` (device array of n u32) is non-NULL, else `init_all`.  With
 * NVL_CRC32C_FLAG_MASK, out[i] = Mask(that).  Replaces n calls of
 * crc32c::Value/Extend at table/table_builder.cc:185-186 (data blocks of one
 * table laid out back to back) and the db_bench crc32c loop
 * (db/db_bench.cc:729-746).  Fast path when base and stride are multiples
 * of 16 and len a multiple of 4096. */
NVL_API int nvl_crc32c_fixed_dev(const void* base, uint64_t stride, uint64_t len, uint64_t n,
                         const uint32_t* init, uint32_t init_all, uint32_t* out,
                         uint32_t flags, void* workspace, size_t workspace_bytes,
                         void* stream);

/* Measurement form of nvl_crc32c_fixed_dev (same arguments and results)
 * for benchmark harnesses: the call's first kernel dispatch records
 * `start_event` and its last records `stop_event` (hipEvent_t, either may be
 * NULL) through hipExtLaunchKernel, so hipEventElapsedTime gives the kernels'
 * own duration -- what rocprofv3's kernel trace reports -- with no marker
 * packet between back-to-back launches.  Not needed by the call sites. */
NVL_API int nvl_crc32c_fixed_dev_timed(const void* base, uint64_t stride, uint64_t len, uint64_t n,
                                       const uint32_t* init, uint32_t init_all, uint32_t* out,
                                       uint32_t flags, void* workspace, size_t workspace_bytes,
                                       void* stream, void* start_event, void* stop_event);

/* Workspace bytes nvl_crc32c_fixed_dev needs for this shape (0 when none). */
NVL_API size_t nvl_crc32c_fixed_workspace_bytes(uint64_t stride, uint64_t len, uint64_t n);

/* Variable-length batch: buffer i is lengths[i] bytes at base + offsets[i]
 * (all three in device memory; pass base = NULL to give absolute device
 * addresses in `offsets`).  Arbitrary alignment and length (0 included).
 * out[i] = Extend(init_i, buffer i) (Mask()ed with NVL_CRC32C_FLAG_MASK).
 * Replaces per-call Value/Extend at table/format.cc:90-92 (block verify),
 * db/log_reader.cc:255-256 and db/log_writer.cc:95 (records).
 * The layout is checked on the device (a plan kernel over the metadata): a
 * region-shaped batch -- sorted by offset, non-overlapping, every buffer at
 * most NVL_CRC32C_REGION_MAX_LEN bytes, the first one not empty, no 4 KiB
 * page between the first and the last byte without a buffer byte (only the
 * buffers' own pages are read: buffers from different allocations are safe),
 * gaps between buffers at most 1/8 of the buffer bytes + 64 KiB, a span of
 * at most 64 GiB -- is checksummed over its own span by the region path (see
 * nvl_crc32c_region_dev); any other batch whose buffers are all exactly 4096
 * bytes (shuffled blocks, pages far apart or overlapping) by the page path
 * (one 4 KiB pass per buffer at the fixed-stride path's rate); the rest by
 * the batch kernels. */
NVL_API int nvl_crc32c_batch_dev(const void* base, const uint64_t* offsets, const uint64_t* lengths,
                         const uint32_t* init, uint32_t init_all, uint32_t* out, uint64_t n,
                         uint32_t flags, void* workspace, size_t workspace_bytes,
                         void* stream);

/* Workspace bytes nvl_crc32c_batch_dev needs for n buffers. */
NVL_API size_t nvl_crc32c_batch_workspace_bytes(uint64_t n);

/* Region batch: buffer i is lengths[i] bytes at region + offsets[i] (device
 * memory; offsets relative to `region`), for buffers that lie inside ONE
 * region [region, region + region_len) sorted by offset and non-overlapping
 * -- an SSTable image's blocks in file order (table/format.cc:90-92 for each),
 * a log image's records, a packed batch.  The region is checksummed in its
 * own page-aligned 4 KiB chunks at the fixed-stride path's rate whatever the
 * buffers' lengths and alignment, and each out[i] is derived from the chunk
 * values (Mask()ed with NVL_CRC32C_FLAG_MASK).  Gaps between buffers cost
 * their bytes (the whole region is read).  The layout is checked on the
 * device first: a batch that is not region-shaped (unsorted, overlapping, a
 * buffer outside the region or longer than NVL_CRC32C_REGION_MAX_LEN) runs
 * as nvl_crc32c_batch_dev runs it (the page path or the batch kernels).
 * NVL_CRC32C_FLAG_REGION_SHAPED
 * skips the check (one launch instead of three). */
NVL_API int nvl_crc32c_region_dev(const void* region, uint64_t region_len, const uint64_t* offsets,
                                  const uint64_t* lengths, const uint32_t* init, uint32_t init_all, uint32_t* out,
                                  uint64_t n, uint32_t flags, void* workspace, size_t workspace_bytes, void* stream);

/* Measurement form (as nvl_crc32c_fixed_dev_timed): the first kernel records
 * start_event, the last stop_event. */
NVL_API int nvl_crc32c_region_dev_timed(const void* region, uint64_t region_len, const uint64_t* offsets,
                                        const uint64_t* lengths, const uint32_t* init, uint32_t init_all,
                                        uint32_t* out, uint64_t n, uint32_t flags, void* workspace,
                                        size_t workspace_bytes, void* stream, void* start_event, void* stop_event);

/* Workspace bytes nvl_crc32c_region_dev needs (4 B per 4 KiB of region + 32 B
 * per buffer for the region path, plus the batch path's workspace). */
NVL_API size_t nvl_crc32c_region_workspace_bytes(uint64_t region_len, uint64_t n);

/* ---- several devices, device-resident, one process ---------------------- */
/* BASELINE config 5's form inside ONE process (a LevelDB process is one
 * process: db/db_impl.cc:920-923 runs compactions on its own threads): the
 * blocks already live on several GPUs, shard k in devices[k]'s HBM, and each
 * shard is checksummed where it lies -- no block ever crosses xGMI.  Shard k
 * is a fixed-stride batch (as nvl_crc32c_fixed_dev) with its results in
 * `out` on the same device; `stream` is a stream of that device (NULL: its
 * null stream).  Every shard is
 * enqueued before the call returns (asynchronous, like nvl_crc32c_fixed_dev:
 * synchronise each shard's stream); the calling thread's current device is
 * left as it was.  A device may hold several shards. */
typedef struct nvl_crc32c_shard {
  int device;         /* HIP device holding base and out */
  const void* base;   /* shard buffer i at base + i * stride, len bytes */
  uint64_t stride;
  uint64_t len;
  uint64_t n;         /* buffers in the shard */
  uint32_t* out;      /* n u32 results, on `device` */
  void* stream;       /* hipStream_t of `device`, or NULL (its null stream) */
} nvl_crc32c_shard;
NVL_API int nvl_crc32c_fixed_dev_multi(const nvl_crc32c_shard* shards, int nshards, uint32_t init_all,
                                       uint32_t flags);

/* The shards' results gathered into ONE device array `dst` (on dst_device,
 * ordered on `stream`, a stream of dst_device or NULL for its null stream),
 * after each shard's stream: up to 16 shards on dst_device or peer-mapped to
 * it (peer access is enabled once per device pair, process-wide) are read in
 * place by one kernel -- over xGMI for a peer, 4 bytes per block: the only
 * cross-device traffic; more shards, or a peer that cannot be mapped, are
 * copied first (hipMemcpyPeerAsync) and then laid out.  Layouts:
 *   NVL_CRC32C_GATHER_CONCAT       shard 0's results, then shard 1's, ...
 *   NVL_CRC32C_GATHER_ROUND_ROBIN  global block i from shard i mod nshards
 *                                  (shard k must hold ceil((N - k) / nshards)
 *                                  blocks of the N in total: config 5's split)
 * Asynchronous on `stream`. */
#define NVL_CRC32C_GATHER_CONCAT 0u
#define NVL_CRC32C_GATHER_ROUND_ROBIN 1u
NVL_API int nvl_crc32c_gather_dev(uint32_t* dst, int dst_device, const nvl_crc32c_shard* shards, int nshards,
                                  uint32_t layout, void* stream);

/* ---- batched, host-resident (end-to-end path) ---------------------------- */

/* Host buffers in, host results out, synchronous: stages the buffers through
 * pinned memory, H2D, GPU batch kernel, D2H.  ptrs/lengths/init/out are host
 * arrays (init may be NULL -> init_all).  This is what the block-batching
 * shims at the four reference call sites use. */
NVL_API int nvl_crc32c_batch_host(const void* const* ptrs, const uint64_t* lengths,
                          const uint32_t* init, uint32_t init_all, uint32_t* out,
                          uint64_t n, uint32_t flags);

/* Host region variant: n buffers that all lie inside ONE host region
 * [region, region + region_len) (a file image, a log block run): buffer i is
 * region[offsets[i] .. offsets[i]+lengths[i]).  The covered range is staged
 * once (one pinned copy, one H2D; none when it lies in a range registered
 * with nvl_crc32c_host_register: DMA from the caller's pages, or with
 * NVL_CRC32C_FLAG_HOST_ZERO_COPY no copy at all), then batched as
 * nvl_crc32c_batch_dev.  Synchronous.  NVL_CRC32C_FLAG_HOST_ZERO_COPY on a
 * range that is not registered: NVL_CRC32C_EINVAL. */
NVL_API int nvl_crc32c_batch_region_host(const void* region, uint64_t region_len, const uint64_t* offsets,
                                         const uint64_t* lengths, const uint32_t* init, uint32_t init_all,
                                         uint32_t* out, uint64_t n, uint32_t flags);

/* Several devices, host-resident (the compaction output of db/db_impl.cc:920-923
 * or an mmap'd table scan, util/env_posix.cc:199-209, over the GPUs of a node):
 * the batch is cut into at most ndev contiguous index ranges of about equal
 * covered bytes -- no more than (bytes / min_bytes_per_device) of them, so a
 * small batch stays on devices[0] -- and range k runs as
 * nvl_crc32c_batch_region_host on devices[k] (its own pinned staging, stream
 * and PCIe link) from a pool thread, results written straight into out.
 * min_bytes_per_device = 0: NVL_CRC32C_MULTI_MIN_BYTES.  A device may appear
 * twice (two pipes into one GPU).  Synchronous; multi calls are serialised. */
#define NVL_CRC32C_MULTI_MIN_BYTES (64ull << 20)
NVL_API int nvl_crc32c_batch_region_host_multi(const void* region, uint64_t region_len, const uint64_t* offsets,
                                               const uint64_t* lengths, const uint32_t* init, uint32_t init_all,
                                               uint32_t* out, uint64_t n, uint32_t flags, const int* devices,
                                               int ndev, uint64_t min_bytes_per_device);

/* The cut nvl_crc32c_batch_region_host_multi makes: part k is buffers
 * [part_first[k], part_first[k+1]) (part_first holds ndev + 1 entries);
 * returns the number of parts (>= 1), or a negative status. */
NVL_API int nvl_crc32c_multi_plan(const uint64_t* offsets, const uint64_t* lengths, uint64_t n, int ndev,
                                  uint64_t min_bytes, uint64_t* part_first);

/* ---- registered host memory: the staging-free host-resident path -------- */
/* The fork's host-resident call sites start in pageable memory -- an mmap'd
 * table (util/env_posix.cc:199-209), a TableBuilder's block buffer
 * (table/table_builder.cc:185-187), a compaction's output -- which the
 * host-resident entry points otherwise first copy into pinned staging on
 * the calling CPU threads.  nvl_crc32c_host_register pins and maps
 * [ptr, ptr + bytes) for every device (hipHostRegister, portable | mapped),
 * once, for as long as the caller keeps it (e.g. the life of an mmap):
 * nvl_crc32c_batch_region_host (and the _multi form, per device) then DMA a
 * window that lies inside one registration straight from the caller's pages
 * -- no CPU copy -- and with NVL_CRC32C_FLAG_HOST_ZERO_COPY run the kernels
 * on the mapped pages themselves (they read over PCIe; nothing is copied to
 * HBM).  Anything else (unregistered, or a window crossing a registration's
 * end) still takes the pinned staging; a failed registration leaves the
 * range unregistered and returns its status.  Registrations may not
 * overlap (NVL_CRC32C_EINVAL).  nvl_crc32c_host_unregister takes the `ptr`
 * that was registered; no call may be using the range. */
#define NVL_CRC32C_FLAG_HOST_ZERO_COPY 0x4u /* host region entry: read registered pages in place */
NVL_API int nvl_crc32c_host_register(const void* ptr, size_t bytes);
NVL_API int nvl_crc32c_host_unregister(const void* ptr);
/* 1 if [ptr, ptr + bytes) lies inside one registration, else 0. */
NVL_API int nvl_crc32c_host_registered(const void* ptr, size_t bytes);

/* Host fixed-stride batch (one contiguous host region, e.g. an mmap'd table
 * file or a pinned bench buffer), pipelined H2D/compute/D2H over two
 * streams.  Synchronous. */
NVL_API int nvl_crc32c_fixed_host(const void* base, uint64_t stride, uint64_t len, uint64_t n,
                          const uint32_t* init, uint32_t init_all, uint32_t* out,
                          uint32_t flags);

/* ---- synthetic inputs (measurement harness) -------------- */

/* Fill device memory with the canonical splitmix64 byte stream: block k
 * (block_bytes long, written at dst + k*block_bytes) receives stream bytes
 * [(first_block + k*block_step)*block_bytes, +block_bytes), where stream word
 * j is splitmix64's (j+1)-th output from state `seed`, little-endian.
 * block_step > 1 lays out a round-robin shard (buffer i on GPU i mod G).
 * block_bytes must be a multiple of 8.  Asynchronous on `stream`. */
NVL_API int nvl_crc32c_fill_splitmix(void* dst, uint64_t nblocks, uint64_t block_bytes,
                                     uint64_t first_block, uint64_t block_step, uint64_t seed,
                                     void* stream);

/* (harness) The measured read ceiling: one launch of a plain streaming
 * kernel that reads `bytes` (a multiple of 16) at `src` (16-byte aligned; else
 * NVL_CRC32C_EINVAL) and XOR-reduces them
 * -- four 16-byte nontemporal loads in flight per thread, grid-strided, 256
 * workgroups of 1024 threads (the best read-only shape measured on gfx950,
 * DESIGN.md §4) -- so that a benchmark can time the HBM read rate beside the
 * engine's kernels in the same run.  Writes 4 bytes at `sink` only when the
 * XOR of the data is 0x12345678.  Asynchronous on `stream`. */
NVL_API int nvl_crc32c_read_probe(const void* src, uint64_t bytes, uint32_t* sink, void* stream);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* NVL_CRC32C_H_ */
