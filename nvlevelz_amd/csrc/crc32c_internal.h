// nvlevelz_amd/csrc/crc32c_internal.h -- internal interfaces between the
// C-ABI layer (crc32c_capi.cpp) and the kernel launchers (crc32c_fixed.hip,
// crc32c_batch.hip, crc32c_region.hip, crc32c_misc.hip,
// crc32c_scan.hip).  Not installed; not part of the ABI.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include <algorithm>

#include "nvl_framing.h"

namespace nvl {

// Device table blob (u32 words), built on the host by build_device_tables():
//   [0,     1024)  slice4[4][256]     util/crc32c.cc:18-281 equivalents
//   [1024,  7168)  comb[6][4][256]    shift by 64*2^k bytes, byte-sliced
//   [7168,  8192)  sh4096[4][256]     shift by 4096 bytes, byte-sliced
//   [8192,  8256)  x2n[64]            x^(2^k) mod P
//   [8256, 16449)  xp8[8193]          x^(8d) mod P, d = 0..8192        (region fold)
//   [16449,20545)  xm8[4096]          x^(-8d) mod P, d = 0..4095       (region fold)
//   [20548,28740)  nib[8][16][64]     T[n][v][j] = shift(v << 4n, 64(63 - j))  (region kernel:
//                                     lane j's piece raw to the chunk end; 16-byte aligned, copied
//                                     verbatim into LDS)
//   [28740,32836) shc[4][4][256]     shift by 4096 d bytes (d = 1..4), byte-sliced (region fold: copied
//                                     into LDS over the nibble tables' upper half once the chunks are done)
//   [32836,33092) pw4k[256]          x^(8*4096*q) mod P, q = 0..255  (region fold: x^(8L) of a long buffer)
constexpr uint32_t kXp8Len = 8193;  // a buffer spanning at most two chunks has at most 8192 bytes
constexpr uint32_t kTabXp8 = 8256, kTabXm8 = kTabXp8 + kXp8Len;
constexpr uint32_t kTabNib = (kTabXm8 + 4096u + 3u) & ~3u;
constexpr uint32_t kTabShc = kTabNib + 8u * 16u * 64u;
constexpr uint32_t kTabPw4k = kTabShc + 4u * 1024u;
constexpr uint32_t kTableWords = kTabPw4k + 256u;

// A portion of one buffer processed inside one work unit (fix-up input).
struct Rec {
  unsigned long long buf;  // buffer index, kNoBuf when unused
  uint32_t raw;            // raw register of the portion (ends at the portion end)
  uint32_t cnt;            // chunks in the portion | kRecEnds if it holds the last chunk
};
constexpr unsigned long long kNoBuf = ~0ull;
constexpr uint32_t kRecEnds = 0x80000000u;

// Per-stream counter block: kCounterBytes, zeroed once when created; every
// kernel that counts in it leaves it zero again, so the launches of one
// stream (ordered) share it.
constexpr size_t kCounterBytes = 256;

struct LaunchCtx {
  hipStream_t stream;
  int num_cu;
  const uint32_t* tables;  // device blob
  uint32_t* counter;       // the stream's counter block (fused kernels), or nullptr
  // Measurement only (nvl_crc32c_fixed_dev_timed): recorded by the call's
  // first / last kernel dispatch itself (hipExtLaunchKernel), so they time the
  // kernels alone and add no marker packet between back-to-back launches.
  hipEvent_t ev_start = nullptr;
  hipEvent_t ev_stop = nullptr;
};

void build_device_tables(uint32_t* words /* kTableWords */);

// ws: fixed_recs_bytes() of workspace (unit records, then head contributions).
hipError_t launch_fixed(const LaunchCtx& lc, const uint8_t* base, uint64_t stride, uint64_t len, uint64_t n,
                        const uint32_t* init, uint32_t init_all, uint32_t* out, uint32_t flags, Rec* ws);
size_t fixed_recs_bytes(int num_cu, uint64_t len, uint64_t n);  // workspace of launch_fixed
size_t var_recs_bytes(int num_cu);                               // record part of launch_var's workspace
size_t var_unit_map_bytes(int num_cu);                           // unit map part of launch_var's workspace

// Plan for the variable-length kernel: small batches in one launch
// (chunk_start + unit map), large ones as counts -> device scan -> unit map.
bool var_plan_small(uint64_t n);
// long_bufs: one u32 of workspace, set by the plan (0: every buffer has at
// most 32 chunks, so the body kernel can give each buffer to one wave).
hipError_t launch_var_plan_small(const LaunchCtx& lc, const uint64_t* lengths, uint64_t n, uint64_t* chunk_start,
                                 uint64_t* unit_first, uint32_t* long_bufs);
hipError_t launch_var_counts(const uint64_t* lengths, uint64_t n, uint64_t* cnt, uint32_t* long_bufs,
                             hipStream_t st);
// have_unit_map: unit_first already written (small plan); otherwise built here.
// hc: n u32 of workspace (head contributions, written by the head kernel
// that every variable-length call launches first).
hipError_t launch_var(const LaunchCtx& lc, const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths,
                      const uint64_t* chunk_start, uint64_t* unit_first, uint64_t n, const uint32_t* init,
                      uint32_t init_all, uint32_t* out, uint32_t flags, Rec* recs, uint32_t* hc, uint32_t* long_bufs,
                      bool have_unit_map);

// A variable-length batch in two launches (lc.counter set): the head kernel
// (heads + the plan's tiles: lpre[n], tiles[2 * head grid]) and the fused
// kernel (chunk positions from the tiles, checksum, fix-up); recs: the
// launch_var workspace records (hold the edge records).  max_len: a bound
// on the lengths the caller knows on the host (UINT64_MAX: none); when it
// makes every tile a short-mode tile (see var_heads_only) the fused kernel,
// which would return at once, is not launched.
hipError_t launch_var_fused(const LaunchCtx& lc, const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths,
                            uint64_t n, const uint32_t* init, uint32_t init_all, uint32_t* out, uint32_t flags,
                            Rec* recs, uint32_t* hc, uint64_t* lpre, uint64_t* tiles, uint64_t max_len = UINT64_MAX);
// The head kernel finishes every buffer of an n-buffer batch whose lengths
// are all <= max_len: two chunks at most, one sub-range per tile.
bool var_heads_only(int num_cu, uint64_t n, uint64_t max_len);

// Region batch (nvl_crc32c_region_dev): n buffers inside [region, region +
// region_len), checksummed over the region's page-aligned 4 KiB chunks and
// folded per buffer in the same launch.  ws: region_ws_bytes(region_len, n)
// (chunk raws and gen-tagged event records; never needs resetting).
size_t region_ws_bytes(uint64_t region_len, uint64_t n);
uint64_t region_cap_chunks(uint64_t region_len);                  // raws the region workspace holds
size_t region_ws_bytes_cap(uint64_t cap_chunks, uint64_t n);      // a region workspace for cap_chunks raws

// Routed batch over device metadata (nvl_crc32c_batch_dev: dyn, the region
// is the batch's own span; nvl_crc32c_region_dev: the caller's region):
// crc32c_route_plan -> crc32c_route_kernel (region path or heads) ->
// crc32c_var_fused_kernel (returns at once on the region path).  Needs the
// stream's counter block (lc.counter), the launch_var_fused workspace (recs,
// hc, lpre, tiles), route_parts_bytes() of plan partials and a region
// workspace of region_ws_bytes_cap(cap_chunks, n) (dyn: cap_chunks =
// route_cap_chunks(n); region_dev: region_cap_chunks(region_len)).
size_t route_parts_bytes();
uint64_t route_cap_chunks(uint64_t n);
hipError_t launch_routed(const LaunchCtx& lc, const uint8_t* base, uint64_t region_len, bool dyn,
                         const uint64_t* offsets, const uint64_t* lengths, uint64_t n, const uint32_t* init,
                         uint32_t init_all, uint32_t* out, uint32_t flags, void* region_ws, uint64_t cap_chunks,
                         void* parts_ws, Rec* recs, uint32_t* hc, uint64_t* lpre, uint64_t* tiles);
// The longest buffer the region path takes (a longer one: the batch path).
constexpr uint64_t kRegionMaxLen = 128ull << 10;
hipError_t launch_region(const LaunchCtx& lc, const uint8_t* region, uint64_t region_len, const uint64_t* offsets,
                         const uint64_t* lengths, const uint32_t* init, uint32_t init_all, uint32_t* out, uint64_t n,
                         uint32_t flags, void* ws);

// nvl_crc32c_gather_dev in one launch: up to kGatherMax shards' result arrays
// on (or peer-mapped to) the destination device, round robin (rr) or
// concatenated (shard k at [pos[k], pos[k+1])).
namespace dev {
constexpr uint32_t kGatherMax = 16;
struct GatherSrc {
  const uint32_t* src[kGatherMax];
  uint64_t pos[kGatherMax + 1];
  uint32_t G, rr;
};
}  // namespace dev
hipError_t launch_gather(const dev::GatherSrc& s, uint64_t N, uint32_t* dst, hipStream_t st);
// dst[i] = shard (i mod G)'s result (i div G) from the shards' results concatenated (nvl_crc32c_gather_dev)
hipError_t launch_interleave_rr(const uint32_t* src, uint64_t N, uint32_t G, uint32_t* dst, hipStream_t st);
hipError_t launch_read_probe(const void* src, uint64_t bytes, uint32_t* sink, hipStream_t st);
hipError_t launch_fill(void* dst, uint64_t nblocks, uint64_t block_bytes, uint64_t first_block, uint64_t block_step,
                       uint64_t seed, hipStream_t st);
// verdict[i] = NVL_BLOCK_* of the trailer at file[off[i] + len1[i] - 1] against crc[i]
hipError_t launch_trailer_verdicts(const void* file, const uint64_t* off, const uint64_t* len1, const uint32_t* crc,
                                   uint64_t n, uint8_t* verdict, hipStream_t st);

// nvl_sstable_verify_table_dev's fast path (crc32c_table_dev.hip): batch
// slots [0, nr) from the entries of a restart-interval-1 index block, parsed
// one per thread (records rec[i]; *bad |= 1 when the block is not in the form
// the sequential walk reads the same way), [nr, nr + nm) the meta blocks
// (host), up to pb zero-length fillers, [pb, pb + np) the index block in
// 4096-byte pieces -- file order; then ReadBlock's trailer checks for every
// slot whose verdict vk[k] is still 0xFF, with counts, piece CRCs and meta
// verdicts in res.
hipError_t launch_index_entries(const void* file, uint64_t file_len, uint64_t index_off, uint64_t size, uint32_t nr,
                                uint32_t np, uint32_t pb, uint64_t* boff, uint64_t* blen, uint8_t* vk,
                                nvl_table_block* rec, uint32_t* bad, hipStream_t st);
hipError_t launch_table_verdicts(const void* file, const uint64_t* boff, const uint64_t* blen, const uint32_t* crc,
                                 uint64_t n, uint32_t nr, uint32_t nm, uint32_t pb, uint32_t np, uint8_t* vk,
                                 void* res, hipStream_t st);
// Its per-thread resources (crc32c_capi.cpp): device memory on `device`,
// pinned host memory (both grown on demand, reused by the thread's next
// call), a second stream and two events on `device`.
void* thread_table_device(int device, size_t bytes);
void* thread_table_pinned(size_t bytes);
bool thread_table_aux(int device, hipStream_t* side, hipEvent_t* ev_a, hipEvent_t* ev_b);

// Exclusive prefix sum over n u64 (crc32c_scan.hip, hipCUB).
size_t scan_temp_bytes(uint64_t n);
hipError_t exclusive_scan_u64(void* temp, size_t temp_bytes, const uint64_t* in, uint64_t* out, uint64_t n,
                              hipStream_t st);

// CPU single-buffer Extend (crc32c_host.cpp) and the tier it chose.
uint32_t host_extend(uint32_t init, const void* data, size_t n);
const char* host_impl_name();
// The host tier host_extend runs: 0 slice-by-8, 1 SSE4.2 crc32q, 2 AVX-512 folding.
int host_tier_id();

}  // namespace nvl
