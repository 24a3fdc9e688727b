// nvlevelz_amd/csrc/crc32c_kernels.hip -- CDNA4 (gfx950) batched CRC32C.
//
// Replaces the per-call hot loops of the reference,
//   port/port_posix_sse.cc:103-105  (8 B crc32q steps)  and
//   util/crc32c.cc:333-339          (slice-by-4 STEP4),
// with a batched, device-resident engine.  Bit-exact with
// leveldb::crc32c::Extend (util/crc32c.cc:299-347).
//
// Work decomposition:
//   * A buffer of L bytes is cut into J = max(1, ceil(L/4096)) "chunks",
//     END-aligned: chunk c covers [e - 4096*(J-c), e - 4096*(J-1-c)) ∩ [p, e)
//     for buffer [p, e).  Only chunk 0 (the head) can be short.
//   * One wavefront processes one chunk: lane l owns the contiguous 64-byte
//     "piece" [ce - 64*(64-l), ce - 64*(63-l)) of the chunk ending at ce, loads
//     it with four (five when misaligned) 16-byte global loads, and runs a
//     serial slice-by-4 over its 16 words.  Bytes before the buffer start are
//     zero (leading zeros do not change a zero-state register), and the
//     buffer's ~init is XORed into its first four bytes
//     (raw(s, w||rest) = raw(0, (w^s)||rest)), so every piece starts from 0.
//   * The 64 per-lane registers are folded with a 6-level butterfly:
//     level k combines neighbouring groups of 2^k pieces with the GF(2)
//     operator "shift by 64*2^k bytes", applied as 4 byte-table lookups that
//     are spread over the group's lanes and XOR-reduced with DPP.
//   * A wave walks a contiguous range of chunk indices; consecutive chunks of
//     one buffer accumulate as acc = shift4096(acc) ^ raw.  A buffer whose
//     chunks span several waves leaves per-wave records that a small fix-up
//     kernel folds (shift by 4096*k bytes, k the later waves' chunk count).
//
// Lookup tables live in LDS.  The four slice-by-4 tables are replicated 32
// times with the replica chosen by lane%32, so a wave's ds_read_b32 of
// data-dependent indices never bank-conflicts (bank = lane%32).  Address of
// table t, byte b, lane l:  (t>>1)<<16 | b<<8 | (t&1)<<7 | (l&31)<<2, formed
// with ONE v_perm_b32 per lookup from the data word and a per-lane base.
#include <hip/hip_ext.h>
#include <atomic>
#include <random>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_internal.h"
#include "crc32c_math.h"

namespace nvl {
namespace dev {

constexpr int kWave = 64;
constexpr int kWavesPerWG = 16;
constexpr int kThreads = kWave * kWavesPerWG;  // 1024
constexpr uint32_t kChunk = 4096;
constexpr uint32_t kUnitsPerWG = 64;  // work units per workgroup (scheduler B)
// Chunks of a buffer of L bytes: END-aligned 4096-byte chunks, the first one
// 1..4096 bytes long (tests/kernel_model.py chunks_of).  (Round 1 tried an
// overhang -- a first chunk of up to 4096+16 bytes as one pass -- and dropped
// it: its registers slowed every body pass more than it saved.)
__host__ __device__ __forceinline__ uint32_t chunks_for(uint64_t L) {
  return L <= kChunk ? 1u : (uint32_t)((L + kChunk - 1) / kChunk);
}

// LDS image (bytes)
// The operator tables sit first so that every table offset of a lookup fits
// the ds_read 16-bit immediate (comb level k at 4096*k, sh4096 at 24576, the
// slice image at 28672); only the data-dependent part is computed per lookup.
constexpr uint32_t kCombOff = 0;                              // comb[6][4][256] u32
constexpr uint32_t kShOff = kCombOff + 6u * 4u * 256u * 4u;   // sh4096[4][256] u32
constexpr uint32_t kSliceOff = kShOff + 4u * 256u * 4u;       // 4 tables x 256 x 32 replicas x 4 B
constexpr uint32_t kRepBytes = 128u * 1024u;
constexpr uint32_t kCtrOff = kSliceOff + kRepBytes;           // per-workgroup work counter
constexpr uint32_t kLdsBytes = kCtrOff + 16u;                 // 159760 B
static_assert(kSliceOff < 65536u && kShOff < 65536u, "table offsets must fit the ds_read immediate");
static_assert(kLdsBytes <= 160u * 1024u, "LDS image exceeds 160 KiB");

// DevTables word offsets (see crc32c_internal.h)
constexpr uint32_t kGSlice = 0, kGComb = 1024, kGX2n = 1024 + 6144 + 1024;  // comb, sh4096 contiguous

// ---------------------------------------------------------------------------
// Wave-uniform copies (lane 0's value in SGPRs).  readfirstlane returns int:
// each half goes through uint32_t so that a low half >= 2^31 is not
// sign-extended into the high half (a device address usually has bit 31 set).
// These four helpers are the ONLY places the kernels may call
// __builtin_amdgcn_readfirstlane / __builtin_amdgcn_readlane
// (tests/test_kernel_source.py enforces it): the 32-bit forms refuse wider
// operands at compile time, the 64-bit forms move two uint32_t halves.
template <class T>
__device__ __forceinline__ uint32_t uniform_u32(T v) {
  static_assert(sizeof(T) <= 4, "uniform_u32 of a 64-bit value: use uniform_u64");
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
  return ((uint64_t)uniform_u32((uint32_t)(v >> 32)) << 32) | (uint64_t)uniform_u32((uint32_t)v);
}
// lane j's value (j wave-uniform)
template <class T>
__device__ __forceinline__ uint32_t lane_u32(T v, uint32_t j) {
  static_assert(sizeof(T) <= 4, "lane_u32 of a 64-bit value: use lane_u64");
  return (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)j);
}
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, uint32_t j) {
  return ((uint64_t)lane_u32((uint32_t)(v >> 32), j) << 32) | (uint64_t)lane_u32((uint32_t)v, j);
}

// cross-lane helpers (all called with EXEC = all 64 lanes)
__device__ __forceinline__ uint32_t dpp_xor1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ uint32_t dpp_xor2(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
}
__device__ __forceinline__ uint32_t swz_xor4(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x101F);  // and 0x1f, xor 4
}
__device__ __forceinline__ uint32_t dpp_xor8(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, true);  // row_ror:8
}
__device__ __forceinline__ uint32_t swz_xor16(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);  // and 0x1f, xor 16
}
__device__ __forceinline__ uint32_t xor32(uint32_t v) {
  return (uint32_t)__shfl_xor((int)v, 32);
}

template <int LEV>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
  if constexpr (LEV == 0) return dpp_xor1(v);
  else if constexpr (LEV == 1) return dpp_xor2(v);
  else if constexpr (LEV == 2) return swz_xor4(v);
  else if constexpr (LEV == 3) return dpp_xor8(v);
  else if constexpr (LEV == 4) return swz_xor16(v);
  else return xor32(v);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

typedef const u32x4 __attribute__((address_space(1))) * gvec_ptr;

// 16-byte streaming load from global memory (read-once data: non-temporal
// hint).  The explicit address space keeps it a global_load (a flat_load would
// also count in lgkmcnt and serialise against the LDS lookups).
__device__ __forceinline__ u32x4 ld16(uintptr_t addr) { return __builtin_nontemporal_load((gvec_ptr)addr); }

// The same through the caches: the head kernel's lane-group loads touch each
// line from several instructions (lanes 64 bytes apart), so non-temporal
// loads would let a line go before its neighbours read it.
__device__ __forceinline__ u32x4 ld16c(uintptr_t addr) { return *(gvec_ptr)addr; }

__device__ __forceinline__ uint32_t lds_u32(const uint8_t* lds, uint32_t off) {
  return *reinterpret_cast<const uint32_t*>(lds + off);
}

// Per-lane replica bases for slice tables t = 3, 2, 1, 0.
struct LaneBase {
  uint32_t t3, t2, t1, t0;
};

__device__ __forceinline__ LaneBase make_lane_base(int lane) {
  const uint32_t r = (uint32_t)(lane & 31) << 2;
  return LaneBase{(1u << 16) | 0x80u | r, (1u << 16) | r, 0x80u | r, r};
}

// One slice-by-4 step (util/crc32c.cc:287-289 STEP4 semantics): x = crc ^ word,
// result = T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3].
__device__ __forceinline__ uint32_t slice4(const uint8_t* lds, uint32_t x, const LaneBase& lb) {
  const uint32_t a0 = __builtin_amdgcn_perm(x, lb.t3, 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, lb.t2, 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, lb.t1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(x, lb.t0, 0x0C020700u);
  const uint8_t* sl = lds + kSliceOff;
  return lds_u32(sl, a0) ^ lds_u32(sl, a1) ^ lds_u32(sl, a2) ^ lds_u32(sl, a3);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));  // gfx950: 3-input XOR via truth table 0x96
  return d;
}

// slice4(x) ^ next, with the five-way XOR as two v_xor3_b32.
__device__ __forceinline__ uint32_t slice4_x(const uint8_t* lds, uint32_t x, uint32_t next, const LaneBase& lb) {
  const uint32_t a0 = __builtin_amdgcn_perm(x, lb.t3, 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, lb.t2, 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, lb.t1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(x, lb.t0, 0x0C020700u);
  const uint8_t* sl = lds + kSliceOff;
  return xor3(xor3(lds_u32(sl, a0), lds_u32(sl, a1), lds_u32(sl, a2)), lds_u32(sl, a3), next);
}

// slice4(x) ^ next -- the chain step with the following word folded in.
__device__ __forceinline__ uint32_t slice4_next(const uint8_t* lds, uint32_t x, uint32_t next, const LaneBase& lb) {
  return slice4_x(lds, x, next, lb);  // two v_bitop3 instead of four v_xor (tools/ab_bench.py: -2 us on cfg2)
}



// A lane-derived value made opaque at its point of use.  The per-lane table
// bases below are cheap to recompute; without this the compiler hoists one
// base per (table, level) out of the main loop, the extra loop-invariant VGPRs
// spill, and every scratch reload waits (vmcnt) on the in-flight prefetch.
__device__ __forceinline__ uint32_t opaque(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}


// Byte j of v looked up in 1 KiB table (TAB, j): the lane supplies j through
// (base = table 0's address for its j, sh = 8j); TAB becomes the ds_read
// immediate offset.
template <uint32_t OFF>
__device__ __forceinline__ uint32_t lane_lookup(const uint8_t* lds, uint32_t base, uint32_t sh, uint32_t v) {
  const uint32_t b = __builtin_amdgcn_ubfe(v, sh, 8);
  return lds_u32(lds + OFF, base + (b << 2));
}

// One butterfly level over lane bit LEV: the lane with bit LEV clear holds the
// group of lower stream positions ("left"), the partner the upper one
// ("right"); left is shifted by the operator in comb table TAB (64*2^TAB
// bytes) and XORed in.  Lanes 0..3 of every quad spread the 4 byte lookups.
template <int LEV, int TAB = LEV, bool OPQ = true>
__device__ __forceinline__ uint32_t fold_level(const uint8_t* lds, uint32_t g, int lane) {
  const uint32_t pt = lane_xor<LEV>(g);
  const bool hi = (lane >> LEV) & 1;
  const uint32_t left = hi ? pt : g;
  const uint32_t right = hi ? g : pt;
  uint32_t s;
  if constexpr (LEV == 0) {  // lane bit 0 picks bytes {0,1} or {2,3}
    const uint32_t h = OPQ ? opaque((uint32_t)lane & 1u) : (uint32_t)lane & 1u;
    const uint32_t base = h << 11, sh = h << 4;
    s = lane_lookup<kCombOff + TAB * 4096u>(lds, base, sh, left) ^
        lane_lookup<kCombOff + TAB * 4096u + 1024u>(lds, base, sh + 8u, left);
    s ^= dpp_xor1(s);
  } else {  // lane & 3 picks the byte
    const uint32_t j = OPQ ? opaque((uint32_t)lane & 3u) : (uint32_t)lane & 3u;
    s = lane_lookup<kCombOff + TAB * 4096u>(lds, j << 10, j << 3, left);
    s ^= dpp_xor1(s);
    s ^= dpp_xor2(s);
  }
  return s ^ right;
}

// shift(acc, 4096) for a wave-uniform acc; every lane gets the result.
__device__ __forceinline__ uint32_t shift4096(const uint8_t* lds, uint32_t acc, int lane) {
  const uint32_t j = opaque((uint32_t)lane & 3u);
  uint32_t s = lane_lookup<kShOff>(lds, j << 10, j << 3, acc);
  s ^= dpp_xor1(s);
  s ^= dpp_xor2(s);
  return s;
}

// The LDS image from the device table blob, in two halves: the loads (issued
// ahead of a wave's first chunk loads, so the fill waits for the blob alone),
// then the stores -- the replicated slice tables as 8192 16-byte slots
// (consecutive lanes write consecutive 16 B: conflict-free ds_write_b128),
// the comb + sh4096 operators (7168 words) verbatim, the work counter.
template <int NW>
struct LdsFill {
  uint32_t rep[(8192 + kWave * NW - 1) / (kWave * NW)];
  uint4 op[(1792 + kWave * NW - 1) / (kWave * NW)];
};
template <int NW>
__device__ __forceinline__ LdsFill<NW> fill_lds_load(const uint32_t* __restrict__ g) {
  constexpr int kT = kWave * NW;
  LdsFill<NW> f;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < (8192 + kT - 1) / kT; ++q) {
    const uint32_t s = (uint32_t)(t + q * kT);
    if ((8192 % kT) != 0 && s >= 8192u) break;
    const uint32_t off = s << 4;
    f.rep[q] = g[kGSlice + (((off >> 16) << 1) | ((off >> 7) & 1u)) * 256u + ((off >> 8) & 0xFFu)];
  }
  const uint4* src = reinterpret_cast<const uint4*>(g + kGComb);
#pragma unroll
  for (int q = 0; q < (1792 + kT - 1) / kT; ++q)
    if (t + q * kT < 1792) f.op[q] = src[t + q * kT];
  return f;
}
template <int NW>
__device__ __forceinline__ void fill_lds_store(uint8_t* lds, const LdsFill<NW>& f, uint32_t ctr0 = NW) {
  constexpr int kT = kWave * NW;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < (8192 + kT - 1) / kT; ++q) {
    const uint32_t s = (uint32_t)(t + q * kT);
    if ((8192 % kT) != 0 && s >= 8192u) break;
    *reinterpret_cast<uint4*>(lds + kSliceOff + (s << 4)) = make_uint4(f.rep[q], f.rep[q], f.rep[q], f.rep[q]);
  }
  uint4* dst = reinterpret_cast<uint4*>(lds + kCombOff);
#pragma unroll
  for (int q = 0; q < (1792 + kT - 1) / kT; ++q)
    if (t + q * kT < 1792) dst[t + q * kT] = f.op[q];
  if (t == 0) *reinterpret_cast<uint32_t*>(lds + kCtrOff) = ctr0;
}

__device__ __forceinline__ uint32_t finish(uint32_t crc, uint32_t flags) {
  return (flags & 1u) ? nvl::mask(crc) : crc;
}

// Buffer geometry as seen by a wave.
struct BufInfo {
  const uint8_t* p;  // first byte
  uint64_t len;      // bytes
  uint32_t J;        // chunks
  uint32_t s;        // ~init, injected into the first 4 bytes
};

// Wave-uniform reads of read-only metadata (lengths, offsets, init, plan
// arrays) through the constant address space: scalar loads (s_load, counted
// in lgkmcnt).  As vector loads they were counted in vmcnt, whose in-order
// retirement made every buffer boundary wait for the prefetched chunk too.
// (Written before the launch only: the scalar cache is invalidated at kernel
// start, cdna_hip_programming.md Guideline 16 Pitfall 6.)
template <class T>
__device__ __forceinline__ T ldc(const T* p, uint64_t i) {
  return ((const __attribute__((address_space(4))) T*)p)[i];
}

// Route plan of a batch over device metadata (nvl_crc32c_batch_dev,
// nvl_crc32c_region_dev): crc32c_route_plan checks the offsets and lengths
// in slices and writes one partial per slice; every later launch of the
// call reduces the same partials (route_region: one wave-wide load, ballots
// and a sum) and takes the same decision -- the region path for a
// region-shaped batch, the head + body kernels otherwise.  No atomics, no
// reset: the partials are plain stores of the plan launch.
struct RoutePart {
  uint64_t sum;  // sum of the slice's lengths, each capped at kRegionMaxLen + 1 (< 2^43 for n < 2^31)
  uint64_t bad;  // kRpBad | kRpNot4k | kRpUnaligned, OR over the slice
};
constexpr uint64_t kRpBad = 1;        // a pair out of order / overlapping, a buffer outside the region or too long
constexpr uint64_t kRpNot4k = 2;      // a buffer whose length is not 4096
constexpr uint64_t kRpUnaligned = 4;  // a buffer not 16-byte aligned
// The launches after the plan: the region path, the page path (every buffer
// exactly one 4 KiB chunk: scheduler A over the batch's own list, aligned or
// realigned), or the head + body kernels.
enum RouteKind : int { kRouteHeads = 0, kRouteRegion = 1, kRoutePages = 2, kRoutePagesAligned = 3 };
constexpr uint32_t kRoutePlanMax = 128;  // plan workgroups (a wave reduces their partials, two per lane)
struct Route {
  const RoutePart* parts = nullptr;  // nullptr: no route (the launch is what it is)
  uint32_t np = 0;
  uint32_t dyn = 0;                  // 1: geometry from the batch (batch_dev), gap rule; 0: the caller's region
  const uint8_t* base = nullptr;     // dyn: the offsets' base (nullptr: absolute addresses)
  const uint64_t* offsets = nullptr; // the batch's metadata (dyn: its span from the first and last buffer)
  const uint64_t* lengths = nullptr;
  uint64_t n = 0;
  uint64_t cap_chunks = 0;           // dyn: region chunks the workspace holds
};

struct KArgs {
  uint32_t* out;
  uint32_t flags;
  Rec* recs;  // 2 per work unit: [2u] = head portion, [2u+1] = tail portion (or nullptr)
  const uint32_t* tables;
  uint32_t* counter;  // the stream's done counter (fused variable kernel); zero between launches
  // Heads (kGeneral): hc[i] = the raw register of buffer i's partial first
  // chunk when the buffer has more chunks, written by crc32c_head_kernel
  // before the body kernel runs (only read for such buffers); nullptr when no
  // buffer of the batch has one.
  uint32_t* hc;
  // Variable-length batches: nonzero when some buffer has more than
  // kBufsMaxJ chunks (set by the plan kernels); zero lets the body kernel use
  // the buffer scheduler (no split buffers).  nullptr: unknown.
  const uint32_t* long_bufs = nullptr;
  // Variable-length plan, written by the head kernel (tile_scan) and read by
  // the body kernel (tiled_plan).  Tile b = buffers [S*b, min(n, S*b + S)):
  // lpre[i] = the tile-local exclusive prefix of the chunk counts,
  // tiles[2b] = the tile's chunk total, tiles[2b+1] = its largest count.
  uint64_t* lpre = nullptr;
  uint64_t* tiles = nullptr;
  uint64_t tile_S = 0;  // buffers per tile
  uint32_t tile_G = 0;  // tiles (the head kernel's workgroups)
  // Head kernel: nonzero allows short mode (every buffer finished in the
  // head kernel, no body kernel) -- for a fixed batch the host's decision,
  // for a tiled variable batch per tile, from its scan.
  uint32_t short_ok = 0;
  // Chunk-parallel aligned batches (crc32c_chunks_kernel): the raw register
  // of every 4 KiB chunk, folded per buffer by crc32c_fold_kernel.
  uint32_t* raws = nullptr;
  // Routed batches (crc32c_route_kernel, crc32c_var_fused_kernel): the plan.
  Route route{};
};

// Inclusive sum over the wave by DPP (row_shr 1/2/4/8, row_bcast 15/31): lane 63 holds the total.
__device__ __forceinline__ uint32_t add_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15 into rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31 into rows 2, 3
  return x;
}

// The wave's total of a u64 whose per-lane values are < 2^43, in two DPP sums
// (bits 20.. and 0..19: each total fits 32 bits).
__device__ __forceinline__ uint64_t wave_total_u64(uint64_t v) {
  const uint32_t h = add_scan((uint32_t)(v >> 20)), l = add_scan((uint32_t)v & 0xFFFFFu);
  return ((uint64_t)lane_u32(h, 63u) << 20) + lane_u32(l, 63u);
}


// The verdict, as every launch after the plan takes it: the partials (lane
// k < np loads slice k's), ballots of their flags and a sum of their
// lengths; a sorted batch's span is [offsets[0], offsets[n-1] + lengths[n-1]).
// lo / hi: the span (dyn).  Region-shaped: the region path.  Otherwise, when
// every buffer is exactly 4096 bytes (pages of a block cache, a shuffled
// batch of 4 KiB blocks, blocks far apart), the page path; else the head +
// body kernels.
__device__ __forceinline__ bool route_region(const Route& r, uint64_t& lo, uint64_t& hi) {
  const int lane = (int)(threadIdx.x & 63u);
  // lane k takes partials k, k + 64, ... (np <= kRoutePlanMax; the loads together, clamped)
  RoutePart q[kRoutePlanMax / 64u];
#pragma unroll
  for (uint32_t m = 0; m < kRoutePlanMax / 64u; ++m)
    q[m] = (m == 0u || 64u * m < r.np) ? r.parts[min(64u * m + (uint32_t)lane, r.np - 1u)] : RoutePart{0u, 0u};
  lo = ldc(r.offsets, 0);
  hi = ldc(r.offsets, r.n - 1u) + ldc(r.lengths, r.n - 1u);
  bool bad = false, some = false;
  uint64_t lsum = 0;
#pragma unroll
  for (uint32_t m = 0; m < kRoutePlanMax / 64u; ++m) {
    const bool mine = 64u * m + (uint32_t)lane < r.np;
    bad |= mine && (q[m].bad & kRpBad) != 0u;
    some |= mine && q[m].sum != 0u;
    lsum += mine ? q[m].sum : 0u;
  }
  if (__ballot(bad)) return false;
  if (!__ballot(some)) return false;  // nothing to checksum
  if (!r.dyn) return true;
  const uint64_t sum = wave_total_u64(lsum);
  // sorted and non-overlapping: hi - lo >= sum; gaps at most 1/8 of the bytes (+64 KiB)
  if (hi - lo - sum > sum / 8u + 65536u) return false;
  const uintptr_t O = ((uintptr_t)r.base + lo) & ~(uintptr_t)(kChunk - 1u);
  return ((uintptr_t)r.base + hi - O + kChunk - 1u) / kChunk <= r.cap_chunks;
}
// Not region-shaped: the page path (kRoutePages / kRoutePagesAligned) or the
// head + body kernels (kRouteHeads), from the partials' flags.
__device__ __forceinline__ int route_other(const Route& r) {
  const int lane = (int)(threadIdx.x & 63u);
  uint64_t fl = 0;
#pragma unroll
  for (uint32_t m = 0; m < kRoutePlanMax / 64u; ++m)
    if (m == 0u || 64u * m < r.np) fl |= 64u * m + (uint32_t)lane < r.np ? r.parts[min(64u * m + (uint32_t)lane, r.np - 1u)].bad : 0u;
  if (__ballot((fl & kRpNot4k) != 0u)) return kRouteHeads;
  return __ballot((fl & kRpUnaligned) != 0u) ? kRoutePages : kRoutePagesAligned;
}


// floor(a / d) for wave-uniform a < 2^63, d > 0, from a double-precision
// estimate (inv_d = 1/d, loop-invariant) corrected by a step or two: the
// integer 64-bit division is a ~100-instruction software sequence, and the
// general loops ran several per work unit (3.6x the aligned kernel's scalar
// instructions, PMC SQ_INSTS_SALU).
__device__ __forceinline__ uint64_t udiv_est(uint64_t a, uint64_t d, double inv_d) {
  uint64_t q = (uint64_t)((double)a * inv_d);
  while (q > 0 && q * d > a) --q;
  while ((q + 1) * d <= a) ++q;
  return q;
}
// The same with a shift when d is a power of two (the grid's unit count on
// a 256-CU part, the chunk count of power-of-two buffers): no VALU at all.
__device__ __forceinline__ uint64_t udiv_u(uint64_t a, uint64_t d) {
  if ((d & (d - 1u)) == 0u) return a >> __builtin_ctzll(d);
  return udiv_est(a, d, 1.0 / (double)d);
}

// Global work units: the grid's NU = gridDim.x * kUnitsPerWG units split the
// chunk space [0, T) evenly; workgroup b owns units [64b, 64b+64).
// F: the estimate-based division (general kernels); the aligned kernel keeps
// the integer one, whose code needs no vector registers (with the estimate's
// double arithmetic in its loop it spilled 23 VGPRs).
template <bool F>
__device__ __forceinline__ uint64_t global_unit_lo(uint64_t T, uint32_t u) {
  const uint64_t nu = (uint64_t)gridDim.x * kUnitsPerWG;
  if constexpr (F) return udiv_u(T * (uint64_t)u, nu);
  else return T * (uint64_t)u / nu;
}
__device__ __forceinline__ void global_put_recs(const KArgs& ka, uint32_t u, const Rec& h, const Rec& t) {
  if (ka.recs) {
    ka.recs[2 * (uint64_t)u] = h;
    ka.recs[2 * (uint64_t)u + 1] = t;
  }
}

struct FixedGeom {
  static constexpr bool kTiled = false;  // no plan: chunk positions are arithmetic
  const uint8_t* base;
  uint64_t stride, len, n;
  uint32_t J;
  const uint32_t* init;
  uint32_t init_all;
  __device__ __forceinline__ uint64_t total() const { return n * (uint64_t)J; }
  // long_heads' raw metadata (offset from base_addr(), length) of buffer i
  __device__ __forceinline__ uint64_t offsets_at(uint64_t i) const { return i * stride; }
  __device__ __forceinline__ uint64_t lengths_at(uint64_t) const { return len; }
  __device__ __forceinline__ uint32_t lengths_lo(uint64_t) const { return (uint32_t)len; }
  // buffer i's offset from base_addr(), length's low word and ~init, wave-uniform (scalar loads)
  __device__ __forceinline__ void meta_s(uint64_t i, uint64_t& o, uint32_t& Llo, uint32_t& s) const {
    o = i * stride;
    Llo = (uint32_t)len;
    s = ~(init ? ldc(init, i) : init_all);
  }
  __device__ __forceinline__ uintptr_t base_addr() const { return (uintptr_t)base; }
  template <bool F = false>
  __device__ __forceinline__ void locate(uint64_t t, uint64_t& i, uint32_t& c) const {
    if constexpr (F) i = udiv_u(t, J);
    else i = t / J;
    c = (uint32_t)(t - i * J);
  }
  __device__ __forceinline__ BufInfo info(uint64_t i) const {
    const uint32_t ini = init ? ldc(init, i) : init_all;
    return BufInfo{base + i * stride, len, J, ~ini};
  }
  template <bool F>
  __device__ __forceinline__ void locate_unit(uint32_t, uint64_t t, uint64_t& i, uint32_t& c) const {
    locate<F>(t, i, c);
  }
  // Buffer i's start, length and ~init in this lane (head kernel).
  __device__ __forceinline__ void lane_meta(uint64_t i, uintptr_t& p, uint64_t& L, uint32_t& sx) const {
    p = (uintptr_t)(base + i * stride);
    L = len;
    sx = ~(init ? init[i] : init_all);
  }
  template <bool F>
  __device__ __forceinline__ uint64_t unit_lo(uint64_t T, uint32_t u) const { return global_unit_lo<F>(T, u); }
  __device__ __forceinline__ void put_recs(const KArgs& ka, uint8_t*, uint32_t u, const Rec& h, const Rec& t) const {
    global_put_recs(ka, u, h, t);
  }
};

// The J 4096-byte chunks of n aligned buffers (16-B aligned base and stride,
// len = 4096 J) as n*J independent one-chunk "buffers" for scheduler A:
// chunk t = buffer t / J, chunk t % J; only chunk 0 carries the buffer's
// ~init.  Scheduler B walked a buffer's chunks through a serial
// acc = shift4096(acc) ^ raw chain and ran ~10 % behind config 2's rate on
// config 4 (5000 x 2 MiB); here every chunk is an independent pass whose raw
// register goes to KArgs::raws, and crc32c_fold_kernel combines each
// buffer's J raws (log-depth, ~0.1 % of the traffic).
struct ChunkGeom {
  static constexpr bool kTiled = false;
  const uint8_t* base;
  uint64_t stride, n;  // n: chunks (buffers * J)
  uint32_t J, jsh;     // jsh = log2(J) when J is a power of two, else 64
  const uint32_t* init;
  uint32_t init_all;
  __device__ __forceinline__ BufInfo info(uint64_t t) const {
    uint64_t i, c;
    if (jsh < 64u) {
      i = t >> jsh;
      c = t & (uint64_t)(J - 1u);
    } else {
      i = udiv_u(t, J);
      c = t - i * J;
    }
    const uint32_t s = c == 0 ? ~(init ? ldc(init, i) : init_all) : 0u;
    return BufInfo{base + i * stride + c * kChunk, kChunk, 1u, s};
  }
};

struct VarGeom {
  static constexpr bool kTiled = true;  // the head kernel writes the plan's tiles
  const uint8_t* base;
  const uint64_t* offsets;
  const uint64_t* lengths;
  const uint64_t* chunk_start;  // n+1 entries, exclusive prefix of J_i
  const uint64_t* unit_first;   // per work unit: the buffer holding its first chunk
  uint64_t n;
  const uint32_t* init;
  uint32_t init_all;
  __device__ __forceinline__ uint64_t total() const { return ldc(chunk_start, n); }
  __device__ __forceinline__ uint64_t offsets_at(uint64_t i) const { return offsets[i]; }
  __device__ __forceinline__ uint64_t lengths_at(uint64_t i) const { return lengths[i]; }
  __device__ __forceinline__ uint32_t lengths_lo(uint64_t i) const {  // (little-endian low word)
    return reinterpret_cast<const uint32_t*>(lengths)[2 * i];
  }
  __device__ __forceinline__ void meta_s(uint64_t i, uint64_t& o, uint32_t& Llo, uint32_t& s) const {
    o = ldc(offsets, i);
    Llo = ldc(reinterpret_cast<const uint32_t*>(lengths), 2 * i);
    s = ~(init ? ldc(init, i) : init_all);
  }
  __device__ __forceinline__ uintptr_t base_addr() const { return (uintptr_t)base; }
  __device__ __forceinline__ void locate(uint64_t t, uint64_t& i, uint32_t& c) const {
    uint64_t lo = 0, hi = n;  // invariant: chunk_start[lo] <= t < chunk_start[hi]
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (chunk_start[mid] <= t) lo = mid; else hi = mid;
    }
    i = lo;
    c = (uint32_t)(t - chunk_start[lo]);
  }
  // Start of work unit u (chunk t = its first): one load instead of a search.
  template <bool F>
  __device__ __forceinline__ void locate_unit(uint32_t u, uint64_t t, uint64_t& i, uint32_t& c) const {
    i = ldc(unit_first, u);
    c = (uint32_t)(t - ldc(chunk_start, i));
  }
  __device__ __forceinline__ BufInfo info(uint64_t i) const {
    const uint64_t L = ldc(lengths, i);
    const uint32_t ini = init ? ldc(init, i) : init_all;
    return BufInfo{base + ldc(offsets, i), L, chunks_for(L), ~ini};
  }
  __device__ __forceinline__ void lane_meta(uint64_t i, uintptr_t& p, uint64_t& L, uint32_t& sx) const {
    p = (uintptr_t)(base + offsets[i]);
    L = lengths[i];
    sx = ~(init ? init[i] : init_all);
  }
  template <bool F>
  __device__ __forceinline__ uint64_t unit_lo(uint64_t T, uint32_t u) const { return global_unit_lo<F>(T, u); }
  __device__ __forceinline__ void put_recs(const KArgs& ka, uint8_t*, uint32_t u, const Rec& h, const Rec& t) const {
    global_put_recs(ka, u, h, t);
  }
};

// Load modes: kAligned = 16-B aligned buffer whose length is a multiple of 4096
// (every chunk full, no masking: configs 2, 4, 5); kGeneral = the full
// 4096-byte chunks of buffers of any alignment and length (realignment).
// Partial first chunks (heads) never reach these kernels: crc32c_head_kernel
// runs them, so the body kernels' registers never hold masking code -- except
// kMasked: fixed-stride batches of one 1025..4095-byte chunk per buffer, run
// as long heads (load_general / realign_general with hd, page_head_words)
// under scheduler A.
enum LoadMode : int { kAligned = 0, kGeneral = 1, kMasked = 2 };

// Bytes of a buffer's first chunk (END-aligned chunks: the only short one).
__host__ __device__ __forceinline__ uint32_t head_bytes(uint64_t L, uint32_t J) {
  return (uint32_t)(L - (uint64_t)kChunk * (J - 1u));
}

// A buffer's first chunk is a head chunk when it starts before the buffer
// (partial: 1..4095 bytes) or the buffer is shorter than 4 bytes (bytewise).
__host__ __device__ __forceinline__ bool head_first(uint64_t L) {
  return L < 4 || L - (uint64_t)kChunk * (chunks_for(L) - 1u) < kChunk;
}

// Registers of one chunk as loaded.  Load j (j = 0..3) is one coalesced 1 KiB
// wave load of chunk bytes [1024j, 1024j+1024) in a permuted lane order: lane
// (a, b) = (lane >> 4, lane & 15) takes the 16 B at 1024j + 64b + 16a, so that
// the 4x4 exchange across 16-lane rows in row_transpose leaves lane P holding
// the 64 contiguous bytes [64P, 64P+64) -- piece P = lane.  In kGeneral the
// loads start at the 4-byte aligned address A4 below the chunk start (gfx950
// serves 4-B aligned dwordx4 at the 16-B aligned rate, byte-misaligned ones at
// ~2/3: tools/diag/ldpat.hip, profiles/r02_ldpat.jsonl).  e[] is one more
// 16-byte load by two lanes: lane 63 reads the 16 bytes ending at A4 + 4100
// (e[3] = the dword just past the last piece), lane 0 the 16 bytes before A4
// on a chunk with an overhang.  Vector loads, not scalar ones: an s_load in
// flight would make every LDS wait of the chains wait for it too (both count
// in lgkmcnt, and scalar loads return out of order).
struct Chunk {
  uint32_t d[16];
  uint32_t e[4];
};

__device__ __forceinline__ uintptr_t chunk_end(const BufInfo& bi, uint32_t c) {
  return (uintptr_t)bi.p + bi.len - (uint64_t)kChunk * (bi.J - 1u - c);
}

// Byte offset of the lane's 16 B within each 1 KiB load.
__device__ __forceinline__ uint32_t lane_load_off(int lane) {
  return ((uint32_t)(lane & 15) << 6) | ((uint32_t)(lane >> 4) << 4);
}

// kGeneral chunk loads, chunk [cs, ce) with cs = ce - 4096: four row loads
// and the edge granule.
//   body chunk (hd false: cs >= p): rows from A4 = cs rounded down to 4 B
//     (gfx950 serves 4-B aligned dwordx4 at the 16-B aligned rate,
//     byte-misaligned at ~2/3: tools/diag/ldpat.hip); A4 >= floor4(p) >= g.
//   head chunk (hd: crc32c_head_kernel's long heads, kMasked passes, cs < p):
//     rows from A4 as well; a row slot wholly below p's granule g is loaded
//     from g instead (its bytes precede the buffer and are masked).  The slot
//     straddling g reads up to 12 bytes below g, inside g's 4 KiB page --
//     unless g is the page's first granule: then it is loaded from g too and
//     page_head_words moves its words into place (kMasked; the head kernel
//     sends such heads to lane-group rounds instead).
// The edge load is the dword holding byte ce - 1 (lane 63's dword past its
// row data when the body rows start below cs).  Fault safety: only 16-B
// granules that hold buffer bytes are touched (tests/kernel_model.py).  The
// same five loads either way, and no branch around them, so the wait counts
// stay exact.
__device__ __forceinline__ void load_general(uintptr_t ce, bool hd, uintptr_t p, int lane, Chunk& ch) {
  const uintptr_t cs = ce - kChunk;
  const uint32_t lo = lane_load_off(lane);
  uintptr_t a[4];
  if (hd) {
    const uintptr_t A4 = cs & ~(uintptr_t)3, g = p & ~(uintptr_t)15;
    const uintptr_t gl = (g & 4095u) ? g - 15u : g;  // below gl: loaded from g
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uintptr_t x = A4 + 1024u * (uint32_t)j + lo;
      a[j] = x < gl ? g : x;
    }
  } else {
    const uintptr_t A4 = cs & ~(uintptr_t)3;
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = A4 + 1024u * (uint32_t)j + lo;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const u32x4 v = ld16(a[j]);
    ch.d[4 * j + 0] = v.x; ch.d[4 * j + 1] = v.y; ch.d[4 * j + 2] = v.z; ch.d[4 * j + 3] = v.w;
  }
  ch.e[3] = *(const __attribute__((address_space(1))) uint32_t*)((ce - 1u) & ~(uintptr_t)3);
}

// A kMasked pass whose buffer starts in a page's first granule g: the row
// slot straddling g was loaded from g (load_general), so its words move up by
// q = (g - x) / 4 dwords to sit at their chunk positions (the words below g
// precede the buffer: head_fix zeroes them).  Wave-uniform branch, taken by
// ~1/256 of random starts.
__device__ __forceinline__ void page_head_words(uintptr_t ce, uintptr_t p, int lane, uint32_t (&w)[16]) {
  const uintptr_t g = p & ~(uintptr_t)15;
  if (g & 4095u) return;
  const uintptr_t A4 = (ce - kChunk) & ~(uintptr_t)3;
  const uint32_t lo = lane_load_off(lane);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uintptr_t x = A4 + 1024u * (uint32_t)j + lo;
    const bool st = x < g && x + 16u > g;
    const uint32_t q = (uint32_t)(g - x) >> 2;  // 1..3 when st
    const uint32_t x0 = w[4 * j], x1 = w[4 * j + 1], x2 = w[4 * j + 2];
    if (st) {
      w[4 * j + 3] = q == 1u ? x2 : (q == 2u ? x1 : x0);
      w[4 * j + 2] = q == 1u ? x1 : x0;
      w[4 * j + 1] = x0;
    }
  }
}

template <int M>
__device__ __forceinline__ void load_chunk(const BufInfo& bi, uint32_t c, int lane, Chunk& ch) {
  const uintptr_t ce = chunk_end(bi, c);
  const uint32_t lo = lane_load_off(lane);
  if constexpr (M == kAligned) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32x4 v = ld16(ce - kChunk + 1024u * (uint32_t)j + lo);
      ch.d[4 * j + 0] = v.x; ch.d[4 * j + 1] = v.y; ch.d[4 * j + 2] = v.z; ch.d[4 * j + 3] = v.w;
    }
  } else {
    load_general(ce, M == kMasked, (uintptr_t)bi.p, lane, ch);
  }
}

// 4x4 transpose of 16-byte slots across the four 16-lane rows: slot j of lane
// (a, b) <- slot a of lane (j, b).  Two v_permlane32_swap + two
// v_permlane16_swap per dword column (16 VALU per chunk), no temporaries.
__device__ __forceinline__ void row_transpose(uint32_t (&d)[16]) {
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const auto r02 = __builtin_amdgcn_permlane32_swap(d[x], d[8 + x], false, false);
    const auto r13 = __builtin_amdgcn_permlane32_swap(d[4 + x], d[12 + x], false, false);
    const auto q01 = __builtin_amdgcn_permlane16_swap(r02[0], r13[0], false, false);
    const auto q23 = __builtin_amdgcn_permlane16_swap(r02[1], r13[1], false, false);
    d[x] = q01[0];
    d[4 + x] = q01[1];
    d[8 + x] = q23[0];
    d[12 + x] = q23[1];
  }
}

// Next lane's dword (DPP wave_shl:1); lane 63 gets `last`.
__device__ __forceinline__ uint32_t next_lane(uint32_t v, uint32_t last) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)last, (int)v, 0x130, 0xF, 0xF, false);
}
// Previous lane's dword (DPP wave_shr:1); lane 0 gets 0.
__device__ __forceinline__ uint32_t prev_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
}

// Zero the bytes of a piece before the buffer start and XOR ~init (s) into the
// 4 bytes at it: rel = bytes of the piece before the start.  Words below
// zk = clamp(rel)/4 are zeroed, word zk keeps its bytes from the start on
// (pm), and s lands as s << 8b in word kk = floor(rel/4) and s >> (32-8b) in
// word kk+1 (b = rel & 3); four per-lane values, two compares per word.
template <int NW>
__device__ __forceinline__ void mask_inject(uint32_t (&w)[NW], int rel, uint32_t s) {
  const int z = min(max(rel, 0), 4 * NW);
  const int zk = z >> 2;
  const uint32_t pm = ~0u << (8u * (uint32_t)(z & 3));
  const int kk = rel >> 2;  // arithmetic: rel in [-3, -1] -> -1
  const uint32_t b = (uint32_t)rel & 3u;
  const uint32_t lo = s << (8u * b);
  const uint32_t hi = b ? s >> (32u - 8u * b) : 0u;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    uint32_t x = k < zk ? 0u : (k == zk ? w[k] & pm : w[k]);
    x ^= k == kk ? lo : (k == kk + 1 ? hi : 0u);
    w[k] = x;
  }
}

// Head chunk masking: rel = p - cs bytes of the chunk precede the buffer
// (wave-uniform, 1 <= rel < 4096 - 1024), i.e. piece lp = rel / 64 holds the
// buffer start at its word kp, byte bp.  Lanes below lp and lp's words before
// kp are zeroed (leading zeros leave a zero register unchanged), word kp keeps
// its bytes from p on and takes ~init << 8bp, the next word ~init's rest.
// The two words at the uniform index kp are read and written through a
// vector with a uniform dynamic index (v_movrels / v_movreld): per-word
// uniform branches cost ~25 % of a long-head pass, and a switch whose cases
// rewrite many words made the compiler copy the whole array at every join.
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ void head_fix(uint32_t (&w)[16], uint32_t rel, uint32_t s, int lane) {
  const uint32_t lp = rel >> 6, kp = (rel >> 2) & 15u, bp = rel & 3u;
  const bool me = (uint32_t)lane == lp;
  const bool below = (uint32_t)lane < lp;
  const uint32_t pm = ~0u << (8u * bp), lo = s << (8u * bp), hi = bp ? s >> (32u - 8u * bp) : 0u;
  u32x16 v;
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = (below || (me && (uint32_t)k < kp)) ? 0u : w[k];
  const uint32_t x = v[kp];
  v[kp] = me ? ((x & pm) ^ lo) : x;
  const uint32_t k1 = kp < 15u ? kp + 1u : 0u;  // kp == 15: ~init's rest goes to lane lp + 1's word 0
  const bool me1 = kp < 15u ? me : (uint32_t)lane == lp + 1u;
  const uint32_t y = v[k1];
  v[k1] = me1 ? y ^ hi : y;
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = v[k];
}

// kGeneral words after the transpose (see load_general): lane P holds the 64
// bytes from the row base + 64P.
//   shift left by r = cs & 3 bytes (lane P's bytes continue in lane P+1,
//   lane 63's in the edge dword); then
//   body chunk: ~init goes into lane 0's first word when the chunk starts
//     0..3 bytes after the buffer start (a short head holds those bytes);
//   head chunk: head_fix.
__device__ __forceinline__ void realign_general(uintptr_t ce, bool hd, uintptr_t p, uint32_t s, int lane,
                                                const Chunk& ch, uint32_t (&w)[16]) {
  const uintptr_t cs = ce - kChunk;
  // (Unconditional -- alignbyte by 0 keeps the low word -- spares the
  // compiler's register copies at the join but measured slower: scheduler C
  // 10^5 x 4097 B 85.5 -> 91.5 us, config 3 223 -> 235 us, same box.)
  const uint32_t r = (uint32_t)(cs & 3u);
  if (r != 0) {
    const uint32_t nx = next_lane(w[0], ch.e[3]);
#pragma unroll
    for (int k = 0; k < 15; ++k) w[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], r);
    w[15] = __builtin_amdgcn_alignbyte(nx, w[15], r);
  }
  if (!hd) {
    if (cs < p + 4 && lane == 0) w[0] ^= s >> (8u * (uint32_t)(cs - p));
  } else {
    head_fix(w, (uint32_t)(p - cs), s, lane);
  }
}

// The lane's 16 words of piece P = lane (64 contiguous bytes), with the ~init
// injection.
template <int M>
__device__ __forceinline__ void build_words(const BufInfo& bi, uint32_t c, int lane, const Chunk& ch,
                                            uint32_t (&w)[16], uint32_t (&ov)[4]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = ch.d[k];
  if constexpr (M == kMasked) page_head_words(chunk_end(bi, c), (uintptr_t)bi.p, lane, w);
  row_transpose(w);
  if constexpr (M == kAligned) {
    if (c == 0 && lane == 0) w[0] ^= bi.s;  // chunk position 0 is lane 0, word 0
  } else {
    (void)ov;
    realign_general(chunk_end(bi, c), M == kMasked, (uintptr_t)bi.p, bi.s, lane, ch, w);
  }
}

// Serial slice-by-4 chains + butterflies of U chunks from their built words,
// interleaved so each wave keeps U independent LDS round trips in flight.
// OPQ: recompute the per-lane butterfly bases at each use.  Every kernel now
// keeps them hoisted (OPQ = false): since the general kernels stopped
// spilling, hoisting costs no spill there and saves 22 us on config 3
// (306 -> 285 us, same-box A/B).
// The region kernel's LDS image: no butterfly tables.  Each lane moves its
// piece raw to the chunk end by its OWN constant, x^(8*64*(63 - lane)), from
// nibble tables T[n][v][lane] = shift(v << 4n, 64(63 - lane)) (8 x 16 rows of
// 64 lanes: a lane reads only its own column, conflict-free); the chunk raw
// and every lane prefix are then plain XORs over lanes (xor_scan, DPP).
// Lane 63 (identity) never reads its column, whose first slot holds the
// workgroup's unit counter.  The slice replicas follow at 32 KiB.
constexpr uint32_t kRNibOff = 0;
constexpr uint32_t kRCtrOff = 252;  // T[0][0][63]
constexpr uint32_t kRSliceOff = 32768;
constexpr uint32_t kRLdsBytes = kRSliceOff + kRepBytes;  // 163840 B
static_assert(kRLdsBytes <= 160u * 1024u, "region LDS image exceeds 160 KiB");
constexpr uint32_t kGNib = kTabNib;  // the blob's nibble tables (crc32c_internal.h)

// The region image: slice replicas at kRSliceOff, nibble tables verbatim,
// the unit counter patched into its slot by the thread that copies it.  In
// two halves so that the blob loads are in flight together with the waves'
// first searches (a fill after the search waited for both in turn: 6 us to
// the first barrier).
struct RegionFill {
  uint32_t rep[8192 / kThreads];
  uint4 nib[2048 / kThreads];
};
__device__ __forceinline__ RegionFill fill_region_load(const uint32_t* __restrict__ g) {
  RegionFill f;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < (int)(8192 / kThreads); ++q) {
    const uint32_t off = (uint32_t)(t + q * (int)kThreads) << 4;
    const uint32_t tab = ((off >> 16) << 1) | ((off >> 7) & 1u);
    f.rep[q] = g[kGSlice + tab * 256u + ((off >> 8) & 0xFFu)];
  }
  const uint4* src = reinterpret_cast<const uint4*>(g + kGNib);
#pragma unroll
  for (int q = 0; q < (int)(2048 / kThreads); ++q) f.nib[q] = src[t + q * (int)kThreads];
  return f;
}
__device__ __forceinline__ void fill_region_store(uint8_t* lds, const RegionFill& f, uint32_t ctr0) {
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < (int)(8192 / kThreads); ++q) {
    const uint32_t off = (uint32_t)(t + q * (int)kThreads) << 4;
    *reinterpret_cast<uint4*>(lds + kRSliceOff + off) = make_uint4(f.rep[q], f.rep[q], f.rep[q], f.rep[q]);
  }
  uint4* dst = reinterpret_cast<uint4*>(lds + kRNibOff);
#pragma unroll
  for (int q = 0; q < (int)(2048 / kThreads); ++q) {
    uint4 v = f.nib[q];
    if (t + q * (int)kThreads == (int)(kRCtrOff >> 4)) v.w = ctr0;  // units 0..ctr0-1 are pre-assigned
    dst[t + q * (int)kThreads] = v;
  }
}
static_assert(8192 % kThreads == 0 && 2048 % kThreads == 0, "region fill: whole rounds per thread");

// shift(lr, 64(63 - lane)): this lane's piece raw moved to the chunk end.
// Address of row (n, v): v << 8 | lane << 2 -- v_perm puts the nibble byte
// over the lane byte; n is the ds_read immediate.
__device__ __forceinline__ uint32_t to_chunk_end(const uint8_t* lds, uint32_t lr, uint32_t jb, int lane) {
  const uint32_t lo = lr & 0x0F0F0F0Fu, hi = (lr >> 4) & 0x0F0F0F0Fu;
  const uint8_t* nb = lds + kRNibOff;
  const uint32_t r0 = lds_u32(nb + 0u * 4096u, __builtin_amdgcn_perm(lo, jb, 0x0C0C0400u));
  const uint32_t r1 = lds_u32(nb + 1u * 4096u, __builtin_amdgcn_perm(hi, jb, 0x0C0C0400u));
  const uint32_t r2 = lds_u32(nb + 2u * 4096u, __builtin_amdgcn_perm(lo, jb, 0x0C0C0500u));
  const uint32_t r3 = lds_u32(nb + 3u * 4096u, __builtin_amdgcn_perm(hi, jb, 0x0C0C0500u));
  const uint32_t r4 = lds_u32(nb + 4u * 4096u, __builtin_amdgcn_perm(lo, jb, 0x0C0C0600u));
  const uint32_t r5 = lds_u32(nb + 5u * 4096u, __builtin_amdgcn_perm(hi, jb, 0x0C0C0600u));
  const uint32_t r6 = lds_u32(nb + 6u * 4096u, __builtin_amdgcn_perm(lo, jb, 0x0C0C0700u));
  const uint32_t r7 = lds_u32(nb + 7u * 4096u, __builtin_amdgcn_perm(hi, jb, 0x0C0C0700u));
  const uint32_t t = xor3(xor3(r0, r1, r2), xor3(r3, r4, r5), r6) ^ r7;
  return lane == 63 ? lr : t;
}

// Inclusive XOR scan over the wave's 64 lanes (rows of 16 by row_shr, then
// row_bcast:15 / :31 across rows).
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_or0(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xF, false);
}
__device__ __forceinline__ uint32_t xor_scan(uint32_t x) {
  x ^= dpp_or0<0x111, 0xF>(x);  // row_shr:1
  x ^= dpp_or0<0x112, 0xF>(x);  // row_shr:2
  x ^= dpp_or0<0x114, 0xF>(x);  // row_shr:4
  x ^= dpp_or0<0x118, 0xF>(x);  // row_shr:8
  x ^= dpp_or0<0x142, 0xA>(x);  // row_bcast:15 into rows 1, 3
  x ^= dpp_or0<0x143, 0xC>(x);  // row_bcast:31 into rows 2, 3
  return x;
}

// NIB: the region LDS image (slice replicas at kRSliceOff, nibble tables at
// 0): each lane's piece raw moved to the chunk end by its own nibble-table
// column and XOR-reduced over the wave (to_chunk_end + xor_scan) instead of
// the byte-sliced butterfly -- fewer VALU per chunk.
template <int U, bool OPQ, bool NIB = false>
__device__ __forceinline__ void chains(const uint8_t* lds, const LaneBase& lb, const uint32_t (&w)[U][16], int lane,
                                       uint32_t (&raw)[U]) {
  uint32_t crc[U];
  const uint8_t* sl = NIB ? lds + (kRSliceOff - kSliceOff) : lds;
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = w[u][0];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
#pragma unroll
    for (int u = 0; u < U; ++u) crc[u] = slice4_next(sl, crc[u], k < 15 ? w[u][k + 1] : 0u, lb);
  }
  if constexpr (NIB) {
    const uint32_t jb = (uint32_t)lane << 2;
#pragma unroll
    for (int u = 0; u < U; ++u) raw[u] = lane_u32(xor_scan(to_chunk_end(lds, crc[u], jb, lane)), 63u);
    return;
  }
  // Lane = stream position P: lane bit k steps 64*2^k bytes (comb table k).
  // Bits 0 and 1 go first: afterwards the lanes of a quad hold equal values,
  // which fold_level's quad-spread byte lookups rely on.
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = fold_level<0, 0, OPQ>(lds, crc[u], lane);
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = fold_level<1, 1, OPQ>(lds, crc[u], lane);
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = fold_level<2, 2, OPQ>(lds, crc[u], lane);
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = fold_level<3, 3, OPQ>(lds, crc[u], lane);
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = fold_level<4, 4, OPQ>(lds, crc[u], lane);
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = fold_level<5, 5, OPQ>(lds, crc[u], lane);
#pragma unroll
  for (int u = 0; u < U; ++u) raw[u] = crc[u];
}

// Raw (zero-state, ~init injected) registers of U chunks, wave-uniform.
template <int M, int U, bool NIB = false>
__device__ __forceinline__ void group_raw(const uint8_t* lds, const LaneBase& lb, const BufInfo (&bi)[U],
                                          const uint32_t (&c)[U], int lane, const Chunk (&ch)[U],
                                          uint32_t (&raw)[U]) {
  uint32_t w[U][16], ov[4];
#pragma unroll
  for (int u = 0; u < U; ++u) build_words<M>(bi[u], c[u], lane, ch[u], w[u], ov);
  chains<U, false, NIB>(lds, lb, w, lane, raw);
}

// Chain + butterfly of one chunk from its built words.
template <int M>
__device__ __forceinline__ uint32_t chain_fold(const uint8_t* lds, const LaneBase& lb, const uint32_t (&w)[16],
                                               int lane) {
  uint32_t w1[1][16], r[1];
#pragma unroll
  for (int k = 0; k < 16; ++k) w1[0][k] = w[k];
  chains<1, false>(lds, lb, w1, lane, r);
  return r[0];
}

template <int M, bool NIB = false>
__device__ __forceinline__ uint32_t chunk_raw(const uint8_t* lds, const LaneBase& lb, const BufInfo& bi,
                                              uint32_t c, int lane, const Chunk& ch) {
  const BufInfo b1[1] = {bi};
  const uint32_t c1[1] = {c};
  const Chunk h1[1] = {ch};
  uint32_t r1[1];
  group_raw<M, 1, NIB>(lds, lb, b1, c1, lane, h1, r1);
  return r1[0];
}

// Position of one chunk.
struct Pos {
  uint64_t i;  // buffer
  uint32_t c;  // chunk within the buffer
  BufInfo bi;
};

template <bool F, class G>
__device__ __forceinline__ Pos unit_start_pos(const G& g, uint32_t u, uint64_t t) {
  Pos p;
  g.template locate_unit<F>(u, t, p.i, p.c);
  p.bi = g.info(p.i);
  return p;
}

template <class G>
__device__ __forceinline__ Pos next_pos(const G& g, const Pos& p) {
  Pos q = p;
  if (p.c + 1 == p.bi.J) {
    q.i = p.i + 1;
    q.c = 0;
    q.bi = g.info(q.i);
  } else {
    q.c = p.c + 1;
  }
  return q;
}

// Accumulation over the consecutive chunks of one work unit (wave-uniform).
struct UnitState {
  uint32_t acc, cnt;
  bool from_zero;
  Rec head;
};

// hx: the raw register of the buffer's head (its partial first chunk,
// prefetched from KArgs::hc) when this chunk is its first body chunk, else 0:
// the head then enters like a preceding chunk (shift(0) = 0 otherwise).
__device__ __forceinline__ void consume(UnitState& st, const Pos& p, uint32_t raw, const uint8_t* lds, int lane,
                                        const KArgs& ka, uint32_t hx = 0u) {
  st.acc = shift4096(lds, st.cnt ? st.acc : hx, lane) ^ raw;
  ++st.cnt;
  if (p.c + 1 == p.bi.J) {
    if (st.from_zero) {
      if (lane == 0) ka.out[p.i] = finish(~st.acc, ka.flags);
    } else {
      st.head = Rec{p.i, st.acc, st.cnt | kRecEnds};
    }
    st.cnt = 0;
    st.from_zero = true;
  }
}

// A portion's raw register normalized to the end of its buffer:
// shift(acc, 4096 * after), `after` = chunks of the buffer after the portion.
// Every record then combines by XOR alone (no serial walk of shifts in the
// fix-up).  Few chunks: `after` shift4096 lookups; more: the GF(2) power
// ladder over the x^(2^k) table.
__device__ __forceinline__ uint32_t normalize(const uint8_t* lds, const uint32_t* tables, uint32_t acc,
                                              uint32_t after, int lane) {
  if (after <= 24) {
    for (uint32_t k = 0; k < after; ++k) acc = shift4096(lds, acc, lane);
    return acc;
  }
  return nvl::shift_bytes(tables + kGX2n, acc, (uint64_t)after * kChunk);
}

__device__ __forceinline__ uint32_t pull_unit(uint8_t* lds, int lane, uint32_t ctr = kCtrOff) {
  uint32_t v = 0;
  if (lane == 0)
    v = __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(lds + ctr), 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
  return uniform_u32(v);
}

// Per-wave timeline hooks (NVL_STAMP0 / NVL_STAMP1 / NVL_COUNT /
// NVL_STAMP_END): no-ops here; tools/diag/stamps.h defines them for a
// diagnostic variant build (make variant VFLAGS="-include .../stamps.h").
#ifndef NVL_STAMP0
#define NVL_STAMP0() do {} while (0)
#define NVL_STAMP1() do {} while (0)
#define NVL_COUNT() do {} while (0)
#define NVL_STAMP_END() do {} while (0)
#endif
#ifndef NVL_TL_DECL  // phase timeline (same header): NVL_TL(k) at phase boundaries
#define NVL_TL_DECL() do {} while (0)
#define NVL_TL(k) do {} while (0)
#define NVL_TL_END() do {} while (0)
#endif
#ifndef NVL_TL_WAIT  // NVL_TL(k) once the wave's loads (and value v) are in
#define NVL_TL_WAIT(k, v) do {} while (0)
#endif

// ---------------------------------------------------------------------------
// Scheduler A -- fixed stride, aligned, J == 1 (every chunk a whole buffer;
// configs 2 and 5).  The workgroup owns a contiguous range of buffers and its
// 16 waves pull units of U buffers from an LDS counter, so fast and slow waves
// of a CU finish together (a static per-wave split left the last wave ~20 %
// behind the mean: older waves win issue arbitration).  U buffers per unit are
// computed with interleaved chains.
constexpr uint32_t kTail = 64;  // single-buffer units at the end of a range (tools/ab_bench.py: 64 > 32 > 96 > 16 > 0)

template <int U, int NW = kWavesPerWG, int M = kAligned, class G = FixedGeom, bool kRaw = false, bool NIB = false>
__device__ __forceinline__ void run_pairs(const G& g, const KArgs& ka, uint8_t* lds) {
  NVL_STAMP0();
  const int lane = threadIdx.x & 63;
  const uint32_t wv = uniform_u32(threadIdx.x >> 6);
  const uint64_t B0 = g.n * blockIdx.x / gridDim.x;
  const uint64_t B1 = g.n * (blockIdx.x + 1) / gridDim.x;
  // The range's last kTail buffers are single-buffer units: a CU's waves
  // then finish within half a unit of each other instead of a whole one.
  const uint32_t cnt = (uint32_t)(B1 - B0);
  const uint32_t nfull = cnt > kTail ? (cnt - kTail) / U : 0u;  // U-buffer units
  const uint32_t nunits = nfull + (cnt - nfull * U);

  auto unit_pos = [&](uint32_t u, int k, Pos& p) -> bool {
    const uint64_t i = u < nfull ? B0 + (uint64_t)u * U + (uint64_t)k : B0 + (uint64_t)nfull * U + (u - nfull);
    if (u >= nunits || (u >= nfull && k > 0)) return false;
    p.i = i;
    p.c = 0;
    p.bi = g.info(i);
    return true;
  };

  uint32_t u = wv;  // first unit pre-assigned; its loads overlap the LDS fill
  Pos gp[U];
  bool ok[U];
  Chunk cur[U];
  // The table blob's loads go out ahead of the first unit's chunk loads, so
  // the fill waits for them alone, not for the chunk burst queued in front
  // (config 2 interleaved A/B: 63.6-63.7 vs 64.0 us back to back,
  // profiles/r05b/ab_blobfirst.jsonl).
  RegionFill rf;
  LdsFill<NW> lf;
  if constexpr (NIB) rf = fill_region_load(ka.tables);
  else lf = fill_lds_load<NW>(ka.tables);
#pragma unroll
  for (int k = 0; k < U; ++k) {
    ok[k] = unit_pos(u, k, gp[k]);
    if (ok[k]) load_chunk<M>(gp[k].bi, 0, lane, cur[k]);
  }
  if constexpr (NIB) fill_region_store(lds, rf, NW);
  else fill_lds_store<NW>(lds, lf, NW);
  __syncthreads();
  const LaneBase lb = make_lane_base(lane);
  NVL_STAMP1();

  while (u < nunits) {
    NVL_COUNT();
    const uint32_t un = pull_unit(lds, lane, NIB ? kRCtrOff : kCtrOff);
    Pos np[U];
    bool nok[U];
    Chunk nxt[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      nok[k] = unit_pos(un, k, np[k]);
      if (nok[k]) load_chunk<M>(np[k].bi, 0, lane, nxt[k]);
    }
    if (ok[U - 1]) {  // full unit
      BufInfo bis[U];
      uint32_t cs[U], raws[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        bis[k] = gp[k].bi;
        cs[k] = 0;
      }
      group_raw<M, U, NIB>(lds, lb, bis, cs, lane, cur, raws);
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
          if constexpr (kRaw) ka.raws[gp[k].i] = raws[k];
          else ka.out[gp[k].i] = finish(~raws[k], ka.flags);
        }
      }
    } else {  // the range's ragged last unit
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (ok[k]) {
          const uint32_t r = chunk_raw<M, NIB>(lds, lb, gp[k].bi, 0, lane, cur[k]);
          if (lane == 0) {
            if constexpr (kRaw) ka.raws[gp[k].i] = r;
            else ka.out[gp[k].i] = finish(~r, ka.flags);
          }
        }
      }
    }
    u = un;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      gp[k] = np[k];
      ok[k] = nok[k];
      cur[k] = nxt[k];
    }
  }
  NVL_STAMP_END();
}

// ---------------------------------------------------------------------------
// Scheduler B -- everything else (any J, any alignment, variable lengths).
// The chunk space [0, T) is cut into NU = grid * kUnitsPerWG contiguous work
// units; workgroup b owns units [64b, 64b+64) and its waves pull them from an
// LDS counter.  A wave walks its unit's chunks in order, accumulating
// consecutive chunks of one buffer (acc = shift4096(acc) ^ raw); buffers
// completed inside the unit are written directly, and a buffer cut by a unit
// boundary leaves a head/tail record for crc32c_fixup_kernel.  The next
// chunk -- including the first chunk of the next unit -- is always in flight
// while the current one computes.
constexpr int kUnitStep = 1;         // chunks per step in scheduler B (2: interleaved pair; A/B'd, no gain)
constexpr int kUnitStepAligned = 2;  // the same for the aligned (kAligned, J > 1) kernel: no spills there (cfg4 -3 %)

template <int M, int NW, class G>
__device__ __forceinline__ void run_units(const G& g, const KArgs& ka, uint8_t* lds) {
  NVL_STAMP0();
  constexpr int kStep = M == kAligned ? kUnitStepAligned : kUnitStep;
  static_assert(M == kAligned || kStep == 1, "the kGeneral loop skips head chunks one step at a time");
  const int lane = threadIdx.x & 63;
  const uint32_t wv = uniform_u32(threadIdx.x >> 6);
  const uint64_t T = g.total();
  const uint32_t ub0 = blockIdx.x * kUnitsPerWG, ub1 = ub0 + kUnitsPerWG;
  constexpr bool kFastDiv = M != kAligned;
  auto lo_of = [&](uint32_t uu) -> uint64_t { return g.template unit_lo<kFastDiv>(T, uu); };
  // kGeneral: a head chunk (partial first chunk, or a buffer of < 4 bytes)
  // belongs to crc32c_head_kernel: the step that reaches one loads and
  // computes nothing; its raw register hc[i] is prefetched with the buffer's
  // first body chunk (hv) and shifted in ahead of it.
  auto skip = [&](const Pos& q) -> bool { return M == kGeneral && q.c == 0 && head_first(q.bi.len); };
  auto first_body = [&](const Pos& q) -> uint32_t { return (M == kGeneral && head_first(q.bi.len)) ? 1u : 0u; };
  auto hc_of = [&](const Pos& q) -> uint32_t {  // vector load, in vmcnt order behind the chunk's own loads
    if (M != kGeneral || !ka.hc || q.c != 1u || !head_first(q.bi.len)) return 0u;
    return __builtin_nontemporal_load((const __attribute__((address_space(1))) uint32_t*)(ka.hc + q.i));
  };

  // One flat loop over steps.  A step is the next two chunks of the current
  // unit u (one at an odd tail; none when u is empty), their chains
  // interleaved.  p0/p1 + c0/c1 hold the step's chunks, loaded while the
  // previous step computed; the next unit un is pulled ahead so the step that
  // ends a unit prefetches the next unit's first step.  Every chunk load of the
  // loop is issued from one place, so the loaded registers carry straight into
  // the next iteration (no copies that would wait on the loads).
  const LdsFill<NW> lf = fill_lds_load<NW>(ka.tables);  // ahead of the first chunk loads (run_pairs)
  uint32_t u = ub0 + wv;
  uint64_t t = lo_of(u), t1 = lo_of(u + 1);
  Pos p0{}, p1{};
  Chunk c0, c1;
  uint32_t hv0 = 0u;
  if (t < t1) {  // the first step's loads overlap the LDS fill
    p0 = unit_start_pos<kFastDiv>(g, u, t);
    if (!skip(p0)) load_chunk<M>(p0.bi, p0.c, lane, c0);
    hv0 = hc_of(p0);
    if (kStep == 2 && t + 1 < t1) {
      p1 = next_pos(g, p0);
      load_chunk<M>(p1.bi, p1.c, lane, c1);
    }
  }
  fill_lds_store<NW>(lds, lf);
  __syncthreads();
  const LaneBase lb = make_lane_base(lane);
  NVL_STAMP1();

  uint32_t un = ub0 + pull_unit(lds, lane);
  uint64_t un_lo = un < ub1 ? lo_of(un) : 0, un_hi = un < ub1 ? lo_of(un + 1) : 0;
  UnitState st{0u, 0u, p0.c <= first_body(p0), Rec{kNoBuf, 0u, 0u}};
  Rec tail{kNoBuf, 0u, 0u};
  while (true) {
    const bool cur = t < t1;
    const bool two = kStep == 2 && t + 1 < t1;
    const uint64_t tn = cur ? t + (two ? 2u : 1u) : t;
    const bool unit_ends = tn == t1;
    Pos q0 = p0, q1 = p0;
    bool q0v = false, q1v = false;
    if (!unit_ends) {
      q0 = two ? next_pos(g, p1) : next_pos(g, p0);
      q0v = true;
      if (kStep == 2 && tn + 1 < t1) {
        q1 = next_pos(g, q0);
        q1v = true;
      }
    } else if (un_lo < un_hi) {  // the next unit's first step
      q0 = unit_start_pos<kFastDiv>(g, un, un_lo);
      q0v = true;
      if (kStep == 2 && un_lo + 1 < un_hi) {
        q1 = next_pos(g, q0);
        q1v = true;
      }
    }
    const bool work = cur && !skip(p0);
    // Build the words first (c0/c1 die), then put the next step's loads in
    // flight, then run the chains.
    uint32_t w[2][16];
    uint32_t ov[2][4];
    if (work) {
      build_words<M>(p0.bi, p0.c, lane, c0, w[0], ov[0]);
      if (two) build_words<M>(p1.bi, p1.c, lane, c1, w[1], ov[1]);
    }
    Chunk n0, n1;
    uint32_t hvn = 0u;
    if (q0v && !skip(q0)) load_chunk<M>(q0.bi, q0.c, lane, n0);
    if (q0v) hvn = hc_of(q0);
    if (q1v) load_chunk<M>(q1.bi, q1.c, lane, n1);
    if (work) {
      NVL_COUNT();
      uint32_t r[2];
      if (two) {
        chains<2, false>(lds, lb, w, lane, r);
      } else {
        r[0] = chain_fold<M>(lds, lb, w[0], lane);
      }
      consume(st, p0, r[0], lds, lane, ka, hv0);
      if (two) consume(st, p1, r[1], lds, lane, ka);
    }
    if (unit_ends) {
      if (st.cnt) {  // the unit ends inside a buffer: its portion, normalized to the buffer end
        const Pos& pl = two ? p1 : p0;  // the step's last chunk
        const uint32_t norm = normalize(lds, ka.tables, st.acc, pl.bi.J - 1u - pl.c, lane);
        if (st.from_zero) tail = Rec{pl.i, norm, st.cnt};
        else st.head = Rec{pl.i, norm, st.cnt};
      }
      if (lane == 0) g.put_recs(ka, lds, u, st.head, tail);
      if (un >= ub1) break;
      u = un;
      t = un_lo;
      t1 = un_hi;
      un = ub0 + pull_unit(lds, lane);
      un_lo = un < ub1 ? lo_of(un) : 0;
      un_hi = un < ub1 ? lo_of(un + 1) : 0;
      st = UnitState{0u, 0u, q0.c <= first_body(q0), Rec{kNoBuf, 0u, 0u}};
      tail = Rec{kNoBuf, 0u, 0u};
    } else {
      t = tn;
    }
    p0 = q0;
    p1 = q1;
    c0 = n0;
    c1 = n1;
    hv0 = hvn;
  }
  NVL_STAMP_END();
}

template <int NW, class G>
__device__ __forceinline__ void run_general(const G& g, const KArgs& ka, uint8_t* lds) {
  run_units<kGeneral, NW>(g, ka, lds);
}

// ---------------------------------------------------------------------------
// Scheduler C -- variable-length batches whose buffers are all short (at most
// kBufsMaxJ chunks).  Workgroup b owns the buffers that START in its chunk
// range [T*b/G, T*(b+1)/G) (balanced to within one buffer), so no buffer is
// split: no records, no fix-up.  Its waves claim groups of consecutive
// buffers from the LDS counter, one buffer per lane (offset, length, ~init in
// the lane's registers: no scalar loads per buffer), and walk each buffer's
// body chunks (a head chunk is crc32c_head_kernel's: its raw register enters
// with the first body chunk).  As in scheduler A the next chunk's loads go
// out before the current chunk's words are built; the unit scheduler (B),
// which also splits buffers across waves, ran the same chunks ~30 % slower
// (fixed-stride: 91.7 vs 70.4 us for 10^5 x 4096 B).
constexpr uint32_t kBufsMaxJ = 32;

// A chunk of scheduler C's stream, wave-uniform (SGPRs): where it ends, its
// buffer, the buffer's ~init and what the chunk is to its buffer.
struct CPos {
  uintptr_t ce;  // chunk end (an invalid position: safe + 4096, the loads read the table blob)
  uint64_t i;    // buffer index
  uint32_t s;    // ~init
  uint32_t f;    // kPos* flags | inj << 8: inj = (chunk start - buffer start) when < 4 (~init lands there), else 0xFF
};
constexpr uint32_t kPosValid = 1u, kPosFirst = 2u, kPosLast = 4u, kPosHeadIn = 8u;

// The chunk's four row loads from A4 (the 4-byte aligned address at or below
// the chunk start), the edge dword (see Chunk), and hc[i] when the chunk is a
// head-first buffer's first body chunk (the table blob otherwise): the same
// loads for every position, valid or not, so the wait counts stay exact.
__device__ __forceinline__ void load_pos(const CPos& q, int lane, uintptr_t safe, const uint32_t* hc, Chunk& ch,
                                         uint32_t& hv) {
  const uint32_t r = (uint32_t)(q.ce & 3u);
  const uintptr_t A4 = q.ce - kChunk - r;
  const uint32_t lo = lane_load_off(lane);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const u32x4 v = ld16(A4 + 1024u * (uint32_t)j + lo);
    ch.d[4 * j + 0] = v.x; ch.d[4 * j + 1] = v.y; ch.d[4 * j + 2] = v.z; ch.d[4 * j + 3] = v.w;
  }
  ch.e[3] = *(const __attribute__((address_space(1))) uint32_t*)(A4 + (r ? kChunk : kChunk - 4u));
  const uintptr_t ha = (q.f & kPosHeadIn) ? (uintptr_t)(hc + q.i) : safe;
  hv = __builtin_nontemporal_load((const __attribute__((address_space(1))) uint32_t*)ha);
}

// The lane's 16 words of piece P = lane of the chunk (build_words<kGeneral>
// from scalars): transpose, realign by r = ce & 3, ~init at the buffer start.
__device__ __forceinline__ void build_pos(const CPos& q, int lane, const Chunk& ch, uint32_t (&w)[16]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = ch.d[k];
  row_transpose(w);
  const uint32_t r = (uint32_t)(q.ce & 3u);
  if (r != 0) {
    const uint32_t nx = next_lane(w[0], ch.e[3]);
#pragma unroll
    for (int k = 0; k < 15; ++k) w[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], r);
    w[15] = __builtin_amdgcn_alignbyte(nx, w[15], r);
  }
  const uint32_t inj = q.f >> 8;
  if (inj < 4u && lane == 0) w[0] ^= q.s >> (8u * inj);
}

template <int NW, class G>
__device__ __forceinline__ void run_bufs(const G& g, const KArgs& ka, uint8_t* lds, uint64_t i0, uint64_t i1,
                                         const uint16_t* perm = nullptr) {
  NVL_STAMP0();
  const int lane = threadIdx.x & 63;
  const uint32_t wv = uniform_u32(threadIdx.x >> 6);
  const uint64_t nb = i1 > i0 ? i1 - i0 : 0;
constexpr int kBufsDiv = 4;  // about this many GS-buffer groups per wave
  const uint32_t GS = (uint32_t)max<uint64_t>(1, min<uint64_t>(kWave, nb / (kBufsDiv * NW)));  // buffers per group
constexpr int kBufsTail = 0;  // single-buffer groups for the range's last buffers (A/B'd: none)
  // Groups of GS buffers (optionally single-buffer groups for the range's
  // last kBT buffers).  The singles once evened out the waves' ends (12 us
  // apart on 10^5 x 4097 B, 27 us on config 3); with the buffers handed out
  // most-chunks-first (lpt_order) and the next group's metadata prefetched
  // they only cost single-chunk steps: 64 -> 0 took 10^5 x 4097 B from 101
  // to 91 us per call and 10^5 x 3364..4109 B from 124 to 115 us, config 3
  // unchanged within the box's spread (tools/diag/ab_variants.sh, same box).
  const uint64_t kBT = kBufsTail;
  const uint64_t nbig = nb > kBT * 2 ? (nb - kBT) / GS : 0;  // GS-buffer groups
  const uint64_t ngroups = nbig + (nb - nbig * GS);
  const uintptr_t safe = (uintptr_t)ka.tables;

  // Groups: the current one (lane j holds buffer gb + j: start, length,
  // ~init) and the next one, claimed and its metadata loads issued one
  // iteration ahead.  Every iteration first builds the words of the chunks
  // in hand (waiting for their loads, which were issued AFTER the next
  // group's metadata), then adopts groups and issues the next loads: an
  // adoption never waits on a load still in flight.  fill_lds starts the LDS
  // counter at 2 * NW: groups wv and NW + wv are pre-assigned.
  // perm (LDS, optional): the range's buffers in the order they are handed
  // out (lpt_order: most chunks first), as indices relative to i0.
  uint64_t todo = 0;  // todo: group lanes whose buffers have body chunks, not started
  uintptr_t lp = 0;
  uint64_t lL = 0;
  uint32_t ls = 0, lr = 0;  // lr: the lane's buffer - i0
  uint64_t ngb = 0;
  uint32_t ngn = 0;
  bool has_nxt = false, nxt_ready = false;
  // The next group's raw metadata, reloaded by EVERY iteration at one place
  // (meta_load, before the chunk loads): the loads are unconditional and
  // nothing is computed from them until the adoption, so they never need a
  // copy at a control-flow join -- such a copy waits for the load (with
  // conditional loads the compiler waited right after issuing them).
  uint64_t no = 0, nL = 0;
  uint32_t ni = 0, nr = 0;
  auto claim_group = [&](uint64_t k) {  // the next group's index (scalars only)
    has_nxt = k < ngroups;
    nxt_ready = false;
    ngb = has_nxt ? i0 + (k < nbig ? k * GS : nbig * GS + (k - nbig)) : 0u;
    ngn = has_nxt ? (k < nbig ? GS : 1u) : 1u;
  };
  const uint32_t* const ibase = g.init ? g.init : reinterpret_cast<const uint32_t*>(safe);
  auto meta_load = [&]() {
    const uint64_t pos = ngb + (uint64_t)min<uint32_t>((uint32_t)lane, ngn - 1u);  // < n (buffer 0 when none)
    const uint64_t i = perm && pos >= i0 ? i0 + perm[pos - i0] : pos;
    nr = (uint32_t)(i - i0);
    no = g.offsets[i];
    nL = g.lengths[i];
    ni = ibase[g.init ? i : 0u];
  };
  auto adopt = [&]() {
    lp = (uintptr_t)g.base + no;
    lL = nL;
    ls = ~(g.init ? ni : g.init_all);
    lr = nr;
    todo = __ballot((uint32_t)lane < ngn && chunks_for(lL) > (head_first(lL) ? 1u : 0u));
    has_nxt = false;
  };
  // the buffer being walked
  uintptr_t cp = 0;
  uint64_t cL = 0, ci = 0;
  uint32_t cJ = 0, cx = 0, cc = 0, cfb = 0;
  bool cvalid = false;
  // the stream's next chunk (invalid when the work is done or the next group
  // is not in registers yet)
  auto next_pos = [&](CPos& q) {
    q.ce = safe + kChunk;
    q.i = 0;
    q.s = 0;
    q.f = 0;
    if (cvalid && cc + 1u < cJ) {
      ++cc;
    } else {
      cvalid = false;
      while (todo == 0) {
        if (!has_nxt || !nxt_ready) return;
        adopt();
        claim_group(pull_unit(lds, lane));  // its metadata: this iteration's meta_load
      }
      const uint32_t j = (uint32_t)__builtin_ctzll(todo);
      todo &= todo - 1u;
      cp = (uintptr_t)lane_u64((uint64_t)lp, j);
      cL = lane_u64(lL, j);
      cx = lane_u32(ls, j);
      ci = i0 + lane_u32(lr, j);
      cJ = chunks_for(cL);
      cfb = head_first(cL) ? 1u : 0u;
      cc = cfb;
      cvalid = true;
    }
    q.ce = cp + cL - (uint64_t)kChunk * (cJ - 1u - cc);
    q.i = ci;
    q.s = cx;
    const uintptr_t cs = q.ce - kChunk;  // >= cp: body chunks start at or after the buffer start
    const uint32_t inj = cs < cp + 4u ? (uint32_t)(cs - cp) : 0xFFu;
    q.f = kPosValid | (cc == cfb ? kPosFirst : 0u) | (cc + 1u == cJ ? kPosLast : 0u) |
          (cc == cfb && cfb == 1u && ka.hc ? kPosHeadIn : 0u) | (inj << 8);
  };
  auto more = [&]() -> bool { return (cvalid && cc + 1u < cJ) || todo != 0 || has_nxt; };

  // pre-assigned: group wv now, group NW + wv as the next one
  claim_group(wv);
  meta_load();
  if (has_nxt) adopt();
  claim_group(NW + wv);
  meta_load();
  CPos p0, p1;
  next_pos(p0);  // (no adoption before the barrier: the next group is not ready)
  next_pos(p1);
  Chunk c0, c1;
  uint32_t hv0, hv1;
  const LdsFill<NW> lf = fill_lds_load<NW>(ka.tables);  // ahead of the first chunk loads (run_pairs)
  load_pos(p0, lane, safe, ka.hc, c0, hv0);  // overlaps the LDS fill
  load_pos(p1, lane, safe, ka.hc, c1, hv1);
  fill_lds_store<NW>(lds, lf, 2u * NW);
  __syncthreads();
  const LaneBase lb = make_lane_base(lane);
  NVL_STAMP1();
  uint32_t acc = 0u;
  // hs: shift4096 of the buffer's head register (hc[i]) for a first body chunk
  auto accumulate = [&](const CPos& q, uint32_t raw, uint32_t hs) {
    const bool first = (q.f & kPosFirst) != 0u;
    acc = (first ? ((q.f & kPosHeadIn) ? hs : 0u) : shift4096(lds, acc, lane)) ^ raw;
    if ((q.f & kPosLast) && lane == 0) ka.out[q.i] = finish(~acc, ka.flags);
  };
  // Two consecutive chunks of the wave's stream per step (the same buffer's or
  // two buffers'), their chains interleaved as in scheduler A.  The step's
  // words are built and its head registers shifted first (c0/c1, hv0/hv1
  // die), then the next two chunks' loads go out into the same registers,
  // then the chains run: no register copies at the loop's back edge (a copy
  // of a loaded register waits for the load).
  while (true) {
    nxt_ready = has_nxt;  // its metadata was loaded before the chunk loads built below
    uint32_t w[2][16];
    const bool work = (p0.f & kPosValid) != 0u;
    if (work) {
      build_pos(p0, lane, c0, w[0]);
      build_pos(p1, lane, c1, w[1]);
    }
    const uint32_t hs0 = shift4096(lds, hv0, lane), hs1 = shift4096(lds, hv1, lane);
    CPos q0, q1;
    next_pos(q0);
    next_pos(q1);
    meta_load();
    load_pos(q0, lane, safe, ka.hc, c0, hv0);
    load_pos(q1, lane, safe, ka.hc, c1, hv1);
    if (work) {
      uint32_t raws[2];
      chains<2, false>(lds, lb, w, lane, raws);
      accumulate(p0, raws[0], hs0);
      if (p1.f & kPosValid) accumulate(p1, raws[1], hs1);
      NVL_COUNT();
    }
    if (!(q0.f & kPosValid) && !more()) break;
    p0 = q0;
    p1 = q1;
  }
  NVL_STAMP_END();
}

// ---------------------------------------------------------------------------
// Head chunks -- crc32c_head_kernel, launched before the kGeneral body
// kernel of the same batch.  A head is a buffer's partial first chunk, h =
// 1..4095 bytes (the whole buffer when it has one chunk).  The chunk pass
// cuts a chunk into 64-byte pieces, one per lane; a head needs only
// ceil(h/64) of them, so a wave runs heads in lane groups of P = 1, 4, 16 or
// 64 lanes (h <= 64, 256, 1024, 4095) -- 64/P heads per round, the chains of
// a group combined by the first log2(P) butterfly levels.  A round costs the
// same 16 chain steps whatever P is: a 6-byte log record no longer takes a
// whole 4 KiB pass.
// Each wave owns a contiguous range of buffers and takes it 64 at a time
// (one buffer per lane: its metadata in the lane's registers).  Buffers of
// < 4 bytes are finished bytewise by their lane (util/crc32c.cc:287 STEP1
// semantics); the heads of each class go out in rounds, lane group q of a
// round holding the class's next q-th head (picked from the class's ballot
// mask and pulled across lanes with ds_bpermute).  The next round's loads are
// issued before the current round computes.  A one-chunk buffer is finished
// (out[i]); a longer one leaves hc[i] = its head's raw register, which the
// body kernel shifts into the buffer's first body chunk.
__device__ __forceinline__ uint32_t nth_set_bit(uint64_t m, uint32_t k) {  // k < popcount(m)
  uint32_t pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint32_t c = (uint32_t)__builtin_popcountll(m & ((1ull << w) - 1ull));
    const bool up = k >= c;
    k -= up ? c : 0u;
    m = up ? m >> w : m;
    pos += up ? (uint32_t)w : 0u;
  }
  return pos;
}

struct HeadLane {  // one lane's part of a head round (5 VGPRs: three rounds are live)
  uintptr_t p;     // buffer start
  uint32_t hl;     // head bytes: the head is [p, p + hl)
  uint32_t s;      // ~init
  uint32_t tag;    // group lane holding the buffer | kHeadOk | kHeadLast
};
constexpr uint32_t kHeadOk = 1u << 8;    // this lane's group has a head this round
constexpr uint32_t kHeadLast = 1u << 9;  // the head is the whole buffer (J == 1)

struct HeadData {
  uint32_t d[17];  // 64 bytes from the 4-byte aligned address at or below the piece start, + 1 dword
};

// The lane's 64-byte piece of its group's head: [ce - 64P + 64k, +64), ce =
// p + hl, k = lane mod P, loaded as four 16-byte slots from A4 (the 4-byte
// aligned address at or below it) plus the dword at A4 + 64.  Fault safety:
// a slot wholly below p's 16-byte granule g is not loaded (zeros); the slot
// straddling g is loaded from g (head_words moves its words up); nothing
// reaches past the head's last dword.
__device__ __forceinline__ uintptr_t head_piece(const HeadLane& h, uint32_t P, int lane) {
  return h.p + h.hl - 64u * P + 64u * ((uint32_t)lane & (P - 1u));
}

// Every load is issued unconditionally (a slot that holds no head bytes reads
// `safe` -- p's own granule, or any valid address when the lane's group has
// no head -- and is zeroed in head_words): loads behind branches would make
// the compiler wait for every load in flight (vmcnt(0)) before each round.
__device__ __forceinline__ bool head_slot_used(const HeadLane& h, uintptr_t A4, uintptr_t g, int j) {
  return (h.tag & kHeadOk) != 0u && A4 + 16u * (uint32_t)j + 16u > g;
}
__device__ __forceinline__ bool head_edge_used(const HeadLane& h, uintptr_t ps, uintptr_t g) {
  return (h.tag & kHeadOk) != 0u && (ps & 3u) != 0u && (ps & ~(uintptr_t)3) + 68u > g;
}

__device__ __forceinline__ void head_load(const HeadLane& h, uint32_t P, int lane, uintptr_t safe, HeadData& hd) {
  const uintptr_t ps = head_piece(h, P, lane);
  const uintptr_t A4 = ps & ~(uintptr_t)3;
  const uintptr_t g = h.p & ~(uintptr_t)15;
  const uintptr_t sf = (h.tag & kHeadOk) ? g : safe;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uintptr_t a = A4 + 16u * (uint32_t)j;
    const u32x4 v = ld16c(head_slot_used(h, A4, g, j) ? (a < g ? g : a) : sf);
    hd.d[4 * j + 0] = v.x; hd.d[4 * j + 1] = v.y; hd.d[4 * j + 2] = v.z; hd.d[4 * j + 3] = v.w;
  }
  hd.d[16] = *(const __attribute__((address_space(1))) uint32_t*)(head_edge_used(h, ps, g) ? A4 + 64u : sf);
}

// The lane's 16 words of its piece: unused slots zeroed, the slot straddling
// g moved into place, realigned to the piece start, bytes before p masked,
// ~init injected.
__device__ __forceinline__ void head_words(const HeadLane& h, const HeadData& hd, uint32_t P, int lane,
                                           uint32_t (&w)[16]) {
  const uintptr_t ps = head_piece(h, P, lane);
  const uintptr_t A4 = ps & ~(uintptr_t)3;
  const uintptr_t g = h.p & ~(uintptr_t)15;
  uint32_t d[17];
  const uint32_t q = (uint32_t)((g - A4) >> 2) & 3u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uintptr_t a = A4 + 16u * (uint32_t)j;
    const bool used = head_slot_used(h, A4, g, j);
    uint32_t x0 = used ? hd.d[4 * j + 0] : 0u, x1 = used ? hd.d[4 * j + 1] : 0u;
    uint32_t x2 = used ? hd.d[4 * j + 2] : 0u, x3 = used ? hd.d[4 * j + 3] : 0u;
    if (a < g) {  // (used) the slot straddling g was loaded from g: its words move up by q dwords
      x3 = q == 1u ? x2 : (q == 2u ? x1 : x0);
      x2 = q == 1u ? x1 : (q == 2u ? x0 : 0u);
      x1 = q == 1u ? x0 : 0u;
      x0 = 0u;
    }
    d[4 * j + 0] = x0; d[4 * j + 1] = x1; d[4 * j + 2] = x2; d[4 * j + 3] = x3;
  }
  d[16] = head_edge_used(h, ps, g) ? hd.d[16] : 0u;
  const uint32_t b = (uint32_t)ps & 3u;
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], b);
  mask_inject<16>(w, (int)(int64_t)(h.p - ps), h.s);
}

// Raw register of the round's heads from their words (every lane of a group
// holds its head's).
__device__ __forceinline__ uint32_t head_chain(const uint8_t* lds, const LaneBase& lb, const uint32_t (&w)[16],
                                               uint32_t nlev, int lane) {
  uint32_t crc = w[0];
#pragma unroll
  for (int k = 0; k < 16; ++k) crc = slice4_next(lds, crc, k < 15 ? w[k + 1] : 0u, lb);
  if (nlev > 0) {
    crc = fold_level<0, 0, false>(lds, crc, lane);
    crc = fold_level<1, 1, false>(lds, crc, lane);
  }
  if (nlev > 2) {
    crc = fold_level<2, 2, false>(lds, crc, lane);
    crc = fold_level<3, 3, false>(lds, crc, lane);
  }
  if (nlev > 4) {
    crc = fold_level<4, 4, false>(lds, crc, lane);
    crc = fold_level<5, 5, false>(lds, crc, lane);
  }
  return crc;
}

// Plan, part 1 (variable-length batches, in the head kernel before its LDS
// fill, with LDS scratch under the table image): workgroup b owns tile b and
// writes lpre/tiles (see KArgs).  Thread t takes 4 consecutive buffers per
// step; one block-wide scan per 4096 buffers.  The body kernel's tiled_plan
// turns the tiles into chunk positions, so a variable-length batch needs no
// plan kernels of its own (the counts -> device scan -> unit map -> fix-up
// launches cost ~20 us on 10^5 buffers).  Returns (block-uniform) whether
// some buffer of the tile has a head that needs the lookup tables (4..4095
// bytes; shorter ones are done bitwise, see bitwise_raw).
template <int NW, class G>
__device__ bool tile_scan(const G& g, const KArgs& ka, uint8_t* lds) {
  constexpr uint32_t kT = kWave * NW, kPer = 4;
  uint64_t* wsum = reinterpret_cast<uint64_t*>(lds);           // [NW]
  uint32_t* wmax = reinterpret_cast<uint32_t*>(lds + 8u * NW);  // [NW]
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint64_t S = ka.tile_S, lo = S * blockIdx.x;
  const uint64_t hi = lo < g.n ? min(g.n, lo + S) : lo;
  uint64_t carry = 0;
  uint32_t mj = 0;
  bool tab = false;
  for (uint64_t base = lo; base < hi; base += (uint64_t)kT * kPer) {  // (uniform trip count)
    const uint64_t i0 = base + (uint64_t)t * kPer;
    uint64_t L[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) L[k] = i0 + k < hi ? g.lengths[i0 + k] : 0;
    uint32_t J[kPer];
    uint64_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      J[k] = i0 + k < hi ? chunks_for(L[k]) : 0u;
      sum += J[k];
      mj = max(mj, J[k]);
      const uint64_t hl = L[k] - (uint64_t)kChunk * (J[k] - 1u);
      tab |= i0 + k < hi && L[k] >= 4 && hl >= 4 && hl < kChunk;
    }
    uint64_t x = sum;  // inclusive scan over the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint64_t before = 0, tot = 0;
#pragma unroll
    for (uint32_t v = 0; v < (uint32_t)NW; ++v) {
      const uint64_t sv = wsum[v];
      before += v < wv ? sv : 0;
      tot += sv;
    }
    uint64_t e = carry + before + x - sum;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      if (i0 + k < hi) ka.lpre[i0 + k] = e;
      e += J[k];
    }
    carry += tot;
    __syncthreads();  // (wsum is rewritten by the next step)
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mj = max(mj, (uint32_t)__shfl_xor((int)mj, o));
  // the wave's largest count, bit 31 = some lane's `tab` (an OR over the
  // workgroup in the scratch: __syncthreads_or would take 256 B of LDS
  // beyond the image, which crc32c_route_kernel's region image cannot spare)
  if (lane == 0) wmax[wv] = mj | (__ballot(tab) ? 0x80000000u : 0u);
  __syncthreads();
  bool need = false;
#pragma unroll
  for (uint32_t v = 0; v < (uint32_t)NW; ++v) need |= (wmax[v] >> 31) != 0u;
  if (t == 0) {
    uint32_t m = 0;
#pragma unroll
    for (uint32_t v = 0; v < (uint32_t)NW; ++v) m = max(m, wmax[v] & 0x7FFFFFFFu);
    ka.tiles[2ull * blockIdx.x] = carry;
    ka.tiles[2ull * blockIdx.x + 1] = max(m, 3u);  // head mode: the body kernel has work (> 2, see run_heads)
  }
  __syncthreads();  // (the scratch becomes the table image)
  return need;
}

// CRC register after n <= 3 bytes at p from state l, bit by bit (the
// reflected polynomial, util/crc32c.cc:287 STEP1 semantics): no tables, so a
// workgroup whose heads are all this short skips its 156 KiB LDS fill
// (10^5 x 4097 B: every head is 1 byte).
__device__ __forceinline__ uint32_t bitwise_raw(const uint8_t* p, uint32_t n, uint32_t l) {
  for (uint32_t k = 0; k < n; ++k) {
    l ^= (uint32_t)p[k];
#pragma unroll
    for (int b = 0; b < 8; ++b) l = (l >> 1) ^ (0x82F63B78u & (0u - (l & 1u)));
  }
  return l;
}

// Head kernel LDS beyond the table image: a sub-range's work list and the
// fused tile scan's scratch.
//   u32 ctl[4]: [0] list A size, [1] slots handed out, [2] list B size
//   u16 list[kHeadSub]: list A (one pass per entry) from the front, list B
//       (two passes per entry) from the back, as indices within the sub-range
//   u64 wsum[16], u32 wmax[16]: per-wave scan totals / largest chunk counts
constexpr uint64_t kHeadSub = (uint64_t)kWave * kWavesPerWG;  // buffers per sub-range: <= 64 per wave
constexpr uint32_t kLongOff = kLdsBytes;
constexpr uint32_t kListOff = kLongOff + 16u;
constexpr uint32_t kScanOff = kListOff + 2u * (uint32_t)kHeadSub;
constexpr uint32_t kHeadLdsBytes = kScanOff + 16u * (8u + 4u);
static_assert(kLongOff % 16u == 0u && kScanOff % 8u == 0u && kHeadLdsBytes <= 160u * 1024u,
              "head kernel LDS exceeds 160 KiB");

// Work-list entries (u16): index within the sub-range (bits 0..9) | kLOut
// when the entry is a whole buffer (J == 1).
constexpr uint32_t kLOut = 1u << 15;
static_assert(kHeadSub <= 1024u, "list entries hold a 10-bit index");

// Drain pass tags: list entry (bits 0..15) | flags.
constexpr uint32_t kTOk = 1u << 16;    // a real pass
constexpr uint32_t kTOut = 1u << 17;   // the whole buffer (J == 1): out[i] = finish(~raw)
constexpr uint32_t kTHc = 1u << 18;    // head mode: the head of a longer buffer, hc[i] = raw
constexpr uint32_t kTInj = 1u << 19;   // short mode: a J == 2 buffer's body, its head's register from hc[i]
constexpr uint32_t kTTiny = 1u << 20;  // (kTInj) a 1..3-byte head: hc[i] is rewritten for the body kernel
constexpr uint32_t kTPair = 1u << 21;  // short mode: a slot holding the head and the body of one J == 2 buffer

// One pass of the drain (wave-uniform): the chunk [ce - 4096, ce) with its
// bytes before ps zeroed and sx XORed into the 4 bytes at ps.  The body pass
// of a two-chunk buffer in list A (kTInj) starts from its head's register
// instead: raw(s, H || B) = raw(raw(s, H), B) = raw(0, B ^ raw(s, H))
// (crc32c_math.h), so raw(s, H) is XORed into the body's first word and the
// pass yields the whole buffer -- no shift, no combine.  raw(s, H) is in
// hc[i] before the drain starts: a 1..3-byte head fed bitwise by its lane
// at classification, a head that starts a page's first granule (which a
// masked pass cannot read: load_general) by a pre-drain lane-group round.
struct SlotPass {
  uintptr_t ce, ps;
  uint32_t sx, tag;
};

// The drain of a sub-range's lists, two passes per step with interleaved
// chains, every wave of the workgroup pulling slots from one LDS counter.
// Slot k < nB is list B's k-th entry (a J == 2 buffer: its head and body);
// later slots hold two list-A entries each.  Pipeline: a step builds the
// words of the slot in hand (waiting for its loads), turns the next slot's
// metadata -- loaded a step earlier, before those chunk loads -- into
// positions, pulls the slot after it and issues its metadata loads, issues
// the next slot's chunk loads, then runs the chains.  Past the end a pass is
// a dummy chunk in the table blob (loaded, not written; a slot of two
// dummies is not run).  The metadata is the offset, the length's low word
// (list entries have at most two chunks or are heads: h = ((L - 1) & 4095)
// + 1, J == 1 from the entry's kLOut) and ~init: the fewer registers the
// next slot's loads hold, the more LDS lookups of the chains the compiler
// keeps in flight.
template <class G>
__device__ __forceinline__ void drain_list(const G& g, const KArgs& ka, uint8_t* lds, const LaneBase& lb,
                                           uint64_t sub0, uint32_t* ctl, const uint16_t* list, bool shortm) {
  const int lane = threadIdx.x & 63;
  const uint32_t nA = uniform_u32(ctl[0]), nB = uniform_u32(ctl[2]);
  const uint32_t nslots = nB + (nA + 1u) / 2u;
  if (nslots == 0) return;
  const uintptr_t safe = (uintptr_t)ka.tables;
  auto pull = [&]() -> uint32_t {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(&ctl[1], 1u);
    return uniform_u32(v);
  };
  // Slot k's entries and their metadata -- scalar loads into SGPRs: the
  // metadata of the next slot holds no vector registers across the chains
  // (with vector loads the scheduler ran out of registers and serialised the
  // two chains' LDS lookups)
  uint64_t mo0, mo1;
  uint32_t mL0, mL1, ms0, ms1, mj0, mj1;
  auto meta = [&](uint32_t k) {
    const bool isb = k < nB;
    const uint32_t a = 2u * (k - nB);
    const uint32_t e0 = uniform_u32(isb ? (uint32_t)list[kHeadSub - 1u - k] : (a < nA ? (uint32_t)list[a] : 0u));
    const uint32_t e1 = uniform_u32(isb || a + 1u >= nA ? 0u : (uint32_t)list[a + 1u]);
    mj0 = isb ? (e0 | kTOk | kTPair) : (a < nA ? e0 | kTOk : 0u);
    mj1 = isb ? mj0 : (a + 1u < nA ? e1 | kTOk : 0u);
    g.meta_s(sub0 + (mj0 & 1023u), mo0, mL0, ms0);
    g.meta_s(sub0 + (mj1 & 1023u), mo1, mL1, ms1);
  };
  // positions of one entry; for a PAIR slot the first pass is the head, the
  // second the body
  auto pos = [&](uint64_t o, uint32_t L, uint32_t s, uint32_t tag, bool second, SlotPass& q) {
    const uint32_t h = ((L - 1u) & (kChunk - 1u)) + 1u;  // (L: the low word, see above)
    const uintptr_t p = g.base_addr() + o;
    q.tag = tag;
    if (!(tag & kTOk)) {
      q.ce = safe + kChunk;
      q.ps = safe;
      q.sx = 0u;
      q.tag = 0u;
    } else if (tag & kTPair) {
      q.ce = second ? p + L : p + h;
      q.ps = second ? p + h : p;
      q.sx = second ? 0u : s;
    } else if (tag & kLOut) {
      q.ce = p + L;
      q.ps = p;
      q.sx = s;
      q.tag |= kTOut;
    } else if (shortm) {  // J == 2: the body, from its head's register (hc[i])
      q.ce = p + L;
      q.ps = q.ce - kChunk;
      q.sx = h < 4u ? s >> (8u * h) : 0u;  // (kTTiny: hc[i]'s rewrite for the body kernel)
      q.tag |= kTInj | (h < 4u ? kTTiny : 0u);
    } else {  // head mode: a long head
      q.ce = p + h;
      q.ps = p;
      q.sx = s;
      q.tag |= kTHc;
    }
  };
  auto aux_load = [&](const SlotPass& q) -> uint32_t {  // hc[i] of a kTInj pass (bypassing L1)
    const uintptr_t a = (q.tag & kTInj) ? (uintptr_t)(ka.hc + sub0 + (q.tag & 1023u)) : safe;
    return __builtin_nontemporal_load((const __attribute__((address_space(1))) uint32_t*)a);
  };
  SlotPass A, B;
  meta(pull());
  pos(mo0, mL0, ms0, mj0, false, A);
  pos(mo1, mL1, ms1, mj1, true, B);
  Chunk cA, cB;
  load_general(A.ce, true, A.ps, lane, cA);
  load_general(B.ce, true, B.ps, lane, cB);
  uint32_t xA = aux_load(A), xB = aux_load(B);
  while (true) {
    if (!(A.tag & kTOk)) break;  // (a slot wholly past the end: its loads just drain)
    meta(pull());  // the next slot's (lands while this slot's words are built)
    uint32_t w[2][16];
#pragma unroll
    for (int q = 0; q < 16; ++q) w[0][q] = cA.d[q];
    row_transpose(w[0]);
    realign_general(A.ce, true, A.ps, (A.tag & kTInj) ? 0u : A.sx, lane, cA, w[0]);
#pragma unroll
    for (int q = 0; q < 16; ++q) w[1][q] = cB.d[q];
    row_transpose(w[1]);
    realign_general(B.ce, true, B.ps, (B.tag & kTInj) ? 0u : B.sx, lane, cB, w[1]);
    // a kTInj body starts from its head's register (word 0 of lane 0)
    const uint32_t iA = (A.tag & kTInj) ? xA : 0u, iB = (B.tag & kTInj) ? xB : 0u;
    if (lane == 0) {
      w[0][0] ^= iA;
      w[1][0] ^= iB;
    }
    // hc of a 1..3-byte head in the body kernel's convention (raw(s, H) ^
    // (s >> 8h): that kernel injects s >> 8h into the body itself), for a
    // mixed batch whose body kernel re-runs this tile's two-chunk bodies
    const uint32_t hcA = iA ^ A.sx, hcB = iB ^ B.sx;
    const uint32_t uA = A.tag, uB = B.tag;
    pos(mo0, mL0, ms0, mj0, false, A);
    pos(mo1, mL1, ms1, mj1, true, B);
    load_general(A.ce, true, A.ps, lane, cA);
    load_general(B.ce, true, B.ps, lane, cB);
    xA = aux_load(A);
    xB = aux_load(B);
    // (The scheduler sinks the second pass's loads into the chains below to
    // keep the two chains' lookups interleaved; forcing every load ahead of
    // the chains -- an asm memory barrier -- serialised the chains and
    // measured 2-6 % slower on r and v; so did pinning the chain steps with
    // sched_group_barrier.)
    uint32_t raws[2];
    chains<2, false>(lds, lb, w, lane, raws);
    // shift4096 spreads its lookups over the lanes of a quad: every lane runs it
    const uint32_t shA = (uA & kTPair) ? shift4096(lds, raws[0], lane) : 0u;
    if (lane == 0) {
      const uint64_t ia = sub0 + (uA & 1023u), ib = sub0 + (uB & 1023u);
      if (uA & kTPair) {  // head + body of one buffer
        ka.out[ia] = finish(~(shA ^ raws[1]), ka.flags);
        if (ka.hc) ka.hc[ia] = raws[0];
      } else {
        if (uA & (kTOut | kTInj)) ka.out[ia] = finish(~raws[0], ka.flags);
        if (uA & (kTHc | kTTiny)) ka.hc[ia] = (uA & kTHc) ? raws[0] : hcA;
        if (uB & (kTOut | kTInj)) ka.out[ib] = finish(~raws[1], ka.flags);
        if (uB & (kTHc | kTTiny)) ka.hc[ib] = (uB & kTHc) ? raws[1] : hcB;
      }
    }
    if (!(uB & kTOk)) break;  // (slots are handed out in order: a half-empty one is the last)
  }
}

// The head kernel: a workgroup takes its buffers (its plan tile when the
// batch is variable-length) in sub-ranges of kHeadSub, a slice of at most 64
// buffers (one per lane) per wave.
//   head mode: the partial first chunks ("heads") of the buffers -- a
//     one-chunk buffer is finished (out[i]), a longer one leaves hc[i] for
//     the body kernel; buffers of < 4 bytes and 1..3-byte heads bitwise,
//     heads of <= 1024 bytes in the wave's own lane-group rounds, longer
//     ones as whole masked chunks from the workgroup's LDS list.
//   short mode (every buffer of the tile has at most 2 chunks, and none
//     needs a page-start masked head: KArgs::short_ok and the tile's scan):
//     EVERY buffer is finished here, so the body kernel has nothing left --
//     one-chunk buffers of > 1024 bytes as one pass (list A), two-chunk
//     buffers as head + body passes in one slot (list B) or, with a 1..3-byte
//     head, as the body pass with the head folded in inline (list A); the
//     rest in lane-group rounds.  tiles[2b+1] (the tile's largest chunk
//     count) stays <= 2 only for a short-mode tile: the body kernel exits at
//     once when every tile is one.
// After the lists are complete each wave runs its own rounds and then joins
// the drain, so a wave with many rounds leaves the list to the others (a
// barrier between rounds and drain made the whole workgroup wait for its
// slowest wave's rounds: up to 13 us on 10^5 buffers of 3364..4109 B).
template <class G>
__device__ __forceinline__ void run_heads(const G& g, const KArgs& ka, uint8_t* lds) {
  NVL_TL_DECL();
  NVL_TL(0);
  const int lane = threadIdx.x & 63;
  const uint32_t wv = uniform_u32(threadIdx.x >> 6);
  // the workgroup's buffers: its plan tile when there is one
  uint64_t w0 = g.n * blockIdx.x / gridDim.x, w1 = g.n * (blockIdx.x + 1) / gridDim.x;
  bool tiled = false;
  if constexpr (G::kTiled) {
    if (ka.lpre) {
      tiled = true;
      w0 = min(g.n, ka.tile_S * blockIdx.x);
      w1 = min(g.n, w0 + ka.tile_S);
    }
  }
  // one sub-range tiles fold their plan scan into the classification pass
  const bool fused_scan = tiled && w1 - w0 <= kHeadSub;
  bool shortm = !tiled && ka.short_ok != 0u;
  if constexpr (G::kTiled) {
    if (tiled && !fused_scan) {
      (void)tile_scan<kWavesPerWG>(g, ka, lds);  // head mode (large tiles)
      NVL_TL(1);
    }
  }
  const LaneBase lb = make_lane_base(lane);
  uint32_t* ctl = reinterpret_cast<uint32_t*>(lds + kLongOff);
  uint16_t* list = reinterpret_cast<uint16_t*>(lds + kListOff);
  uint64_t* wsum = reinterpret_cast<uint64_t*>(lds + kScanOff);
  uint32_t* wmax = reinterpret_cast<uint32_t*>(lds + kScanOff + 16u * 8u);
  uintptr_t lp = 0;  // the lane's buffer of the current sub-range: start, length, ~init
  uint64_t lL = 0;
  uint32_t ls = 0;
  // the wave's slice of a sub-range [s0, s1): at most 64 buffers
  auto slice = [&](uint64_t s0, uint64_t s1, uint64_t& a, uint64_t& b) {
    a = s0 + (s1 - s0) * wv / kWavesPerWG;
    b = s0 + (s1 - s0) * (wv + 1) / kWavesPerWG;
  };
  const LdsFill<kWavesPerWG> lf = fill_lds_load<kWavesPerWG>(ka.tables);  // ahead of the metadata loads
  {
    uint64_t a, b;
    slice(w0, min(w1, w0 + kHeadSub), a, b);
    if (a + (uint64_t)lane < b) g.lane_meta(a + (uint64_t)lane, lp, lL, ls);  // in flight during the fill
  }
  if (threadIdx.x < 4) ctl[threadIdx.x] = 0u;
  fill_lds_store<kWavesPerWG>(lds, lf);
  // Every path passes this barrier before its first table lookup and its
  // first list append: it orders the LDS fill AND wave 0's zeroing of the
  // list counters ctl before them (round 3 faulted a parity test,
  // test_varlen_plan_paths[32769], when an append could land before the
  // zeroing; the fused path's scan barrier below no longer carries that).
  __syncthreads();
  NVL_TL(2);
  if (fused_scan) {  // (the first -- and only -- sub-range's lanes hold their metadata)
    uint64_t gb, ge;
    slice(w0, w1, gb, ge);
    const bool valid = gb + (uint64_t)lane < ge;
    const uint64_t i = gb + (uint64_t)lane;
    const uint32_t J = valid ? chunks_for(lL) : 0u;
      // the tile's plan (tile_scan's lpre / tiles) from the lanes' lengths:
      // the waves' slices are consecutive, so one wave scan + one barrier
      uint64_t x = J;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
      }
      uint32_t mj = J;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mj = max(mj, (uint32_t)__shfl_xor((int)mj, o));
      if (lane == 63) wsum[wv] = x;
      if (lane == 0) wmax[wv] = mj;
      __syncthreads();  // wsum / wmax complete
      // the 16 waves' totals and flags across lanes 0..15 (a wave scan, not
      // 48 LDS reads held in registers at once)
      const bool lw = (uint32_t)lane < kWavesPerWG;
      const uint64_t sv = lw ? wsum[lane] : 0;
      uint32_t mv = lw ? wmax[lane] : 0u;
      uint64_t inc = sv;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const uint64_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
        mv = max(mv, (uint32_t)__shfl_xor((int)mv, o));
      }
      const uint64_t tot = lane_u64(inc, kWavesPerWG - 1u);
      const uint64_t before = lane_u64(inc - sv, wv);
      const uint32_t m = lane_u32(mv, 0u);
      shortm = ka.short_ok != 0u && m <= 2u;
      if (valid) ka.lpre[i] = before + x - J;
      if (threadIdx.x == 0) {
        ka.tiles[2ull * blockIdx.x] = tot;
        ka.tiles[2ull * blockIdx.x + 1] = shortm ? m : max(m, 3u);  // > 2: the body kernel has work
      }
      NVL_TL(1);
    }
  for (uint64_t sub0 = w0; sub0 < w1; sub0 += kHeadSub) {  // (workgroup-uniform trip count)
    const uint64_t sub1 = min(w1, sub0 + kHeadSub);
    uint64_t gb, ge;
    slice(sub0, sub1, gb, ge);
    const bool valid = gb + (uint64_t)lane < ge;
    const uint64_t i = gb + (uint64_t)lane;
    if (sub0 != w0) {
      lp = 0;
      lL = 0;
      ls = 0;
      if (valid) g.lane_meta(i, lp, lL, ls);
    }
    const bool tiny = valid && lL < 4;
    const uint32_t J = valid ? chunks_for(lL) : 0u;
    const uint64_t hl = lL - (uint64_t)kChunk * (J - 1u);  // first chunk's bytes (when valid)
    const bool pstart = ((lp >> 4) & 255u) == 0u;          // p in a 4 KiB page's first 16 bytes
    const uint32_t cls = hl <= 64u ? 0u : (hl <= 256u ? 1u : (hl <= 1024u ? 2u : 3u));
    bool inA, inB, round, shrt, pre = false;
    if (shortm) {  // (workgroup-uniform)
      // a two-chunk buffer whose 4..4095-byte head starts a page's first
      // granule: the head in a round before the drain (a masked pass would
      // read below the page), its register handed to the body pass via hc
      pre = valid && !tiny && J == 2u && hl >= 4u && hl < kChunk && pstart;
      inA = valid && !tiny && ((J == 1u && hl > 1024u && (hl == kChunk || !pstart)) || (J == 2u && (hl < 4u || pre)));
      inB = valid && !tiny && J == 2u && hl >= 4u && !pre;
      round = valid && !tiny && J == 1u && !inA;
      shrt = false;
    } else {
      shrt = valid && !tiny && hl < 4;  // 1..3-byte head of a longer buffer
      const bool head = valid && !tiny && !shrt && hl < kChunk;
      // Long heads (1025..4095 bytes) run as whole masked chunks from the
      // list (as P = 64 lane-group rounds, whose 64-byte-per-lane loads touch
      // 32 lines per instruction, this class ran at ~2.7 TB/s), except where
      // the buffer starts in a page's first 16 bytes (load_general reads up to
      // 12 bytes below p's granule).
      inA = head && cls == 3u && !pstart;
      inB = false;
      round = head && !inA;
    }
    // what setup pulls across lanes: head bytes (< 4096) | kHeadLast << 16
    const uint32_t hlx = (uint32_t)(hl & 0xFFFFu) | (J == 1u ? kHeadLast << 16 : 0u);
    if (tiny) ka.out[i] = finish(~bitwise_raw(reinterpret_cast<const uint8_t*>(lp), (uint32_t)lL, ls), ka.flags);
    // hc = raw(0, head ^ s's low bytes) = raw(s, head) ^ (s >> 8 hl): the body
    // injects s's remaining bytes into its first word itself
    if (shrt) ka.hc[i] = bitwise_raw(reinterpret_cast<const uint8_t*>(lp), (uint32_t)hl, ls) ^ (ls >> (8u * (uint32_t)hl));
    // short mode: a 1..3-byte head's register raw(s, H) for its body pass
    // (list A, kTInj), stored before the lists-complete barrier
    if (shortm && valid && !tiny && J == 2u && hl < 4u)
      ka.hc[i] = bitwise_raw(reinterpret_cast<const uint8_t*>(lp), (uint32_t)hl, ls);
    {  // append to the workgroup's lists (index within the sub-range)
      const uint64_t ma = __ballot(inA), mb = __ballot(inB);
      const uint32_t rank_a = __builtin_amdgcn_mbcnt_hi((uint32_t)(ma >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ma, 0u));
      const uint32_t rank_b = __builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u));
      uint32_t ba = 0, bb = 0;
      if (lane == 0) {
        if (ma) ba = atomicAdd(&ctl[0], (uint32_t)__builtin_popcountll(ma));
        if (mb) bb = atomicAdd(&ctl[2], (uint32_t)__builtin_popcountll(mb));
      }
      ba = uniform_u32(ba);
      bb = uniform_u32(bb);
      if (inA) list[ba + rank_a] = (uint16_t)((uint32_t)(i - sub0) | (J == 1u ? kLOut : 0u));
      if (inB) list[kHeadSub - 1u - (bb + rank_b)] = (uint16_t)(i - sub0);
    }
    uint64_t m[4];
    uint32_t nr[4], NR = 0;
    // phase 0: the pre-drain heads (short mode); then the lists are complete;
    // phase 1: the wave's own rounds
    for (int ph = 0; ph < 2; ++ph) {  // (workgroup-uniform)
    NR = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      m[c] = __ballot((ph == 0 ? pre : round) && cls == (uint32_t)c);
      const uint32_t per = 64u >> (2 * c);
      nr[c] = ((uint32_t)__builtin_popcountll(m[c]) + per - 1u) / per;
      NR += nr[c];
    }
    // Round R -> class c and the class's round t (wave-uniform), then each
    // lane's head: lane group q = lane / P takes the class's (t*64/P + q)-th.
    auto setup = [&](uint32_t R, HeadLane& h, uint32_t& P, uint32_t& nlev) {
      uint32_t c = 0, t = R;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const bool past = c == (uint32_t)k && t >= nr[k];
        t -= past ? nr[k] : 0u;
        c += past ? 1u : 0u;
      }
      nlev = 2u * c;
      P = 1u << nlev;
      const uint64_t mc = c == 0 ? m[0] : (c == 1 ? m[1] : (c == 2 ? m[2] : m[3]));
      const uint32_t per = 64u >> nlev;
      const uint32_t rank = t * per + ((uint32_t)lane >> nlev);
      const bool ok = rank < (uint32_t)__builtin_popcountll(mc);
      const uint32_t src = ok ? nth_set_bit(mc, rank) : (uint32_t)lane;
      const int sa = (int)(src << 2);
      const uint32_t plo = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)(uint32_t)lp);
      const uint32_t phi = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)(uint32_t)(lp >> 32));
      const uint32_t hx = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)hlx);
      h.s = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)ls);
      h.p = ((uintptr_t)phi << 32) | plo;
      h.hl = hx & 0xFFFFu;
      h.tag = src | (ok ? kHeadOk : 0u) | (hx >> 16);
    };
    if (NR != 0) {
    // Two buffers, A and B, in ping-pong: a buffer's next round is loaded
    // right after its words are built (the registers carry over, no copies),
    // so each round's loads have two rounds of chains to arrive.  Past the
    // last round a buffer reloads its own round (valid addresses, unused).
    const uintptr_t safe = (uintptr_t)ka.tables;
    HeadLane hA, hB;
    HeadData dA, dB;
    uint32_t PA, LA, PB, LB;
    setup(0, hA, PA, LA);
    head_load(hA, PA, lane, safe, dA);
    // (A's loads issue before B's on entry as on the back edge: the wait
    // counts the compiler derives for the loop then let B's stay in flight)
    asm volatile("" ::: "memory");
    hB = hA;
    PB = PA;
    LB = LA;
    if (NR > 1) setup(1, hB, PB, LB);
    head_load(hB, PB, lane, safe, dB);
    auto finish_round = [&](uint32_t raw, uint32_t tag, uint32_t P) {
      if ((tag & kHeadOk) && ((uint32_t)lane & (P - 1u)) == 0u) {
        const uint64_t ib = gb + (tag & 63u);
        if (tag & kHeadLast) ka.out[ib] = finish(~raw, ka.flags);
        else ka.hc[ib] = raw;
      }
    };
    for (uint32_t R = 0; R < NR; R += 2) {
      uint32_t w[16];
      head_words(hA, dA, PA, lane, w);
      uint32_t tag = hA.tag, P = PA, nl = LA;
      if (R + 2 < NR) setup(R + 2, hA, PA, LA);
      head_load(hA, PA, lane, safe, dA);
      asm volatile("" ::: "memory");
      finish_round(head_chain(lds, lb, w, nl, lane), tag, P);
      // B's half runs even past the last round (then on its own reloaded
      // round, not written): a branch around its loads would make the wait
      // counts at the loop head assume the worst order
      head_words(hB, dB, PB, lane, w);
      tag = R + 1 < NR ? hB.tag : 0u;
      P = PB;
      nl = LB;
      if (R + 3 < NR) setup(R + 3, hB, PB, LB);
      head_load(hB, PB, lane, safe, dB);
      asm volatile("" ::: "memory");
      finish_round(head_chain(lds, lb, w, nl, lane), tag, P);
    }
    // (the last reloads drain before the list's first loads are issued)
    }
    if (ph == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the hc stores (pre-drain rounds, 1..3-byte heads) done
      __syncthreads();  // the lists are complete (and the tables in LDS)
      NVL_TL(3);
    }
    }
    NVL_TL(4);
    drain_list(g, ka, lds, lb, sub0, ctl, list, shortm);
    NVL_TL(5);
    if (sub0 + kHeadSub < w1) {  // (workgroup-uniform) the lists are reused by the next sub-range
      __syncthreads();
      if (threadIdx.x < 4) ctl[threadIdx.x] = 0u;
      __syncthreads();
    }
  }
  NVL_TL_END();
}

template <class G>
__global__ __launch_bounds__(kThreads, 1) void crc32c_head_kernel(G g, KArgs ka) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kHeadLdsBytes];
  run_heads(g, ka, lds);
}

constexpr int kFastU = 2;  // buffers per unit in scheduler A (tools/ab_bench.py: 2 > 1 > 4)

constexpr int kGenWaves = 16;  // waves per workgroup of the kGeneral kernels
constexpr int kGenPairU = 2;   // buffers per unit (g: 67.7 us at 2, 70.4 at 1, 91.7 through run_units)
template <int M>
constexpr int waves_of() { return M == kGeneral ? kGenWaves : kWavesPerWG; }

// Aligned one-chunk batches of at least kLongFixedMin blocks (config 5's
// whole-rank step) run this copy of crc32c_fixed_kernel<kAligned>'s J == 1
// path: the same code under its own name, so a profile's per-kernel
// statistics keep config 2-sized launches (~64 us) apart from ms-long ones.
constexpr uint64_t kLongFixedMin = 1ull << 18;
__global__ __launch_bounds__(kThreads, 1) void crc32c_fixed_long_kernel(FixedGeom g, KArgs ka) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes > kRLdsBytes ? kLdsBytes : kRLdsBytes];
  run_pairs<kFastU, kWavesPerWG, kAligned, FixedGeom, false, true>(g, ka, lds);
}

template <int M>
__global__ __launch_bounds__(kWave * waves_of<M>(), 1) void crc32c_fixed_kernel(FixedGeom g, KArgs ka) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes > kRLdsBytes ? kLdsBytes : kRLdsBytes];
  if constexpr (M == kAligned) {
    if (g.J == 1) {
      run_pairs<kFastU, kWavesPerWG, kAligned, FixedGeom, false, true>(g, ka, lds);
      return;
    }
  }
  if constexpr (M == kGeneral) {
    // one whole chunk per buffer (len == 4096, any alignment): scheduler A,
    // one buffer per unit, no records
    if (g.J == 1 && !head_first(g.len)) {
      run_pairs<kGenPairU, waves_of<M>(), kGeneral>(g, ka, lds);
      return;
    }
    // one partial chunk per buffer, 1025..4095 bytes (launch_fixed): each
    // buffer a long head, in scheduler A's order (10^5 x 3500 B at stride
    // 4128: 75.3 -> 71.3 us against the head kernel, profiles/r03_ablations).
    // (launch_fixed sends these batches here without a head kernel.)
    if (g.J == 1) {
      run_pairs<kGenPairU, waves_of<M>(), kMasked>(g, ka, lds);
      return;
    }
  }
  if constexpr (M == kGeneral) run_general<waves_of<M>()>(g, ka, lds);
  else run_units<M, waves_of<M>()>(g, ka, lds);
}

// Aligned multi-chunk fixed batches (config 4): every 4 KiB chunk an
// independent scheduler-A pass (ChunkGeom), raw registers to KArgs::raws.
__global__ __launch_bounds__(kThreads, 1) void crc32c_chunks_kernel(ChunkGeom g, KArgs ka) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes > kRLdsBytes ? kLdsBytes : kRLdsBytes];
  run_pairs<kFastU, kWavesPerWG, kAligned, ChunkGeom, true, true>(g, ka, lds);
}

// Buffer i of J chunks: raw = XOR_c shift(raws[iJ + c], 4096 (J - 1 - c)).
// One wave per buffer: lane l folds the R = ceil(J/64) raws of its run
// [J - R(64 - l), J - R(63 - l)) serially through the shift-by-4096 operator
// (byte-sliced, in LDS), shifts its run to the buffer end with one GF(2)
// multiply by m_l = x^(8 * 4096 R (63 - l)) (built once per wave from the
// x^(2^k) powers), and the 64 lanes XOR-reduce.
__global__ __launch_bounds__(256) void crc32c_fold_kernel(const uint32_t* __restrict__ raws, uint64_t n, uint32_t J,
                                                          const uint32_t* __restrict__ tables,
                                                          uint32_t* __restrict__ out, uint32_t flags) {
  __shared__ uint32_t sh[1024];  // sh4096[4][256]
  for (uint32_t t = threadIdx.x; t < 1024u; t += blockDim.x) sh[t] = tables[kGComb + 6u * 1024u + t];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t R = (J + 63u) / 64u;
  const uint32_t* x2n = tables + kGX2n;
  uint32_t m = nvl::kOne, P = nvl::xpow8(x2n, (uint64_t)kChunk * R);
  const uint32_t e = 63u - lane;
  for (int b = 0; b < 6; ++b) {
    if ((e >> b) & 1u) m = nvl::gf_mul(P, m);
    P = nvl::gf_mul(P, P);
  }
  const uint64_t wpb = blockDim.x >> 6;
  const uint64_t nw = (uint64_t)gridDim.x * wpb;
  for (uint64_t i = (uint64_t)blockIdx.x * wpb + uniform_u32(threadIdx.x >> 6); i < n; i += nw) {
    const int64_t c0 = (int64_t)J - (int64_t)R * (int64_t)(64u - lane);
    const uint32_t* rb = raws + i * J;
    uint32_t acc = 0;
    for (uint32_t k = 0; k < R; ++k) {
      const int64_t c = c0 + (int64_t)k;
      const uint32_t r = c >= 0 ? rb[c] : 0u;
      acc = sh[acc & 255u] ^ sh[256u + ((acc >> 8) & 255u)] ^ sh[512u + ((acc >> 16) & 255u)] ^ sh[768u + (acc >> 24)] ^ r;
    }
    acc = nvl::gf_mul(m, acc);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, o);
    if (lane == 0) out[i] = finish(~acc, flags);
  }
}

// Two-level fold for buffers of more than kChunkParallelMaxJ chunks (a lone
// 1 GiB buffer: J = 262144): level 1 folds segments of S chunk raws (one
// wave each, the whole grid busy), level 2 folds each buffer's G segment
// raws -- the same fold with the step "S chunks".  Row `row` holds J
// elements, element e sits at its end, consecutive elements `step` apart
// (x^(8 * bytes)); segment g = elements [J - (G - g) S, J - (G - g - 1) S)
// (the first one clipped at 0).  A wave's lane l folds the run of R =
// ceil(S / 64) elements ending R (63 - l) before the segment end through the
// byte-sliced step table (built in LDS), multiplies by m[l] = step^(R (63 -
// l)) (host-computed), and the lanes XOR-reduce: G > 1 writes the segment's
// raw to dst[row * G + g], G == 1 writes finish(~raw) to dst[row].
struct FoldSeg {
  const uint32_t* src;
  uint64_t rows;
  uint32_t J, S, G, step;
  uint32_t m[64];
  uint32_t* dst;
  uint32_t flags;
};
__global__ __launch_bounds__(256) void crc32c_fold_seg_kernel(FoldSeg a) {
  __shared__ uint32_t sh[1024];  // sh[j][b] = (b << 8j) * step
  for (uint32_t t = threadIdx.x; t < 1024u; t += blockDim.x) sh[t] = nvl::gf_mul(a.step, (t & 255u) << (8u * (t >> 8)));
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t R = (a.S + 63u) / 64u;
  const uint32_t m = a.m[lane];
  const uint64_t items = a.rows * a.G;
  const uint64_t wpb = blockDim.x >> 6;
  const uint64_t nw = (uint64_t)gridDim.x * wpb;
  for (uint64_t it = (uint64_t)blockIdx.x * wpb + uniform_u32(threadIdx.x >> 6); it < items; it += nw) {
    const uint64_t row = it / a.G;
    const uint32_t g = (uint32_t)(it - row * a.G);
    const int64_t seg0 = (int64_t)a.J - (int64_t)(a.G - g) * (int64_t)a.S;  // first element of the segment
    const int64_t c0 = seg0 + (int64_t)a.S - (int64_t)R * (int64_t)(64u - lane);
    const uint32_t* rb = a.src + row * a.J;
    uint32_t acc = 0;
    for (uint32_t k = 0; k < R; ++k) {
      const int64_t c = c0 + (int64_t)k;
      const uint32_t r = (c >= 0 && c >= seg0) ? rb[c] : 0u;
      acc = sh[acc & 255u] ^ sh[256u + ((acc >> 8) & 255u)] ^ sh[512u + ((acc >> 16) & 255u)] ^ sh[768u + (acc >> 24)] ^ r;
    }
    acc = nvl::gf_mul(m, acc);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, o);
    if (lane == 0) {
      if (a.G > 1) a.dst[it] = acc;
      else a.dst[row] = finish(~acc, a.flags);
    }
  }
}

__global__ __launch_bounds__(kWave * kGenWaves, 1) void crc32c_var_kernel(VarGeom g, KArgs ka) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  if (ka.long_bufs && ldc(ka.long_bufs, 0) == 0u) {
    // Workgroup b: the buffers that start in its chunk range [lo(64b),
    // lo(64b+64)): unit_first[u] holds the buffer containing chunk lo(u),
    // which starts there or earlier (then it is the previous workgroup's).
    const uint64_t T = g.total();
    const uint32_t ub0 = blockIdx.x * kUnitsPerWG, nu = gridDim.x * kUnitsPerWG;
    auto first_at = [&](uint32_t u) -> uint64_t {
      if (u >= nu) return g.n;
      const uint64_t lo = global_unit_lo<true>(T, u);
      if (lo >= T) return g.n;
      const uint64_t b = ldc(g.unit_first, u);
      return ldc(g.chunk_start, b) == lo ? b : b + 1u;
    };
    const uint64_t i0 = first_at(ub0), i1 = first_at(ub0 + kUnitsPerWG);
    if (threadIdx.x < kUnitsPerWG && ka.recs) {  // no split buffers: empty records for the fix-up
      ka.recs[2ull * (ub0 + threadIdx.x)] = Rec{kNoBuf, 0u, 0u};
      ka.recs[2ull * (ub0 + threadIdx.x) + 1] = Rec{kNoBuf, 0u, 0u};
    }
    run_bufs<kGenWaves>(g, ka, lds, i0, i1);
    return;
  }
  run_general<kGenWaves>(g, ka, lds);
}

// Per-buffer chunk counts for the variable-length plan: cnt[i] = J_i, cnt[n] = 0.
__global__ void crc32c_var_counts(const uint64_t* __restrict__ lengths, uint64_t n,
                                  uint64_t* __restrict__ cnt, uint32_t* __restrict__ long_bufs) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    cnt[i] = chunks_for(lengths[i]);
  } else if (i == n) {
    cnt[i] = 0;
    *long_bufs = 0u;  // (crc32c_unit_map, two launches later, sets it)
  }
}

// unit_first[u] = the buffer holding chunk floor(T*u/NU), T = chunk_start[n]:
// buffer i owns the units u with cs_i <= floor(T*u/NU) < cs_{i+1}, i.e.
// u in [ceil(cs_i*NU/T), ceil(cs_{i+1}*NU/T)).
__global__ void crc32c_unit_map(const uint64_t* __restrict__ cs, uint64_t n, uint64_t NU,
                                uint64_t* __restrict__ unit_first, uint32_t* __restrict__ long_bufs) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t T = cs[n];
  const uint64_t a = cs[i], b = cs[i + 1];
  if (b - a > kBufsMaxJ) *long_bufs = 1u;  // (every writer stores the same value)
  uint64_t u0 = (a * NU + T - 1) / T, u1 = (b * NU + T - 1) / T;
  if (u1 > NU) u1 = NU;
  for (uint64_t u = u0; u < u1; ++u) unit_first[u] = i;
}

// ceil(a / d) for a < 2^62, d > 0: a double-precision estimate corrected by
// at most a step or two (a full 64-bit division is a long software loop).
__device__ __forceinline__ uint64_t ceil_div_u64(uint64_t a, uint64_t d) {
  uint64_t q = (uint64_t)((double)a / (double)d);
  while (q * d < a) ++q;
  while (q > 0 && (q - 1) * d >= a) --q;
  return q;
}

// The whole variable-length plan in one workgroup, for batches of up to
// kPlanSmallMax buffers: chunk counts, their exclusive prefix (chunk_start,
// cs[n] = T) and the unit map -- one launch instead of counts + device scan +
// unit map.  The chunk counts are staged in LDS by one coalesced pass; thread
// t then owns the contiguous buffer run [t*per, t*per + per): one block-wide
// scan of the run sums, and each thread walks its run in registers.
constexpr uint64_t kPlanThreads = 1024;
constexpr uint64_t kPlanSmallMax = 32768;

__device__ __forceinline__ uint32_t plan_pad(uint32_t i) { return i + (i >> 5); }  // 33 words per 32: no bank conflicts

__global__ __launch_bounds__(kPlanThreads) void crc32c_plan_small(const uint64_t* __restrict__ lengths, uint64_t n,
                                                                uint64_t NU, uint64_t* __restrict__ cs,
                                                                uint64_t* __restrict__ unit_first,
                                                                uint32_t* __restrict__ long_bufs) {
  __shared__ uint32_t js[kPlanSmallMax + kPlanSmallMax / 32];  // chunk counts, then run-relative prefixes
  __shared__ uint64_t wsum[kPlanThreads / kWave];
  __shared__ uint64_t rstart[kPlanThreads];  // first chunk of each thread's run
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t nn = (uint32_t)n;
  {  // all of the thread's lengths in flight at once (a loop issues them one latency at a time)
    constexpr int kPer = (int)(kPlanSmallMax / kPlanThreads);
    uint64_t Ls[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = t + (uint32_t)k * (uint32_t)kPlanThreads;
      Ls[k] = i < nn ? lengths[i] : 0;
    }
    bool lng = false;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = t + (uint32_t)k * (uint32_t)kPlanThreads;
      const uint32_t J = chunks_for(Ls[k]);
      lng |= J > kBufsMaxJ;
      if (i < nn) js[plan_pad(i)] = J;
    }
    const int any = __syncthreads_or(lng ? 1 : 0);
    if (t == 0) *long_bufs = any ? 1u : 0u;
  }
  const uint32_t per = (nn + (uint32_t)kPlanThreads - 1) / (uint32_t)kPlanThreads;
  const uint32_t i0 = min(nn, t * per), i1 = min(nn, i0 + per);
  // The run's counts become run-relative exclusive prefixes in place (u32: a
  // device-resident buffer is < 2^38 bytes = 2^26 chunks, a run <= 32 of them).
  uint32_t sum = 0;
  for (uint32_t i = i0; i < i1; ++i) {
    const uint32_t j = js[plan_pad(i)];
    js[plan_pad(i)] = sum;
    sum += j;
  }
  uint64_t x = sum;  // inclusive scan of the run sums over the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  uint64_t before = 0, T = 0;
#pragma unroll
  for (uint32_t v = 0; v < kPlanThreads / kWave; ++v) {
    const uint64_t sv = wsum[v];
    before += v < wv ? sv : 0;
    T += sv;
  }
  const uint64_t run0 = before + x - sum;
  rstart[t] = run0;
  __syncthreads();
  // chunk_start, coalesced: cs[i] = start of i's run + its run-relative prefix.
  for (uint32_t i = t; i < nn; i += kPlanThreads) cs[i] = rstart[i / per] + js[plan_pad(i)];
  if (t == 0) cs[n] = T;
  // Unit map: unit u starts in buffer i iff cs_i*NU <= T*u < cs_{i+1}*NU
  // (lo(u) = floor(T*u/NU), see crc32c_unit_map).  Walk the run with the
  // running products cn = cs_{i+1}*NU and tu = T*u: one division per thread.
  uint64_t u = ceil_div_u64(run0 * NU, T);
  uint64_t tu = T * u;
  for (uint32_t i = i0; i < i1; ++i) {
    const uint64_t next = run0 + (i + 1 < i1 ? js[plan_pad(i + 1)] : sum);
    const uint64_t cn = next * NU;
    for (; u < NU && tu < cn; ++u, tu += T) unit_first[u] = i;
  }
}

// Fold the per-unit records of buffers cut by work-unit boundaries.  Records
// are normalized (each portion already shifted to its buffer's end), so a
// buffer's CRC is the XOR of its portions: unit w's head record, when it
// holds the LAST portion, plus the head records (middle portions) and the
// tail record (first portion) of the units before it; units with an empty
// chunk range carry no records.  One wave per unit w walks back 64 units per
// step (one record pair per lane), so a buffer spanning thousands of units
// costs tens of steps, not thousands of serial ones.
__global__ __launch_bounds__(256) void crc32c_fixup_kernel(const Rec* __restrict__ recs, uint32_t nw,
                                                           uint32_t* __restrict__ out, uint32_t flags) {
  const uint32_t w = uniform_u32(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  if (w >= nw) return;
  const Rec h = recs[2 * (uint64_t)w];
  if (h.buf == kNoBuf || !(h.cnt & kRecEnds)) return;
  uint32_t acc = lane == 0 ? h.raw : 0u;
  for (int64_t base = (int64_t)w - 1; base >= 0; base -= kWave) {
    const int64_t x = base - lane;
    Rec hx{kNoBuf, 0u, 0u}, tx{kNoBuf, 0u, 0u};
    if (x >= 0) {
      hx = recs[2 * x];
      tx = recs[2 * x + 1];
    }
    const bool mid = hx.buf == h.buf;                  // a middle portion
    const bool first = !mid && tx.buf == h.buf;        // the first portion: the walk ends here
    const bool other = !mid && !first && (hx.buf != kNoBuf || tx.buf != kNoBuf || x < 0);
    const unsigned long long stop = __ballot(first || other);
    const int lim = stop ? __builtin_ctzll(stop) : kWave;  // lanes below lim: middle or empty units
    if ((lane < lim && mid) || (lane == lim && first)) acc ^= lane < lim ? hx.raw : tx.raw;
    if (stop) break;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, o);
  if (lane == 0) out[h.buf] = finish(~acc, flags);
}

// ---------------------------------------------------------------------------
// Fused variable-length batch (n <= kPlanSmallMax): plan, checksum and fix-up
// in ONE launch instead of three (config 3: plan 26 + kernel 255 + fix-up
// 7 us, plus two launch gaps).
//   * Plan prologue, in the LDS the tables later occupy: every workgroup
//     scans all n chunk counts (n * 8 B, L2-resident after the first reader):
//     coalesced counts, run-relative prefixes, block scan.  Workgroup b owns
//     chunks [T*b/G, T*(b+1)/G), cut into 64 work units whose (buffer, chunk)
//     starts 64 threads find by binary search.
//   * Records of buffers cut by unit boundaries stay in LDS and the workgroup
//     folds them itself.  A buffer crossing a WORKGROUP boundary leaves edge
//     records: E_in, its portion here when it began in an earlier workgroup
//     (flagged when it also ends here), and E_out, the portion of a buffer
//     that begins here and runs on.  Hand-off per MI355X_MICROARCH.md's
//     visibility table, row 1 (cdna_hip_programming.md Guideline 16): edge
//     records stored sc1 (agent-scope atomic stores), the storing wave drains
//     (vmcnt(0)), ONE lane adds to the stream's done counter; the workgroup
//     whose add returns G-1 reads every edge record with sc1 loads, folds the
//     cross-workgroup buffers and re-zeroes the counter (zeroed when the
//     stream's counter was created; every launch leaves it zero).
constexpr uint32_t kUnitOff = kLdsBytes;                                           // u32 ubuf[64], uc[64]
constexpr uint32_t kRecOff = kUnitOff + 2u * kUnitsPerWG * 4u;                     // Rec[2 * 64]
constexpr uint32_t kEdgeOff = kRecOff + 2u * kUnitsPerWG * (uint32_t)sizeof(Rec);  // Rec e_in, e_out; u32 last
constexpr uint32_t kFusedLdsBytes = kEdgeOff + 2u * (uint32_t)sizeof(Rec) + 16u;
static_assert(kFusedLdsBytes <= 160u * 1024u, "fused LDS image exceeds 160 KiB");
constexpr uint32_t kPlanJsBytes = (uint32_t)(kPlanSmallMax + kPlanSmallMax / 32) * 4u;
constexpr uint32_t kPlanWsumOff = kPlanJsBytes;             // u64 [16]
constexpr uint32_t kPlanRunOff = kPlanWsumOff + 16u * 8u;   // u64 run starts [1024]
static_assert(kPlanRunOff + 1024u * 8u <= kSliceOff + kRepBytes, "plan scratch must fit under the table image");
constexpr uint32_t kMaxFusedGrid = 4096;  // the last workgroup folds 2 edge records per workgroup in LDS
static_assert(2u * kMaxFusedGrid * sizeof(Rec) <= kSliceOff + kRepBytes, "edge fold must fit under the table image");

struct VarGeomFused {
  const uint8_t* base;
  const uint64_t* offsets;
  const uint64_t* lengths;
  uint64_t n;
  const uint32_t* init;
  uint32_t init_all;
  uint64_t C0, C1;        // this workgroup's chunk range
  const uint32_t* ubuf;   // LDS: buffer holding the first chunk of local unit k
  const uint32_t* uc;     // LDS: that chunk's index within the buffer
  uint32_t ub0;
  __device__ __forceinline__ uint64_t total() const { return C1 - C0; }
  template <bool F>
  __device__ __forceinline__ uint64_t unit_lo(uint64_t span, uint32_t u) const {
    return C0 + span * (uint64_t)(u - ub0) / kUnitsPerWG;
  }
  template <bool F>
  __device__ __forceinline__ void locate_unit(uint32_t u, uint64_t, uint64_t& i, uint32_t& c) const {
    i = ubuf[u - ub0];
    c = uc[u - ub0];
  }
  __device__ __forceinline__ BufInfo info(uint64_t i) const {
    const uint64_t L = ldc(lengths, i);
    const uint32_t ini = init ? ldc(init, i) : init_all;
    return BufInfo{base + ldc(offsets, i), L, chunks_for(L), ~ini};
  }
  __device__ __forceinline__ void put_recs(const KArgs&, uint8_t* lds, uint32_t u, const Rec& h, const Rec& t) const {
    Rec* r = reinterpret_cast<Rec*>(lds + kRecOff);
    r[2 * (u - ub0)] = h;
    r[2 * (u - ub0) + 1] = t;
  }
};



// Plan, part 2, from the head kernel's tiles (tile_scan), in the LDS the
// tables later occupy: the tile totals' block scan gives each tile's first
// chunk (tb[], T = tb[Gt]); the workgroup's chunk range is [T*b/G, T*(b+1)/G).
// Chunk q lies in the last tile k with tb[k] <= q (binary search in LDS) and
// there in the last buffer a with tb[k] + lpre[a] <= q: a 16-ary search over
// lpre by 16 lanes (ballot of the 16 probes), about log16(S) rounds of
// global loads.  Scheduler B needs the first chunk of each of the 64 units
// (64 searches, 16 lanes each: the whole block); scheduler C only the first
// buffers starting at or after C0 and C1 (2 searches).
constexpr uint32_t kMaxTiles = 1023;
constexpr uint32_t kTbWsumOff = 8u * (kMaxTiles + 1u);  // u64 [16]
constexpr uint32_t kTbResOff = kTbWsumOff + 16u * 8u;   // u64 B0, B1
static_assert(kTbResOff + 16u <= kSliceOff + kRepBytes, "tiled plan scratch must fit under the table image");

template <int NW>
__device__ __forceinline__ void tiled_plan(uint8_t* lds, const VarGeom& g, const KArgs& ka, uint64_t& C0,
                                           uint64_t& C1, bool& long_bufs, uint64_t& B0, uint64_t& B1,
                                           bool& multi) {
  constexpr uint32_t kT = kWave * NW;
  static_assert(kT == 1024, "64 searches of 16 lanes fill the block");
  uint64_t* tb = reinterpret_cast<uint64_t*>(lds);
  uint64_t* wsum = reinterpret_cast<uint64_t*>(lds + kTbWsumOff);
  uint64_t* res = reinterpret_cast<uint64_t*>(lds + kTbResOff);
  uint32_t* ubuf = reinterpret_cast<uint32_t*>(lds + kUnitOff);
  uint32_t* uc = ubuf + kUnitsPerWG;
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t Gt = ka.tile_G;  // <= kMaxTiles (host)
  const uint64_t tot = t < Gt ? ka.tiles[2ull * t] : 0;
  const uint64_t mj = t < Gt ? ka.tiles[2ull * t + 1] : 0;
  multi = __syncthreads_or(mj > 2 ? 1 : 0) != 0;
  if (!multi) return;  // every tile finished by the head kernel (short mode): the caller returns too
  long_bufs = __syncthreads_or(mj > kBufsMaxJ ? 1 : 0) != 0;
  uint64_t x = tot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  uint64_t before = 0, T = 0;
#pragma unroll
  for (uint32_t v = 0; v < (uint32_t)NW; ++v) {
    const uint64_t sv = wsum[v];
    before += v < wv ? sv : 0;
    T += sv;
  }
  if (t <= Gt) tb[t] = before + x - tot;  // tb[Gt] = T
  __syncthreads();
  T = uniform_u64(T);
  C0 = T * blockIdx.x / gridDim.x;
  C1 = T * (blockIdx.x + 1) / gridDim.x;
  const uint32_t s = t >> 4, j = t & 15u;  // search s, probe lane j
  const uint32_t nsearch = long_bufs ? kUnitsPerWG : 2u;
  if (s < nsearch) {
    const uint64_t q = long_bufs ? C0 + (C1 - C0) * s / kUnitsPerWG : (s == 0 ? C0 : C1);
    if (q < T && (!long_bufs || q < C1)) {
      uint32_t klo = 0, khi = Gt;  // tb[klo] <= q < tb[khi]
      while (khi - klo > 1) {
        const uint32_t mid = (klo + khi) >> 1;
        if (tb[mid] <= q) klo = mid; else khi = mid;
      }
      const uint64_t kb = tb[klo];
      const uint64_t S = ka.tile_S;
      uint64_t lo = S * klo, hi = min(g.n, lo + S);  // kb + lpre[lo] = kb <= q
      while (hi - lo > 1) {  // (the same trip count in the group's 16 lanes)
        const uint64_t step = (hi - lo + 15u) / 16u;
        const uint64_t a = lo + step * j;
        const bool le = a < hi && kb + ka.lpre[a] <= q;
        const uint32_t bits = (uint32_t)(__ballot(le) >> (lane & 48u)) & 0xFFFFu;
        lo += step * (uint64_t)(__builtin_popcount(bits) - 1);
        hi = min(hi, lo + step);
      }
      const uint64_t key = kb + ka.lpre[lo];
      if (j == 0) {
        if (long_bufs) {
          ubuf[s] = (uint32_t)lo;
          uc[s] = (uint32_t)(q - key);
        } else {
          res[s] = key == q ? lo : lo + 1u;
        }
      }
    } else if (j == 0 && !long_bufs) {
      res[s] = g.n;
    }
  }
  __syncthreads();
  B0 = long_bufs ? 0 : res[0];
  B1 = long_bufs ? 0 : res[1];
  __syncthreads();  // (the scratch becomes the table image)
}

// XOR into `total` the earlier portions of buffer `buf` (LDS records of units
// x < k, normalized): middle portions are head records, the first portion a
// tail record.  True when the first portion is in this workgroup.
__device__ __forceinline__ bool fold_back(const Rec* lr, int k, unsigned long long buf, uint32_t& total) {
  for (int x = k - 1; x >= 0; --x) {
    const Rec hx = lr[2 * x];
    if (hx.buf == buf) {
      total ^= hx.raw;
      continue;
    }
    const Rec tx = lr[2 * x + 1];
    if (tx.buf == buf) {
      total ^= tx.raw;
      return true;
    }
    if (hx.buf != kNoBuf || tx.buf != kNoBuf) return false;  // unreachable for a consistent plan
  }
  return false;
}

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;

// Edge records as two 8-B agent-scope atomic accesses (sc1 stores / loads).
__device__ __forceinline__ void store_edge(gu64* g, const Rec& r) {
  __hip_atomic_store(g, r.buf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(g + 1, (unsigned long long)r.raw | ((unsigned long long)r.cnt << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ Rec load_edge(gu64* g) {
  const unsigned long long b = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long v = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return Rec{b, (uint32_t)v, (uint32_t)(v >> 32)};
}

// Longest-processing-time order for scheduler C (fused kernel, whole
// buffers): the workgroup's buffers by body chunks, most first, so the last
// groups handed out are the smallest.  In range order the waves of a
// workgroup finished 26..43 us apart on config 3 (buffers of up to 16
// chunks, ~4.6 us per two-chunk step: tools/diag/bstamps.py).  A counting
// sort over the 33 chunk counts in LDS beyond the table image (scheduler B's
// unit/record area, unused here); nullptr when the range is larger than the
// permutation space.
constexpr uint32_t kPermOff = kLdsBytes;             // u32 bucket[33], then u16 perm[kPermMax]
constexpr uint32_t kPermMax = 1792;  // (the compiler adds ~264 B of its own to this kernel)
constexpr uint32_t kPermLdsBytes = kPermOff + 136u + 2u * kPermMax;
static_assert(kPermLdsBytes <= 160u * 1024u, "permutation exceeds LDS");

template <int NW>
__device__ const uint16_t* lpt_order(const VarGeom& g, uint8_t* lds, uint64_t i0, uint64_t i1) {
  const uint64_t nb = i1 - i0;
  if (nb == 0 || nb > kPermMax) return nullptr;
  constexpr uint32_t kT = kWave * NW;
  uint32_t* bucket = reinterpret_cast<uint32_t*>(lds + kPermOff);
  uint16_t* perm = reinterpret_cast<uint16_t*>(lds + kPermOff + 136u);
  const uint32_t t = threadIdx.x;
  if (t < 33) bucket[t] = 0u;
  __syncthreads();
  constexpr int kPer = (int)((kPermMax + kT - 1) / kT);
  uint32_t key[kPer], rank[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const uint64_t x = (uint64_t)t + (uint64_t)q * kT;
    key[q] = 0u;
    rank[q] = 0u;
    if (x < nb) {
      const uint64_t L = g.lengths[i0 + x];
      const uint32_t w = chunks_for(L) - (head_first(L) ? 1u : 0u);  // body chunks, 0..32
      key[q] = 32u - min(w, 32u);
      rank[q] = atomicAdd(&bucket[key[q]], 1u);
    }
  }
  __syncthreads();
  if (t < kWave) {  // exclusive prefix of the 33 buckets (key 0 = most chunks first)
    const uint32_t v = t < 33 ? bucket[t] : 0u;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
      if (t >= (uint32_t)o) x += y;
    }
    if (t < 33) bucket[t] = x - v;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const uint64_t x = (uint64_t)t + (uint64_t)q * kT;
    if (x < nb) perm[bucket[key[q]] + rank[q]] = (uint16_t)x;
  }
  __syncthreads();
  return perm;
}

__global__ __launch_bounds__(kWave * kGenWaves, 1) void crc32c_var_fused_kernel(VarGeom gv, KArgs ka) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kFusedLdsBytes > kPermLdsBytes ? kFusedLdsBytes : kPermLdsBytes];
  if (ka.route.parts) {
    // the route kernel's verdict (written by its workgroup 0 before anything
    // else; this launch follows it on the stream)
    const int rv = (int)ldc(&ka.route.parts[kRoutePlanMax].bad, 0);
    if (rv == kRouteRegion) return;  // the region path ran
    if (rv == kRoutePagesAligned) {  // every buffer one aligned 4 KiB chunk: config 2's loop over the list
      run_pairs<kFastU, kGenWaves, kAligned, VarGeom>(gv, ka, lds);  // (the kLdsBytes image: the region one
                                                                     // and this kernel's own LDS exceed 160 KiB)
      return;
    }
    if (rv == kRoutePages) {  // every buffer 4096 bytes, some misaligned
      run_pairs<kGenPairU, kGenWaves, kGeneral, VarGeom>(gv, ka, lds);
      return;
    }
  }
  const uint32_t ub0 = blockIdx.x * kUnitsPerWG;
  uint64_t C0, C1, B0, B1;
  bool long_bufs = false, multi;
  tiled_plan<kGenWaves>(lds, gv, ka, C0, C1, long_bufs, B0, B1, multi);
  // Every tile's largest chunk count <= 2: the head kernel ran each tile in
  // short mode and finished every buffer (run_heads) -- nothing left here.
  if (!multi) return;
  // The range is uniform, but the 64-bit divisions that made it ran on the
  // VALU: pin it to SGPRs, or it stays in VGPRs through the main loop and
  // that spills (25 VGPRs, 108 B/lane scratch, cfg3 287 -> 430 us).
  C0 = uniform_u64(C0);
  C1 = uniform_u64(C1);
  const uint32_t* ubuf = reinterpret_cast<const uint32_t*>(lds + kUnitOff);
  const VarGeomFused g{gv.base, gv.offsets, gv.lengths, gv.n, gv.init, gv.init_all, C0, C1, ubuf,
                       ubuf + kUnitsPerWG, ub0};
  if (!long_bufs) {
    // whole buffers: no records, so no edge fold either -- no grid-wide
    // hand-off (its sc1 stores, drain and counter round trip cost ~5 us of
    // tail; the stream's counter is left untouched, i.e. zero)
    B0 = uniform_u64(B0);
    B1 = uniform_u64(B1);
    const uint16_t* perm = multi ? lpt_order<kGenWaves>(gv, lds, B0, B1) : nullptr;
    run_bufs<kGenWaves>(gv, ka, lds, B0, B1, perm);
    return;
  }
  run_general<kGenWaves>(g, ka, lds);
  const Rec* lr = reinterpret_cast<const Rec*>(lds + kRecOff);
  Rec* edge = reinterpret_cast<Rec*>(lds + kEdgeOff);
  uint32_t* last = reinterpret_cast<uint32_t*>(lds + kEdgeOff + 2u * sizeof(Rec));
  const uint32_t t = threadIdx.x;
  if (t < 2) edge[t] = Rec{kNoBuf, 0u, 0u};
  __syncthreads();  // every unit's records are in LDS
  if (t < kUnitsPerWG) {  // a buffer that ends in unit t and began in an earlier unit
    const Rec h = lr[2 * t];
    if (h.buf != kNoBuf && (h.cnt & kRecEnds)) {
      uint32_t total = h.raw;
      if (fold_back(lr, (int)t, h.buf, total)) ka.out[h.buf] = finish(~total, ka.flags);
      else edge[0] = Rec{h.buf, total, kRecEnds};  // began before C0
    }
  } else if (t == kUnitsPerWG) {  // the buffer of the range's last chunk, if it runs past C1
    int L = (int)kUnitsPerWG - 1;
    while (L >= 0 && lr[2 * L].buf == kNoBuf && lr[2 * L + 1].buf == kNoBuf) --L;
    if (L >= 0) {
      const Rec h = lr[2 * L], tl = lr[2 * L + 1];
      if (tl.buf != kNoBuf) {
        edge[1] = tl;
      } else if (!(h.cnt & kRecEnds)) {  // a middle portion: the buffer covers unit L
        uint32_t total = h.raw;
        if (fold_back(lr, L, h.buf, total)) edge[1] = Rec{h.buf, total, 0u};
        else edge[0] = Rec{h.buf, total, 0u};  // began before C0 and runs past C1
      }
    }
  }
  __syncthreads();
  if (t == 0) {  // publish: sc1 stores, drain, ONE counter add
    gu64* eg = (gu64*)ka.recs + 4ull * blockIdx.x;
    store_edge(eg, edge[0]);
    store_edge(eg + 2, edge[1]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t d = __hip_atomic_fetch_add((gu32*)ka.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *last = d == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!*last) return;
  // The last workgroup: every edge record (sc1 loads) into the now free table
  // image, then one thread per workgroup whose E_in ends a buffer XORs in the
  // earlier workgroups' (normalized) edge records of that buffer.
  const uint32_t G = gridDim.x;
  Rec* E = reinterpret_cast<Rec*>(lds);  // [2b] = E_in of workgroup b, [2b+1] = E_out
  gu64* eg = (gu64*)ka.recs;
  for (uint32_t b = t; b < 2 * G; b += blockDim.x) E[b] = load_edge(eg + 2ull * b);
  __syncthreads();
  for (uint32_t b = t; b < G; b += blockDim.x) {
    const Rec e = E[2 * b];
    if (e.buf == kNoBuf || !(e.cnt & kRecEnds)) continue;
    uint32_t total = e.raw;
    for (int bb = (int)b - 1; bb >= 0; --bb) {
      const Rec ei = E[2 * bb], eo = E[2 * bb + 1];
      if (ei.buf == e.buf) {  // a workgroup wholly inside the buffer
        total ^= ei.raw;
        continue;
      }
      if (eo.buf == e.buf) {  // the workgroup where it began
        total ^= eo.raw;
        break;
      }
      if (ei.buf != kNoBuf || eo.buf != kNoBuf) break;  // unreachable for a consistent plan
    }
    ka.out[e.buf] = finish(~total, ka.flags);
  }
  if (t == 0) (void)__hip_atomic_exchange((gu32*)ka.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ReadBlock's trailer checks (table/format.cc:88-135) for blocks whose CRCs
// a batch just computed over the device-resident table: len1[i] = size + 1
// (block | type), the trailer's type byte at off + size, its masked CRC after.
__global__ void crc32c_trailer_verdicts(const uint8_t* __restrict__ f, const uint64_t* __restrict__ off,
                                        const uint64_t* __restrict__ len1, const uint32_t* __restrict__ crc,
                                        uint64_t n, uint8_t* __restrict__ verdict) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* t = f + off[i] + len1[i] - 1u;
  const uint32_t stored = (uint32_t)t[1] | ((uint32_t)t[2] << 8) | ((uint32_t)t[3] << 16) | ((uint32_t)t[4] << 24);
  verdict[i] = crc[i] != nvl::unmask(stored) ? 2u /* NVL_BLOCK_CHECKSUM_MISMATCH */
                                             : (t[0] > 1u ? 3u /* NVL_BLOCK_BAD_TYPE */ : 0u);
}

// ---------------------------------------------------------------------------
// Region batches (nvl_crc32c_region_dev): the n buffers lie inside ONE region
// (an SSTable image's blocks, a log image's records, config 3's packed
// buffers), sorted by offset and non-overlapping.  Instead of one pass per
// buffer-aligned chunk -- a 3.4..4.1 KiB block costs a whole 4 KiB pass and
// its head a second -- the region is streamed in ITS OWN page-aligned 4 KiB
// chunks at scheduler A's rate, and every buffer is derived from chunk-level
// values (model: tests/kernel_model.py region_batch):
//   chunk c = [4096c, 4096c + 4096) from the grid origin O = region & ~4095,
//   raws[c] = raw(0, chunk c);
//   for a buffer boundary ("event") at in-chunk offset p (not 0), lane L = p/64
//     holds it: Qe = the butterfly over the lanes below L with the others
//     zeroed = raw(0, chunk bytes [0, 64L)) shifted to the chunk end;
//   the fold kernel re-reads the piece bytes [64L, p) (R = their raw) and
//     combines: Ze(p) = Qe ^ shift(R, 4096 - p) is the chunk prefix before p
//     at the chunk end, so a buffer [s, e) is
//       acc = raws[c0] ^ Ze(s) (^ ~init injected at s), shift4096 ^ raws[c]
//       over the chunks in between, then unshifted from the end of e's chunk:
//       raw = (acc' ^ Qe(e)) * x^(-8(4096 - p_e)) ^ R(e).
// The buffers are found per work unit from a 64-buffer window of the
// metadata (lane j = buffer cursor + j) whose cursor the previous unit's
// window gives, so there is no plan launch; a 64-ary search places each
// wave's first cursor.  Events need the ends to be non-decreasing: the waves
// check the batch (sorted, non-overlapping, inside the region) and any
// violation sets a flag with which the fold kernel checksums every buffer
// serially instead (correct, slow).
constexpr uint32_t kRegionDirect = 64;  // shorter buffers: checksummed whole by the fold kernel

struct RegionGeom {
  const uint8_t* grid;  // O: chunk c at grid + 4096c
  uint64_t nc;          // chunks
  uint64_t rel0;        // buffer i starts at grid position rel0 + offsets[i] (u64, wrapping)
  uint64_t rs, re;      // the region [rs, re) in grid positions (rs < 4096)
  const uint64_t* offsets;
  const uint64_t* lengths;
  uint64_t n;
  const uint32_t* init;  // per-buffer Extend seeds (nullptr: init_all)
  uint32_t init_all;
  uint32_t* raws;  // [nc]
  uint4* qs;       // [n] buffer i's start event: {Qe, lane L's chain checkpoint x_4c, gen, i}
  uint4* qe;       // [n] its end event
  uint32_t gen;    // this call's generation: a record without it (and its own index) was not written by this call
};

typedef const __attribute__((address_space(1))) uint64_t* g64_ptr;
__device__ __forceinline__ uint64_t ldg64(const uint64_t* p, uint64_t i) { return ((g64_ptr)p)[i]; }

// One lane's buffer of a 64-buffer metadata window.
struct WinRaw {
  uint64_t off, len;
};
struct Win {
  uint64_t s, e;  // grid-relative [s, e)
  bool valid;     // cursor + lane < n
  bool big;       // valid and at least kRegionDirect bytes (has events)
};

// Loads of the window at `cur` (the index is clamped so that the loads are
// unconditional: a load behind a branch makes the compiler wait for it).
__device__ __forceinline__ WinRaw load_win(const RegionGeom& g, uint64_t cur, int lane) {
  const uint64_t b = min(cur + (uint64_t)lane, g.n - 1u);
  return WinRaw{ldg64(g.offsets, b), ldg64(g.lengths, b)};
}
__device__ __forceinline__ Win make_win(const RegionGeom& g, const WinRaw& r, uint64_t cur, int lane) {
  Win w;
  w.valid = cur + (uint64_t)lane < g.n;
  w.s = g.rel0 + r.off;
  w.e = w.s + r.len;
  w.big = w.valid && r.len >= kRegionDirect;
  return w;
}

// First buffer b with e_b > A (n when none), for non-decreasing ends: a
// 64-ary search, one wave-wide load per level.  The first level, a window at
// the interpolated index (a packed region of similar buffers: the answer),
// is loaded by region_probe so that the caller can issue it early.
struct SearchProbe {
  uint64_t w0, e;
};
__device__ __forceinline__ SearchProbe region_probe(const RegionGeom& g, uint64_t A, int lane) {
  const double f = (double)A / (double)(g.re + 1u);
  const uint64_t gi = min((uint64_t)(f * (double)g.n), g.n - 1u);
  const uint64_t w0 = gi > 32u ? gi - 32u : 0u;
  const uint64_t b = min(w0 + (uint64_t)lane, g.n - 1u);
  return SearchProbe{w0, g.rel0 + ldg64(g.offsets, b) + ldg64(g.lengths, b)};
}
__device__ uint64_t region_search(const RegionGeom& g, uint64_t A, int lane, const SearchProbe& p);
__device__ __forceinline__ uint64_t region_search(const RegionGeom& g, uint64_t A, int lane) {
  return region_search(g, A, lane, region_probe(g, A, lane));
}
__device__ uint64_t region_search(const RegionGeom& g, uint64_t A, int lane, const SearchProbe& p) {
  uint64_t lo = 0, hi = g.n;  // every b < lo has e_b <= A; the answer is <= hi
  {
    const uint64_t w0 = p.w0;
    const uint64_t m = __ballot(w0 + (uint64_t)lane < g.n && p.e > A);
    if (m & 1u) {
      if (w0 == 0) return 0;
      hi = w0;  // the answer lies below the window
    } else if (m) {
      return w0 + (uint64_t)__builtin_ctzll(m);
    } else {
      lo = min(w0 + 64u, g.n);  // above it
    }
  }
  while (hi - lo > 64u) {
    const uint64_t step = (hi - lo + 63u) / 64u;
    const uint64_t b = min(lo + (uint64_t)lane * step, hi - 1u);
    const uint64_t e = g.rel0 + ldg64(g.offsets, b) + ldg64(g.lengths, b);
    const uint64_t m = __ballot(e > A);
    if (m == 0) {
      lo = min(lo + 63u * step, hi - 1u) + 1u;
    } else {
      const uint32_t k = (uint32_t)__builtin_ctzll(m);
      const uint64_t pk = min(lo + (uint64_t)k * step, hi - 1u);
      lo = k ? lo + (uint64_t)(k - 1u) * step + 1u : lo;
      hi = pk;
    }
  }
  const uint64_t b = lo + (uint64_t)lane;
  const uint64_t bc = min(b, g.n - 1u);
  const uint64_t e = g.rel0 + ldg64(g.offsets, bc) + ldg64(g.lengths, bc);
  const uint64_t m = __ballot(b < hi && e > A);
  return m ? lo + (uint64_t)__builtin_ctzll(m) : hi;
}

// Chains of U chunks, then per chunk: raw[u] = raw(0, chunk) (wave-uniform)
// and pre[u] = this lane's exclusive prefix, the chunk bytes [0, 64 lane) at
// the chunk end -- Qe(L) of an event on lane L is pre at lane L.
// cp[u][c - 1] = the chain register before word 4c (c = 1, 2, 3): the state
// after 4c words with word 4c XORed in (x_4c = S_4c ^ w[4c]); an event's
// record carries its lane's checkpoint, so the fold kernel re-runs at most 3
// words of the piece instead of 15.  `lsl` = the LDS image shifted so that
// the chain's kSliceOff lands on kRSliceOff.
template <int U>
__device__ __forceinline__ void chains_scan(const uint8_t* lds, const LaneBase& lb, const uint32_t (&w)[U][16],
                                            int lane, uint32_t (&raw)[U], uint32_t (&pre)[U],
                                            uint32_t (&cp)[U][3]) {
  const uint8_t* lsl = lds + (kRSliceOff - kSliceOff);
  uint32_t crc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = w[u][0];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
#pragma unroll
    for (int u = 0; u < U; ++u) crc[u] = slice4_next(lsl, crc[u], k < 15 ? w[u][k + 1] : 0u, lb);
    if (k == 3 || k == 7 || k == 11) {
#pragma unroll
      for (int u = 0; u < U; ++u) cp[u][k >> 2] = crc[u];
    }
  }
  const uint32_t jb = (uint32_t)lane << 2;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t t = to_chunk_end(lds, crc[u], jb, lane);
    const uint32_t inc = xor_scan(t);
    raw[u] = lane_u32(inc, 63u);
    pre[u] = inc ^ t;
  }
}

// This lane's events in the unit [A, B) (its window buffer): in-unit
// positions of its start / end when they are events.
struct LaneEv {
  uint32_t ps, pe;
  bool sv, ev;
};
__device__ __forceinline__ LaneEv lane_events(const Win& w, uint64_t A, uint64_t B) {
  LaneEv le;
  le.sv = w.big && (w.s & (kChunk - 1u)) != 0u && w.s >= A && w.s < B;
  le.ev = w.big && (w.e & (kChunk - 1u)) != 0u && w.e > A && w.e < B;
  le.ps = (uint32_t)(w.s - A);
  le.pe = (uint32_t)(w.e - A);
  return le;
}

// The first event lane of each chunk of the unit (0 when none).  Events are
// in lane order by position (a lane's start before its end).
template <int U>
__device__ __forceinline__ void first_lanes(const LaneEv& le, uint32_t (&Lf)[U]) {
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const bool sk = le.sv && (le.ps >> 12) == (uint32_t)k, ek = le.ev && (le.pe >> 12) == (uint32_t)k;
    const uint64_t m = __ballot(sk || ek);
    Lf[k] = 0u;
    if (m) Lf[k] = (lane_u32(sk ? le.ps : le.pe, (uint32_t)__builtin_ctzll(m)) & (kChunk - 1u)) >> 6;
  }
}

// The events of chunks [ca, ca + cu) (pre[k], cp[k]: chunk ca + k's lane
// prefixes and chain checkpoints): every window lane records its own start
// and end ({Qe, its piece lane's checkpoint x_4c}, one coalesced store) when
// the event sits on its chunk's first event lane -- that lane's values read
// once per chunk; the other events (a second boundary lane in one chunk) go
// one by one.  `w` is the window at `cur`; further windows are loaded while
// the last buffer of the current one still starts before the unit's end.
template <int U>
__device__ __forceinline__ void region_events(const RegionGeom& g, Win w, uint64_t cur, uint64_t ca, uint32_t cu,
                                              const uint32_t (&pre)[U], const uint32_t (&Lf)[U],
                                              const uint32_t (&cp)[U][3], LaneEv le, int lane) {
  const uint64_t A = ca * kChunk, B = (ca + cu) * kChunk;
  uint32_t qf[U], cpf[U][3];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    qf[k] = lane_u32(pre[k], Lf[k]);
#pragma unroll
    for (int m = 0; m < 3; ++m) cpf[k][m] = lane_u32(cp[k][m], Lf[k]);
  }
  // fast record of the event at in-unit position pos (uniform-indexed selects)
  auto rec = [&](uint32_t pos, uint2& r) -> bool {
    const uint32_t k = pos >> 12, L = (pos & (kChunk - 1u)) >> 6, c = (pos >> 4) & 3u;
    uint32_t lf = Lf[0], q = qf[0], x = 0u;
#pragma unroll
    for (int kk = 0; kk < U; ++kk) {
      if (kk) {
        lf = k == (uint32_t)kk ? Lf[kk] : lf;
        q = k == (uint32_t)kk ? qf[kk] : q;
      }
#pragma unroll
      for (int m = 0; m < 3; ++m) x = (k == (uint32_t)kk && c == (uint32_t)m + 1u) ? cpf[kk][m] : x;
    }
    r = make_uint2(q, x);
    return L == lf;
  };
  for (;;) {
    uint2 rs, re;
    const bool fs = le.sv && rec(le.ps, rs), fe = le.ev && rec(le.pe, re);
    if (fs) g.qs[cur + (uint64_t)lane] = make_uint4(rs.x, rs.y, g.gen, (uint32_t)(cur + (uint64_t)lane));
    if (fe) g.qe[cur + (uint64_t)lane] = make_uint4(re.x, re.y, g.gen, (uint32_t)(cur + (uint64_t)lane));
    const uint64_t ms = __ballot(le.sv && !fs), me = __ballot(le.ev && !fe);
    uint64_t all = ms | me;
    while (all) {  // events on another lane than their chunk's first
      const uint32_t j = (uint32_t)__builtin_ctzll(all);
      all &= all - 1u;
#pragma unroll
      for (int t = 0; t < 2; ++t) {  // start, then end
        if (!(((t ? me : ms) >> j) & 1u)) continue;
        const uint32_t pos = lane_u32(t ? le.pe : le.ps, j);
        const uint32_t k = pos >> 12, L = (pos & (kChunk - 1u)) >> 6, c = (pos >> 4) & 3u;
        uint32_t v = pre[0], x = 0u;
#pragma unroll
        for (int q = 0; q < U; ++q) {
          if (q) v = k == (uint32_t)q ? pre[q] : v;
#pragma unroll
          for (int m = 0; m < 3; ++m) x = (k == (uint32_t)q && c == (uint32_t)m + 1u) ? cp[q][m] : x;
        }
        const uint4 r = make_uint4(lane_u32(v, L), lane_u32(x, L), g.gen, (uint32_t)(cur + j));
        if (lane == 0) (t ? g.qe : g.qs)[cur + j] = r;
      }
    }
    if (cur + 64u >= g.n || lane_u64(w.s, 63) >= B) break;
    cur += 64u;  // the unit's buffers run past the window (short buffers): the next one
    w = make_win(g, load_win(g, cur, lane), cur, lane);
    le = lane_events(w, A, B);
  }
}

__device__ __forceinline__ uint32_t fold_slice4(const uint32_t* t, uint32_t x) {
  return t[768u + (x & 255u)] ^ t[512u + ((x >> 8) & 255u)] ^ t[256u + ((x >> 16) & 255u)] ^ t[x >> 24];
}
__device__ __forceinline__ uint32_t fold_step1(const uint32_t* t, uint32_t crc, uint32_t b) {
  return t[(crc ^ b) & 255u] ^ (crc >> 8);
}

// raw(s, [p, p + L)) serially: bytes to a 4-byte boundary, STEP4 words (32
// bytes' loads in flight at a time), bytes.
__device__ uint32_t serial_raw(const uint32_t* t, uint32_t crc, const uint8_t* p, uint64_t L) {
  while (L && ((uintptr_t)p & 3u)) {
    crc = fold_step1(t, crc, *p++);
    --L;
  }
  for (; L >= 32; L -= 32, p += 32) {
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = reinterpret_cast<const uint32_t*>(p)[k];
#pragma unroll
    for (int k = 0; k < 8; ++k) crc = fold_slice4(t, crc ^ w[k]);
  }
  for (; L >= 4; L -= 4, p += 4) crc = fold_slice4(t, crc ^ *reinterpret_cast<const uint32_t*>(p));
  while (L--) crc = fold_step1(t, crc, *p++);
  return crc;
}

// R = raw(0, the first o bytes of a 64-byte piece), o = 16c + 4m + r, from
// the chunk kernel's checkpoint x (x_4c = S_4c ^ w[4c]; c = 0: S_0 = 0) and
// the piece's 16-byte quad c: at most 3 words and 3 bytes, fixed trip count.
__device__ __forceinline__ uint32_t quad_prefix(const uint32_t* t, uint32_t x, const u32x4& v, uint32_t o) {
  const uint32_t c = o >> 4, m = (o >> 2) & 3u, r = o & 3u;
  uint32_t crc = c ? x ^ v[0] : 0u, cur = v[0];
#pragma unroll
  for (uint32_t j = 0; j < 3u; ++j) {
    const uint32_t nx = fold_slice4(t, crc ^ v[j]);
    crc = j < m ? nx : crc;
    cur = j + 1u == m ? v[j + 1u] : cur;
  }
#pragma unroll
  for (uint32_t b = 0; b < 3u; ++b) {
    const uint32_t nx = fold_step1(t, crc, (cur >> (8u * b)) & 255u);
    crc = b < r ? nx : crc;
  }
  return crc;
}

__device__ __forceinline__ uint32_t fold_sh4096(const uint32_t* sh, uint32_t acc) {
  return sh[acc & 255u] ^ sh[256u + ((acc >> 8) & 255u)] ^ sh[512u + ((acc >> 16) & 255u)] ^ sh[768u + (acc >> 24)];
}

// The fold of one region buffer, in two halves.  fold_in: what depends on
// the batch alone -- its metadata, the two 16-byte quads re-read for the
// piece prefixes R (the end's clamped into the grid when it is a chunk end),
// the powers -- issued before the workgroup's last unit is done.  fold_out:
// the chunk raws and gen-tagged event records this workgroup wrote (after
// its barrier), then the arithmetic; false when a record is missing (not
// written by this call: the batch was not region-shaped there) -- the
// caller then checksums the buffer serially.
struct FoldIn {
  uint64_t s, L;
  uint32_t ninit, xs, xe, xt;  // x^(8(4096 - os)), x^(-8(4096 - oe)), x^(8L) (one or two chunks)
  u32x4 vs, ve;
  bool fast;  // inside the region, >= kRegionDirect bytes, every chunk streamed by this workgroup
};
__device__ __forceinline__ FoldIn fold_in(const RegionGeom& g, const uint32_t* tables, uint64_t i, uint64_t c0w,
                                          uint64_t B1) {
  FoldIn f;
  const uint64_t off = ldg64(g.offsets, i), L = ldg64(g.lengths, i);
  f.ninit = ~(g.init ? g.init[i] : g.init_all);
  f.s = g.rel0 + off;
  f.L = L;
  const bool inside = f.s >= g.rs && f.s <= g.re && L <= g.re - f.s;
  f.fast = inside && L >= kRegionDirect && (f.s >> 12) >= c0w && ((f.s + L - 1u) >> 12) < B1;
  const uint64_t s = f.fast ? f.s : 0u, e = f.fast ? f.s + L : 64u;  // (the grid's first chunk otherwise)
  const uint64_t c1 = (e - 1u) >> 12;
  const uint32_t os = (uint32_t)(s & (kChunk - 1u)), oe = (uint32_t)(e - (c1 << 12));  // oe in [1, 4096]
  f.vs = ld16c((uintptr_t)g.grid + (s & ~(uint64_t)15));
  f.ve = ld16c((uintptr_t)g.grid + (oe == kChunk ? e - 16u : (e & ~(uint64_t)15)));
  f.xs = tables[kTabXp8 + kChunk - os];
  f.xe = tables[kTabXm8 + (kChunk - oe)];
  const uint64_t c0 = s >> 12;
  f.xt = tables[kTabXp8 + (c1 <= c0 + 1u ? e - s : 0u)];  // (L <= 8192 there)
  return f;
}

// quad_prefix over the LDS slice replicas (lsl, lb: as the chains).
__device__ __forceinline__ uint32_t quad_prefix_lds(const uint8_t* lsl, const LaneBase& lb, uint32_t x, const u32x4& v,
                                                    uint32_t o) {
  const uint32_t c = o >> 4, m = (o >> 2) & 3u, r = o & 3u;
  uint32_t crc = c ? x ^ v[0] : 0u, cur = v[0];
#pragma unroll
  for (uint32_t j = 0; j < 3u; ++j) {
    const uint32_t nx = slice4(lsl, crc ^ v[j], lb);
    crc = j < m ? nx : crc;
    cur = j + 1u == m ? v[j + 1u] : cur;
  }
  const uint8_t* sl = lsl + kSliceOff;
#pragma unroll
  for (uint32_t b = 0; b < 3u; ++b) {  // T0[(crc ^ byte) & 255] ^ crc >> 8 (table 0 = byte 3's slot of slice4)
    const uint32_t nx = lds_u32(sl, __builtin_amdgcn_perm(crc ^ (cur >> (8u * b)), lb.t0, 0x0C020400u)) ^ (crc >> 8);
    crc = b < r ? nx : crc;
  }
  return crc;
}

// gf_mul(a, b) (crc32c_math.h) by bytes of a, Horner in x^8: with
// B_j = b x^j (j < 8), C_k = sum_j a_{8k+j} B_j, a b = C_0 ^ x^8 (C_1 ^ x^8 (C_2
// ^ x^8 C_3)), and v x^8 = T0[v & 255] ^ v >> 8 -- one LDS lookup (slice
// table 0's replica) per byte instead of eight shift-reduce steps.  Bit
// 31 - i of a is its x^i coefficient (reflected).
__device__ __forceinline__ uint32_t gf_mul_lds(const uint8_t* lsl, const LaneBase& lb, uint32_t a, uint32_t b) {
  uint32_t B[8];
  B[0] = b;
#pragma unroll
  for (int j = 1; j < 8; ++j)
    B[j] = (B[j - 1] >> 1) ^ ((uint32_t)__builtin_amdgcn_sbfe((int)B[j - 1], 0, 1) & kPolyReflected);
  const uint8_t* sl = lsl + kSliceOff;
  uint32_t p = 0u;
#pragma unroll
  for (int k = 3; k >= 0; --k) {
    if (k < 3) p = lds_u32(sl, __builtin_amdgcn_perm(p, lb.t0, 0x0C020400u)) ^ (p >> 8);  // p x^8
#pragma unroll
    for (int j = 0; j < 8; ++j) p ^= (uint32_t)__builtin_amdgcn_sbfe((int)a, 31 - (8 * k + j), 1) & B[j];
  }
  return p;
}

// shift(v, 64 (63 - j)) through column j of the nibble tables (jb = 4j).
__device__ __forceinline__ uint32_t col_shift(const uint8_t* lds, uint32_t v, uint32_t jb) {
  const uint32_t lo = v & 0x0F0F0F0Fu, hi = (v >> 4) & 0x0F0F0F0Fu;
  const uint8_t* nb = lds + kRNibOff;
  const uint32_t r0 = lds_u32(nb + 0u * 4096u, __builtin_amdgcn_perm(lo, jb, 0x0C0C0400u));
  const uint32_t r1 = lds_u32(nb + 1u * 4096u, __builtin_amdgcn_perm(hi, jb, 0x0C0C0400u));
  const uint32_t r2 = lds_u32(nb + 2u * 4096u, __builtin_amdgcn_perm(lo, jb, 0x0C0C0500u));
  const uint32_t r3 = lds_u32(nb + 3u * 4096u, __builtin_amdgcn_perm(hi, jb, 0x0C0C0500u));
  const uint32_t r4 = lds_u32(nb + 4u * 4096u, __builtin_amdgcn_perm(lo, jb, 0x0C0C0600u));
  const uint32_t r5 = lds_u32(nb + 5u * 4096u, __builtin_amdgcn_perm(hi, jb, 0x0C0C0600u));
  const uint32_t r6 = lds_u32(nb + 6u * 4096u, __builtin_amdgcn_perm(lo, jb, 0x0C0C0700u));
  const uint32_t r7 = lds_u32(nb + 7u * 4096u, __builtin_amdgcn_perm(hi, jb, 0x0C0C0700u));
  return xor3(xor3(r0, r1, r2), xor3(r3, r4, r5), r6) ^ r7;
}

// shift(acc, 4096) as two column shifts, 64 a and 64 (64 - a) bytes with
// a = (lane & 31) + 1: the 32 lanes of a half read 32 distinct columns
// (banks) -- one shared column would serialise them.
__device__ __forceinline__ uint32_t sh4096_lds(const uint8_t* lds, uint32_t acc, int lane) {
  const uint32_t a = ((uint32_t)lane & 31u) + 1u;
  return col_shift(lds, col_shift(lds, acc, (63u - a) << 2), (a - 1u) << 2);
}

__device__ __forceinline__ bool fold_out(const RegionGeom& g, const uint8_t* lds, const uint8_t* lsl,
                                         const LaneBase& lb, int lane, const FoldIn& f, const uint4& q_s,
                                         const uint4& q_e, uint32_t ti, uint32_t& v) {
  const uint64_t s = f.s, e = f.s + f.L;
  const uint64_t c0 = s >> 12, c1 = (e - 1u) >> 12;
  const uint32_t os = (uint32_t)(s & (kChunk - 1u)), oe = (uint32_t)(e - (c1 << 12));  // oe in [1, 4096]
  const uint32_t r0 = g.raws[c0], r1 = g.raws[c1], rm = g.raws[min(c0 + 1u, c1)];
  if ((os && (q_s.z != g.gen || q_s.w != ti)) || (oe != kChunk && (q_e.z != g.gen || q_e.w != ti))) return false;
  const uint32_t qs = os ? q_s.x : 0u;                                   // chunk c0's bytes before s, at its end
  const uint32_t T = (os ? quad_prefix_lds(lsl, lb, q_s.y, f.vs, s & 63u) : 0u) ^ f.ninit;  // R(s) ^ ~init, at s
  const uint32_t ze = oe == kChunk ? r1 : q_e.x;                         // chunk c1's bytes before e, at its end
  const uint32_t re = oe == kChunk ? 0u : quad_prefix_lds(lsl, lb, q_e.y, f.ve, e & 63u);  // R(e), at e
  if (c1 <= c0 + 1u) {
    // one or two chunks, one formula (a slice holding both kinds would run
    // both branches): the data terms at chunk c1's end -- Qe(s) (one chunk)
    // or shift4096(Qe(s) ^ raw c0) (two) -- ^ Ze, unshifted to e, and T
    // straight to e:  (X ^ Ze) x^(-8(4096 - oe)) ^ T x^(8L) ^ R(e)
    // (for two chunks x^(-8(4096 - oe)) x^(8(8192 - os)) = x^(8L))
    const uint32_t sh = sh4096_lds(lds, qs ^ r0, lane);
    v = gf_mul_lds(lsl, lb, f.xe, (c1 == c0 ? qs : sh) ^ ze) ^ gf_mul_lds(lsl, lb, f.xt, T) ^ re;
    return true;
  }
  // Longer: Ze'(s) = Qe(s) ^ T x^(8(4096 - os)) at chunk c0's end, the chunks in between, unshifted from c1's end
  uint32_t acc = qs ^ gf_mul_lds(lsl, lb, f.xs, T) ^ r0;
  acc = sh4096_lds(lds, acc, lane) ^ rm;
  for (uint64_t c = c0 + 2u; c < c1; c += 4u) {  // further chunks in between, four loads at a time
    uint32_t rr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) rr[k] = g.raws[min(c + (uint64_t)k, c1)];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c + (uint64_t)k < c1) acc = sh4096_lds(lds, acc, lane) ^ rr[k];
  }
  acc = sh4096_lds(lds, acc, lane);
  v = gf_mul_lds(lsl, lb, f.xe, acc ^ ze) ^ re;
  return true;
}

// LDS slots in the region image's lane-63 column (never read by the lane
// shifts): row r at r * 256 + 252.  Row 16 (T[1][0][63]) is 0 in the blob.
// (generic pointer: the volatile accesses become flat loads, which count in
// vmcnt as well; an LDS-qualified pointer was measured slower, see load_unit)
typedef volatile uint32_t lds_vu32;
__device__ __forceinline__ lds_vu32* region_slot(uint8_t* lds, uint32_t r) {
  return (lds_vu32*)(lds + kRNibOff + r * 256u + 252u);
}
constexpr uint32_t kSlotOwnLo = 1, kSlotOwnHi = 2, kSlotEndLo = 3, kSlotEndHi = 4, kSlotHalo = 5;
// (rows 16, 32, 48, 64, 80, 96: T[n][0][63] = 0 in the blob; row 96 counts the
// workgroup's waves per SIMD, one byte each)
constexpr uint32_t kSlotReady = 16, kSlotTail = 32, kSlotWaves = 96;

// Scheduler A over the region's chunks, and the per-buffer fold in the same
// launch.  Workgroup b owns the chunk range [B0, B1) and the buffers
// [I_b, I_b+1), I_b = the first buffer ending after chunk B0's start (I_0 = 0,
// I_G = n): every buffer's end event lies in its owner's range.  The one
// owned buffer that starts in an earlier range (I_b) has its chunks there
// re-streamed by the owner ("halo" units after its own), so the fold needs
// nothing from another workgroup: after its units the workgroup folds its
// buffers from the records and raws it wrote itself.  Its waves pull 2-chunk
// units from an LDS counter; the next unit's chunks and metadata window are
// in flight while this one computes.
//
// Any batch comes out right: the owned ranges of the workgroups cover
// [0, n) whatever the searches return (I_0 = 0 <= x < n = I_G), a record
// carries this call's generation only when this call wrote it, and a buffer
// without its records or with chunks outside the workgroup's streamed range
// is checksummed serially (unsorted or overlapping batches: correct, slow).
// Buffers must lie inside the region (the entry point's contract).
constexpr uint32_t kRTail = 8;  // single-chunk units at the end of a range (64 / 16 / 8 / 0 A/B'd: DESIGN §3.7)

template <int U>
__device__ __forceinline__ void run_region(const RegionGeom& g, const KArgs& ka, uint8_t* lds, uint32_t G) {
  NVL_TL_DECL();
  NVL_TL(0);
  const int lane = threadIdx.x & 63;
  const uint32_t wv = uniform_u32(threadIdx.x >> 6);
  const uint64_t B0 = g.nc * blockIdx.x / G;  // (G workgroups: blockIdx.x < G)
  const uint64_t B1 = g.nc * (blockIdx.x + 1) / G;
  const uint32_t cnt = (uint32_t)(B1 - B0);
  const uint32_t nfull = cnt > kRTail ? (cnt - kRTail) / U : 0u;
  const uint32_t nunits = nfull + (cnt - nfull * U);
  // Unit u's chunks [first, first + count): own units from [B0, B1), halo
  // units (u >= nunits) from the halo [C0, B0) that wave 0 publishes after
  // the LDS fill barrier.  One function gives both, and a halo unit's first
  // chunk is formed only after the published halo has been read: a halo
  // unit never addresses a chunk from an origin it has not read.  (Round 4
  // computed them in two lambdas whose halo origin was valid only when the
  // count was asked first; a variant that called them the other way round
  // addressed chunks past the region -- DESIGN.md §3.7.)  Every chunk of a
  // unit lies in [C0, B1) with C0 <= B0 <= B1 <= nc (tests/kernel_model.py
  // region_schedule asserts it, zero-chunk workgroups and one-buffer
  // batches included); a unit with count 0 loads nothing.
  uint64_t C0 = B0;      // the halo's first chunk -- valid once nhalo != ~0u
  uint32_t nhalo = ~0u;  // halo units, ~0u until read
  auto span_of = [&](uint32_t u, uint64_t& first) -> uint32_t {
    if (u < nunits) {
      first = u < nfull ? B0 + (uint64_t)u * U : B0 + (uint64_t)nfull * U + (u - nfull);
      return u < nfull ? (uint32_t)U : 1u;
    }
    if (nhalo == ~0u) {  // wave 0 publishes right after the LDS fill: long done by now
      uint32_t r;
      while ((r = *region_slot(lds, kSlotReady)) == 0u) __builtin_amdgcn_s_sleep(1);
      nhalo = uniform_u32(r - 1u);
      const uint64_t h = *region_slot(lds, kSlotHalo);
      C0 = B0 - uniform_u64(h);
    }
    first = B0;
    if (u - nunits >= nhalo) return 0u;
    first = C0 + (uint64_t)(u - nunits) * U;
    return (uint32_t)min((uint64_t)U, B0 - first);
  };
  // (Loads behind the branch: the compiler then waits vmcnt(0) at the top
  // of the unit, the next unit's chunks included.  Unconditional loads with
  // exact wait counts were measured 1.5-2 us slower on v / r -- waves that
  // run further ahead only queue more requests -- and were rejected.)
  auto load_unit = [&](uint64_t ca, uint32_t cu, Chunk (&ch)[U]) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if ((uint32_t)k >= cu) continue;
      const uint64_t c = ca + (uint64_t)k;
      const uintptr_t cs = (uintptr_t)g.grid + c * kChunk;
      const uint32_t lo = lane_load_off(lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const u32x4 v = ld16(cs + 1024u * (uint32_t)j + lo);
        ch[k].d[4 * j + 0] = v.x; ch[k].d[4 * j + 1] = v.y; ch[k].d[4 * j + 2] = v.z; ch[k].d[4 * j + 3] = v.w;
      }
    }
  };

  // First unit pre-assigned.  Issue order matters: vmcnt retires in order,
  // so what the waves wait for before the fill barrier -- the table blob
  // and the search's first probe -- goes out ahead of the unit's chunks.
  // (Two pre-assigned units per wave, 64 MB in flight at the start, delayed
  // the probes' return to ~10 us and lost ~8 us: rejected.)
  uint32_t u = wv;
  uint64_t ca = B0;  // (a wave without a pre-assigned unit pulls one after the barrier)
  uint32_t cu = u < nunits ? span_of(u, ca) : 0u;
  uint32_t un = 0u, cun = 0u;
  uint64_t can = 0u;
  Chunk cur[U], nxt[U];
  const RegionFill fill = fill_region_load(ka.tables);
  const SearchProbe probe = region_probe(g, ca * kChunk, lane);
  asm volatile("" ::: "memory");
  load_unit(ca, cu, cur);
  // The first search after the LDS fill barrier, which then waits for the
  // fill alone (r 68.75 -> 68.25 us, v 72.58 -> 72.42 us in interleaved A/B).
  fill_region_store(lds, fill, min(nunits, (uint32_t)kWavesPerWG));
  __syncthreads();
  NVL_TL(1);
  // this wave's SIMD (HW_ID bits 5:4), counted for the fold's slice dealing
  const uint32_t simd = uniform_u32(__builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4) & 3u);
  if (lane == 0)
    __hip_atomic_fetch_add(const_cast<uint32_t*>(region_slot(lds, kSlotWaves)), 1u << (8u * simd), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
  uint64_t cursor = cu ? region_search(g, ca * kChunk, lane, probe) : g.n;
  NVL_TL(6);
  WinRaw wr = load_win(g, cursor, lane);
  // wave 0, after the barrier (searches before it held every wave there):
  // the owned buffers [I_b, I_b+1) -- I_b is its own first cursor -- and the
  // halo (the chunks of I_b before B0), published for the halo units and
  // the fold; its first unit's loads are in flight meanwhile
  if (wv == 0) {
    const uint64_t Ib = blockIdx.x == 0 ? 0u : (cu ? cursor : region_search(g, B0 * kChunk, lane));
    const uint64_t Ib1 = blockIdx.x + 1u == G ? g.n : region_search(g, B1 * kChunk, lane);
    const uint64_t sb = Ib < g.n ? g.rel0 + ldg64(g.offsets, Ib) : 0u;
    const uint64_t hc = (Ib < Ib1 && sb < B0 * kChunk) ? B0 - (sb >> 12) : 0u;  // halo chunks
    if (lane == 0) {
      *region_slot(lds, kSlotOwnLo) = (uint32_t)Ib;
      *region_slot(lds, kSlotOwnHi) = (uint32_t)(Ib >> 32);
      *region_slot(lds, kSlotEndLo) = (uint32_t)Ib1;
      *region_slot(lds, kSlotEndHi) = (uint32_t)(Ib1 >> 32);
      *region_slot(lds, kSlotHalo) = (uint32_t)hc;
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      *region_slot(lds, kSlotReady) = (uint32_t)((hc + U - 1u) / U) + 1u;
    }
  }
  const LaneBase lb = make_lane_base(lane);
  if (!cu) {  // no pre-assigned unit (a range of fewer than 16 units): pull one, maybe a halo unit
    u = pull_unit(lds, lane, kRCtrOff);
    cu = span_of(u, ca);
    load_unit(ca, cu, cur);
    cursor = cu && u < nunits ? region_search(g, ca * kChunk, lane) : g.n;
    wr = load_win(g, cursor, lane);
  }

  // Per unit: the next unit is pulled and its chunks go out (in flight
  // while this one computes), this unit's window (loaded a unit ago) gives
  // the next unit's cursor and window load, this unit computes -- one fixed
  // count of loads per unit.  (Loads at the end of the unit, ping-pong
  // buffers: 8 % slower on v, rejected.)
  while (cu) {
    un = pull_unit(lds, lane, kRCtrOff);
    cun = span_of(un, can);
    load_unit(can, cun, nxt);
    const bool halo = u >= nunits;
    const Win w = make_win(g, wr, cursor, lane);
    uint64_t ncur = g.n;
    if (cun && un < nunits) {  // the next unit's cursor: the first buffer of this window ending after its start
      const uint64_t m = __ballot(w.valid && w.e > can * kChunk);
      ncur = m ? cursor + (uint64_t)__builtin_ctzll(m) : min(cursor + 64u, g.n);
    }
    const WinRaw nwr = load_win(g, ncur, lane);

    const LaneEv le = lane_events(w, ca * kChunk, (ca + cu) * kChunk);
    const bool any_ev = !halo && __ballot(le.sv || le.ev) != 0u;
    uint32_t Lf[U];
#pragma unroll
    for (int k = 0; k < U; ++k) Lf[k] = 0u;
    if (any_ev) first_lanes<U>(le, Lf);
    uint32_t raw[U], pre[U], cp[U][3];
    if (cu == (uint32_t)U) {
      uint32_t wd[U][16];
#pragma unroll
      for (int k = 0; k < U; ++k) {
#pragma unroll
        for (int q = 0; q < 16; ++q) wd[k][q] = cur[k].d[q];
        row_transpose(wd[k]);
      }
      chains_scan<U>(lds, lb, wd, lane, raw, pre, cp);
    } else {  // the range's single-chunk units
      uint32_t wd[1][16], r1[1], p1[1], c1[1][3];
#pragma unroll
      for (int q = 0; q < 16; ++q) wd[0][q] = cur[0].d[q];
      row_transpose(wd[0]);
      chains_scan<1>(lds, lb, wd, lane, r1, p1, c1);
#pragma unroll
      for (int k = 0; k < U; ++k) {
        raw[k] = r1[0];
        pre[k] = p1[0];
#pragma unroll
        for (int m = 0; m < 3; ++m) cp[k][m] = c1[0][m];
      }
    }
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < U; ++k)
        if ((uint32_t)k < cu) g.raws[ca + k] = raw[k];
    }
    if (halo) {
      if (ca == C0) {  // the halo's first chunk holds I_b's start: its one record
        const uint64_t ib = ((uint64_t)*region_slot(lds, kSlotOwnHi) << 32) | *region_slot(lds, kSlotOwnLo);
        const uint64_t s = g.rel0 + ldg64(g.offsets, uniform_u64(ib));
        const uint32_t os = uniform_u32((uint32_t)(s & (kChunk - 1u)));
        if (os) {
          const uint32_t L = os >> 6, c = (os >> 4) & 3u;
          const uint32_t x = c == 1u ? cp[0][0] : (c == 2u ? cp[0][1] : cp[0][2]);
          const uint4 r = make_uint4(lane_u32(pre[0], L), c ? lane_u32(x, L) : 0u, g.gen, (uint32_t)ib);
          if (lane == 0) g.qs[ib] = r;
        }
      }
    } else if (any_ev || (cursor + 64u < g.n && lane_u64(w.s, 63) < (ca + cu) * kChunk)) {
      // (a unit with no event and no buffer running past its window -- most
      // of config 3's -- has nothing to record)
      region_events<U>(g, w, cursor, ca, cu, pre, Lf, cp, le, lane);
    }

    u = un;
    ca = can;
    cu = cun;
    cursor = ncur;
    wr = nwr;
#pragma unroll
    for (int k = 0; k < U; ++k) cur[k] = nxt[k];
  }

  // The fold of the owned buffers, one thread each, from this workgroup's
  // own records and raws (visible after the barrier), in 64-buffer slices
  // claimed from an LDS counter: a wave claims its first slice as it runs
  // out of units and has that slice's batch-only inputs in flight across the
  // barrier, so the last waves to finish find the slices taken.
  NVL_TL(2);
  uint32_t r;
  while ((r = *region_slot(lds, kSlotReady)) == 0u) __builtin_amdgcn_s_sleep(1);  // (wave 0 has published)
  const uint64_t ib = ((uint64_t)*region_slot(lds, kSlotOwnHi) << 32) | *region_slot(lds, kSlotOwnLo);
  const uint64_t ib1 = ((uint64_t)*region_slot(lds, kSlotEndHi) << 32) | *region_slot(lds, kSlotEndLo);
  const uint64_t c0w = B0 - *region_slot(lds, kSlotHalo);  // the first chunk streamed here
  const uint64_t nsl = ib1 > ib ? (ib1 - ib + 63u) / 64u : 0u;
  // slices k = s (mod 4) go to the waves on SIMD s: the fold is VALU-bound,
  // so a SIMD holding two folding waves finishes last.  A SIMD that holds
  // none of the workgroup's waves (at <= 64 VGPRs a SIMD may take 5+ of the
  // 16, or another kernel's waves may fill one) has its slices adopted by
  // the waves of the lowest populated SIMD once their own run out (the wave
  // counts are complete at the fold barrier), so every slice is claimed.
  uint32_t cs = simd;  // the SIMD whose slices this wave claims
  auto claim = [&]() -> uint64_t {
    uint32_t v = 0;
    if (lane == 0)
      v = __hip_atomic_fetch_add(const_cast<uint32_t*>(region_slot(lds, kSlotTail + 16u * cs)), 1u,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return (uint64_t)cs + 4u * (uint64_t)uniform_u32(v);
  };
  uint64_t k = claim();
  FoldIn f;
  if (k < nsl) f = fold_in(g, ka.tables, min(ib + 64u * k + (uint64_t)lane, ib1 - 1u), c0w, B1);
  __syncthreads();
  NVL_TL(3);
  const uint8_t* lsl = lds + (kRSliceOff - kSliceOff);
  uint32_t adopt = 0u;  // empty SIMDs whose slices this wave takes over
  {
    const uint32_t wc = *region_slot(lds, kSlotWaves);
    uint32_t empty = 0u;
#pragma unroll
    for (uint32_t j = 0; j < 4u; ++j) empty |= ((wc >> (8u * j)) & 255u) == 0u ? 1u << j : 0u;
    adopt = simd == (uint32_t)__builtin_ctz(~empty & 15u) ? uniform_u32(empty) : 0u;
  }
  for (;;) {
    while (k < nsl) {
      const uint64_t i = ib + 64u * k + (uint64_t)lane;
      if (i < ib1) {
        const uint4 q_s = g.qs[i], q_e = g.qe[i];  // (not written for a buffer without that event: unused then)
        NVL_TL_WAIT(4, q_s.x);
        uint32_t v = 0u;
        if (!(f.fast && fold_out(g, lds, lsl, lb, lane, f, q_s, q_e, (uint32_t)i, v)))
          v = serial_raw(ka.tables + kGSlice, f.ninit, g.grid + f.s, f.L);  // (outside the region too: the caller's memory)
        NVL_TL_WAIT(5, v);
        ka.out[i] = finish(~v, ka.flags);
      }
      k = claim();
      if (k < nsl) f = fold_in(g, ka.tables, min(ib + 64u * k + (uint64_t)lane, ib1 - 1u), c0w, B1);
    }
    if (!adopt) break;
    cs = (uint32_t)__builtin_ctz(adopt);
    adopt &= adopt - 1u;
    k = claim();
    if (k < nsl) f = fold_in(g, ka.tables, min(ib + 64u * k + (uint64_t)lane, ib1 - 1u), c0w, B1);
  }
  NVL_TL_END();
}

__global__ __launch_bounds__(kThreads, 1) void crc32c_region_kernel(RegionGeom g, KArgs ka) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kRLdsBytes];
  run_region<kFastU>(g, ka, lds, gridDim.x);
}

// ---------------------------------------------------------------------------
// Routed batches: one plan, then the region path or the batch path.
//
// A batch over device metadata is region-shaped when its buffers are sorted
// by offset and do not overlap (table/format.cc:90-92 over a table image in
// file order, db/log_reader.cc:255-256 over a log's records, a packed batch),
// none is longer than kRegionMaxLen (a longer one would be re-streamed as a
// halo and folded serially by its owner), and -- for nvl_crc32c_batch_dev,
// whose region is the batch's own span -- no page of the span is without a
// buffer byte and the gaps are few bytes against the buffer bytes (the
// region path reads the gaps).  Only the
// device knows, so a call is three launches: crc32c_route_plan (partials),
// crc32c_route_kernel (the region path, or the head kernel's work) and
// crc32c_var_fused_kernel (returns at once on the region path).
// Partial k: buffers [n k / P, n (k+1) / P) and each one's successor (four
// pairs per thread and step, their loads issued together: the plan is a
// latency-bound scan).  Bad: a pair out of order or overlapping, a length
// over kRegionMaxLen, a buffer outside [0, lim) (region_dev: lim =
// region_len; batch_dev: ~0, i.e. only a wrapping end).  batch_dev (`pages`)
// also: a 4 KiB page of the batch's span that holds no buffer byte -- the
// region path reads every page of the span, and only the pages a buffer
// touches are known to be mapped (two buffers from different allocations
// may have an unmapped page between them).  Page-wise, in address space
// (A(x) = base + x): a non-empty buffer starts at most one page after the
// page of the previous buffer's last byte, an empty one no later than that
// byte's page ends (page(A(o) - 1) <= page(A(e_prev) - 1)), and the first
// buffer is not empty -- so the last byte's page of every prefix is touched
// and no page is skipped.
constexpr uint32_t kPlanT = 512, kPlanPer = 2;  // (shapes A/B'd: tools/diag/abl_plan.sh)
__global__ __launch_bounds__(kPlanT) void crc32c_route_plan(const uint64_t* __restrict__ off,
                                                           const uint64_t* __restrict__ len, uint64_t n, uint64_t lim,
                                                           uintptr_t base, uint32_t pages,
                                                           RoutePart* __restrict__ parts) {
  __shared__ uint64_t wsum[kPlanT / kWave];
  __shared__ uint32_t wbad[kPlanT / kWave];
  const uint64_t P = gridDim.x, k = blockIdx.x;
  const uint64_t i0 = n * k / P, i1 = n * (k + 1) / P;
  uint64_t sum = 0;  // (lengths capped at kRegionMaxLen + 1: a longer one makes the slice bad anyway)
  bool bad = false, not4k = false, unal = false;
  for (uint64_t b = i0 + (uint64_t)threadIdx.x * kPlanPer; b < i1; b += (uint64_t)kPlanT * kPlanPer) {
    uint64_t o[kPlanPer + 1], L[kPlanPer + 1];
#pragma unroll
    for (uint32_t q = 0; q <= kPlanPer; ++q) o[q] = off[min(b + q, n - 1u)];  // (clamped: every load issued)
#pragma unroll
    for (uint32_t q = 0; q <= kPlanPer; ++q) L[q] = len[min(b + q, n - 1u)];
#pragma unroll
    for (uint32_t q = 0; q < kPlanPer; ++q) {
      if (b + q >= i1) break;
      const uint64_t e = o[q] + L[q];
      bad |= e < o[q] || L[q] > kRegionMaxLen || o[q] > lim || L[q] > lim - o[q];
      if (b + q + 1u < n) {
        bad |= e > o[q + 1];
        if (pages) {
          const bool nz = L[q + 1] != 0u;
          const uint64_t pn = ((uint64_t)base + o[q + 1] - (nz ? 0u : 1u)) >> 12;
          const uint64_t pe = ((uint64_t)base + e - 1u) >> 12;
          bad |= pn > pe + (nz ? 1u : 0u);
        }
      }
      if (pages && b + q == 0u) bad |= L[q] == 0u;
      not4k |= L[q] != (uint64_t)kChunk;
      unal |= ((base + o[q]) & 15u) != 0u;
      sum += min<uint64_t>(L[q], kRegionMaxLen + 1u);
    }
  }
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint64_t tot = wave_total_u64(sum);
  const uint32_t wb = (__ballot(bad) ? (uint32_t)kRpBad : 0u) | (__ballot(not4k) ? (uint32_t)kRpNot4k : 0u) |
                      (__ballot(unal) ? (uint32_t)kRpUnaligned : 0u);
  if (lane == 0u) {
    wsum[w] = tot;
    wbad[w] = wb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t s = 0, bb = 0;
#pragma unroll
    for (uint32_t v = 0; v < kPlanT / kWave; ++v) {
      s += wsum[v];
      bb |= wbad[v];
    }
    parts[k] = RoutePart{s, bb};
  }
}

// The second launch of a routed call: the region path over the batch (its
// geometry from the plan for batch_dev), or the head kernel's work.  Launched
// with one workgroup per CU; the region path runs on the region grid
// (grid_for), the head work on the plan's tiles; the other workgroups return.
__global__ __launch_bounds__(kThreads, 1) void crc32c_route_kernel(RegionGeom rg, VarGeom vg, KArgs ka) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kHeadLdsBytes > kRLdsBytes ? kHeadLdsBytes : kRLdsBytes];
  uint64_t lo, hi;
  // (workgroup 0 stores the verdict for the body kernel: one word after the
  // partials, written in each branch so nothing extra stays live)
  uint64_t* const verdict = &const_cast<RoutePart*>(ka.route.parts)[kRoutePlanMax].bad;
  if (route_region(ka.route, lo, hi)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *verdict = kRouteRegion;
    if (ka.route.dyn) {
      const uintptr_t base = (uintptr_t)ka.route.base, start = base + lo;
      const uintptr_t O = start & ~(uintptr_t)(kChunk - 1u);
      rg.grid = reinterpret_cast<const uint8_t*>(O);
      rg.rel0 = (uint64_t)(base - O);  // (wrapping: buffer i at rel0 + offsets[i] >= start - O)
      rg.rs = (uint64_t)(start - O);
      rg.re = (uint64_t)(base + hi - O);
      rg.nc = (rg.re + kChunk - 1u) / kChunk;
    }
    const uint64_t gw = (rg.nc + kWavesPerWG - 1u) / kWavesPerWG;  // (the host's grid_for)
    const uint32_t G = (uint32_t)max<uint64_t>(1u, min<uint64_t>(gridDim.x, gw));
    if (blockIdx.x >= G) return;
    run_region<kFastU>(rg, ka, lds, G);
  } else {
    const int kind = route_other(ka.route);
    if (blockIdx.x == 0 && threadIdx.x == 0) *verdict = (uint64_t)kind;
    if (kind != kRouteHeads || blockIdx.x >= ka.tile_G) return;
    run_heads(vg, ka, lds);
  }  // (the page path runs in crc32c_var_fused_kernel: here its registers would spill the region path's SGPRs)
}

// The read ceiling probe (nvl_crc32c_read_probe): grid-strided, four
// independent 16-byte nontemporal loads per thread per step.
__global__ __launch_bounds__(1024) void read_probe_kernel(const u32x4* __restrict__ p, uint64_t n16,
                                                          uint32_t* __restrict__ sink) {
  uint32_t x = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3u * stride < n16; i += 4u * stride) {
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(p + i + (uint64_t)k * stride);
#pragma unroll
    for (int k = 0; k < 4; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  for (; i < n16; i += stride) {
    const u32x4 v = p[i];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) sink[0] = x;
}

// Synthetic stream: one thread per 8-byte word.
__global__ void fill_splitmix_kernel(uint64_t* __restrict__ dst, uint64_t words_per_block, uint64_t nwords,
                                     uint64_t first_block, uint64_t block_step, uint64_t seed) {
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
       w += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = w / words_per_block;
    const uint64_t j = (first_block + k * block_step) * words_per_block + (w - k * words_per_block);
    uint64_t z = seed + (j + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    dst[w] = z ^ (z >> 31);
  }
}

}  // namespace dev

// ---------------------------------------------------------------------------
// launchers (host)

hipError_t launch_trailer_verdicts(const void* file, const uint64_t* off, const uint64_t* len1, const uint32_t* crc,
                                   uint64_t n, uint8_t* verdict, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(dev::crc32c_trailer_verdicts, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st,
                     static_cast<const uint8_t*>(file), off, len1, crc, n, verdict);
  return hipGetLastError();
}

hipError_t launch_fill(void* dst, uint64_t nblocks, uint64_t block_bytes, uint64_t first_block, uint64_t block_step,
                       uint64_t seed, hipStream_t st) {
  const uint64_t wpb = block_bytes / 8;
  const uint64_t nwords = nblocks * wpb;
  if (nwords == 0) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>((nwords + 255) / 256, 65536);
  hipLaunchKernelGGL(dev::fill_splitmix_kernel, dim3((uint32_t)blocks), dim3(256), 0, st,
                     static_cast<uint64_t*>(dst), wpb, nwords, first_block, block_step, seed);
  return hipGetLastError();
}

hipError_t launch_read_probe(const void* src, uint64_t bytes, uint32_t* sink, hipStream_t st) {
  hipLaunchKernelGGL(dev::read_probe_kernel, dim3(256), dim3(1024), 0, st, static_cast<const dev::u32x4*>(src),
                     bytes / 16u, sink);
  return hipGetLastError();
}

static inline hipError_t launch_fixup(const Rec* recs, uint32_t nw, uint32_t* out, uint32_t flags, hipStream_t st,
                                      hipEvent_t ev_stop = nullptr) {
  const uint32_t wpb = 4;  // one wave per unit
  const dim3 grid((nw + wpb - 1) / wpb), block(dev::kWave * wpb);
  if (ev_stop)
    hipExtLaunchKernelGGL(dev::crc32c_fixup_kernel, grid, block, 0, st, nullptr, ev_stop, 0u, recs, nw, out, flags);
  else
    hipLaunchKernelGGL(dev::crc32c_fixup_kernel, grid, block, 0, st, recs, nw, out, flags);
  return hipGetLastError();
}

static inline uint32_t grid_for(int num_cu, uint64_t T) {
  uint64_t g = (T + dev::kWavesPerWG - 1) / dev::kWavesPerWG;
  if (g > (uint64_t)num_cu) g = (uint64_t)num_cu;
  return g ? (uint32_t)g : 1u;
}

static inline uint32_t chunks_of(uint64_t len) { return dev::chunks_for(len); }

// The head kernel over a geometry's n buffers; its dispatch records
// ev_start when given (it is then the call's first kernel).
constexpr uint32_t kHeadGridMult = 1;  // head kernel workgroups per CU (A/B'd; the fused plan takes <= 1023 tiles)
static inline uint32_t head_grid(int num_cu, uint64_t n) {
  const uint64_t per_wg = 8u * dev::kWavesPerWG;  // at least ~8 buffers per wave
  const uint64_t cap = std::min<uint64_t>((uint64_t)num_cu * kHeadGridMult, dev::kMaxTiles);
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(cap, (n + per_wg - 1) / per_wg));
}

template <class G>
static hipError_t launch_heads(const LaunchCtx& lc, const G& g, uint32_t* out, uint32_t flags, uint32_t* hc,
                               hipEvent_t ev_start, uint64_t* lpre = nullptr, uint64_t* tiles = nullptr,
                               bool short_ok = false, hipEvent_t ev_stop = nullptr) {
  const uint32_t grid = head_grid(lc.num_cu, g.n);
  dev::KArgs ka{out, flags, nullptr, lc.tables, nullptr, hc};
  ka.short_ok = short_ok ? 1u : 0u;
  if (lpre) {  // tiles of the variable-length plan: one per workgroup
    ka.lpre = lpre;
    ka.tiles = tiles;
    ka.tile_G = grid;
    ka.tile_S = (g.n + grid - 1) / grid;
  }
  if (ev_start || ev_stop)
    hipExtLaunchKernelGGL(dev::crc32c_head_kernel<G>, dim3(grid), dim3(dev::kThreads), 0, lc.stream, ev_start,
                          ev_stop, 0u, g, ka);
  else
    hipLaunchKernelGGL(dev::crc32c_head_kernel<G>, dim3(grid), dim3(dev::kThreads), 0, lc.stream, g, ka);
  return hipGetLastError();
}

static inline size_t recs_part(int num_cu, uint64_t len, uint64_t n) {
  if (n == 0 || chunks_of(len) == 1) return 0;
  return 2ull * grid_for(num_cu, n * (uint64_t)chunks_of(len)) * dev::kUnitsPerWG * sizeof(Rec);
}

// Fixed-stride workspace: [unit records (J > 1)][hc: n u32 (partial first chunks with J > 1)]
// or, for a shape that can take the chunk-parallel path (len a multiple of
// 4096, J > 1: aligned when base and stride are), the n*J chunk raws if larger.
constexpr uint32_t kChunkParallelMaxJ = 1024;  // fold runs of <= 16 raws per lane (config 4: J = 512, R = 8)

constexpr uint32_t kFoldSeg = 1024;  // level-1 segment of the two-level fold (runs of 16 raws per lane)

static inline uint64_t fold_segments(uint32_t J) { return (J + kFoldSeg - 1u) / kFoldSeg; }

// the n*J chunk raws, and for J > kChunkParallelMaxJ the n*G segment raws after them
static inline size_t chunk_raws_bytes(uint64_t len, uint64_t n) {
  if (!(len > dev::kChunk && len % dev::kChunk == 0)) return 0;
  const uint64_t J = len / dev::kChunk;
  const size_t raws = (n * J * sizeof(uint32_t) + 255u) / 256u * 256u;
  return J <= kChunkParallelMaxJ ? n * J * sizeof(uint32_t) : raws + n * fold_segments((uint32_t)J) * sizeof(uint32_t);
}

// x^(8 bytes) and the lane multipliers step^(R (63 - l)) of a fold whose
// lanes take runs of R elements (host GF(2) arithmetic, crc32c_math.h).
static void fold_powers(uint64_t step_bytes, uint32_t S, uint32_t* step, uint32_t m[64]) {
  PowTable pw;
  build_pow_table(&pw);
  *step = xpow8(pw.x2n, step_bytes);
  const uint32_t R = (S + 63u) / 64u;
  const uint32_t sR = xpow8(pw.x2n, step_bytes * R);
  m[63] = kOne;
  for (int l = 62; l >= 0; --l) m[l] = gf_mul(m[l + 1], sR);
}
size_t fixed_recs_bytes(int num_cu, uint64_t len, uint64_t n) {
  const size_t cr = chunk_raws_bytes(len, n);
  const size_t r0 = (recs_part(num_cu, len, n) + 255) / 256 * 256;
  const size_t r = r0 > cr ? r0 : cr;
  const bool hcs = n && chunks_of(len) > 1 && dev::head_first(len);
  return r + (hcs ? n * sizeof(uint32_t) : 0);
}

hipError_t launch_fixed(const LaunchCtx& lc, const uint8_t* base, uint64_t stride, uint64_t len, uint64_t n,
                        const uint32_t* init, uint32_t init_all, uint32_t* out, uint32_t flags, Rec* ws) {
  if (n == 0) return hipSuccess;
  const uint32_t J = chunks_of(len);
  const uint32_t grid = grid_for(lc.num_cu, n * (uint64_t)J);
  const bool aligned = len > 0 && (len % dev::kChunk) == 0 && ((uintptr_t)base % 16) == 0 && (stride % 16) == 0;
  dev::FixedGeom g{base, stride, len, n, J, init, init_all};
  Rec* recs = J > 1 ? ws : nullptr;
  const bool masked = !aligned && J == 1 && len >= 1025 && len < dev::kChunk;
  const bool heads = !aligned && dev::head_first(len) && !masked;  // every buffer's first chunk is a head chunk
  // Short mode (run_heads): two-chunk buffers with a 1..3-byte head (block |
  // type of 4096-byte blocks at a fixed stride) are finished by the head
  // kernel, body chunk and all; no masked head can start a page there.
  const bool short_all = heads && J == 2 && dev::head_bytes(len, J) < 4u;
  const bool body = !(heads && (J == 1 || short_all));  // some buffer has a chunk left for a body kernel
  uint32_t* hc = heads && J > 1
                     ? reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(ws) +
                                                   (recs_part(lc.num_cu, len, n) + 255) / 256 * 256)
                     : nullptr;
  hipEvent_t ev_start = lc.ev_start;
  if (heads) {
    hipError_t eh = launch_heads(lc, g, out, flags, hc, ev_start, nullptr, nullptr, short_all,
                                 body ? nullptr : lc.ev_stop);
    if (eh != hipSuccess || !body) return eh;
    ev_start = nullptr;
  }
  // Chunk-parallel: every chunk a scheduler-A pass, then the per-buffer
  // fold -- one wave per buffer while a lane's serial run R = ceil(J/64)
  // stays short (J <= 1024), else two levels (crc32c_fold_seg_kernel:
  // segments of 1024 chunks over the whole grid, then the segments per
  // buffer), so a lone 1 GiB buffer (bench_configs `big1`) streams at
  // scheduler A's rate too.
  if (aligned && J > kChunkParallelMaxJ) {
    const uint64_t T = n * (uint64_t)J;
    const uint32_t jsh = (J & (J - 1u)) == 0u ? (uint32_t)__builtin_ctz(J) : 64u;
    dev::ChunkGeom cg{base, stride, T, J, jsh, init, init_all};
    dev::KArgs kc{out, flags, nullptr, lc.tables, nullptr, nullptr};
    kc.raws = reinterpret_cast<uint32_t*>(ws);
    const uint32_t gc = grid_for(lc.num_cu, T);
    if (ev_start)
      hipExtLaunchKernelGGL(dev::crc32c_chunks_kernel, dim3(gc), dim3(dev::kThreads), 0, lc.stream, ev_start, nullptr,
                            0u, cg, kc);
    else
      hipLaunchKernelGGL(dev::crc32c_chunks_kernel, dim3(gc), dim3(dev::kThreads), 0, lc.stream, cg, kc);
    hipError_t ec = hipGetLastError();
    if (ec != hipSuccess) return ec;
    const uint32_t G = (uint32_t)fold_segments(J);
    uint32_t* segs = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(ws) +
                                                 (n * (uint64_t)J * sizeof(uint32_t) + 255u) / 256u * 256u);
    dev::FoldSeg f1{kc.raws, n, J, kFoldSeg, G, 0u, {}, segs, flags};
    fold_powers(dev::kChunk, kFoldSeg, &f1.step, f1.m);
    dev::FoldSeg f2{segs, n, G, G, 1u, 0u, {}, out, flags};
    fold_powers((uint64_t)dev::kChunk * kFoldSeg, G, &f2.step, f2.m);
    const uint32_t g1 = (uint32_t)std::min<uint64_t>((n * G + 3) / 4, 65535);
    hipLaunchKernelGGL(dev::crc32c_fold_seg_kernel, dim3(g1), dim3(256), 0, lc.stream, f1);
    ec = hipGetLastError();
    if (ec != hipSuccess) return ec;
    const uint32_t g2 = (uint32_t)std::min<uint64_t>((n + 3) / 4, 65535);
    if (lc.ev_stop)
      hipExtLaunchKernelGGL(dev::crc32c_fold_seg_kernel, dim3(g2), dim3(256), 0, lc.stream, nullptr, lc.ev_stop, 0u, f2);
    else
      hipLaunchKernelGGL(dev::crc32c_fold_seg_kernel, dim3(g2), dim3(256), 0, lc.stream, f2);
    return hipGetLastError();
  }
  if (aligned && J > 1 && J <= kChunkParallelMaxJ) {
    const uint64_t T = n * (uint64_t)J;
    const uint32_t jsh = (J & (J - 1u)) == 0u ? (uint32_t)__builtin_ctz(J) : 64u;
    dev::ChunkGeom cg{base, stride, T, J, jsh, init, init_all};
    dev::KArgs kc{out, flags, nullptr, lc.tables, nullptr, nullptr};
    kc.raws = reinterpret_cast<uint32_t*>(ws);
    const uint32_t gc = grid_for(lc.num_cu, T);
    if (ev_start)
      hipExtLaunchKernelGGL(dev::crc32c_chunks_kernel, dim3(gc), dim3(dev::kThreads), 0, lc.stream, ev_start, nullptr,
                            0u, cg, kc);
    else
      hipLaunchKernelGGL(dev::crc32c_chunks_kernel, dim3(gc), dim3(dev::kThreads), 0, lc.stream, cg, kc);
    hipError_t ec = hipGetLastError();
    if (ec != hipSuccess) return ec;
    const uint32_t gf = (uint32_t)std::min<uint64_t>((n + 3) / 4, 65535);
    if (lc.ev_stop)
      hipExtLaunchKernelGGL(dev::crc32c_fold_kernel, dim3(gf), dim3(256), 0, lc.stream, nullptr, lc.ev_stop, 0u,
                            kc.raws, n, J, lc.tables, out, flags);
    else
      hipLaunchKernelGGL(dev::crc32c_fold_kernel, dim3(gf), dim3(256), 0, lc.stream, kc.raws, n, J, lc.tables, out,
                         flags);
    return hipGetLastError();
  }
  dev::KArgs ka{out, flags, recs, lc.tables, nullptr, hc};
  hipEvent_t stop_main = J == 1 ? lc.ev_stop : nullptr;  // else the fix-up records it
  const bool timed = ev_start || stop_main;
  if (aligned && J == 1 && n >= dev::kLongFixedMin) {
    if (timed)
      hipExtLaunchKernelGGL(dev::crc32c_fixed_long_kernel, dim3(grid), dim3(dev::kThreads), 0, lc.stream, ev_start,
                            stop_main, 0u, g, ka);
    else
      hipLaunchKernelGGL(dev::crc32c_fixed_long_kernel, dim3(grid), dim3(dev::kThreads), 0, lc.stream, g, ka);
    return hipGetLastError();
  }
  if (aligned) {
    if (timed)
      hipExtLaunchKernelGGL(dev::crc32c_fixed_kernel<dev::kAligned>, dim3(grid), dim3(dev::kThreads), 0, lc.stream,
                            ev_start, stop_main, 0u, g, ka);
    else
      hipLaunchKernelGGL(dev::crc32c_fixed_kernel<dev::kAligned>, dim3(grid), dim3(dev::kThreads), 0, lc.stream, g,
                         ka);
  } else {
    if (timed)
      hipExtLaunchKernelGGL(dev::crc32c_fixed_kernel<dev::kGeneral>, dim3(grid), dim3(dev::kWave * dev::kGenWaves),
                            0, lc.stream, ev_start, stop_main, 0u, g, ka);
    else
      hipLaunchKernelGGL(dev::crc32c_fixed_kernel<dev::kGeneral>, dim3(grid), dim3(dev::kWave * dev::kGenWaves), 0,
                         lc.stream, g, ka);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || J == 1) return e;
  return launch_fixup(recs, grid * dev::kUnitsPerWG, out, flags, lc.stream, lc.ev_stop);
}

size_t var_recs_bytes(int num_cu) { return 2ull * (uint64_t)num_cu * dev::kUnitsPerWG * sizeof(Rec); }
size_t var_unit_map_bytes(int num_cu) { return (uint64_t)num_cu * dev::kUnitsPerWG * sizeof(uint64_t); }


bool var_plan_small(uint64_t n) { return n <= dev::kPlanSmallMax; }

// Short mode (run_heads) needs a tile's largest chunk count <= 2 and the
// tile scan fused into the classification (a tile of <= kHeadSub buffers).
bool var_heads_only(int num_cu, uint64_t n, uint64_t max_len) {
  const uint64_t G = head_grid(num_cu, n);
  return max_len <= 2ull * dev::kChunk && (n + G - 1) / G <= dev::kHeadSub;
}

hipError_t launch_var_fused(const LaunchCtx& lc, const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths,
                            uint64_t n, const uint32_t* init, uint32_t init_all, uint32_t* out, uint32_t flags,
                            Rec* recs, uint32_t* hc, uint64_t* lpre, uint64_t* tiles, uint64_t max_len) {
  if (n == 0) return hipSuccess;
  if (!lc.counter || !lpre || !tiles || lc.num_cu > (int)dev::kMaxTiles) return hipErrorInvalidValue;
  dev::VarGeom g{base, offsets, lengths, nullptr, nullptr, n, init, init_all};
  hipError_t eh = launch_heads(lc, g, out, flags, hc, nullptr, lpre, tiles, /*short_ok=*/true);
  if (eh != hipSuccess || var_heads_only(lc.num_cu, n, max_len)) return eh;
  dev::KArgs ka{out, flags, recs, lc.tables, lc.counter, hc};
  ka.lpre = lpre;
  ka.tiles = tiles;
  ka.tile_G = head_grid(lc.num_cu, n);
  ka.tile_S = (n + ka.tile_G - 1) / ka.tile_G;
  hipLaunchKernelGGL(dev::crc32c_var_fused_kernel, dim3((uint32_t)lc.num_cu), dim3(dev::kWave * dev::kGenWaves), 0,
                     lc.stream, g, ka);
  return hipGetLastError();
}

hipError_t launch_var_plan_small(const LaunchCtx& lc, const uint64_t* lengths, uint64_t n, uint64_t* chunk_start,
                                 uint64_t* unit_first, uint32_t* long_bufs) {
  const uint64_t NU = (uint64_t)lc.num_cu * dev::kUnitsPerWG;
  hipLaunchKernelGGL(dev::crc32c_plan_small, dim3(1), dim3((uint32_t)dev::kPlanThreads), 0, lc.stream, lengths, n, NU,
                     chunk_start, unit_first, long_bufs);
  return hipGetLastError();
}

hipError_t launch_var_counts(const uint64_t* lengths, uint64_t n, uint64_t* cnt, uint32_t* long_bufs,
                             hipStream_t st) {
  const uint32_t tpb = 256;
  const uint64_t blocks = (n + 1 + tpb - 1) / tpb;
  hipLaunchKernelGGL(dev::crc32c_var_counts, dim3((uint32_t)blocks), dim3(tpb), 0, st, lengths, n, cnt, long_bufs);
  return hipGetLastError();
}

hipError_t launch_var(const LaunchCtx& lc, const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths,
                      const uint64_t* chunk_start, uint64_t* unit_first, uint64_t n, const uint32_t* init,
                      uint32_t init_all, uint32_t* out, uint32_t flags, Rec* recs, uint32_t* hc, uint32_t* long_bufs,
                      bool have_unit_map) {
  if (n == 0) return hipSuccess;
  {
    const dev::VarGeom gh{base, offsets, lengths, nullptr, nullptr, n, init, init_all};
    hipError_t eh = launch_heads(lc, gh, out, flags, hc, nullptr);
    if (eh != hipSuccess) return eh;
  }
  const uint32_t grid = (uint32_t)lc.num_cu;  // chunk count is only known on the device
  const uint64_t NU = (uint64_t)grid * dev::kUnitsPerWG;
  if (!have_unit_map) {
    hipLaunchKernelGGL(dev::crc32c_unit_map, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, lc.stream, chunk_start,
                       n, NU, unit_first, long_bufs);
    hipError_t e0 = hipGetLastError();
    if (e0 != hipSuccess) return e0;
  }
  dev::VarGeom g{base, offsets, lengths, chunk_start, unit_first, n, init, init_all};
  dev::KArgs ka{out, flags, recs, lc.tables, nullptr, hc, long_bufs};
  hipLaunchKernelGGL(dev::crc32c_var_kernel, dim3(grid), dim3(dev::kWave * dev::kGenWaves), 0, lc.stream, g, ka);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_fixup(recs, grid * dev::kUnitsPerWG, out, flags, lc.stream);
}

static inline size_t align256(size_t v) { return (v + 255u) / 256u * 256u; }

// A process-wide call generation (never 0, the zeroed workspace's value),
// seeded at random so that leftover memory is unlikely to hold it: the
// region fold trusts an event record only when it carries this call's
// generation AND its own buffer index (workspace memory is never
// zeroed).
static uint32_t next_generation() {
  static std::atomic<uint32_t> s_gen{(uint32_t)std::random_device{}()};
  uint32_t gen = s_gen.fetch_add(1u, std::memory_order_relaxed) + 1u;
  if (gen == 0u) gen = s_gen.fetch_add(1u, std::memory_order_relaxed) + 1u;
  return gen;
}

// Routed calls (crc32c_route_plan -> crc32c_route_kernel -> crc32c_var_fused_kernel).
// the plan's partials and, after them, the route kernel's verdict
size_t route_parts_bytes() { return ((dev::kRoutePlanMax + 1u) * sizeof(dev::RoutePart) + 255u) / 256u * 256u; }
// Region chunks a region-shaped batch_dev batch can span: sorted, each buffer
// <= kRegionMaxLen (32 chunks), gaps <= 1/8 of the bytes + 64 KiB -> at most
// 36 chunks per buffer + 18 + 2 (route_region checks it).
// Capped at 2^24 chunks (64 MiB of raws, a 64 GiB span): a larger batch
// takes the batch path rather than a workspace of 4 bytes per 4 KiB of the
// worst case (10^7 buffers would have reserved 1.4 GB).
uint64_t route_cap_chunks(uint64_t n) { return std::min<uint64_t>(36u * n + 20u, 1ull << 24); }
// Plan workgroups: one step of kPlanT x kPlanPer = 1024 pairs each, but at
// least ~64 of them from 16K pairs on (the scan is latency-bound: spreading
// it over more CUs shortens it -- config 3's 32 672 pairs 175.2 -> 173.3 us
// on 64 workgroups instead of 8, v / r 1.5 us on 98 instead of 25).
static inline uint32_t route_plan_grid(uint64_t n) {
  const uint64_t per = (uint64_t)dev::kPlanT * dev::kPlanPer;
  const uint64_t want = std::max<uint64_t>(std::min<uint64_t>(64, (n + 255u) / 256u), (n + per - 1u) / per);
  return (uint32_t)std::min<uint64_t>(dev::kRoutePlanMax, std::max<uint64_t>(1, want));
}

hipError_t launch_routed(const LaunchCtx& lc, const uint8_t* base, uint64_t region_len, bool dyn,
                         const uint64_t* offsets, const uint64_t* lengths, uint64_t n, const uint32_t* init,
                         uint32_t init_all, uint32_t* out, uint32_t flags, void* region_ws, uint64_t cap_chunks,
                         void* parts_ws, Rec* recs, uint32_t* hc, uint64_t* lpre, uint64_t* tiles) {
  if (n == 0) return hipSuccess;
  if (!lc.counter || !lpre || !tiles || lc.num_cu > (int)dev::kMaxTiles) return hipErrorInvalidValue;
  const uint32_t P = route_plan_grid(n);
  dev::RoutePart* parts = static_cast<dev::RoutePart*>(parts_ws);
  const uint64_t lim = dyn ? ~0ull : region_len;
  dev::Route rt;
  rt.parts = parts;
  rt.np = P;
  rt.dyn = dyn ? 1u : 0u;
  rt.base = base;
  rt.offsets = offsets;
  rt.lengths = lengths;
  rt.n = n;
  rt.cap_chunks = cap_chunks;
  if (lc.ev_start)
    hipExtLaunchKernelGGL(dev::crc32c_route_plan, dim3(P), dim3(dev::kPlanT), 0, lc.stream, lc.ev_start, nullptr, 0u,
                          offsets, lengths, n, lim, (uintptr_t)base, dyn ? 1u : 0u, parts);
  else
    hipLaunchKernelGGL(dev::crc32c_route_plan, dim3(P), dim3(dev::kPlanT), 0, lc.stream, offsets, lengths, n, lim,
                       (uintptr_t)base, dyn ? 1u : 0u, parts);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // the region path's geometry: the caller's region, or (dyn) set in the kernel from the plan
  uint8_t* w = static_cast<uint8_t*>(region_ws);
  uint32_t* raws = reinterpret_cast<uint32_t*>(w);
  uint4* qs = reinterpret_cast<uint4*>(w + align256(cap_chunks * 4u));
  uint4* qe = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(qs) + align256(n * 16u));
  const uintptr_t O = dyn ? 0u : (uintptr_t)base & ~(uintptr_t)(dev::kChunk - 1u);
  const uint64_t rel0 = dyn ? 0u : (uintptr_t)base - O;
  const uint64_t nc = dyn ? 0u : (rel0 + region_len + dev::kChunk - 1u) / dev::kChunk;
  dev::RegionGeom rg{reinterpret_cast<const uint8_t*>(O), nc, rel0, rel0, rel0 + region_len, offsets, lengths, n,
                     init, init_all, raws, qs, qe, next_generation()};
  const dev::VarGeom vg{base, offsets, lengths, nullptr, nullptr, n, init, init_all};
  const uint32_t hg = head_grid(lc.num_cu, n);
  dev::KArgs ka{out, flags, nullptr, lc.tables, nullptr, hc};
  ka.lpre = lpre;
  ka.tiles = tiles;
  ka.tile_G = hg;
  ka.tile_S = (n + hg - 1) / hg;
  ka.short_ok = 1u;
  ka.route = rt;
  hipLaunchKernelGGL(dev::crc32c_route_kernel, dim3((uint32_t)lc.num_cu), dim3(dev::kThreads), 0, lc.stream, rg, vg,
                     ka);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  dev::KArgs kf{out, flags, recs, lc.tables, lc.counter, hc};
  kf.lpre = lpre;
  kf.tiles = tiles;
  kf.tile_G = hg;
  kf.tile_S = ka.tile_S;
  kf.route = rt;
  if (lc.ev_stop)
    hipExtLaunchKernelGGL(dev::crc32c_var_fused_kernel, dim3((uint32_t)lc.num_cu), dim3(dev::kWave * dev::kGenWaves),
                          0, lc.stream, nullptr, lc.ev_stop, 0u, vg, kf);
  else
    hipLaunchKernelGGL(dev::crc32c_var_fused_kernel, dim3((uint32_t)lc.num_cu), dim3(dev::kWave * dev::kGenWaves), 0,
                       lc.stream, vg, kf);
  return hipGetLastError();
}

// Region workspace: [raws: chunks u32][qs: n x 8 B][qe: n x 8 B] (chunks bounded
// by region_len / 4096 + 2 whatever the region's alignment).
size_t region_ws_bytes_cap(uint64_t cap_chunks, uint64_t n) { return align256(cap_chunks * 4u) + 2u * align256(n * 16u); }
uint64_t region_cap_chunks(uint64_t region_len) { return region_len / dev::kChunk + 2u; }
size_t region_ws_bytes(uint64_t region_len, uint64_t n) { return region_ws_bytes_cap(region_cap_chunks(region_len), n); }

hipError_t launch_region(const LaunchCtx& lc, const uint8_t* region, uint64_t region_len, const uint64_t* offsets,
                         const uint64_t* lengths, const uint32_t* init, uint32_t init_all, uint32_t* out, uint64_t n,
                         uint32_t flags, void* ws) {
  if (n == 0) return hipSuccess;
  const uintptr_t O = (uintptr_t)region & ~(uintptr_t)(dev::kChunk - 1u);
  const uint64_t rel0 = (uintptr_t)region - O;
  const uint64_t nc = (rel0 + region_len + dev::kChunk - 1u) / dev::kChunk;
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint32_t* raws = reinterpret_cast<uint32_t*>(w);
  uint4* qs = reinterpret_cast<uint4*>(w + align256((region_len / dev::kChunk + 2u) * 4u));
  uint4* qe = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(qs) + align256(n * 16u));
  const uint32_t gen = next_generation();
  dev::RegionGeom g{reinterpret_cast<const uint8_t*>(O), nc, rel0, rel0, rel0 + region_len, offsets, lengths, n, init, init_all,
                    raws, qs, qe, gen};
  dev::KArgs ka{out, flags, nullptr, lc.tables, nullptr, nullptr};
  const uint32_t grid = grid_for(lc.num_cu, nc);  // >= 1 (nc >= 1: n > 0 buffers inside the region)
  if (lc.ev_start || lc.ev_stop)
    hipExtLaunchKernelGGL(dev::crc32c_region_kernel, dim3(grid), dim3(dev::kThreads), 0, lc.stream, lc.ev_start,
                          lc.ev_stop, 0u, g, ka);
  else
    hipLaunchKernelGGL(dev::crc32c_region_kernel, dim3(grid), dim3(dev::kThreads), 0, lc.stream, g, ka);
  return hipGetLastError();
}

}  // namespace nvl
