// nvlevelz_amd/csrc/crc32c_dev.h -- CDNA4 (gfx950) batched CRC32C: the device
// primitives every kernel shares (lane helpers, LDS table images, loads and
// realignment, per-chunk chains, geometries, the route plan's verdict).
// Schedulers A/B/C: crc32c_dev_sched.h; heads: crc32c_dev_heads.h; region
// path: crc32c_dev_region.h; kernels and launchers: crc32c_fixed.hip,
// crc32c_batch.hip, crc32c_region.hip, crc32c_misc.hip (one TU,
// crc32c_kernels.hip, until round 5).
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
#pragma once
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
// The fold's chunk shifts (the blob's shc tables, 16 KiB) over the nibble
// tables' rows 64..127, written once the workgroup's chunks are done.
constexpr uint32_t kRShcOff = 16384;
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
    // column 63 of rows 0..15 holds the unit counter (units 0..ctr0-1 are
    // pre-assigned) and the workgroup's slots (crc32c_dev_region.h), zeroed
    // here; the lane shifts never read that column
    const int gi = t + q * (int)kThreads;
    if (gi < 256 && (gi & 15) == 15) v.w = gi == (int)(kRCtrOff >> 4) ? ctr0 : 0u;
    dst[gi] = v;
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

}  // namespace dev
}  // namespace nvl
