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

// LDS image (bytes)
constexpr uint32_t kRepBytes = 128u * 1024u;           // 4 tables x 256 x 32 replicas x 4 B
constexpr uint32_t kCombOff = kRepBytes;               // comb[6][4][256] u32
constexpr uint32_t kShOff = kCombOff + 6u * 4u * 256u * 4u;  // sh4096[4][256] u32
constexpr uint32_t kCtrOff = kShOff + 4u * 256u * 4u;         // per-workgroup work counter
constexpr uint32_t kLdsBytes = kCtrOff + 16u;                 // 159760 B
static_assert(kLdsBytes <= 160u * 1024u, "LDS image exceeds 160 KiB");

// DevTables word offsets (see crc32c_internal.h)
constexpr uint32_t kGSlice = 0, kGComb = 1024, kGX2n = 1024 + 6144 + 1024;  // comb, sh4096 contiguous

// ---------------------------------------------------------------------------
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

#if defined(NVL_ABL_STRIDED) || defined(NVL_ABL_NOLOAD)
#define NVL_ABL_LAYOUT_STRIDED 1
#else
#define NVL_ABL_LAYOUT_STRIDED 0
#endif

typedef const u32x4 __attribute__((address_space(1))) * gvec_ptr;

// 16-byte streaming load from global memory (read-once data: non-temporal
// hint).  The explicit address space keeps it a global_load (a flat_load would
// also count in lgkmcnt and serialise against the LDS lookups).
__device__ __forceinline__ u32x4 ld16(uintptr_t addr) {
#if defined(NVL_ABL_NO_NT)
  return *(gvec_ptr)addr;
#else
  return __builtin_nontemporal_load((gvec_ptr)addr);
#endif
}

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
  return lds_u32(lds, a0) ^ lds_u32(lds, a1) ^ lds_u32(lds, a2) ^ lds_u32(lds, a3);
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
  return xor3(xor3(lds_u32(lds, a0), lds_u32(lds, a1), lds_u32(lds, a2)), lds_u32(lds, a3), next);
}

// slice4(x) ^ next -- the chain step with the following word folded in.
__device__ __forceinline__ uint32_t slice4_next(const uint8_t* lds, uint32_t x, uint32_t next, const LaneBase& lb) {
#if defined(NVL_XOR3)
  return slice4_x(lds, x, next, lb);
#else
  return slice4(lds, x, lb) ^ next;
#endif
}



__device__ __forceinline__ uint32_t comb_lookup(const uint8_t* lds, int lev, int j, uint32_t v) {
  return lds_u32(lds, kCombOff + ((uint32_t)((lev * 4 + j) << 8) + ((v >> (8 * j)) & 0xFFu)) * 4u);
}

// One butterfly level over lane bit LEV: the lane with bit LEV clear holds the
// group of lower stream positions ("left"), the partner the upper one
// ("right"); left is shifted by the operator in comb table TAB (64*2^TAB
// bytes) and XORed in.  Lanes 0..3 of every quad spread the 4 byte lookups.
template <int LEV, int TAB = LEV>
__device__ __forceinline__ uint32_t fold_level(const uint8_t* lds, uint32_t g, int lane) {
  const uint32_t pt = lane_xor<LEV>(g);
  const bool hi = (lane >> LEV) & 1;
  const uint32_t left = hi ? pt : g;
  const uint32_t right = hi ? g : pt;
  uint32_t s;
  if constexpr (LEV == 0) {
    const int j = hi ? 2 : 0;
    s = comb_lookup(lds, TAB, j, left) ^ comb_lookup(lds, TAB, j + 1, left);
    s ^= dpp_xor1(s);
  } else {
    s = comb_lookup(lds, TAB, lane & 3, left);
    s ^= dpp_xor1(s);
    s ^= dpp_xor2(s);
  }
  return s ^ right;
}

// XOR_l shift(g_l, 64*(63-l)) over the wave; every lane gets the result.
__device__ __forceinline__ uint32_t wave_fold(const uint8_t* lds, uint32_t g, int lane) {
  g = fold_level<0>(lds, g, lane);
  g = fold_level<1>(lds, g, lane);
  g = fold_level<2>(lds, g, lane);
  g = fold_level<3>(lds, g, lane);
  g = fold_level<4>(lds, g, lane);
  g = fold_level<5>(lds, g, lane);
  return g;
}

// shift(acc, 4096) for a wave-uniform acc; every lane gets the result.
__device__ __forceinline__ uint32_t shift4096(const uint8_t* lds, uint32_t acc, int lane) {
  const int j = lane & 3;
  uint32_t s = lds_u32(lds, kShOff + ((uint32_t)(j << 8) + ((acc >> (8 * j)) & 0xFFu)) * 4u);
  s ^= dpp_xor1(s);
  s ^= dpp_xor2(s);
  return s;
}

// Fill the LDS image from the device table blob.
__device__ __forceinline__ void fill_lds(uint8_t* lds, const uint32_t* __restrict__ g) {
  const int t = threadIdx.x;
  // replicated slice tables: 8192 16-byte stores, consecutive lanes write
  // consecutive 16 B (conflict-free ds_write_b128).
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t s = (uint32_t)(t + q * kThreads);  // 16-byte slot index
    const uint32_t off = s << 4;
    const uint32_t tab = ((off >> 16) << 1) | ((off >> 7) & 1u);
    const uint32_t b = (off >> 8) & 0xFFu;
    const uint32_t v = g[kGSlice + tab * 256u + b];
    *reinterpret_cast<uint4*>(lds + off) = make_uint4(v, v, v, v);
  }
  // comb + sh4096 copied verbatim (7168 words = 1792 uint4)
  const uint4* src = reinterpret_cast<const uint4*>(g + kGComb);
  uint4* dst = reinterpret_cast<uint4*>(lds + kCombOff);
  for (int q = t; q < 1792; q += kThreads) dst[q] = src[q];
  if (t == 0) *reinterpret_cast<uint32_t*>(lds + kCtrOff) = (uint32_t)kWavesPerWG;  // units 0..15 are pre-assigned
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

struct FixedGeom {
  const uint8_t* base;
  uint64_t stride, len, n;
  uint32_t J;
  const uint32_t* init;
  uint32_t init_all;
  __device__ __forceinline__ uint64_t total() const { return n * (uint64_t)J; }
  __device__ __forceinline__ void locate(uint64_t t, uint64_t& i, uint32_t& c) const {
    i = t / J;
    c = (uint32_t)(t - i * J);
  }
  __device__ __forceinline__ BufInfo info(uint64_t i) const {
    const uint32_t ini = init ? init[i] : init_all;
    return BufInfo{base + i * stride, len, J, ~ini};
  }
};

struct VarGeom {
  const uint8_t* base;
  const uint64_t* offsets;
  const uint64_t* lengths;
  const uint64_t* chunk_start;  // n+1 entries, exclusive prefix of J_i
  uint64_t n;
  const uint32_t* init;
  uint32_t init_all;
  __device__ __forceinline__ uint64_t total() const { return chunk_start[n]; }
  __device__ __forceinline__ void locate(uint64_t t, uint64_t& i, uint32_t& c) const {
    uint64_t lo = 0, hi = n;  // invariant: chunk_start[lo] <= t < chunk_start[hi]
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (chunk_start[mid] <= t) lo = mid; else hi = mid;
    }
    i = lo;
    c = (uint32_t)(t - chunk_start[lo]);
  }
  __device__ __forceinline__ BufInfo info(uint64_t i) const {
    const uint64_t L = lengths[i];
    const uint32_t J = L <= kChunk ? 1u : (uint32_t)((L + kChunk - 1) / kChunk);
    const uint32_t ini = init ? init[i] : init_all;
    return BufInfo{base + offsets[i], L, J, ~ini};
  }
};

// Loaded bytes of one lane's piece (20 dwords covers a misaligned piece).
struct Piece {
  uint32_t d[20];
};

// 4x4 transpose of 16-byte slots inside each lane quad (DPP quad_perm):
// afterwards lane 4q+r holds, in slot s, what lane 4q+s held in slot r.
__device__ __forceinline__ void quad_transpose(int lane, uint32_t (&d)[20]) {
  const int r = lane & 3;
  uint32_t t[16];
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // stage 1: swap 2x2 blocks across lane bit 1
    const bool take = ((j >> 1) & 1) != ((r >> 1) & 1);
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const uint32_t o = dpp_xor2(d[4 * (j ^ 2) + x]);
      t[4 * j + x] = take ? o : d[4 * j + x];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // stage 2: swap within 2x2 blocks across lane bit 0
    const bool take = (j & 1) != (r & 1);
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const uint32_t o = dpp_xor1(t[4 * (j ^ 1) + x]);
      d[4 * j + x] = take ? o : t[4 * j + x];
    }
  }
}

// Fast path (16-B aligned, full 4 KiB chunks): four fully coalesced 1 KiB
// loads (row j = bytes [1024j, 1024j+1024) of the chunk, lane l at 16l).  After
// quad_transpose (in build_words) lane 4q+r holds the contiguous 64-byte piece
// at chunk position P = 16r + q.
template <bool kFast>
__device__ __forceinline__ void load_piece(const BufInfo& bi, uint32_t c, int lane, Piece& pc) {
  const uintptr_t ce = (uintptr_t)bi.p + bi.len - (uint64_t)kChunk * (bi.J - 1u - c);
  const uintptr_t ps = ce - (uintptr_t)(64 * (64 - lane));
  if constexpr (kFast) {
#if defined(NVL_ABL_NOLOAD)  // ablation: synthetic data, no global loads
#pragma unroll
    for (int k = 0; k < 16; ++k) pc.d[k] = (uint32_t)(ps >> 4) * 2654435761u + (uint32_t)k * 40503u;
    return;
#endif
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#if defined(NVL_ABL_STRIDED)  // ablation: the v1 lane-contiguous (64-B stride) loads
      const u32x4 v = ld16(ps + 16u * (uint32_t)j);
#else
      const u32x4 v = ld16(ce - kChunk + 1024u * (uint32_t)j + 16u * (uint32_t)lane);
#endif
      pc.d[4 * j + 0] = v.x; pc.d[4 * j + 1] = v.y; pc.d[4 * j + 2] = v.z; pc.d[4 * j + 3] = v.w;
    }
  } else {
    if (bi.len < 4) return;  // tiny path reads its own bytes
    const uint32_t m = (uint32_t)(ce & 15u);
    const uintptr_t a = ps - m;
    const uintptr_t p = (uintptr_t)bi.p;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const bool ok = (j < 4 || m != 0) && (a + 16u * (uint32_t)j + 16u > p);
      u32x4 v = {0u, 0u, 0u, 0u};
      if (ok) v = ld16(a + 16u * (uint32_t)j);
      pc.d[4 * j + 0] = v.x; pc.d[4 * j + 1] = v.y; pc.d[4 * j + 2] = v.z; pc.d[4 * j + 3] = v.w;
    }
  }
}

template <int Q0>
__device__ __forceinline__ void realign(const Piece& pc, uint32_t r, uint32_t (&w)[16]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = __builtin_amdgcn_alignbyte(pc.d[Q0 + k + 1], pc.d[Q0 + k], r);
}

// The 16 little-endian words of this lane's piece, realigned, with the head
// masking and ~init injection applied (wave-uniform control flow).
template <bool kFast>
__device__ __forceinline__ void build_words(const BufInfo& bi, uint32_t c, int lane, const Piece& pc,
                                            uint32_t (&w)[16]) {
  if constexpr (kFast) {
    Piece t = pc;
#if !defined(NVL_ABL_STRIDED) && !defined(NVL_ABL_NOLOAD)
    quad_transpose(lane, t.d);
#endif
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = t.d[k];
    if (c == 0 && lane == 0) w[0] ^= bi.s;  // position 0 is lane 0 in both layouts
  } else {
    const uintptr_t ce = (uintptr_t)bi.p + bi.len - (uint64_t)kChunk * (bi.J - 1u - c);
    const uint32_t m = (uint32_t)(ce & 15u);
    const uint32_t r = m & 3u;
    switch (m >> 2) {
      case 0: realign<0>(pc, r, w); break;
      case 1: realign<1>(pc, r, w); break;
      case 2: realign<2>(pc, r, w); break;
      default: realign<3>(pc, r, w); break;
    }
    const uintptr_t p = (uintptr_t)bi.p;
    if (ce - kChunk < p + 4) {  // chunk holds the buffer head (or the tail of its ~init)
      const uintptr_t ps = ce - (uintptr_t)(64 * (64 - lane));
      int64_t rel = (int64_t)(p - ps);  // bytes of this piece before the buffer
      rel = rel < -8 ? -8 : (rel > 72 ? 72 : rel);
      const uint32_t s = bi.s;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int sh = (int)rel - 4 * k;
        const uint32_t keep = sh <= 0 ? 0xFFFFFFFFu : (sh >= 4 ? 0u : (0xFFFFFFFFu << (8 * sh)));
        uint32_t inj = 0;
        if (sh >= 0 && sh < 4) inj = s << (8 * sh);
        else if (sh < 0 && sh > -4) inj = s >> (-8 * sh);
        w[k] = (w[k] & keep) ^ inj;
      }
    }
  }
}

// Raw (zero-state, ~init injected) registers of U chunks, wave-uniform.  The
// U serial slice-by-4 chains and U butterflies are interleaved so each wave
// keeps U independent LDS round trips in flight (the kernel is bound by the
// chain's LDS latency, not by LDS bandwidth).
template <bool kFast, int U>
__device__ __forceinline__ void group_raw(const uint8_t* lds, const LaneBase& lb, const BufInfo (&bi)[U],
                                          const uint32_t (&c)[U], int lane, const Piece (&pc)[U],
                                          uint32_t (&raw)[U]) {
  uint32_t w[U][16];
#pragma unroll
  for (int u = 0; u < U; ++u) build_words<kFast>(bi[u], c[u], lane, pc[u], w[u]);
  uint32_t crc[U];
#if defined(NVL_ABL_NOCOMPUTE)  // ablation: keep the loads live, skip every lookup
#pragma unroll
  for (int u = 0; u < U; ++u) {
    crc[u] = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) crc[u] ^= w[u][k];
    raw[u] = crc[u] ^ lane_xor<5>(crc[u]);
  }
  return;
#endif
  {
#pragma unroll
    for (int u = 0; u < U; ++u) crc[u] = w[u][0];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
#pragma unroll
      for (int u = 0; u < U; ++u) crc[u] = slice4_next(lds, crc[u], k < 15 ? w[u][k + 1] : 0u, lb);
    }
  }

  // Lane -> stream position: general path P = lane; fast path (transposed
  // rows) P = 16*(lane&3) + (lane>>2), so lane bits 0,1 step 1024/2048 bytes
  // and bits 2..5 step 64..512 bytes.
  constexpr bool kT = kFast && !NVL_ABL_LAYOUT_STRIDED;
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = fold_level<0, kT ? 4 : 0>(lds, crc[u], lane);
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = fold_level<1, kT ? 5 : 1>(lds, crc[u], lane);
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = fold_level<2, kT ? 0 : 2>(lds, crc[u], lane);
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = fold_level<3, kT ? 1 : 3>(lds, crc[u], lane);
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = fold_level<4, kT ? 2 : 4>(lds, crc[u], lane);
#pragma unroll
  for (int u = 0; u < U; ++u) crc[u] = fold_level<5, kT ? 3 : 5>(lds, crc[u], lane);
#pragma unroll
  for (int u = 0; u < U; ++u) raw[u] = crc[u];
}

template <bool kFast>
__device__ __forceinline__ uint32_t chunk_raw(const uint8_t* lds, const LaneBase& lb, const BufInfo& bi,
                                              uint32_t c, int lane, const Piece& pc) {
  const BufInfo b1[1] = {bi};
  const uint32_t c1[1] = {c};
  const Piece p1[1] = {pc};
  uint32_t r1[1];
  group_raw<kFast, 1>(lds, lb, b1, c1, lane, p1, r1);
  return r1[0];
}

// Buffers shorter than 4 bytes: bytewise (util/crc32c.cc:287 STEP1), lane-uniform.
__device__ __forceinline__ uint32_t tiny_crc(const uint8_t* lds, const BufInfo& bi) {
  uint32_t l = bi.s;  // = ~init
  for (uint32_t k = 0; k < (uint32_t)bi.len; ++k) {
    const uint32_t b = bi.p[k];
    l = lds_u32(lds, ((l ^ b) & 0xFFu) << 8) ^ (l >> 8);  // T0, replica 0
  }
  return ~l;
}

struct KArgs {
  uint32_t* out;
  uint32_t flags;
  Rec* recs;  // 2 per wave: [2w] = head portion, [2w+1] = tail portion (or nullptr)
  const uint32_t* tables;
};

// Position of one chunk inside a wave's range.
struct Pos {
  uint64_t i;  // buffer
  uint32_t c;  // chunk within the buffer
  BufInfo bi;
};

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

// Per-wave accumulation over consecutive chunks (wave-uniform).
struct WaveState {
  uint32_t acc, cnt;
  bool from_zero;
  Rec head;
};

__device__ __forceinline__ void consume(WaveState& st, const Pos& p, uint32_t raw, const uint8_t* lds, int lane,
                                        const KArgs& ka) {
  st.acc = st.cnt ? (shift4096(lds, st.acc, lane) ^ raw) : raw;
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

#if defined(NVL_DIAG_STAMPS)
// Diagnostic build only: per-wave {start, after-fill, end} s_memtime stamps
// and the XCC id, read back with nvl_diag_stamps().
__device__ unsigned long long g_stamps[4 * 65536];
#endif

template <bool kFast, int U, class G>
__device__ __forceinline__ void run_waves(const G& g, const KArgs& ka, uint8_t* lds) {
#if defined(NVL_DIAG_STAMPS)
  const unsigned long long ts0 = __builtin_amdgcn_s_memrealtime();
#endif

  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerWG + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * kWavesPerWG;

  const uint64_t T = g.total();
  const uint64_t t0 = T * wave / nw;
  const uint64_t t1 = T * (wave + 1) / nw;

  // Issue the first chunks' HBM loads before building the LDS tables so the
  // table fill hides under their latency.
  Pos p;
  Pos gp[U];
  Piece cur[U];
  const bool grouped = (U > 1) && (t0 + U <= t1);
  if (t0 < t1) {
    g.locate(t0, p.i, p.c);
    p.bi = g.info(p.i);
    if (grouped) {
      gp[0] = p;
#pragma unroll
      for (int u = 1; u < U; ++u) gp[u] = next_pos(g, gp[u - 1]);
#pragma unroll
      for (int u = 0; u < U; ++u) load_piece<kFast>(gp[u].bi, gp[u].c, lane, cur[u]);
    } else {
      load_piece<kFast>(p.bi, p.c, lane, cur[0]);
    }
  }
  fill_lds(lds, ka.tables);
  __syncthreads();
  const LaneBase lb = make_lane_base(lane);
#if defined(NVL_DIAG_STAMPS)
  const unsigned long long ts1 = __builtin_amdgcn_s_memrealtime();
#endif

  Rec tail{kNoBuf, 0u, 0u};
  WaveState st{0u, 0u, true, Rec{kNoBuf, 0u, 0u}};
  if (t0 < t1) {
    st.from_zero = (p.c == 0);
    uint64_t t = t0;
    // ---- U chunks per step, next U prefetched while these compute ----
    if constexpr (U > 1) {
      if (grouped) {
        while (true) {
          const bool more = t + 2 * U <= t1;
          Pos np[U];
          Piece nxt[U];
          if (more) {
            np[0] = next_pos(g, gp[U - 1]);
#pragma unroll
            for (int u = 1; u < U; ++u) np[u] = next_pos(g, np[u - 1]);
#pragma unroll
            for (int u = 0; u < U; ++u) load_piece<kFast>(np[u].bi, np[u].c, lane, nxt[u]);
          }
          BufInfo bis[U];
          uint32_t cs[U], raws[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            bis[u] = gp[u].bi;
            cs[u] = gp[u].c;
          }
          group_raw<kFast, U>(lds, lb, bis, cs, lane, cur, raws);
#pragma unroll
          for (int u = 0; u < U; ++u) consume(st, gp[u], raws[u], lds, lane, ka);
          t += U;
          if (!more) break;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            gp[u] = np[u];
            cur[u] = nxt[u];
          }
        }
        p = (t < t1) ? next_pos(g, gp[U - 1]) : gp[U - 1];  // chunk t, or the last one consumed
        if (t < t1) load_piece<kFast>(p.bi, p.c, lane, cur[0]);
      }
    }
    // ---- remaining chunks one at a time (cur[0] holds chunk t) ----
    for (; t < t1; ++t) {
      Pos q = p;
      Piece nxt;
      if (t + 1 < t1) {
        q = next_pos(g, p);
        load_piece<kFast>(q.bi, q.c, lane, nxt);
      }
      if (!kFast && p.bi.len < 4) {
        const uint32_t v = tiny_crc(lds, p.bi);
        if (lane == 0) ka.out[p.i] = finish(v, ka.flags);
        st.cnt = 0;
        st.from_zero = true;
      } else {
        consume(st, p, chunk_raw<kFast>(lds, lb, p.bi, p.c, lane, cur[0]), lds, lane, ka);
      }
      if (t + 1 < t1) {
        p = q;
        cur[0] = nxt;
      }
    }
    if (st.cnt) {
      if (st.from_zero) tail = Rec{p.i, st.acc, st.cnt};
      else st.head = Rec{p.i, st.acc, st.cnt};
    }
  }
  if (ka.recs && lane == 0) {
    ka.recs[2 * wave] = st.head;
    ka.recs[2 * wave + 1] = tail;
  }
#if defined(NVL_DIAG_STAMPS)
  if (lane == 0 && wave < 65536) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_stamps[4 * wave + 0] = ts0;
    g_stamps[4 * wave + 1] = ts1;
    g_stamps[4 * wave + 2] = __builtin_amdgcn_s_memrealtime();
    g_stamps[4 * wave + 3] = ((unsigned long long)xcc << 32) | (t1 - t0);
  }
#endif
}

// Fixed stride with J == 1 (every chunk is a whole buffer; config 2): the
// workgroup owns a contiguous range of buffers and its 16 waves pull units of
// U buffers from an LDS counter, so fast and slow waves of a CU finish
// together (a static per-wave split left the last wave ~20% behind the mean).
template <int U>
__device__ __forceinline__ void run_dynamic(const FixedGeom& g, const KArgs& ka, uint8_t* lds) {
#if defined(NVL_DIAG_STAMPS)
  const unsigned long long ts0 = __builtin_amdgcn_s_memrealtime();
  uint32_t nproc = 0;
#endif
  const int lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t B0 = g.n * blockIdx.x / gridDim.x;
  const uint64_t B1 = g.n * (blockIdx.x + 1) / gridDim.x;
  const uint32_t nunits = (uint32_t)((B1 - B0 + U - 1) / U);
  uint32_t* ctr = reinterpret_cast<uint32_t*>(lds + kCtrOff);

  auto unit_pos = [&](uint32_t u, int k, Pos& p) -> bool {
    const uint64_t i = B0 + (uint64_t)u * U + (uint64_t)k;
    if (u >= nunits || i >= B1) return false;
    p.i = i;
    p.c = 0;
    p.bi = g.info(i);
    return true;
  };

  uint32_t u = wv;  // first unit pre-assigned; its loads overlap the LDS fill
  Pos gp[U];
  bool ok[U];
  Piece cur[U];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    ok[k] = unit_pos(u, k, gp[k]);
    if (ok[k]) load_piece<true>(gp[k].bi, 0, lane, cur[k]);
  }
  fill_lds(lds, ka.tables);
  __syncthreads();
  const LaneBase lb = make_lane_base(lane);
#if defined(NVL_DIAG_STAMPS)
  const unsigned long long ts1 = __builtin_amdgcn_s_memrealtime();
#endif

  while (u < nunits) {
#if defined(NVL_DIAG_STAMPS)
    ++nproc;
#endif
    uint32_t un = 0;
    if (lane == 0) un = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    un = __builtin_amdgcn_readfirstlane(un);
    Pos np[U];
    bool nok[U];
    Piece nxt[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      nok[k] = unit_pos(un, k, np[k]);
      if (nok[k]) load_piece<true>(np[k].bi, 0, lane, nxt[k]);
    }
    if (ok[U - 1]) {  // full unit
      BufInfo bis[U];
      uint32_t cs[U], raws[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        bis[k] = gp[k].bi;
        cs[k] = 0;
      }
      group_raw<true, U>(lds, lb, bis, cs, lane, cur, raws);
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < U; ++k) ka.out[gp[k].i] = finish(~raws[k], ka.flags);
      }
    } else {  // the range's ragged last unit
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (ok[k]) {
          const uint32_t r = chunk_raw<true>(lds, lb, gp[k].bi, 0, lane, cur[k]);
          if (lane == 0) ka.out[gp[k].i] = finish(~r, ka.flags);
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
#if defined(NVL_DIAG_STAMPS)
  const uint32_t wave = blockIdx.x * kWavesPerWG + wv;
  if (lane == 0 && wave < 65536) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_stamps[4 * wave + 0] = ts0;
    g_stamps[4 * wave + 1] = ts1;
    g_stamps[4 * wave + 2] = __builtin_amdgcn_s_memrealtime();
    g_stamps[4 * wave + 3] = ((unsigned long long)xcc << 32) | nproc;
  }
#endif
}

#ifndef NVL_FAST_U
#define NVL_FAST_U 2  // chunks per wave step on the fast path (tools/ab_bench.py: 2 > 1 > 4)
#endif

template <bool kFast>
__global__ __launch_bounds__(kThreads, 1) void crc32c_fixed_kernel(FixedGeom g, KArgs ka) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
#if !defined(NVL_STATIC_ONLY)
  if constexpr (kFast) {
    if (g.J == 1) {
      run_dynamic<NVL_FAST_U>(g, ka, lds);
      return;
    }
  }
#endif
  run_waves<kFast, kFast ? NVL_FAST_U : 1>(g, ka, lds);
}

__global__ __launch_bounds__(kThreads, 1) void crc32c_var_kernel(VarGeom g, KArgs ka) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  run_waves<false, 1>(g, ka, lds);
}

// Per-buffer chunk counts for the variable-length plan: cnt[i] = J_i, cnt[n] = 0.
__global__ void crc32c_var_counts(const uint64_t* __restrict__ lengths, uint64_t n,
                                  uint64_t* __restrict__ cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint64_t L = lengths[i];
    cnt[i] = L <= kChunk ? 1u : (L + kChunk - 1) / kChunk;
  } else if (i == n) {
    cnt[i] = 0;
  }
}

// Fold the per-wave records of buffers that straddle waves.  One thread per
// wave; the wave where a buffer ENDS walks back over earlier waves.
__global__ void crc32c_fixup_kernel(const Rec* __restrict__ recs, uint32_t nw,
                                    const uint32_t* __restrict__ tables, uint32_t* __restrict__ out,
                                    uint32_t flags) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nw) return;
  const Rec h = recs[2 * w];
  if (h.buf == kNoBuf || !(h.cnt & kRecEnds)) return;
  const uint32_t* x2n = tables + kGX2n;
  uint32_t total = h.raw;
  uint64_t after = h.cnt & ~kRecEnds;  // chunks after the current portion
  // Waves between the buffer's first and last portion either hold a middle
  // portion (head record of this buffer) or have an empty chunk range (no
  // records); the first portion is the tail record of an earlier wave.
  for (int64_t x = (int64_t)w - 1; x >= 0; --x) {
    const Rec hx = recs[2 * x];
    if (hx.buf == h.buf) {  // a middle portion
      total ^= nvl::shift_bytes(x2n, hx.raw, after * kChunk);
      after += hx.cnt & ~kRecEnds;
      continue;
    }
    const Rec tx = recs[2 * x + 1];
    if (tx.buf == h.buf) {  // the first portion
      total ^= nvl::shift_bytes(x2n, tx.raw, after * kChunk);
      break;
    }
    if (hx.buf != kNoBuf || tx.buf != kNoBuf) break;  // unreachable for a consistent plan
  }
  out[h.buf] = finish(~total, flags);
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

static inline hipError_t launch_fixup(const Rec* recs, uint32_t nw, const uint32_t* tables,
                                      uint32_t* out, uint32_t flags, hipStream_t st) {
  const uint32_t tpb = 256;
  hipLaunchKernelGGL(dev::crc32c_fixup_kernel, dim3((nw + tpb - 1) / tpb), dim3(tpb), 0, st, recs, nw,
                     tables, out, flags);
  return hipGetLastError();
}

hipError_t launch_fixed(const LaunchCtx& lc, const uint8_t* base, uint64_t stride, uint64_t len, uint64_t n,
                        const uint32_t* init, uint32_t init_all, uint32_t* out, uint32_t flags, Rec* recs) {
  if (n == 0) return hipSuccess;
  const uint32_t J = len <= dev::kChunk ? 1u : (uint32_t)((len + dev::kChunk - 1) / dev::kChunk);
  const uint64_t T = n * (uint64_t)J;
  uint32_t grid = (uint32_t)std::min<uint64_t>((uint64_t)lc.num_cu, (T + dev::kWavesPerWG - 1) / dev::kWavesPerWG);
  if (grid == 0) grid = 1;
  const bool fast = len > 0 && (len % dev::kChunk) == 0 && ((uintptr_t)base % 16) == 0 && (stride % 16) == 0;
  dev::FixedGeom g{base, stride, len, n, J, init, init_all};
  dev::KArgs ka{out, flags, J > 1 ? recs : nullptr, lc.tables};
  if (fast)
    hipLaunchKernelGGL(dev::crc32c_fixed_kernel<true>, dim3(grid), dim3(dev::kThreads), 0, lc.stream, g, ka);
  else
    hipLaunchKernelGGL(dev::crc32c_fixed_kernel<false>, dim3(grid), dim3(dev::kThreads), 0, lc.stream, g, ka);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || J == 1) return e;
  return launch_fixup(recs, grid * dev::kWavesPerWG, lc.tables, out, flags, lc.stream);
}

uint32_t fixed_grid(int num_cu, uint64_t len, uint64_t n) {
  const uint32_t J = len <= dev::kChunk ? 1u : (uint32_t)((len + dev::kChunk - 1) / dev::kChunk);
  const uint64_t T = n * (uint64_t)J;
  uint32_t grid = (uint32_t)std::min<uint64_t>((uint64_t)num_cu, (T + dev::kWavesPerWG - 1) / dev::kWavesPerWG);
  return grid ? grid : 1;
}

uint32_t waves_per_wg() { return dev::kWavesPerWG; }

#if defined(NVL_DIAG_STAMPS)
extern "C" __attribute__((visibility("default"))) int nvl_diag_stamps(unsigned long long* host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dev::g_stamps), n * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_var_counts(const uint64_t* lengths, uint64_t n, uint64_t* cnt, hipStream_t st) {
  const uint32_t tpb = 256;
  const uint64_t blocks = (n + 1 + tpb - 1) / tpb;
  hipLaunchKernelGGL(dev::crc32c_var_counts, dim3((uint32_t)blocks), dim3(tpb), 0, st, lengths, n, cnt);
  return hipGetLastError();
}

hipError_t launch_var(const LaunchCtx& lc, const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths,
                      const uint64_t* chunk_start, uint64_t n, const uint32_t* init, uint32_t init_all,
                      uint32_t* out, uint32_t flags, Rec* recs) {
  if (n == 0) return hipSuccess;
  const uint32_t grid = (uint32_t)lc.num_cu;
  dev::VarGeom g{base, offsets, lengths, chunk_start, n, init, init_all};
  dev::KArgs ka{out, flags, recs, lc.tables};
  hipLaunchKernelGGL(dev::crc32c_var_kernel, dim3(grid), dim3(dev::kThreads), 0, lc.stream, g, ka);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_fixup(recs, grid * dev::kWavesPerWG, lc.tables, out, flags, lc.stream);
}

}  // namespace nvl
