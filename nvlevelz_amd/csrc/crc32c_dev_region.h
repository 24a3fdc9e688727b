// nvlevelz_amd/csrc/crc32c_dev_region.h -- the region path (run_region: a
// region's own 4 KiB chunks, event records, the in-launch fold; DESIGN.md
// §3.7), run by crc32c_region_kernel and crc32c_route_kernel.
#pragma once
#include "crc32c_dev_sched.h"

namespace nvl {
namespace dev {

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

// x^(8L) for a buffer longer than two chunks: x^(8 (L mod 4096)) x^(8*4096*(q mod 256))
// (tables) and x^(2^(23 + b)) for every bit b of q >> 8, q = L div 4096.
__device__ uint32_t xpow8_long(const uint32_t* tables, const uint8_t* lsl, const LaneBase& lb, uint64_t L) {
  uint32_t p = gf_mul_lds(lsl, lb, tables[kTabXp8 + (L & (kChunk - 1u))], tables[kTabPw4k + ((L >> 12) & 255u)]);
  uint32_t b = 23;
  for (uint64_t q = L >> 20; q && b < 64u; q >>= 1, ++b)  // (x2n holds k < 64: L < 2^61)
    if (q & 1u) p = gf_mul_lds(lsl, lb, p, tables[kGX2n + b]);
  return p;
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
  uint32_t ninit, xe, xt;  // x^(-8(4096 - oe)), x^(8L)
  u32x4 vs, ve;
  bool fast;  // inside the region, >= kRegionDirect bytes, every chunk streamed by this workgroup
};
__device__ __forceinline__ FoldIn fold_in(const RegionGeom& g, const uint32_t* tables, const uint8_t* lsl,
                                          const LaneBase& lb, uint64_t i, uint64_t c0w, uint64_t B1) {
  FoldIn f;
  const uint64_t off = ldg64(g.offsets, i), L = ldg64(g.lengths, i);
  f.ninit = ~(g.init ? g.init[i] : g.init_all);
  f.s = g.rel0 + off;
  f.L = L;
  const bool inside = f.s >= g.rs && f.s <= g.re && L <= g.re - f.s;
  f.fast = inside && L >= kRegionDirect && (f.s >> 12) >= c0w && ((f.s + L - 1u) >> 12) < B1;
  const uint64_t s = f.fast ? f.s : 0u, e = f.fast ? f.s + L : 64u;  // (the grid's first chunk otherwise)
  const uint64_t c1 = (e - 1u) >> 12;
  const uint32_t oe = (uint32_t)(e - (c1 << 12));  // in [1, 4096]
  f.vs = ld16c((uintptr_t)g.grid + (s & ~(uint64_t)15));
  f.ve = ld16c((uintptr_t)g.grid + (oe == kChunk ? e - 16u : (e & ~(uint64_t)15)));
  f.xe = tables[kTabXm8 + (kChunk - oe)];
  const uint64_t d = e - s;  // (L, or 64 for a buffer the fold checksums serially)
  f.xt = tables[kTabXp8 + min(d, (uint64_t)(kXp8Len - 1u))];
  if (d >= kXp8Len) f.xt = xpow8_long(tables, lsl, lb, d);  // longer than two chunks: metadata only
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

// shift(v, 4096 d) for d = 1..4 from the fold's byte-sliced tables (tab =
// (d - 1) * 4096, per lane): one level of four lookups (one copy: bank
// conflicts, but half the fold's LDS reads and a quarter of its VALU of the
// two dependent nibble-column shifts it replaces, which measured the same on
// r / v and 1.2 us slower on config 3).  Valid after the fold's table copy.
__device__ __forceinline__ uint32_t shc_lds(const uint8_t* lds, uint32_t v, uint32_t tab) {
  const uint8_t* b = lds + kRShcOff;
  const uint32_t a0 = ((v & 255u) << 2) + tab, a1 = (((v >> 8) & 255u) << 2) + tab;
  const uint32_t a2 = (((v >> 16) & 255u) << 2) + tab, a3 = ((v >> 24) << 2) + tab;
  return xor3(lds_u32(b, a0), lds_u32(b + 1024u, a1), lds_u32(b + 2048u, a2)) ^ lds_u32(b + 3072u, a3);
}

__device__ __forceinline__ bool fold_out(const RegionGeom& g, const uint8_t* lds, const uint8_t* lsl,
                                         const LaneBase& lb, int lane, const FoldIn& f, const uint4& q_s,
                                         const uint4& q_e, uint32_t ti, uint32_t& v) {
  const uint64_t s = f.s, e = f.s + f.L;
  const uint64_t c0 = s >> 12, c1 = (e - 1u) >> 12;
  const uint32_t os = (uint32_t)(s & (kChunk - 1u)), oe = (uint32_t)(e - (c1 << 12));  // oe in [1, 4096]
  const uint32_t r0 = g.raws[c0], r1 = g.raws[c1];
  if ((os && (q_s.z != g.gen || q_s.w != ti)) || (oe != kChunk && (q_e.z != g.gen || q_e.w != ti))) return false;
  const uint32_t qs = os ? q_s.x : 0u;                                   // chunk c0's bytes before s, at its end
  const uint32_t T = (os ? quad_prefix_lds(lsl, lb, q_s.y, f.vs, s & 63u) : 0u) ^ f.ninit;  // R(s) ^ ~init, at s
  const uint32_t ze = oe == kChunk ? r1 : q_e.x;                         // chunk c1's bytes before e, at its end
  const uint32_t re = oe == kChunk ? 0u : quad_prefix_lds(lsl, lb, q_e.y, f.ve, e & 63u);  // R(e), at e
  // One formula for every length: the data terms at chunk c1's end -- X =
  // Qe(s) (one chunk), shift4096(Qe(s) ^ raw c0) (two), or that chained
  // over the chunks in between (longer) -- ^ Ze, unshifted to e, and T
  // straight to e:  (X ^ Ze) x^(-8(4096 - oe)) ^ T x^(8L) ^ R(e)
  // (x^(8L) from fold_in, so T stays off the chain; one- and two-chunk
  // buffers in one slice run no branch of their own).
  uint32_t X = c1 == c0 ? qs : shc_lds(lds, qs ^ r0, 0u);
  if (c1 > c0 + 1u) {
    // longer: from chunk c0's end up to four chunks per step -- acc at
    // chunk c + k's end = shift(acc, 4096 k) ^ the raws of chunks c + 1 ..
    // c + k below c1, each shifted by its own distance (independent of acc:
    // one dependent lookup level per step); the next step's raws in flight
    uint32_t acc = qs ^ r0;
    uint32_t rr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) rr[j] = g.raws[min(c0 + 1u + (uint64_t)j, c1 - 1u)];
    for (uint64_t c = c0; c < c1;) {
      const uint32_t k = (uint32_t)min(c1 - c, (uint64_t)4);
      const uint64_t cn = c + k;
      uint32_t rn[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) rn[j] = g.raws[min(cn + 1u + (uint64_t)j, c1 - 1u)];
      uint32_t x = shc_lds(lds, acc, (k - 1u) << 12);
#pragma unroll
      for (uint32_t j = 1; j <= 4u; ++j) {  // chunk c + j: below c1 iff c + j < c1 (then j <= k)
        const uint32_t rj = c + j < c1 ? rr[j - 1u] : 0u;
        x ^= j < k ? shc_lds(lds, rj, (k - j - 1u) << 12) : rj;  // (j > k: rj = 0)
      }
      acc = x;
#pragma unroll
      for (int j = 0; j < 4; ++j) rr[j] = rn[j];
      c = cn;
    }
    X = acc;
  }
  v = gf_mul_lds(lsl, lb, f.xe, X ^ ze) ^ gf_mul_lds(lsl, lb, f.xt, T) ^ re;
  return true;
}

// LDS slots in the region image's lane-63 column (never read by the lane
// shifts): row r at r * 256 + 252, rows 0..15, zeroed by the fill (rows
// 64..127 take the fold's chunk-shift tables once the chunks are done).
// (generic pointer: the volatile accesses become flat loads, which count in
// vmcnt as well; an LDS-qualified pointer was measured slower, see load_unit)
typedef volatile uint32_t lds_vu32;
__device__ __forceinline__ lds_vu32* region_slot(uint8_t* lds, uint32_t r) {
  return (lds_vu32*)(lds + kRNibOff + r * 256u + 252u);
}
constexpr uint32_t kSlotOwnLo = 1, kSlotOwnHi = 2, kSlotEndLo = 3, kSlotEndHi = 4, kSlotHalo = 5;
// (row 6: the halo published; rows 7..10: the fold's slice counters per SIMD;
// row 11 counts the workgroup's waves per SIMD, one byte each)
constexpr uint32_t kSlotReady = 6, kSlotTail = 7, kSlotWaves = 11;

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
      v = __hip_atomic_fetch_add(const_cast<uint32_t*>(region_slot(lds, kSlotTail + cs)), 1u,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return (uint64_t)cs + 4u * (uint64_t)uniform_u32(v);
  };
  const uint8_t* lsl = lds + (kRSliceOff - kSliceOff);
  uint64_t k = claim();
  FoldIn f;
  if (k < nsl) f = fold_in(g, ka.tables, lsl, lb, min(ib + 64u * k + (uint64_t)lane, ib1 - 1u), c0w, B1);
  const uint4 shc = reinterpret_cast<const uint4*>(ka.tables + kTabShc)[threadIdx.x];  // 16 KiB: one per thread
  static_assert(kTabShc % 4u == 0 && 4u * 1024u == 4u * (uint32_t)kThreads, "fold tables: one uint4 per thread");
  __syncthreads();  // every unit done: the nibble tables are free
  reinterpret_cast<uint4*>(lds + kRShcOff)[threadIdx.x] = shc;
  __syncthreads();
  NVL_TL(3);
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
      if (k < nsl) f = fold_in(g, ka.tables, lsl, lb, min(ib + 64u * k + (uint64_t)lane, ib1 - 1u), c0w, B1);
    }
    if (!adopt) break;
    cs = (uint32_t)__builtin_ctz(adopt);
    adopt &= adopt - 1u;
    k = claim();
    if (k < nsl) f = fold_in(g, ka.tables, lsl, lb, min(ib + 64u * k + (uint64_t)lane, ib1 - 1u), c0w, B1);
  }
  NVL_TL_END();
}


}  // namespace dev
}  // namespace nvl
