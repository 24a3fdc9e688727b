// nvlevelz_amd/csrc/crc32c_dev_sched.h -- schedulers A (fixed stride,
// whole-chunk units), B (chunk-range work units with records) and C (whole
// buffers per wave) over the crc32c_dev.h primitives.
#pragma once
#include "crc32c_dev.h"

namespace nvl {
namespace dev {

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


constexpr int kFastU = 2;  // buffers per unit in scheduler A (tools/ab_bench.py: 2 > 1 > 4)

constexpr int kGenWaves = 16;  // waves per workgroup of the kGeneral kernels
constexpr int kGenPairU = 2;   // buffers per unit (g: 67.7 us at 2, 70.4 at 1, 91.7 through run_units)
template <int M>
constexpr int waves_of() { return M == kGeneral ? kGenWaves : kWavesPerWG; }

// Tiles of the variable-length plan (head kernel workgroups): list entries hold a 10-bit index.
constexpr uint32_t kMaxTiles = 1023;

}  // namespace dev
}  // namespace nvl
