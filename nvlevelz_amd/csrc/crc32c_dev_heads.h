// nvlevelz_amd/csrc/crc32c_dev_heads.h -- the head path (run_heads: every
// buffer's partial first chunk, short mode, the variable-length plan's tile
// scan) and its kernel template crc32c_head_kernel<G>.
#pragma once
#include "crc32c_dev_sched.h"

namespace nvl {
namespace dev {

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

}  // namespace dev
}  // namespace nvl
