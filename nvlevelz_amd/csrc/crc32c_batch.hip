// nvlevelz_amd/csrc/crc32c_batch.hip -- variable-length batches
// (nvl_crc32c_batch_dev's batch path, the host entries' batches): the
// plan kernels, scheduler B/C's variable kernel, the fused body kernel
// (tiled plan, edge records) and the page path.
#include "crc32c_launch.h"

namespace nvl {
namespace dev {
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

}  // namespace dev

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

// The routed call's third launch (launch_routed): the body kernel over the
// route kernel's verdict -- returns at once on the region path, runs the page
// path, or the batch path's body after the route kernel's heads.
hipError_t launch_var_body(const LaunchCtx& lc, const dev::VarGeom& vg, const dev::KArgs& kf) {
  if (lc.ev_stop)
    hipExtLaunchKernelGGL(dev::crc32c_var_fused_kernel, dim3((uint32_t)lc.num_cu), dim3(dev::kWave * dev::kGenWaves),
                          0, lc.stream, nullptr, lc.ev_stop, 0u, vg, kf);
  else
    hipLaunchKernelGGL(dev::crc32c_var_fused_kernel, dim3((uint32_t)lc.num_cu), dim3(dev::kWave * dev::kGenWaves), 0,
                       lc.stream, vg, kf);
  return hipGetLastError();
}

}  // namespace nvl
