// nvlevelz_amd/csrc/crc32c_region.hip -- region batches and routed calls:
// crc32c_region_kernel (nvl_crc32c_region_dev with
// NVL_CRC32C_FLAG_REGION_SHAPED, the host region entry), the route plan
// and the route kernel (nvl_crc32c_batch_dev / checked region_dev:
// DESIGN.md §3.7-3.8).
#include <atomic>
#include <random>

#include "crc32c_dev_region.h"
#include "crc32c_launch.h"

namespace nvl {
namespace dev {
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

}  // namespace dev

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
  return launch_var_body(lc, vg, kf);
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
