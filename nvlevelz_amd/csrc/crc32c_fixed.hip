// nvlevelz_amd/csrc/crc32c_fixed.hip -- fixed-stride batches
// (nvl_crc32c_fixed_dev: configs 2, 4, 5, db_bench's crc32c loop): the
// scheduler-A kernels, the chunk-parallel kernel and its folds, the
// general / record kernels and their fix-up.
#include "crc32c_launch.h"

namespace nvl {
namespace dev {

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

}  // namespace dev

hipError_t launch_fixup(const Rec* recs, uint32_t nw, uint32_t* out, uint32_t flags, hipStream_t st,
                        hipEvent_t ev_stop) {
  const uint32_t wpb = 4;  // one wave per unit
  const dim3 grid((nw + wpb - 1) / wpb), block(dev::kWave * wpb);
  if (ev_stop)
    hipExtLaunchKernelGGL(dev::crc32c_fixup_kernel, grid, block, 0, st, nullptr, ev_stop, 0u, recs, nw, out, flags);
  else
    hipLaunchKernelGGL(dev::crc32c_fixup_kernel, grid, block, 0, st, recs, nw, out, flags);
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

}  // namespace nvl
