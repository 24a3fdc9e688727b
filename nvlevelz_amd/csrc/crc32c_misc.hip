// nvlevelz_amd/csrc/crc32c_misc.hip -- small kernels beside the engine:
// ReadBlock's trailer checks over a device-resident table, the read-ceiling
// probe and the synthetic-stream fill.
#include "crc32c_launch.h"

namespace nvl {
namespace dev {
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

// Round-robin interleave of gathered shard results (nvl_crc32c_gather_dev):
// src holds shard 0's c_0 results, then shard 1's, ... (c_k = ceil((N-k)/G));
// dst[i] = shard (i mod G)'s result (i div G).
__global__ void interleave_rr_kernel(const uint32_t* __restrict__ src, uint64_t N, uint32_t G,
                                     uint32_t* __restrict__ dst) {
  const uint64_t q = N / G, r = N % G;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = i % G, j = i / G;
    dst[i] = src[k * q + min<uint64_t>(k, r) + j];  // shard k starts after k shards of q (+1 for the first r)
  }
}

// The gather in one launch (nvl_crc32c_gather_dev with at most kGatherMax
// shards, every one on the destination device or peer-mapped to it): each
// result read where its shard wrote it -- no staging copies, no interleave
// pass.  rr: dst[i] = shard (i mod G)'s result (i div G); else shard k's
// results at [pos[k], pos[k+1]).
__global__ void gather_kernel(GatherSrc s, uint64_t N, uint32_t* __restrict__ dst) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t k = 0;
    uint64_t j;
    if (s.rr) {
      k = (uint32_t)(i % s.G);
      j = i / s.G;
    } else {
      while (k + 1u < s.G && i >= s.pos[k + 1]) ++k;
      j = i - s.pos[k];
    }
    dst[i] = s.src[k][j];
  }
}

}  // namespace dev

hipError_t launch_gather(const dev::GatherSrc& s, uint64_t N, uint32_t* dst, hipStream_t st) {
  if (N == 0) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>((N + 255) / 256, 8192);
  hipLaunchKernelGGL(dev::gather_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, s, N, dst);
  return hipGetLastError();
}

hipError_t launch_interleave_rr(const uint32_t* src, uint64_t N, uint32_t G, uint32_t* dst, hipStream_t st) {
  if (N == 0) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>((N + 255) / 256, 65536);
  hipLaunchKernelGGL(dev::interleave_rr_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, src, N, G, dst);
  return hipGetLastError();
}

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

}  // namespace nvl
