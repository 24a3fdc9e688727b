// The measured read-only ceiling SURVEY.md §8d asks for beside the 8 TB/s
// spec: plain streaming kernels that only read a 410 MB buffer (config 2's
// bytes) and XOR-reduce it, in several launch shapes and load forms; per
// shape the sustained period over 200 back-to-back launches after warm-up
// (HIP events), in us and TB/s.  Build: hipcc -O3 --offload-arch=gfx950
// tools/diag/hbm_ceiling.hip -o tools/diag/hbm_ceiling
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// grid-stride, UNROLL independent 16-byte loads per thread per step
template <int UNROLL, bool NT>
__global__ void stream_k(const u32x4* __restrict__ p, uint64_t n16, uint32_t* out) {
  uint32_t x = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) v[k] = NT ? __builtin_nontemporal_load(p + i + k * stride) : p[i + k * stride];
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  for (; i < n16; i += stride) {
    const u32x4 v = p[i];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) out[0] = x;
}

// contiguous 4 KiB blocks per workgroup (the engine's access shape): block b
// of 64 lanes x 16 B x 4 rows, workgroups take blocks b, b + G, ...
template <bool NT>
__global__ void blocks_k(const uint8_t* __restrict__ p, uint64_t nblocks, uint32_t* out) {
  uint32_t x = 0;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (uint64_t b = (uint64_t)blockIdx.x * nw + wv; b < nblocks; b += (uint64_t)gridDim.x * nw) {
    const u32x4* q = reinterpret_cast<const u32x4*>(p + b * 4096u);
    u32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = NT ? __builtin_nontemporal_load(q + 64 * j + lane) : q[64 * j + lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) x ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  if (x == 0x12345678u) out[0] = x;
}

// D 4-KiB blocks per wave per step, loaded together (bytes in flight per
// wave = D x 4 KiB), at the engine's occupancy (256 x 1024)
template <int D>
__global__ void blocksD_k(const uint8_t* __restrict__ p, uint64_t nblocks, uint32_t* out) {
  uint32_t x = 0;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint64_t W = (uint64_t)gridDim.x * nw;
  for (uint64_t b = ((uint64_t)blockIdx.x * nw + wv) * D; b < nblocks; b += W * D) {
    u32x4 v[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const u32x4* q = reinterpret_cast<const u32x4*>(p + min(b + d, nblocks - 1) * 4096u);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[d][j] = __builtin_nontemporal_load(q + 64 * j + lane);
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int j = 0; j < 4; ++j) x ^= v[d][j].x ^ v[d][j].y ^ v[d][j].z ^ v[d][j].w;
  }
  if (x == 0x12345678u) out[0] = x;
}

// 4 blocks per wave at a quarter of the batch apart, taken row by row: step
// j loads row j (1 KiB) of each of the 4 blocks -- 4 KiB per wave in flight,
// as blocks_k, but from four distant places (the grid-stride streamer's
// spread) -- a layout a CRC kernel could use (each row is 16 whole pieces).
__global__ void blocks_spread_k(const uint8_t* __restrict__ p, uint64_t nblocks, uint32_t* out) {
  uint32_t x = 0;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint64_t Q = nblocks / 4, W = (uint64_t)gridDim.x * nw;
  for (uint64_t b = (uint64_t)blockIdx.x * nw + wv; b < Q; b += W) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      u32x4 v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        v[c] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (b + (uint64_t)c * Q) * 4096u) + 64 * j + lane);
#pragma unroll
      for (int c = 0; c < 4; ++c) x ^= v[c].x ^ v[c].y ^ v[c].z ^ v[c].w;
    }
  }
  if (x == 0x12345678u) out[0] = x;
}
// the same four blocks adjacent (b, b+1, b+2, b+3), row by row
__global__ void blocks_rows_adj_k(const uint8_t* __restrict__ p, uint64_t nblocks, uint32_t* out) {
  uint32_t x = 0;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint64_t W = (uint64_t)gridDim.x * nw;
  for (uint64_t b = ((uint64_t)blockIdx.x * nw + wv) * 4; b + 3 < nblocks; b += W * 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      u32x4 v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        v[c] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (b + (uint64_t)c) * 4096u) + 64 * j + lane);
#pragma unroll
      for (int c = 0; c < 4; ++c) x ^= v[c].x ^ v[c].y ^ v[c].z ^ v[c].w;
    }
  }
  if (x == 0x12345678u) out[0] = x;
}

// blocks_k with a dynamic LDS allocation that caps workgroups per CU
// (occupancy sweep: waves per CU at 1 or 2 workgroups per CU)
__global__ void blocks_dyn_k(const uint8_t* __restrict__ p, uint64_t nblocks, uint32_t* out) {
  extern __shared__ uint32_t dyn[];
  uint32_t x = 0;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (uint64_t b = (uint64_t)blockIdx.x * nw + wv; b < nblocks; b += (uint64_t)gridDim.x * nw) {
    const u32x4* q = reinterpret_cast<const u32x4*>(p + b * 4096u);
    u32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = __builtin_nontemporal_load(q + 64 * j + lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) x ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  if (x == 0x12345678u) { dyn[threadIdx.x] = x; out[0] = dyn[(threadIdx.x + 1) % blockDim.x]; }
}

template <class F>
static float period(F launch, int R = 200) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 100; ++i) launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < R; ++i) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.0f / R;
}

int main() {
  const uint64_t bytes = 410000000ull / 4096 * 4096;  // 100096 KiB-blocks ~ config 2's 4.1e8 B
  uint8_t* p;
  uint32_t* out;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(p, 0x5a, bytes);
  const uint64_t n16 = bytes / 16, nblk = bytes / 4096;
  auto rep = [&](const char* what, float us) {
    printf("{\"shape\": \"%s\", \"bytes\": %llu, \"period_us\": %.2f, \"TB_s\": %.3f, \"frac_of_8TBs\": %.4f}\n", what,
           (unsigned long long)bytes, us, bytes / (us * 1e-6) / 1e12, bytes / (us * 1e-6) / 8e12);
  };
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  if (getenv("OCC_SWEEP")) {
    (void)hipFuncSetAttribute((const void*)blocks_dyn_k, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024);
    char what[128];
    for (int pass = 0; pass < 2; ++pass) {
      for (int T : {1024, 768}) {  // one workgroup per CU (100 KiB LDS)
        snprintf(what, sizeof what, "4 KiB blocks per wave, 256 x %d, 1 WG/CU (%d waves/CU)", T, T / 64);
        rep(what, period([&] { hipLaunchKernelGGL(blocks_dyn_k, dim3(256), dim3(T), 100 * 1024, 0, p, nblk, out); }));
      }
      for (int T : {512, 640, 768, 896, 1024}) {  // two per CU (72 KiB LDS)
        snprintf(what, sizeof what, "4 KiB blocks per wave, 512 x %d, 2 WG/CU (%d waves/CU)", T, 2 * T / 64);
        rep(what, period([&] { hipLaunchKernelGGL(blocks_dyn_k, dim3(512), dim3(T), 72 * 1024, 0, p, nblk, out); }));
      }
      for (int T : {256, 320, 384}) {  // four per CU (36 KiB LDS)
        snprintf(what, sizeof what, "4 KiB blocks per wave, 1024 x %d, 4 WG/CU (%d waves/CU)", T, 4 * T / 64);
        rep(what, period([&] { hipLaunchKernelGGL(blocks_dyn_k, dim3(1024), dim3(T), 36 * 1024, 0, p, nblk, out); }));
      }
    }
    return 0;
  }
  for (int pass = 0; pass < 2; ++pass) {
    rep("grid-stride 256 x 1024, 1 x 16 B nt", period([&] { hipLaunchKernelGGL((stream_k<1, true>), dim3(256), dim3(1024), 0, 0, q, n16, out); }));
    rep("grid-stride 256 x 1024, 4 x 16 B nt", period([&] { hipLaunchKernelGGL((stream_k<4, true>), dim3(256), dim3(1024), 0, 0, q, n16, out); }));
    rep("grid-stride 256 x 1024, 4 x 16 B", period([&] { hipLaunchKernelGGL((stream_k<4, false>), dim3(256), dim3(1024), 0, 0, q, n16, out); }));
    rep("grid-stride 1024 x 256, 4 x 16 B nt", period([&] { hipLaunchKernelGGL((stream_k<4, true>), dim3(1024), dim3(256), 0, 0, q, n16, out); }));
    rep("grid-stride 2048 x 512, 2 x 16 B nt", period([&] { hipLaunchKernelGGL((stream_k<2, true>), dim3(2048), dim3(512), 0, 0, q, n16, out); }));
    rep("4 KiB blocks per wave, 256 x 1024 nt", period([&] { hipLaunchKernelGGL((blocks_k<true>), dim3(256), dim3(1024), 0, 0, p, nblk, out); }));
    rep("4 KiB blocks per wave, 256 x 1024", period([&] { hipLaunchKernelGGL((blocks_k<false>), dim3(256), dim3(1024), 0, 0, p, nblk, out); }));
    rep("4 KiB blocks per wave, 2048 x 256 nt", period([&] { hipLaunchKernelGGL((blocks_k<true>), dim3(2048), dim3(256), 0, 0, p, nblk, out); }));
    rep("2 x 4 KiB blocks per wave per step, 256 x 1024 nt", period([&] { hipLaunchKernelGGL((blocksD_k<2>), dim3(256), dim3(1024), 0, 0, p, nblk, out); }));
    rep("3 x 4 KiB blocks per wave per step, 256 x 1024 nt", period([&] { hipLaunchKernelGGL((blocksD_k<3>), dim3(256), dim3(1024), 0, 0, p, nblk, out); }));
    rep("4 x 4 KiB blocks per wave per step, 256 x 1024 nt", period([&] { hipLaunchKernelGGL((blocksD_k<4>), dim3(256), dim3(1024), 0, 0, p, nblk, out); }));
    rep("4 distant blocks per wave row by row, 256 x 1024 nt", period([&] { hipLaunchKernelGGL(blocks_spread_k, dim3(256), dim3(1024), 0, 0, p, nblk, out); }));
    rep("4 adjacent blocks per wave row by row, 256 x 1024 nt", period([&] { hipLaunchKernelGGL(blocks_rows_adj_k, dim3(256), dim3(1024), 0, 0, p, nblk, out); }));
  }
  return 0;
}
