// Does gfx950 serve byte-misaligned global_load_dwordx4 (ROCm unaligned mode),
// and at what streaming bandwidth?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const u32x4 __attribute__((address_space(1)))* gp;

__global__ void probe(const uint8_t* buf, uint32_t off, u32x4* out) {
  out[threadIdx.x] = __builtin_nontemporal_load((gp)(buf + off + 16 * threadIdx.x));
}

template <int MIS>
__global__ __launch_bounds__(1024) void stream(const uint8_t* buf, uint64_t nchunks, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * 16;
  uint32_t acc = 0;
  for (uint64_t t = wave; t < nchunks; t += nw) {
    const uintptr_t base = (uintptr_t)buf + t * 4096 + MIS;
    u32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = __builtin_nontemporal_load((gp)(base + 1024 * j + 16 * lane));
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  if (lane == 0) out[wave] = acc;
}

int main() {
  const uint64_t n = 262144;  // 1 GiB
  uint8_t* buf; hipMalloc(&buf, n * 4096 + 64);
  std::vector<uint8_t> h(1 << 20);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)(i * 131 + (i >> 8));
  hipMemcpy(buf, h.data(), h.size(), hipMemcpyHostToDevice);
  u32x4* out; hipMalloc(&out, 64 * 16);
  int bad = 0;
  for (uint32_t off : {0u, 1u, 2u, 3u, 4u, 5u, 7u, 8u, 13u, 15u, 4093u}) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, buf, off, out);
    std::vector<uint8_t> o(64 * 16);
    hipError_t e = hipMemcpy(o.data(), out, o.size(), hipMemcpyDeviceToHost);
    int b = 0;
    for (int i = 0; i < 64 * 16; ++i) b += o[i] != h[off + i];
    printf("offset %4u: %s (%s)\n", off, b ? "MISMATCH" : "ok", hipGetErrorString(e));
    bad += b;
  }
  uint32_t* o2; hipMalloc(&o2, 1 << 20);
  hipEvent_t a, bb; hipEventCreate(&a); hipEventCreate(&bb);
  #define RUN(M) { std::vector<float> ts; for (int r = 0; r < 25; ++r) { hipEventRecord(a); \
      hipLaunchKernelGGL(stream<M>, dim3(256), dim3(1024), 0, 0, buf, n, o2); hipEventRecord(bb); \
      hipEventSynchronize(bb); float ms; hipEventElapsedTime(&ms, a, bb); if (r > 4) ts.push_back(ms); } \
      std::sort(ts.begin(), ts.end()); float us = ts[ts.size()/2] * 1000; \
      printf("misalign %2d: %8.1f us  %7.1f GB/s\n", M, us, n * 4096.0 / us / 1e3); }
  RUN(0) RUN(1) RUN(3) RUN(4) RUN(8) RUN(13)
  return bad ? 1 : 0;
}
