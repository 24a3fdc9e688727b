// Streaming-load ceiling of the chunk access pattern used by the CRC kernels,
// as a function of (a) the loads each wave keeps in flight and (b) the
// alignment of the chunk start.  One 1024-thread workgroup per CU, 16 waves,
// the kernels' permuted lane order (lane (a,b) reads 1024j + 64b + 16a).
//   D = chunks in flight per wave (software pipeline depth 1..3)
//   MIS = byte offset of every chunk start (0, 4, 1, 13)
// Loads only: each wave XORs what it loaded so nothing is dead.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const u32x4 __attribute__((address_space(1)))* gp;

__device__ __forceinline__ u32x4 ld(uintptr_t a) { return __builtin_nontemporal_load((gp)a); }

template <int D, int MIS>
__global__ __launch_bounds__(1024, 1) void stream(const uint8_t* buf, uint64_t nchunks, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const uint32_t lo = ((uint32_t)(lane & 15) << 6) | ((uint32_t)(lane >> 4) << 4);
  const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * 16;
  uint32_t acc = 0;
  u32x4 v[D][4];
  uint64_t t = wave;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const uint64_t c = t + (uint64_t)d * nw;
    const uintptr_t base = (uintptr_t)buf + (c < nchunks ? c : 0) * 4096 + MIS;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[d][j] = ld(base + 1024 * j + lo);
  }
  for (; t < nchunks; t += nw) {
    u32x4 w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = v[0][j];
#pragma unroll
    for (int d = 0; d + 1 < D; ++d)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[d][j] = v[d + 1][j];
    const uint64_t c = t + (uint64_t)D * nw;
    const uintptr_t base = (uintptr_t)buf + (c < nchunks ? c : 0) * 4096 + MIS;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[D - 1][j] = ld(base + 1024 * j + lo);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= w[j].x ^ w[j].y ^ w[j].z ^ w[j].w;
  }
  if (lane == 0) out[wave] = acc;
}

int main() {
  const uint64_t n = 262144;  // 1 GiB of chunks
  uint8_t* buf;
  if (hipMalloc(&buf, n * 4096 + 4096) != hipSuccess) return 2;
  hipMemset(buf, 0x5a, n * 4096 + 4096);
  uint32_t* o2;
  hipMalloc(&o2, 1 << 20);
  int cu = 0;
  hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
#define RUN(D, M)                                                                              \
  {                                                                                            \
    std::vector<float> ts;                                                                     \
    for (int r = 0; r < 30; ++r) {                                                             \
      hipEventRecord(a);                                                                       \
      hipLaunchKernelGGL((stream<D, M>), dim3(cu), dim3(1024), 0, 0, buf, n, o2);              \
      hipEventRecord(b);                                                                       \
      hipEventSynchronize(b);                                                                  \
      float ms;                                                                                \
      hipEventElapsedTime(&ms, a, b);                                                          \
      if (r > 4) ts.push_back(ms);                                                             \
    }                                                                                          \
    std::sort(ts.begin(), ts.end());                                                           \
    const float us = ts[ts.size() / 2] * 1000;                                                 \
    printf("{\"depth\": %d, \"misalign\": %d, \"us\": %.1f, \"GB/s\": %.1f}\n", D, M, us,       \
           n * 4096.0 / us / 1e3);                                                             \
  }
  RUN(1, 0) RUN(2, 0) RUN(3, 0)
  RUN(1, 4) RUN(2, 4) RUN(3, 4)
  RUN(1, 1) RUN(2, 1) RUN(3, 1)
  RUN(2, 13) RUN(3, 13)
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
