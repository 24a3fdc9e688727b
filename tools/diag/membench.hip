// Read-bandwidth micro-benchmark for the CRC engine's access pattern.
// Each wave reads 4 KiB chunks as four coalesced 1 KiB rows (dwordx4/lane),
// XOR-reduces them (keeps loads live) and writes one word per chunk.
//   mode 0: contiguous chunk range per wave (the engine's partition)
//   mode 1: grid-stride (wave w reads chunks w, w+W, ...)
// DEPTH = chunks in flight per wave (software prefetch), WPG = waves per WG.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const u32x4 __attribute__((address_space(1)))* gp;

template <int DEPTH, bool NT>
__device__ __forceinline__ void ld(uintptr_t base, int lane, u32x4 (&v)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    gp a = (gp)(base + 1024u * j + 16u * lane);
    v[j] = NT ? __builtin_nontemporal_load(a) : *a;
  }
}

template <int DEPTH, bool NT, int MODE>
__global__ __launch_bounds__(1024) void rd(const uint8_t* buf, uint64_t n, uint32_t* out, int wpg) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * wpg + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * wpg;
  uint64_t t0, t1, step;
  if (MODE == 0) { t0 = n * wave / nw; t1 = n * (wave + 1) / nw; step = 1; }
  else { t0 = wave; t1 = n; step = nw; }
  u32x4 q[DEPTH][4];
  uint64_t t = t0;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) if (t + d * step < t1) ld<DEPTH, NT>((uintptr_t)buf + (t + d * step) * 4096, lane, q[d]);
  uint32_t acc = 0;
  for (; t < t1; t += DEPTH * step) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const uint64_t tt = t + d * step;
      if (tt < t1) {
        u32x4 x = q[d][0] ^ q[d][1] ^ q[d][2] ^ q[d][3];
        acc ^= x.x ^ x.y ^ x.z ^ x.w;
        const uint64_t nx = tt + DEPTH * step;
        if (nx < t1) ld<DEPTH, NT>((uintptr_t)buf + nx * 4096, lane, q[d]);
      }
    }
  }
  acc ^= __shfl_xor(acc, 32);
  if (lane == 0) out[wave] = acc;
}

template <int DEPTH, bool NT, int MODE>
float run(const uint8_t* buf, uint64_t n, uint32_t* out, int grid, int wpg) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  std::vector<float> ts;
  for (int r = 0; r < 30; ++r) {
    hipEventRecord(a);
    hipLaunchKernelGGL((rd<DEPTH, NT, MODE>), dim3(grid), dim3(64 * wpg), 0, 0, buf, n, out, wpg);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); if (r >= 5) ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2] * 1000.f;
}

int main() {
  const uint64_t nmax = 1000000;
  uint8_t* buf; uint32_t* out;
  hipMalloc(&buf, nmax * 4096); hipMalloc(&out, 1 << 20);
  hipMemset(buf, 1, nmax * 4096);
  for (uint64_t n : {100000ull, 1000000ull}) {
    for (int wpg : {16, 8}) {
      int grid = 256 * (16 / wpg);  // same total waves: 4096
      #define R(D, NT, M) do { float us = run<D, NT, M>(buf, n, out, grid, wpg); \
        printf("n=%-8llu wpg=%-2d depth=%d nt=%d mode=%d  %8.2f us  %7.1f GB/s\n", (unsigned long long)n, wpg, D, NT, M, us, n * 4096.0 / us / 1e3); } while (0)
      R(1, true, 0); R(2, true, 0); R(3, true, 0); R(4, true, 0);
      R(2, false, 0); R(2, true, 1); R(4, true, 1);
    }
    // more waves: 2 WGs/CU of 1024 (no LDS here) -> 8192 waves
    float us = run<2, true, 0>(buf, n, out, 512, 16);
    printf("n=%-8llu grid=512x16 depth=2 nt=1 mode=0  %8.2f us  %7.1f GB/s\n", (unsigned long long)n, us, n * 4096.0 / us / 1e3);
    us = run<2, true, 1>(buf, n, out, 512, 16);
    printf("n=%-8llu grid=512x16 depth=2 nt=1 mode=1  %8.2f us  %7.1f GB/s\n", (unsigned long long)n, us, n * 4096.0 / us / 1e3);
  }
  return 0;
}
