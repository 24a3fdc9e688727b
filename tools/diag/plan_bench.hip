// Timing of the one-workgroup variable-length plan kernel in isolation,
// with ablations (PLAN_VARIANT): 0 = as shipped, 1 = no cs/unit_first stores,
// 2 = stores but no unit map, 3 = only the length loads + LDS staging.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I nvlevelz_amd/csrc tools/diag/plan_bench.hip -o tools/diag/plan_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <random>
#include "crc32c_kernels.hip"

using namespace nvl::dev;

template <int V>
__global__ __launch_bounds__(kPlanThreads) void plan_v(const uint64_t* __restrict__ lengths, uint64_t n, uint64_t NU,
                                                       uint64_t* __restrict__ cs, uint64_t* __restrict__ unit_first) {
  __shared__ uint32_t js[kPlanSmallMax + kPlanSmallMax / 32];
  __shared__ uint64_t wsum[kPlanThreads / kWave];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t nn = (uint32_t)n;
  {
    constexpr int kPer = (int)(kPlanSmallMax / kPlanThreads);
    uint64_t Ls[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = t + (uint32_t)k * (uint32_t)kPlanThreads;
      Ls[k] = i < nn ? lengths[i] : 0;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = t + (uint32_t)k * (uint32_t)kPlanThreads;
      if (i < nn) js[plan_pad(i)] = Ls[k] <= kChunk ? 1u : (uint32_t)((Ls[k] + kChunk - 1) / kChunk);
    }
  }
  __syncthreads();
  if (V == 3) { if (t == 0) cs[0] = js[5]; return; }
  const uint32_t per = (nn + (uint32_t)kPlanThreads - 1) / (uint32_t)kPlanThreads;
  const uint32_t i0 = min(nn, t * per), i1 = min(nn, i0 + per);
  uint64_t sum = 0;
  for (uint32_t i = i0; i < i1; ++i) sum += js[plan_pad(i)];
  uint64_t x = sum;
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
  uint64_t run = before + x - sum;
  if (t == 0) cs[n] = T;
  uint64_t u = ceil_div_u64(run * NU, T);
  uint64_t tu = T * u, cn = run * NU;
  uint64_t acc = 0;
  for (uint32_t i = i0; i < i1; ++i) {
    if (V != 1) cs[i] = run; else acc += run;
    const uint32_t j = js[plan_pad(i)];
    run += j;
    cn += (uint64_t)j * NU;
    if (V == 2) continue;
    for (; u < NU && tu < cn; ++u, tu += T) { if (V != 1) unit_first[u] = i; else acc ^= i; }
  }
  if (V == 1 && acc == 12345) cs[0] = acc;
}

int main() {
  const uint64_t n = 32672, NU = 256 * 64;
  std::vector<uint64_t> L(n);
  std::mt19937_64 r(3);
  for (auto& x : L) x = 512 + r() % 65025;
  uint64_t *dL, *dcs, *duf;
  hipMalloc(&dL, n * 8); hipMalloc(&dcs, (n + 1) * 8); hipMalloc(&duf, NU * 8);
  hipMemcpy(dL, L.data(), n * 8, hipMemcpyHostToDevice);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto run = [&](const char* name, auto kern) {
    for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(kern, dim3(1), dim3(1024), 0, 0, dL, n, NU, dcs, duf);
    hipEventRecord(a);
    for (int w = 0; w < 50; ++w) hipLaunchKernelGGL(kern, dim3(1), dim3(1024), 0, 0, dL, n, NU, dcs, duf);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-28s %8.2f us/launch\n", name, ms * 1000 / 50);
  };
  run("shipped crc32c_plan_small", crc32c_plan_small);
  run("v0 (copy)", plan_v<0>);
  run("v1 no stores", plan_v<1>);
  run("v2 cs stores, no unit map", plan_v<2>);
  run("v3 loads+LDS only", plan_v<3>);
  return 0;
}
