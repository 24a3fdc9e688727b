// Fixed per-launch cost on gfx950: back-to-back launches of kernels that do
// (almost) nothing, with the engine's launch shape (256 x 1024 threads, 156 KiB
// LDS) and smaller shapes, timed with HIP events over R launches.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int LDS>
__global__ __launch_bounds__(1024) void empty_k(uint32_t* out) {
  __shared__ uint32_t lds[LDS / 4 > 0 ? LDS / 4 : 1];
  if (LDS > 0) {
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = LDS > 0 ? lds[5] : blockIdx.x;
}

template <class F>
static void time_it(const char* name, F launch) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) launch();
  hipDeviceSynchronize();
  const int R = 500;
  hipEventRecord(a);
  for (int i = 0; i < R; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  printf("%-40s %8.2f us/launch\n", name, ms * 1000.0f / R);
}

int main() {
  uint32_t* out;
  hipMalloc(&out, 1 << 20);
  time_it("256 x 1024 thr, 156 KiB LDS", [&] { empty_k<159760><<<256, 1024>>>(out); });
  time_it("256 x 1024 thr, no LDS", [&] { empty_k<0><<<256, 1024>>>(out); });
  time_it("256 x 256 thr, no LDS", [&] { empty_k<0><<<256, 256>>>(out); });
  time_it("1 x 64 thr, no LDS", [&] { empty_k<0><<<1, 64>>>(out); });
  time_it("1024 x 256 thr, no LDS", [&] { empty_k<0><<<1024, 256>>>(out); });
  hipFree(out);
  return 0;
}
