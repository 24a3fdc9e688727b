// What a device-side route costs on gfx950: a streaming kernel (400 MB read,
// the engine's 256 x 1024 launch shape) followed back to back by kernels that
// read a flag and return (the batch kernels skipped by a region-shaped batch),
// and a plan-shaped kernel (metadata scan) in front.  Per-sequence period over
// R repetitions, HIP events; the added cost = period - the streaming kernel's.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(1024) void stream_k(const u32x4* __restrict__ p, uint64_t n16, uint32_t* out) {
  uint32_t x = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) out[0] = x;
}

template <int LDS>
__global__ __launch_bounds__(1024) void guarded_k(const uint32_t* flag, uint32_t* out) {
  __shared__ uint32_t lds[LDS / 4 > 0 ? LDS / 4 : 1];
  if (*flag == 0u) return;  // the route says: not this path
  if (LDS > 0) {
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = LDS > 0 ? lds[5] : blockIdx.x;
}

// plan-shaped: each block checks a slice of n (offset, length) pairs for
// sortedness and reduces min/max/sum with device atomics.
__global__ __launch_bounds__(256) void plan_k(const uint64_t* off, const uint64_t* len, uint64_t n, uint64_t* res) {
  uint64_t bad = 0, sum = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t e = off[i] + len[i];
    sum += len[i];
    if (i + 1 < n && e > off[i + 1]) bad = 1;
  }
  for (int s = 32; s; s >>= 1) {
    bad |= __shfl_xor(bad, s);
    sum += __shfl_xor(sum, s);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicOr((unsigned long long*)&res[0], (unsigned long long)bad);
    atomicAdd((unsigned long long*)&res[1], (unsigned long long)sum);
  }
}

template <class F>
static float period(F seq, int R = 200) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 50; ++i) seq();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < R; ++i) seq();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms * 1000.0f / R;
}

int main() {
  const uint64_t bytes = 409600000ull, n = 100000;
  u32x4* p;
  uint32_t *out, *flag;
  uint64_t *meta, *res;
  hipMalloc(&p, bytes);
  hipMemset(p, 1, bytes);
  hipMalloc(&out, 1 << 20);
  hipMalloc(&flag, 256);
  hipMemset(flag, 0, 256);
  hipMalloc(&meta, 2 * n * 8);
  hipMalloc(&res, 256);
  uint64_t* h = (uint64_t*)malloc(2 * n * 8);
  for (uint64_t i = 0; i < n; ++i) {
    h[i] = i * 4101;
    h[n + i] = 4097;
  }
  hipMemcpy(meta, h, 2 * n * 8, hipMemcpyHostToDevice);
  const uint64_t n16 = bytes / 16;
  auto S = [&] { stream_k<<<256, 1024>>>(p, n16, out); };
  for (int rep = 0; rep < 3; ++rep) {
    const float base = period([&] { S(); });
    printf("rep %d: stream alone                       %8.2f us\n", rep, base);
    printf("  + guarded 256x1024 156KiB LDS           %+8.2f us\n",
           period([&] { S(); guarded_k<159760><<<256, 1024>>>(flag, out); }) - base);
    printf("  + 2 x guarded 256x1024 156KiB LDS       %+8.2f us\n",
           period([&] { S(); guarded_k<159760><<<256, 1024>>>(flag, out); guarded_k<159760><<<256, 1024>>>(flag, out); }) - base);
    printf("  + guarded 256x1024 no LDS               %+8.2f us\n",
           period([&] { S(); guarded_k<0><<<256, 1024>>>(flag, out); }) - base);
    printf("  + guarded 1x64                          %+8.2f us\n",
           period([&] { S(); guarded_k<0><<<1, 64>>>(flag, out); }) - base);
    printf("  + plan 64x256 (1e5 pairs) in front      %+8.2f us\n",
           period([&] { plan_k<<<64, 256>>>(meta, meta + n, n, res); S(); }) - base);
    printf("  + plan 256x256 (1e5 pairs) in front     %+8.2f us\n",
           period([&] { plan_k<<<256, 256>>>(meta, meta + n, n, res); S(); }) - base);
    printf("  + plan 256x256 + guarded 156KiB x2      %+8.2f us\n",
           period([&] {
             plan_k<<<256, 256>>>(meta, meta + n, n, res);
             S();
             guarded_k<159760><<<256, 1024>>>(flag, out);
             guarded_k<159760><<<256, 1024>>>(flag, out);
           }) - base);
  }
  return 0;
}
