// What a cooperative launch costs on gfx950 (hipLaunchCooperativeKernel, one
// workgroup of 1024 threads per CU, 156 KiB LDS) against an ordinary launch
// of the same kernel, and what one grid-wide barrier inside it costs:
// per-call period over R back-to-back calls behind a 400 MB streaming
// kernel, HIP events.  The barrier: one device-scope counter per launch
// generation, every workgroup's thread 0 adds and spins (s_sleep) until all
// have arrived -- safe only because a cooperative launch has every
// workgroup resident.
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

template <int BARRIERS>
__global__ __launch_bounds__(1024) void body_k(uint32_t* ctr, uint32_t gen, uint32_t* out) {
  __shared__ uint32_t lds[159760 / 4];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  for (int b = 0; b < BARRIERS; ++b) {
    if (threadIdx.x == 0) {
      const uint32_t target = (gen * BARRIERS + (uint32_t)b + 1u) * gridDim.x;
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = lds[5];
}

template <class F>
static float period(F seq, int R = 200) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) seq();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < R; ++i) seq();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms * 1000.0f / R;
}

int main() {
  const uint64_t bytes = 409600000ull;
  u32x4* p;
  uint32_t *out, *ctr;
  (void)hipMalloc(&p, bytes);
  (void)hipMemset(p, 1, bytes);
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMalloc(&ctr, 256);
  (void)hipMemset(ctr, 0, 256);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const uint64_t n16 = bytes / 16;
  hipStream_t st;
  (void)hipStreamCreate(&st);
  auto S = [&] { hipLaunchKernelGGL(stream_k, dim3(256), dim3(1024), 0, st, p, n16, out); };
  uint32_t gen = 0;
  auto coop = [&](auto kern, bool barrier) {
    uint32_t g = barrier ? gen++ : 0u;
    void* args[] = {&ctr, &g, &out};
    hipError_t e = hipLaunchCooperativeKernel((const void*)kern, dim3(cus), dim3(1024), args, 0, st);
    if (e != hipSuccess) printf("cooperative launch failed: %s\n", hipGetErrorString(e));
  };
  for (int rep = 0; rep < 3; ++rep) {
    const float base = period([&] { S(); });
    printf("rep %d: stream alone                             %8.2f us\n", rep, base);
    printf("  + ordinary launch, 0 barriers                 %+8.2f us\n",
           period([&] { S(); hipLaunchKernelGGL(body_k<0>, dim3(cus), dim3(1024), 0, st, ctr, 0u, out); }) - base);
    printf("  + cooperative launch, 0 barriers              %+8.2f us\n", period([&] { S(); coop(body_k<0>, false); }) - base);
    (void)hipMemsetAsync(ctr, 0, 4, st);
    gen = 0;
    printf("  + cooperative launch, 1 grid barrier          %+8.2f us\n", period([&] { S(); coop(body_k<1>, true); }) - base);
    (void)hipMemsetAsync(ctr, 0, 4, st);
    gen = 0;
    printf("  + cooperative launch, 2 grid barriers         %+8.2f us\n", period([&] { S(); coop(body_k<2>, true); }) - base);
    (void)hipMemsetAsync(ctr, 0, 4, st);
    gen = 0;
    printf("  + 2 ordinary launches, 0 barriers             %+8.2f us\n",
           period([&] {
             S();
             hipLaunchKernelGGL(body_k<0>, dim3(cus), dim3(1024), 0, st, ctr, 0u, out);
             hipLaunchKernelGGL(body_k<0>, dim3(cus), dim3(1024), 0, st, ctr, 0u, out);
           }) - base);
  }
  (void)hipStreamSynchronize(st);
  uint32_t c = 0;
  (void)hipMemcpy(&c, ctr, 4, hipMemcpyDeviceToHost);
  printf("counter %u\n", c);
  return 0;
}
