// tools/diag/pmc_calib.hip -- calibration of the L2 memory-side read counters
// (FETCH_SIZE, TCC_EA0_RDREQ / _128B) on gfx950 for the access widths the
// batch kernels use (the batch path on shuffled config 3
// reads 0.93 x its algorithmic bytes by those counters; MI355X_MICROARCH.md
// calls every width but 16-B/lane streams uncalibrated).  Each kernel reads
// exactly BYTES once (grid-stride, 256 x 1024 threads, XOR into a sink that is
// never written), one launch each after a flush pass that streams 1 GiB of
// other data with cached loads (the 256 MiB Infinity Cache holds none of the measured bytes):
//   s16nt   16 B/lane, nontemporal (the calibrated case: FETCH_SIZE = 1/2)
//   s16c    16 B/lane, cached
//   s4nt    4 B/lane, nontemporal, 256 B per wave instruction
//   s4nt4   the same from base + 4 (every 128-B line split across requests)
//   s4c     4 B/lane, cached
//   s16mis  the misaligned-chunk pattern of the batch kernels: per 4 KiB
//           chunk five 16-B rows per lane starting 16 B early (the row before
//           overlaps the previous chunk's last row)
// Under rocprofv3 --pmc, each dispatch's counters divided by BYTES give the
// counted fraction for that pattern.
//   hipcc -O3 --offload-arch=gfx950 tools/diag/pmc_calib.hip -o tools/diag/pmc_calib
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d out -o p1 -- ./tools/diag/pmc_calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t BYTES = 1ull << 30;

__global__ __launch_bounds__(1024) void s16nt(const u32x4* p, uint64_t n16, uint32_t* sink) {
  uint32_t x = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x9E3779B9u) sink[0] = x;
}
__global__ __launch_bounds__(1024) void s16c(const u32x4* p, uint64_t n16, uint32_t* sink) {
  uint32_t x = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const u32x4 v = p[i];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x9E3779B9u) sink[0] = x;
}
__global__ __launch_bounds__(1024) void s4nt(const uint32_t* p, uint64_t n4, uint32_t* sink) {
  uint32_t x = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
    x ^= __builtin_nontemporal_load(p + i);
  if (x == 0x9E3779B9u) sink[0] = x;
}
__global__ __launch_bounds__(1024) void s4c(const uint32_t* p, uint64_t n4, uint32_t* sink) {
  uint32_t x = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
    x ^= p[i];
  if (x == 0x9E3779B9u) sink[0] = x;
}
// one wave per 4 KiB chunk: lane l, rows j = 0..4 at chunk - 16 + 1024 j + 16 l (clamped into the buffer)
__global__ __launch_bounds__(1024) void s16mis(const uint8_t* p, uint64_t bytes, uint32_t* sink) {
  uint32_t x = 0;
  const uint64_t nch = bytes / 4096, lane = threadIdx.x & 63u;
  const uint64_t w0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t c = w0; c < nch; c += nw) {
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      int64_t o = (int64_t)(c * 4096) - 16 + 1024 * j + 16 * (int64_t)lane;
      if (j == 4 && lane > 0) o = (int64_t)(c * 4096) + 4096 - 16;  // the fifth row: one extra 16 B per chunk
      if (o < 0) o = 0;
      const u32x4 v = __builtin_nontemporal_load((const u32x4*)(p + o));
      x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (x == 0x9E3779B9u) sink[0] = x;
}

int main() {
  uint8_t *a = nullptr, *flush = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&a, BYTES + 4096) != hipSuccess || hipMalloc(&flush, BYTES) != hipSuccess ||
      hipMalloc(&sink, 64) != hipSuccess) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  (void)hipMemset(a, 0x5A, BYTES + 4096);
  (void)hipMemset(flush, 0x33, BYTES);
  const dim3 g(256), b(1024);
  auto fl = [&] { hipLaunchKernelGGL(s16c, g, b, 0, 0, (const u32x4*)flush, BYTES / 16, sink); };  // (cached: fills the Infinity Cache with other data)
  const char* names[] = {"s16nt", "s16c", "s4nt", "s4nt4", "s4c", "s16mis"};
  for (int rep = 0; rep < 2; ++rep) {
    for (int k = 0; k < 6; ++k) {
      fl();
      switch (k) {
        case 0: hipLaunchKernelGGL(s16nt, g, b, 0, 0, (const u32x4*)a, BYTES / 16, sink); break;
        case 1: hipLaunchKernelGGL(s16c, g, b, 0, 0, (const u32x4*)a, BYTES / 16, sink); break;
        case 2: hipLaunchKernelGGL(s4nt, g, b, 0, 0, (const uint32_t*)a, BYTES / 4, sink); break;
        case 3: hipLaunchKernelGGL(s4nt, g, b, 0, 0, (const uint32_t*)(a + 4), BYTES / 4, sink); break;
        case 4: hipLaunchKernelGGL(s4c, g, b, 0, 0, (const uint32_t*)a, BYTES / 4, sink); break;
        case 5: hipLaunchKernelGGL(s16mis, g, b, 0, 0, (const uint8_t*)a, BYTES, sink); break;
      }
      if (hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "kernel %s failed\n", names[k]);
        return 1;
      }
    }
  }
  // s16mis touches BYTES unique bytes; each chunk's first row re-reads the previous chunk's last 16 B
  // (one 128-B line per chunk more if that line is no longer in L2)
  printf("{\"bytes\": %llu, \"s16mis_max_bytes\": %llu, \"order\": \"per rep: flush(s16c over another 1 GiB) then s16nt s16c s4nt s4nt4 s4c s16mis\"}\n",
         (unsigned long long)BYTES, (unsigned long long)(BYTES + (BYTES / 4096) * 128));
  return 0;
}
