// tools/diag/stamps_clk.h -- stamps.h plus the shader clock: per wave
// {start, after the LDS fill, end} s_memrealtime (100 MHz), {XCC id, units},
// and s_memtime (shader-clock cycles) at start and end, so that a wave's
// average shader clock = d(memtime) / d(memrealtime) x 100 MHz.  DIAGNOSTIC
// variant of one kernel TU only (why an isolated call
// runs slower than a back-to-back one):
//   make -C nvlevelz_amd/csrc variant NAME=stampsclk VFLAGS_crc32c_fixed="-include ../../tools/diag/stamps_clk.h"
// read back by tools/diag/iso_clock.py through nvl_diag_stamps8().
#pragma once
#include <hip/hip_runtime.h>

namespace nvl {
namespace dev {
__device__ unsigned long long g_stamps8[8 * 65536];
}
}  // namespace nvl

#define NVL_STAMP0()                                                   \
  const unsigned long long ts0 = __builtin_amdgcn_s_memrealtime();     \
  const unsigned long long ck0 = __builtin_amdgcn_s_memtime();         \
  uint32_t nproc = 0
#define NVL_STAMP1() const unsigned long long ts1 = __builtin_amdgcn_s_memrealtime()
#define NVL_COUNT() (++nproc)
#define NVL_STAMP_END()                                                                     \
  do {                                                                                      \
    const unsigned long long ck1_ = __builtin_amdgcn_s_memtime();                           \
    const unsigned long long te_ = __builtin_amdgcn_s_memrealtime();                        \
    const uint32_t wave_ = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);              \
    if ((threadIdx.x & 63) == 0 && wave_ < 65536) {                                         \
      unsigned xcc_;                                                                        \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                   \
      ::nvl::dev::g_stamps8[8 * wave_ + 0] = ts0;                                           \
      ::nvl::dev::g_stamps8[8 * wave_ + 1] = ts1;                                           \
      ::nvl::dev::g_stamps8[8 * wave_ + 2] = te_;                                           \
      ::nvl::dev::g_stamps8[8 * wave_ + 3] = ((unsigned long long)xcc_ << 32) | nproc;      \
      ::nvl::dev::g_stamps8[8 * wave_ + 4] = ck0;                                           \
      ::nvl::dev::g_stamps8[8 * wave_ + 5] = ck1_;                                          \
    }                                                                                       \
  } while (0)

extern "C" __attribute__((visibility("default"))) int nvl_diag_stamps8(unsigned long long* host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(::nvl::dev::g_stamps8), n * sizeof(unsigned long long)) == hipSuccess
             ? 0
             : -1;
}
