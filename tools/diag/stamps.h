// tools/diag/stamps.h -- per-wave timeline instrumentation for a DIAGNOSTIC
// variant build of ONE kernel TU (never the shipped library).  Force-included
// ahead of that TU's source (its readers are defined once per library):
//   make -C nvlevelz_amd/csrc variant NAME=stamps VFLAGS_crc32c_fixed="-include ../../tools/diag/stamps.h"
// (crc32c_region for run_region's timelines, crc32c_batch for the body kernels)
// It defines the hook macros the kernel source leaves as no-ops: per wave
// {start, after the LDS table fill, end} s_memrealtime stamps (100 MHz) and
// {XCC id, units processed}, read back by tools/diag/stamps.py through
// nvl_diag_stamps().  The stamp stores go to a buffer of their own that no
// product code reads.
#pragma once
#include <hip/hip_runtime.h>

namespace nvl {
namespace dev {
__device__ unsigned long long g_stamps[4 * 65536];
}
}  // namespace nvl

#define NVL_STAMP0() const unsigned long long ts0 = __builtin_amdgcn_s_memrealtime(); uint32_t nproc = 0
#define NVL_STAMP1() const unsigned long long ts1 = __builtin_amdgcn_s_memrealtime()
#define NVL_COUNT() (++nproc)
#define NVL_STAMP_END()                                                                     \
  do {                                                                                      \
    const uint32_t wave_ = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);              \
    if ((threadIdx.x & 63) == 0 && wave_ < 65536) {                                         \
      unsigned xcc_;                                                                        \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                   \
      ::nvl::dev::g_stamps[4 * wave_ + 0] = ts0;                                            \
      ::nvl::dev::g_stamps[4 * wave_ + 1] = ts1;                                            \
      ::nvl::dev::g_stamps[4 * wave_ + 2] = __builtin_amdgcn_s_memrealtime();               \
      ::nvl::dev::g_stamps[4 * wave_ + 3] = ((unsigned long long)xcc_ << 32) | nproc;       \
    }                                                                                       \
  } while (0)

extern "C" __attribute__((visibility("default"))) int nvl_diag_stamps(unsigned long long* host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(::nvl::dev::g_stamps), n * sizeof(unsigned long long)) == hipSuccess
             ? 0
             : -1;
}

// Multi-point timeline (up to 8 stamps per wave) for kernels with phases:
// NVL_TL_DECL() at entry, NVL_TL(k) at phase boundaries, NVL_TL_END() at
// exit; read back with nvl_diag_tl() (tools/diag/tl.py).
namespace nvl {
namespace dev {
__device__ unsigned long long g_tl[8 * 65536];
}
}  // namespace nvl
#define NVL_TL_DECL() unsigned long long tl_[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define NVL_TL(k) (tl_[(k)] = __builtin_amdgcn_s_memrealtime())
#define NVL_TL_WAIT(k, v)                        \
  do {                                           \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::"v"(v)); \
    NVL_TL(k);                                   \
  } while (0)
#define NVL_TL_END()                                                                        \
  do {                                                                                      \
    const uint32_t wave_ = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);              \
    if ((threadIdx.x & 63) == 0 && wave_ < 65536) {                                         \
      tl_[7] = __builtin_amdgcn_s_memrealtime();                                            \
      for (int k_ = 0; k_ < 8; ++k_) ::nvl::dev::g_tl[8 * wave_ + k_] = tl_[k_];            \
    }                                                                                       \
  } while (0)

extern "C" __attribute__((visibility("default"))) int nvl_diag_tl(unsigned long long* host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(::nvl::dev::g_tl), n * sizeof(unsigned long long)) == hipSuccess ? 0
                                                                                                               : -1;
}
