// nvlevelz_amd/csrc/crc32c_scan.hip -- exclusive prefix sum of per-buffer
// chunk counts for the variable-length plan (hipCUB / rocPRIM device scan).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "crc32c_internal.h"

namespace nvl {

size_t scan_temp_bytes(uint64_t n) {
  size_t bytes = 0;
  const uint64_t* in = nullptr;
  uint64_t* out = nullptr;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, (int)n, (hipStream_t)0);
  return bytes;
}

hipError_t exclusive_scan_u64(void* temp, size_t temp_bytes, const uint64_t* in, uint64_t* out, uint64_t n,
                              hipStream_t st) {
  return hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, in, out, (int)n, st);
}

}  // namespace nvl
