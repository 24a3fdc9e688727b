// nvlevelz_amd/csrc/crc32c_framing_dev.cpp -- nvl_sstable_verify_table_dev:
// whole-table verification of an SSTable image already in device memory
// (include/nvl_framing.h).  The table logic is crc32c_framing.cpp's
// verify_table_core; this file supplies the device-side source (HIP), so the
// host framing code stays free of HIP calls (tests/native/fuzz_framing.cc
// builds it under ASan without a GPU).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "crc32c_framing_core.h"
#include "crc32c_internal.h"
#include "nvl_crc32c.h"
#include "nvl_framing.h"

namespace nvl {
namespace {

// A table already in device memory: structure reads are small D2H copies on
// the stream; the batch runs nvl_crc32c_batch_dev over the image in place and
// a kernel compares every trailer, so only the verdicts come back.
struct DeviceTable : TableSource {
  const uint8_t* f;
  uint64_t len;
  hipStream_t st;
  int read(uint64_t off, uint64_t n, uint8_t* dst) override {
    if (hipMemcpyAsync(dst, f + off, n, hipMemcpyDeviceToHost, st) != hipSuccess) return NVL_CRC32C_EHIP;
    return hipStreamSynchronize(st) == hipSuccess ? NVL_CRC32C_OK : NVL_CRC32C_EHIP;
  }
  int verify(const std::vector<nvl_block_handle>& h, std::vector<uint8_t>* verdict) override {
    verdict->assign(h.size(), NVL_BLOCK_TRUNCATED);
    std::vector<uint64_t> off, ln;
    std::vector<size_t> which;
    for (size_t i = 0; i < h.size(); ++i) {
      if (!block_in_file(h[i], len)) continue;  // "truncated block read" (format.cc:82-85)
      off.push_back(h[i].offset);
      ln.push_back(h[i].size + 1);
      which.push_back(i);
    }
    const size_t m = off.size();
    if (m == 0) return NVL_CRC32C_OK;
    const size_t wsb = nvl_crc32c_batch_workspace_bytes(m);
    const size_t a = (m * 8 + 255) / 256 * 256, c = (m * 4 + 255) / 256 * 256;
    uint8_t* d = nullptr;
    if (hipMallocAsync(reinterpret_cast<void**>(&d), 2 * a + c + a + wsb, st) != hipSuccess) return NVL_CRC32C_EHIP;
    uint64_t* doff = reinterpret_cast<uint64_t*>(d);
    uint64_t* dlen = reinterpret_cast<uint64_t*>(d + a);
    uint32_t* dcrc = reinterpret_cast<uint32_t*>(d + 2 * a);
    uint8_t* dv = d + 2 * a + c;
    void* ws = d + 3 * a + c;
    std::vector<uint8_t> v(m);
    int rc = NVL_CRC32C_EHIP;
    if (hipMemcpyAsync(doff, off.data(), m * 8, hipMemcpyHostToDevice, st) == hipSuccess &&
        hipMemcpyAsync(dlen, ln.data(), m * 8, hipMemcpyHostToDevice, st) == hipSuccess) {
      rc = nvl_crc32c_batch_dev(f, doff, dlen, nullptr, 0, dcrc, m, 0, ws, wsb, st);
      if (rc == NVL_CRC32C_OK)
        rc = launch_trailer_verdicts(f, doff, dlen, dcrc, m, dv, st) == hipSuccess ? NVL_CRC32C_OK : NVL_CRC32C_EHIP;
      if (rc == NVL_CRC32C_OK && (hipMemcpyAsync(v.data(), dv, m, hipMemcpyDeviceToHost, st) != hipSuccess ||
                                  hipStreamSynchronize(st) != hipSuccess))
        rc = NVL_CRC32C_EHIP;
    }
    (void)hipFreeAsync(d, st);
    if (rc != NVL_CRC32C_OK) return rc;
    for (size_t k = 0; k < m; ++k) (*verdict)[which[k]] = v[k];
    return NVL_CRC32C_OK;
  }
};

}  // namespace
}  // namespace nvl

extern "C" {

int nvl_sstable_verify_table_dev(const void* file, uint64_t file_len, nvl_table_block* blocks, size_t cap,
                                 size_t* n_blocks, uint32_t* table_status, uint64_t* n_bad, void* stream) {
  if (n_blocks) *n_blocks = 0;
  if (n_bad) *n_bad = 0;
  if ((!file && file_len) || !n_blocks || !table_status) return NVL_CRC32C_EINVAL;
  nvl::DeviceTable src;
  src.f = static_cast<const uint8_t*>(file);
  src.len = file_len;
  src.st = static_cast<hipStream_t>(stream);
  return nvl::verify_table_core(src, file_len, blocks, cap, n_blocks, table_status, n_bad);
}

}  // extern "C"
