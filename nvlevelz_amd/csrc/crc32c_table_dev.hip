// nvlevelz_amd/csrc/crc32c_table_dev.hip -- the device side of
// nvl_sstable_verify_table_dev's fast path (crc32c_framing_dev.cpp): the
// index block of a table already in HBM is parsed on the GPU, one thread per
// entry, and ReadBlock's trailer checks (table/format.cc:88-135) write the
// output records in place, so a 10^5-block table's index never crosses PCIe.
//
// The index block TableBuilder writes has restart interval 1
// (table/table_builder.cc:59,88): entry i starts at restart point i.  The
// walk of Block::Iter (table/block.cc:17-37, 47-72, 219-246; restated on the
// host by crc32c_framing.cpp's block_handles) visits exactly those entries
// when every entry starts at its restart point, ends where the next one
// starts (the last at the restart array), and shares no key bytes; a block
// for which that does not hold sets *bad and the host reruns the table
// through its sequential parse -- the GPU result is only kept when it is the
// walk's.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_internal.h"
#include "crc32c_math.h"
#include "nvl_framing.h"

namespace nvl {
namespace dev {
namespace {

__device__ __forceinline__ uint32_t ld_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// GetVarint64Ptr / GetVarint32Ptr (util/coding.cc): at most (max_shift/7 + 1)
// bytes, never past limit; nullptr when it does not end.
__device__ __forceinline__ const uint8_t* dvarint(const uint8_t* p, const uint8_t* limit, unsigned max_shift,
                                                  uint64_t* v) {
  uint64_t r = 0;
  for (unsigned shift = 0; shift <= max_shift && p < limit; shift += 7) {
    const uint64_t b = *p++;
    if (b & 128) {
      r |= (b & 127) << shift;
    } else {
      *v = r | (b << shift);
      return p;
    }
  }
  return nullptr;
}

__device__ __forceinline__ bool in_file(uint64_t off, uint64_t size, uint64_t file_len) {  // format.cc:82-85
  return size <= file_len && off <= file_len - size && file_len - size - off >= (uint64_t)NVL_BLOCK_TRAILER_SIZE;
}

constexpr uint8_t kCompute = 0xFF;  // verdict slot still to be computed from the batch
constexpr uint64_t kPiece = 4096;    // index block piece (crc32c_framing_dev.cpp: kIndexPiece)
constexpr uint64_t kResHead = 32;    // res: u32 bad, pad, u64 n_bad, u64 n_fix, pad

}  // namespace

// Batch slots, in file order (TableBuilder writes data blocks, meta blocks,
// the metaindex, the index: table_builder.cc:241-266) so that the batch runs
// as one region (nvl_crc32c_region_dev): [0, nr) the data blocks the index
// entries point at, [nr, pb) zero-length fillers at the index block's offset
// (the meta blocks' places: they get a batch of their own), [pb, pb + np) the
// index block itself in np pieces of 4096 bytes (the last one shorter; their
// CRCs are combined on the host).
// Thread i < nr parses entry i of the index block [blk, blk + size) with nr
// restart points -> slot i (offset, size + 1: block | type; length 0 with a
// verdict preset when the handle is bad or out of the file) and output record
// rec[i] = {offset, size, NVL_TBLOCK_DATA, preset or OK}; *bad |= 1 when the
// entry is not where the sequential walk would find it.  Thread nr + k writes
// piece slot pb + k, thread nr + np + j filler slot nr + j.
__global__ void crc32c_index_entries(const uint8_t* __restrict__ file, uint64_t file_len, uint64_t index_off,
                                     uint64_t size, uint32_t nr, uint32_t np, uint32_t pb,
                                     uint64_t* __restrict__ boff, uint64_t* __restrict__ blen,
                                     uint8_t* __restrict__ vk, nvl_table_block* __restrict__ rec,
                                     uint32_t* __restrict__ bad) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (uint64_t)pb + np) return;
  if (t >= (uint64_t)nr + np) {  // a filler: nothing to read, no verdict of its own
    const uint64_t i = t - np;
    boff[i] = index_off;
    blen[i] = 0;
    vk[i] = (uint8_t)NVL_BLOCK_OK;
    return;
  }
  if (t >= nr) {
    const uint64_t k = t - nr, o = k * kPiece, ilen = size + 1, i = pb + k;
    boff[i] = index_off + o;
    blen[i] = ilen - o < kPiece ? ilen - o : kPiece;
    vk[i] = (uint8_t)NVL_BLOCK_OK;  // no verdict of its own
    return;
  }
  const uint64_t i = t;
  const uint8_t* blk = file + index_off;
  const uint64_t restarts = size - (1ull + nr) * 4ull;
  const uint8_t* limit = blk + restarts;
  const uint64_t start = ld_le32(blk + restarts + 4ull * i);
  const uint64_t next = i + 1 < nr ? ld_le32(blk + restarts + 4ull * (i + 1)) : restarts;
  bool ok = start < restarts;
  nvl_block_handle h{0, 0};
  bool handle_ok = false;
  if (ok) {
    const uint8_t* p = blk + start;
    uint64_t shared = 0, non_shared = 0, value_len = 0;
    if (limit - p < 3) {
      ok = false;
    } else if ((p[0] | p[1] | p[2]) < 128) {
      shared = p[0], non_shared = p[1], value_len = p[2];
      p += 3;
    } else if (!(p = dvarint(p, limit, 28, &shared)) || !(p = dvarint(p, limit, 28, &non_shared)) ||
               !(p = dvarint(p, limit, 28, &value_len))) {
      ok = false;
    }
    if (ok) {
      shared = (uint32_t)shared;  // GetVarint32PtrFallback keeps the low 32 bits
      non_shared = (uint32_t)non_shared;
      value_len = (uint32_t)value_len;
      ok = shared == 0 && (uint64_t)(limit - p) >= non_shared + value_len;
      if (ok) {
        const uint8_t* value = p + non_shared;
        ok = (uint64_t)(value + value_len - blk) == next;
        const uint8_t* q = dvarint(value, value + value_len, 63, &h.offset);
        handle_ok = q && dvarint(q, value + value_len, 63, &h.size);
      }
    }
  }
  if (!ok) atomicOr(bad, 1u);
  if (!handle_ok) h = nvl_block_handle{0, 0};
  const bool fits = handle_ok && in_file(h.offset, h.size, file_len);
  boff[i] = h.offset;
  blen[i] = fits ? h.size + 1u : 0u;
  const uint8_t pre = !handle_ok ? (uint8_t)NVL_BLOCK_BAD_HANDLE : (fits ? kCompute : (uint8_t)NVL_BLOCK_TRUNCATED);
  vk[i] = pre;
  rec[i] = nvl_table_block{h.offset, h.size, NVL_TBLOCK_DATA, pre == kCompute ? (uint32_t)NVL_BLOCK_OK : pre};
}

// ReadBlock's trailer checks for every batch slot whose verdict is still to
// be computed (vk == kCompute): the trailer's type byte at off + len1 - 1,
// its masked CRC after.  Results for the host in res: res64[1] = slots not
// OK, res64[2] = data slots (k < nr) whose checked verdict is not the OK
// their record was given, then the np piece CRCs (u32, slots [pb, pb + np))
// and the nm meta slots' verdicts (u8, slots [nr, nr + nm)).
__global__ void crc32c_table_verdicts(const uint8_t* __restrict__ file, const uint64_t* __restrict__ boff,
                                      const uint64_t* __restrict__ blen, const uint32_t* __restrict__ crc,
                                      uint64_t n, uint32_t nr, uint32_t nm, uint32_t pb, uint32_t np,
                                      uint8_t* __restrict__ vk, uint8_t* __restrict__ res) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  uint8_t v = vk[k];
  const bool computed = v == kCompute;
  if (computed) {
    const uint8_t* t = file + boff[k] + blen[k] - 1u;
    const uint32_t stored = ld_le32(t + 1);
    v = crc[k] != nvl::unmask(stored) ? (uint8_t)NVL_BLOCK_CHECKSUM_MISMATCH
                                      : (t[0] > 1u ? (uint8_t)NVL_BLOCK_BAD_TYPE : (uint8_t)NVL_BLOCK_OK);
    vk[k] = v;
  }
  if (k >= pb && k < (uint64_t)pb + np) reinterpret_cast<uint32_t*>(res + kResHead)[k - pb] = crc[k];
  if (k >= nr && k < (uint64_t)nr + nm) res[kResHead + 4ull * np + (k - nr)] = v;
  unsigned long long* c = reinterpret_cast<unsigned long long*>(res);
  const unsigned long long mb = __ballot(v != NVL_BLOCK_OK);
  const unsigned long long mf = __ballot(computed && k < nr && v != NVL_BLOCK_OK);
  const uint32_t lane = threadIdx.x & 63u;
  if (mb && lane == (uint32_t)__builtin_ctzll(mb)) atomicAdd(c + 1, (unsigned long long)__builtin_popcountll(mb));
  if (mf && lane == (uint32_t)__builtin_ctzll(mf)) atomicAdd(c + 2, (unsigned long long)__builtin_popcountll(mf));
}

}  // namespace dev

hipError_t launch_index_entries(const void* file, uint64_t file_len, uint64_t index_off, uint64_t size, uint32_t nr,
                                uint32_t np, uint32_t pb, uint64_t* boff, uint64_t* blen, uint8_t* vk,
                                nvl_table_block* rec, uint32_t* bad, hipStream_t st) {
  const uint64_t threads = (uint64_t)pb + np;  // data entries, index pieces, fillers [nr, pb)
  if (threads == 0) return hipSuccess;
  hipLaunchKernelGGL(dev::crc32c_index_entries, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, st,
                     static_cast<const uint8_t*>(file), file_len, index_off, size, nr, np, pb, boff, blen, vk, rec,
                     bad);
  return hipGetLastError();
}

hipError_t launch_table_verdicts(const void* file, const uint64_t* boff, const uint64_t* blen, const uint32_t* crc,
                                 uint64_t n, uint32_t nr, uint32_t nm, uint32_t pb, uint32_t np, uint8_t* vk,
                                 void* res, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(dev::crc32c_table_verdicts, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st,
                     static_cast<const uint8_t*>(file), boff, blen, crc, n, nr, nm, pb, np, vk,
                     static_cast<uint8_t*>(res));
  return hipGetLastError();
}

}  // namespace nvl
