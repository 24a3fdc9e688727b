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
#include "crc32c_math.h"
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
    int dev = 0;
    if (st ? hipStreamGetDevice(st, &dev) != hipSuccess : hipGetDevice(&dev) != hipSuccess) return NVL_CRC32C_EHIP;
    uint8_t* d = static_cast<uint8_t*>(thread_table_device(dev, 2 * a + c + a + wsb));
    if (!d) return NVL_CRC32C_EHIP;
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
    if (rc != NVL_CRC32C_OK) {
      (void)hipStreamSynchronize(st);  // the workspace is the thread's: nothing may still use it
      return rc;
    }
    for (size_t k = 0; k < m; ++k) (*verdict)[which[k]] = v[k];
    return NVL_CRC32C_OK;
  }
};

inline uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

inline size_t up256(size_t x) { return (x + 255) / 256 * 256; }

constexpr uint64_t kTailWin = 4096;       // last bytes of the file read first: footer (+ index tail, usually)
constexpr uint64_t kMetaMax = 64u << 10;  // metaindex (+ trailer) bytes the fast path reads
constexpr uint64_t kIndexPiece = 4096;    // the index block is checked as pieces of this size (crc32c_table_dev.hip)
constexpr uint64_t kResHead = 32;         // device results: u32 bad, pad, u64 n_bad, u64 n_fix, pad
constexpr uint64_t kRecSideMin = 4096;    // more data blocks: their records come back on the side stream
constexpr uint8_t kCompute = 0xFF;

// CRC32C(A || B) = shift(CRC32C(A), |B|) ^ CRC32C(B): the index block's
// Value from its pieces' Values, with "shift by kIndexPiece bytes" as a
// byte-sliced operator table (crc32c_math.h).
struct PieceFold {
  PowTable pt;
  uint32_t op[4][256];
  PieceFold() {
    build_pow_table(&pt);
    build_shift_op(pt.x2n, kIndexPiece, op);
  }
  uint32_t fold(const uint32_t* crc, uint64_t np, uint64_t total) const {
    uint32_t u = 0;
    for (uint64_t k = 0; k + 1 < np; ++k)
      u = (op[0][u & 255] ^ op[1][(u >> 8) & 255] ^ op[2][(u >> 16) & 255] ^ op[3][u >> 24]) ^ crc[k];
    const uint64_t last = total - (np - 1) * kIndexPiece;
    return shift_bytes(pt.x2n, u, last) ^ crc[np - 1];
  }
};

// *done = false: the caller runs the generic core (nothing written here is
// kept).  On *done = true the result is final.
//
// One host round trip before the batch -- the file's tail: the footer, the
// index block's tail and, for a table without filter blocks (a few-byte
// metaindex right before the index), the metaindex -- then everything on the
// streams at once: on `st` the index parse (data slots, records, the meta
// blocks' places as zero-length fillers, the index pieces), ONE region batch
// in file order, the trailer checks and the results copy; on the thread's
// side stream, once the parse is done, the records copy.  A metaindex outside
// the tail is copied first on `st` and parsed on the host while the batch
// runs, and meta blocks (filter blocks) get a batch of their own after the
// main one.  Results and records land in pinned memory (a copy into the
// caller's pageable array waits for the stream inside the copy call).
// Records carry the verdict OK for every checked block; only when a check
// fails (n_fix > 0) are the verdicts copied and patched in.
int table_fast(const uint8_t* f, uint64_t len, nvl_table_block* blocks, size_t cap, size_t* n_blocks,
               uint32_t* table_status, uint64_t* n_bad, hipStream_t st, bool* done) {
  *done = false;
  if (!blocks || len < NVL_FOOTER_SIZE) return NVL_CRC32C_OK;
  int dev = 0;
  if (st ? hipStreamGetDevice(st, &dev) != hipSuccess : hipGetDevice(&dev) != hipSuccess) return NVL_CRC32C_EHIP;
  hipStream_t side = nullptr;
  hipEvent_t ev_meta = nullptr, ev_parse = nullptr;
  if (!thread_table_aux(dev, &side, &ev_meta, &ev_parse)) return NVL_CRC32C_EHIP;
  uint8_t* pin = static_cast<uint8_t*>(thread_table_pinned(kTailWin));
  if (!pin) return NVL_CRC32C_EHIP;
  // 1. the file's last bytes (TableBuilder writes the metaindex, the index
  //    and the footer last, table_builder.cc:241-266)
  const uint64_t w = len < kTailWin ? len : kTailWin, w0 = len - w;
  if (hipMemcpyAsync(pin, f + w0, w, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return NVL_CRC32C_EHIP;
  const uint8_t* footer = pin + w - NVL_FOOTER_SIZE;
  const uint64_t magic = (uint64_t)le32(footer + 40) | ((uint64_t)le32(footer + 44) << 32);
  nvl_block_handle meta_h, index_h;
  const uint8_t* fp = decode_handle(footer, footer + NVL_FOOTER_SIZE, &meta_h);
  if (magic != kTableMagic || !fp || !decode_handle(fp, footer + NVL_FOOTER_SIZE, &index_h) ||
      !block_in_file(index_h, len) || index_h.size < 4)
    return NVL_CRC32C_OK;
  const bool meta_in = block_in_file(meta_h, len);
  const uint64_t meta_bytes = meta_in ? meta_h.size + NVL_BLOCK_TRAILER_SIZE : 0;
  if (meta_bytes > kMetaMax) return NVL_CRC32C_OK;
  std::vector<uint8_t> meta_img;  // the metaindex when it came with the tail
  if (meta_in && meta_h.offset >= w0) meta_img.assign(pin + (meta_h.offset - w0), pin + (meta_h.offset - w0) + meta_bytes);
  const bool meta_copy = meta_in && meta_img.empty();  // (else copied on the stream below)
  // the index tail: num_restarts (its last 4 bytes), type byte, masked CRC
  const uint64_t tail_off = index_h.offset + index_h.size - 4;
  uint8_t tail[9];
  if (tail_off >= w0) {
    memcpy(tail, pin + (tail_off - w0), 9);
  } else if (hipMemcpyAsync(pin, f + tail_off, 9, hipMemcpyDeviceToHost, st) != hipSuccess ||
             hipStreamSynchronize(st) != hipSuccess) {
    return NVL_CRC32C_EHIP;
  } else {
    memcpy(tail, pin, 9);
  }
  const uint64_t nr = le32(tail);
  if (tail[4] != 0 || nr == 0 || nr > (index_h.size - 4) / 4 || nr > 0xFFFFFFFFull - (1u << 24))
    return NVL_CRC32C_OK;  // compressed / bad type / empty or bad restart array: the generic walk
  const uint64_t ilen = index_h.size + 1;
  const uint64_t np = (ilen + kIndexPiece - 1) / kIndexPiece;
  if (np > (1u << 24)) return NVL_CRC32C_OK;
  const uint64_t nm_max = meta_in ? meta_h.size / 3 + 1 : 0;  // entries take >= 3 bytes
  if (2 + nr > cap) return NVL_CRC32C_OK;                     // the generic walk reports ENOSPC

  // 2. device workspace: [results][records][boff][blen][crc][vk][region
  //    workspace] [meta batch: off | len1, crc, verdicts, workspace].  Slots in
  //    file order: data [0, nr), zero-length fillers at the index block's
  //    offset [nr, pb) (the meta blocks' places), index pieces [pb, pb + np).
  const uint64_t pb = nr + nm_max, nmax = pb + np;
  if (nmax > 0xFFFFFFFFull) return NVL_CRC32C_OK;
  const size_t s_res = up256(kResHead + 4 * np), s8 = up256(nmax * 8), s4 = up256(nmax * 4), s1 = up256(nmax),
               s_rec = up256(nr * sizeof(nvl_table_block));
  const size_t wsb = nvl_crc32c_region_workspace_bytes(len, nmax);
  const size_t s_main = s_res + 2 * s8 + s4 + s1 + s_rec + up256(wsb);
  const size_t m16 = up256(nm_max * 16), m4 = up256(nm_max * 4), m1 = up256(nm_max);
  const size_t mwsb = nm_max ? nvl_crc32c_batch_workspace_bytes(nm_max) : 0;
  uint8_t* d = static_cast<uint8_t*>(thread_table_device(dev, s_main + m16 + m4 + m1 + mwsb));
  if (!d) return NVL_CRC32C_EHIP;
  uint8_t* dres = d;
  nvl_table_block* rec = reinterpret_cast<nvl_table_block*>(d + s_res);  // (right after: one copy back for both)
  uint64_t* boff = reinterpret_cast<uint64_t*>(d + s_res + s_rec);
  uint64_t* blen = reinterpret_cast<uint64_t*>(d + s_res + s_rec + s8);
  uint32_t* crc = reinterpret_cast<uint32_t*>(d + s_res + s_rec + 2 * s8);
  uint8_t* vk = d + s_res + s_rec + 2 * s8 + s4;
  void* ws = d + s_res + s_rec + 2 * s8 + s4 + s1;
  uint64_t* moff = reinterpret_cast<uint64_t*>(d + s_main);  // [nm_max offsets][nm_max len1]
  uint32_t* mcrc = reinterpret_cast<uint32_t*>(d + s_main + m16);
  uint8_t* mver = d + s_main + m16 + m4;
  void* mws = d + s_main + m16 + m4 + m1;
  // pinned: [metaindex][meta slots: off | len1][meta verdicts][results][records]
  const size_t p_meta = 0, p_slots = up256(kMetaMax), p_mver = p_slots + m16, p_res = p_mver + m1,
               p_rec = p_res + s_res;
  pin = static_cast<uint8_t*>(thread_table_pinned(p_rec + s_rec));
  if (!pin) return NVL_CRC32C_EHIP;

  // 3. everything on the streams
  const bool rec_side = nr > kRecSideMin;  // (see below)
  auto drain = [&]() {  // (the workspace and the pinned buffers are the thread's: nothing may still use them)
    (void)hipStreamSynchronize(st);
    if (rec_side) (void)hipStreamSynchronize(side);
  };
  if (hipMemsetAsync(dres, 0, kResHead, st) != hipSuccess ||
      (meta_copy &&
       hipMemcpyAsync(pin + p_meta, f + meta_h.offset, meta_bytes, hipMemcpyDeviceToHost, st) != hipSuccess)) {
    drain();
    return NVL_CRC32C_EHIP;
  }
  // The records (24 B per data block) come back with the results after the
  // batch -- or, for a large index, on the side stream once the parse has
  // written them, overlapping the batch (10^5 blocks: 2.4 MB).
  if ((meta_copy && hipEventRecord(ev_meta, st) != hipSuccess) ||
      launch_index_entries(f, len, index_h.offset, index_h.size, (uint32_t)nr, (uint32_t)np, (uint32_t)pb, boff, blen,
                           vk, rec, reinterpret_cast<uint32_t*>(dres), st) != hipSuccess ||
      (rec_side && hipEventRecord(ev_parse, st) != hipSuccess)) {
    drain();
    return NVL_CRC32C_EHIP;
  }
  // Up to kShapedMaxSlots slots, one launch (NVL_CRC32C_FLAG_REGION_SHAPED):
  // a table's slots are in file order by construction (table/table_builder.cc
  // writes data blocks, meta blocks, the metaindex and the index in sequence,
  // and the index lists the data blocks in key = file order), so the routed
  // call's plan and body launches (~8 µs per call) would only
  // confirm it.  A corrupt or crafted index whose handles are out of order or
  // overlap still gets every CRC right from the region kernel's per-buffer
  // path -- slowly: 10^4 shuffled 4 KiB blocks 6.9 ms, 10^5 62 ms
  // (tools/shaped_fallback_time.py, profiles/r06/shaped_fallback.jsonl) --
  // so larger tables keep the checked entry, whose plan sends such a batch to
  // the batch kernels (tests/test_table_verify.py::test_table_dev_out_of_order_index).
  constexpr uint64_t kShapedMaxSlots = 8192;
  int rc = nvl_crc32c_region_dev(f, len, boff, blen, nullptr, 0, crc, nmax,
                                 nmax <= kShapedMaxSlots ? NVL_CRC32C_FLAG_REGION_SHAPED : 0u, ws, wsb, st);
  if (rc == NVL_CRC32C_OK &&
      (launch_table_verdicts(f, boff, blen, crc, nmax, (uint32_t)nr, 0u, (uint32_t)pb, (uint32_t)np, vk, dres, st) !=
           hipSuccess ||
       hipMemcpyAsync(pin + p_res, dres, rec_side ? kResHead + 4 * np : s_res + nr * sizeof(nvl_table_block),
                      hipMemcpyDeviceToHost, st) != hipSuccess ||
       (rec_side && (hipStreamWaitEvent(side, ev_parse, 0) != hipSuccess ||
                     hipMemcpyAsync(pin + p_rec, rec, nr * sizeof(nvl_table_block), hipMemcpyDeviceToHost, side) !=
                         hipSuccess))))
    rc = NVL_CRC32C_EHIP;
  if (rc != NVL_CRC32C_OK) {
    drain();
    return rc;
  }

  // 4. the metaindex on the host while the batch runs, then its meta blocks'
  //    own batch and trailer checks after the main one
  if (meta_copy && hipEventSynchronize(ev_meta) != hipSuccess) {
    drain();
    return NVL_CRC32C_EHIP;
  }
  uint8_t v_meta = NVL_BLOCK_TRUNCATED;
  std::vector<nvl_block_handle> meta_blocks;
  std::vector<uint8_t> meta_bad;
  if (meta_in) {
    const uint8_t* mb = meta_copy ? pin + p_meta : meta_img.data();
    v_meta = host_block_verdict(mb, meta_h.size);
    if (v_meta == NVL_BLOCK_OK && mb[meta_h.size] == 0) block_handles(mb, meta_h.size, &meta_blocks, &meta_bad);
  }
  const uint64_t nm = meta_blocks.size(), cnt = 2 + nm + nr;
  if (nm > nm_max || cnt > cap) {  // (nm_max bounds it) / the generic walk reports ENOSPC
    drain();
    return NVL_CRC32C_OK;
  }
  std::vector<uint8_t> mv(nm);  // the meta blocks' verdicts (kCompute: from the meta batch, in order)
  uint64_t nq = 0;
  uint64_t* ms = reinterpret_cast<uint64_t*>(pin + p_slots);
  for (uint64_t j = 0; j < nm; ++j) {
    const nvl_block_handle& b = meta_blocks[j];
    mv[j] = meta_bad[j] ? (uint8_t)NVL_BLOCK_BAD_HANDLE
                        : (block_in_file(b, len) ? kCompute : (uint8_t)NVL_BLOCK_TRUNCATED);
    if (mv[j] == kCompute) {
      ms[nq] = b.offset;
      ms[nm_max + nq] = b.size + 1;
      ++nq;
    }
  }
  if (nq) {
    if (hipMemcpyAsync(moff, ms, nm_max * 16, hipMemcpyHostToDevice, st) != hipSuccess) rc = NVL_CRC32C_EHIP;
    if (rc == NVL_CRC32C_OK) rc = nvl_crc32c_batch_dev(f, moff, moff + nm_max, nullptr, 0, mcrc, nq, 0, mws, mwsb, st);
    if (rc == NVL_CRC32C_OK &&
        (launch_trailer_verdicts(f, moff, moff + nm_max, mcrc, nq, mver, st) != hipSuccess ||
         hipMemcpyAsync(pin + p_mver, mver, nq, hipMemcpyDeviceToHost, st) != hipSuccess))
      rc = NVL_CRC32C_EHIP;
  }
  const hipError_t e1 = hipStreamSynchronize(st), e2 = rec_side ? hipStreamSynchronize(side) : hipSuccess;
  if (rc != NVL_CRC32C_OK) return rc;
  if (e1 != hipSuccess || e2 != hipSuccess) return NVL_CRC32C_EHIP;

  // 5. the index block's own check (Table::Open, table.cc:58-66) from its pieces
  const uint8_t* res = pin + p_res;
  uint32_t bad;
  uint64_t nb, nfix;
  memcpy(&bad, res, 4);
  memcpy(&nb, res + 8, 8);
  memcpy(&nfix, res + 16, 8);
  static const PieceFold pf;
  const uint32_t* pc = reinterpret_cast<const uint32_t*>(res + kResHead);
  const bool index_ok = pf.fold(pc, np, ilen) == unmask(le32(tail + 5));
  if (bad || !index_ok) return NVL_CRC32C_OK;  // not the walk's list, or the index fails: generic
  memcpy(blocks + 2 + nm, pin + p_rec, nr * sizeof(nvl_table_block));
  if (nfix) {  // some data block failed its check: its verdict replaces the record's OK
    std::vector<uint8_t> v(nr);
    if (hipMemcpyAsync(v.data(), vk, nr, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return NVL_CRC32C_EHIP;
    for (uint64_t i = 0; i < nr; ++i) blocks[2 + nm + i].verdict = v[i];
  }
  blocks[0] = nvl_table_block{index_h.offset, index_h.size, NVL_TBLOCK_INDEX, NVL_BLOCK_OK};
  blocks[1] = nvl_table_block{meta_h.offset, meta_h.size, NVL_TBLOCK_METAINDEX, v_meta};
  uint64_t meta_not_ok = 0;
  for (uint64_t j = 0, q = 0; j < nm; ++j) {
    const uint8_t v = mv[j] == kCompute ? pin[p_mver + q++] : mv[j];
    blocks[2 + j] = nvl_table_block{meta_blocks[j].offset, meta_blocks[j].size, NVL_TBLOCK_META, v};
    meta_not_ok += v != NVL_BLOCK_OK;
  }
  *n_blocks = cnt;
  *table_status = NVL_TABLE_OK;
  if (n_bad) *n_bad = nb + meta_not_ok + (v_meta != NVL_BLOCK_OK);
  *done = true;
  return NVL_CRC32C_OK;
}

}  // namespace
}  // namespace nvl

extern "C" {

int nvl_sstable_verify_table_dev(const void* file, uint64_t file_len, nvl_table_block* blocks, size_t cap,
                                 size_t* n_blocks, uint32_t* table_status, uint64_t* n_bad, void* stream) {
  if (n_blocks) *n_blocks = 0;
  if (n_bad) *n_bad = 0;
  if ((!file && file_len) || !n_blocks || !table_status) return NVL_CRC32C_EINVAL;
  hipStream_t st = static_cast<hipStream_t>(stream);
  bool done = false;
  const int rc = nvl::table_fast(static_cast<const uint8_t*>(file), file_len, blocks, cap, n_blocks, table_status,
                                 n_bad, st, &done);
  if (rc != NVL_CRC32C_OK || done) return rc;
  nvl::DeviceTable src;
  src.f = static_cast<const uint8_t*>(file);
  src.len = file_len;
  src.st = st;
  return nvl::verify_table_core(src, file_len, blocks, cap, n_blocks, table_status, n_bad);
}

}  // extern "C"
