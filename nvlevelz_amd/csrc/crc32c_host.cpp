// nvlevelz_amd/csrc/crc32c_host.cpp -- the single-buffer host path of the
// util/crc32c.h API (leveldb::crc32c::Extend, util/crc32c.cc:299-347).
//
// This is the reference API's per-call CPU semantics -- one buffer, on the
// calling thread -- kept because a GPU round trip for one ~4 KiB buffer costs
// more than the checksum.  It is NOT used by any batch entry point.
//
// Two implementations, chosen once (thread-safe static) like the reference's
// CanAccelerateCRC32C probe (util/crc32c.cc:290-303):
//   * SSE4.2 crc32 instruction, three independent 8-byte streams over the
//     bulk of long buffers recombined with the GF(2) shift operator (the
//     instruction has 3-cycle latency and 1/cycle throughput), else
//   * portable slice-by-8.
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#if defined(__x86_64__)
#include <cpuid.h>
#include <nmmintrin.h>
#endif

#include "crc32c_internal.h"
#include "crc32c_math.h"

namespace nvl {
namespace {

struct HostTables {
  uint32_t t[8][256];
  PowTable pw;
  uint32_t sh_op[4][256];  // shift by kStream bytes
};

constexpr size_t kStream = 1024;  // bytes per stream per round (3 streams)

const HostTables& host_tables() {
  static const HostTables* tabs = [] {
    HostTables* h = new HostTables;
    for (uint32_t b = 0; b < 256; ++b) h->t[0][b] = byte_table0(b);
    for (int k = 1; k < 8; ++k)
      for (uint32_t b = 0; b < 256; ++b) h->t[k][b] = (h->t[k - 1][b] >> 8) ^ h->t[0][h->t[k - 1][b] & 0xffu];
    build_pow_table(&h->pw);
    build_shift_op(h->pw.x2n, kStream, h->sh_op);
    return h;
  }();
  return *tabs;
}

inline uint32_t shift_stream(const HostTables& h, uint32_t v) {
  return h.sh_op[0][v & 0xff] ^ h.sh_op[1][(v >> 8) & 0xff] ^ h.sh_op[2][(v >> 16) & 0xff] ^
         h.sh_op[3][v >> 24];
}

uint32_t raw_slice8(uint32_t l, const uint8_t* p, size_t n) {
  const HostTables& h = host_tables();
  while (n && ((uintptr_t)p & 7u)) {
    l = h.t[0][(l ^ *p++) & 0xffu] ^ (l >> 8);
    --n;
  }
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= l;
    l = h.t[7][lo & 0xff] ^ h.t[6][(lo >> 8) & 0xff] ^ h.t[5][(lo >> 16) & 0xff] ^ h.t[4][lo >> 24] ^
        h.t[3][hi & 0xff] ^ h.t[2][(hi >> 8) & 0xff] ^ h.t[1][(hi >> 16) & 0xff] ^ h.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) l = h.t[0][(l ^ *p++) & 0xffu] ^ (l >> 8);
  return l;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t raw_sse42(uint32_t l, const uint8_t* p, size_t n) {
  while (n && ((uintptr_t)p & 7u)) {
    l = _mm_crc32_u8(l, *p++);
    --n;
  }
  if (n >= 3 * kStream) {
    const HostTables& h = host_tables();
    while (n >= 3 * kStream) {
      uint64_t a = l, b = 0, c = 0;
      const uint8_t* pa = p;
      const uint8_t* pb = p + kStream;
      const uint8_t* pc = p + 2 * kStream;
      for (size_t k = 0; k < kStream; k += 8) {
        uint64_t wa, wb, wc;
        memcpy(&wa, pa + k, 8);
        memcpy(&wb, pb + k, 8);
        memcpy(&wc, pc + k, 8);
        a = _mm_crc32_u64(a, wa);
        b = _mm_crc32_u64(b, wb);
        c = _mm_crc32_u64(c, wc);
      }
      // raw(l, A||B||C) = shift(shift(raw(l,A),|B|) ^ raw(0,B), |C|) ^ raw(0,C)
      l = shift_stream(h, shift_stream(h, (uint32_t)a) ^ (uint32_t)b) ^ (uint32_t)c;
      p += 3 * kStream;
      n -= 3 * kStream;
    }
  }
  uint64_t l64 = l;
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    l64 = _mm_crc32_u64(l64, w);
    p += 8;
    n -= 8;
  }
  l = (uint32_t)l64;
  while (n--) l = _mm_crc32_u8(l, *p++);
  return l;
}

bool have_sse42() {
  unsigned int eax, ebx, ecx, edx;
  if (!__get_cpuid(1, &eax, &ebx, &ecx, &edx)) return false;
  return (ecx & (1u << 20)) != 0;
}
#endif

}  // namespace

uint32_t host_extend(uint32_t init, const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
#if defined(__x86_64__)
  static const bool sse = [] {
    // self-test mirrors util/crc32c.cc:290-297
    static const char kTest[] = "TestCRCBuffer";
    return have_sse42() &&
           (raw_sse42(0xffffffffu, reinterpret_cast<const uint8_t*>(kTest), 13) ^ 0xffffffffu) == 0xdcbc59fau;
  }();
  if (sse) return raw_sse42(init ^ 0xffffffffu, p, n) ^ 0xffffffffu;
#endif
  return raw_slice8(init ^ 0xffffffffu, p, n) ^ 0xffffffffu;
}

}  // namespace nvl
