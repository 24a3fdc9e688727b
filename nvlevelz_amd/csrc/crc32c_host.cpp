// nvlevelz_amd/csrc/crc32c_host.cpp -- the single-buffer host path of the
// util/crc32c.h API (leveldb::crc32c::Extend, util/crc32c.cc:299-347).
//
// This is the reference API's per-call CPU semantics -- one buffer, on the
// calling thread -- kept because a GPU round trip for one ~4 KiB buffer costs
// more than the checksum.  It is NOT used by any batch entry point.
//
// Three implementations, chosen once (thread-safe static) like the
// reference's CanAccelerateCRC32C probe (util/crc32c.cc:290-303), each only
// after it passes the probe's known answer and a 4 KiB cross-check:
//   * AVX-512 carry-less multiply folding (VPCLMULQDQ: 256 bytes per step in
//     four 512-bit accumulators, the residue finished by the crc32
//     instruction) for buffers of 256 bytes and more, SSE4.2 below that;
//   * SSE4.2 crc32 instruction, three independent 8-byte streams over the
//     bulk of long buffers recombined with the GF(2) shift operator (the
//     instruction has 3-cycle latency and 1/cycle throughput), else
//   * portable slice-by-8.
// NVL_CRC32C_HOST=sse|table in the environment forces a lower tier (tests).
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
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

// AVX-512F/VL/BW + VPCLMULQDQ + PCLMULQDQ, and the OS saving ZMM state.
bool have_vpclmul512() {
  unsigned int eax, ebx, ecx, edx;
  if (!__get_cpuid(1, &eax, &ebx, &ecx, &edx)) return false;
  if (!(ecx & (1u << 1)) || !(ecx & (1u << 27)) || !(ecx & (1u << 20))) return false;  // pclmul, osxsave, sse4.2
  unsigned int xlo, xhi;
  __asm__ volatile("xgetbv" : "=a"(xlo), "=d"(xhi) : "c"(0));
  if ((xlo & 0xE6u) != 0xE6u) return false;  // XMM, YMM, opmask, ZMM_Hi256, Hi16_ZMM
  if (!__get_cpuid_count(7, 0, &eax, &ebx, &ecx, &edx)) return false;
  const bool f = ebx & (1u << 16), bw = ebx & (1u << 30), vl = ebx & (1u << 31), vpcl = ecx & (1u << 10);
  return f && bw && vl && vpcl;
}

// Folding.  A 16-byte block read as a little-endian
// 128-bit integer is the message polynomial with bit p = the coefficient of
// x^(127-p) (the reflected order of the crc32 instruction): its first 8
// bytes A1 are degrees 127..64, its last 8 bytes A0 degrees 63..0.  Moving it
// d bytes forward multiplies it by x^(8d): A1 x^(8d+64) + A0 x^(8d), with
// each power reduced mod P to 32 bits.  A carry-less product of two
// reflected 64-bit operands lands one degree low (bit p = degree 126 - p),
// so each constant carries an extra x^-1: the fold of A is
//   clmul(A1, x^(8d+63) mod P) ^ clmul(A0, x^(8d-1) mod P),
// a polynomial of degree < 96 congruent to A x^(8d), XORed into the block d
// bytes later.  The 128-bit residue left at the end is congruent to the
// whole prefix, so the crc32 instruction run over its 16 bytes from 0 gives
// the prefix's register (raw(0, .) is linear), and the tail follows.
inline uint32_t mul_xinv(uint32_t v) {  // v * x^-1 mod P (reflected)
  return (v & kOne) ? (((v ^ kPolyReflected) << 1) | 1u) : (v << 1);
}
struct FoldK {
  uint64_t a1, a0;  // constants for A1 and A0 (reflected, degree < 32: the upper half)
};
FoldK fold_k(const PowTable& pw, uint64_t d) {
  return FoldK{(uint64_t)mul_xinv(xpow8(pw.x2n, d + 8)) << 32, (uint64_t)mul_xinv(xpow8(pw.x2n, d)) << 32};
}
struct FoldTables {
  FoldK k256, k192, k128, k64, k48, k32, k16;
};
const FoldTables& fold_tables() {
  static const FoldTables* t = [] {
    FoldTables* f = new FoldTables;
    const PowTable& pw = host_tables().pw;
    f->k256 = fold_k(pw, 256);
    f->k192 = fold_k(pw, 192);
    f->k128 = fold_k(pw, 128);
    f->k64 = fold_k(pw, 64);
    f->k48 = fold_k(pw, 48);
    f->k32 = fold_k(pw, 32);
    f->k16 = fold_k(pw, 16);
    return f;
  }();
  return *t;
}

#define NVL_AVX512_TARGET __attribute__((target("avx512f,avx512vl,avx512bw,vpclmulqdq,pclmul,sse4.2")))

NVL_AVX512_TARGET inline __m512i kvec512(const FoldK& k) {
  return _mm512_broadcast_i32x4(_mm_set_epi64x((long long)k.a0, (long long)k.a1));
}
NVL_AVX512_TARGET inline __m512i fold512(__m512i x, __m512i k, __m512i next) {
  return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x, k, 0x00), _mm512_clmulepi64_epi128(x, k, 0x11), next,
                                   0x96);
}
NVL_AVX512_TARGET inline __m128i fold128(__m128i x, const FoldK& k, __m128i next) {
  const __m128i kv = _mm_set_epi64x((long long)k.a0, (long long)k.a1);
  return _mm_ternarylogic_epi64(_mm_clmulepi64_si128(x, kv, 0x00), _mm_clmulepi64_si128(x, kv, 0x11), next, 0x96);
}

// raw(l, p[0, n)) for n >= 256.
NVL_AVX512_TARGET uint32_t raw_vpclmul(uint32_t l, const uint8_t* p, size_t n) {
  const FoldTables& t = fold_tables();
  __m512i x0 = _mm512_loadu_si512(p), x1 = _mm512_loadu_si512(p + 64), x2 = _mm512_loadu_si512(p + 128),
          x3 = _mm512_loadu_si512(p + 192);
  x0 = _mm512_xor_si512(x0, _mm512_zextsi128_si512(_mm_cvtsi32_si128((int)l)));  // raw(l, w||r) = raw(0, (w^l)||r)
  p += 256;
  n -= 256;
  const __m512i k256 = kvec512(t.k256);
  while (n >= 256) {
    x0 = fold512(x0, k256, _mm512_loadu_si512(p));
    x1 = fold512(x1, k256, _mm512_loadu_si512(p + 64));
    x2 = fold512(x2, k256, _mm512_loadu_si512(p + 128));
    x3 = fold512(x3, k256, _mm512_loadu_si512(p + 192));
    p += 256;
    n -= 256;
  }
  // the four accumulators into the last one, its four lanes into one
  x3 = fold512(x0, kvec512(t.k192), x3);
  x3 = fold512(x1, kvec512(t.k128), x3);
  x3 = fold512(x2, kvec512(t.k64), x3);
  __m128i r = _mm512_extracti32x4_epi32(x3, 3);
  r = fold128(_mm512_extracti32x4_epi32(x3, 0), t.k48, r);
  r = fold128(_mm512_extracti32x4_epi32(x3, 1), t.k32, r);
  r = fold128(_mm512_extracti32x4_epi32(x3, 2), t.k16, r);
  while (n >= 16) {
    r = fold128(r, t.k16, _mm_loadu_si128(reinterpret_cast<const __m128i*>(p)));
    p += 16;
    n -= 16;
  }
  uint64_t c = _mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(r));
  c = _mm_crc32_u64(c, (uint64_t)_mm_extract_epi64(r, 1));
  uint32_t v = (uint32_t)c;
  if (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    v = (uint32_t)_mm_crc32_u64(v, w);
    p += 8;
    n -= 8;
  }
  while (n--) v = _mm_crc32_u8(v, *p++);
  return v;
}
#endif

}  // namespace

namespace {
// 0: slice-by-8, 1: SSE4.2, 2: AVX-512 folding (>= 256 bytes) over SSE4.2
int host_tier() {
  static const int tier = [] {
    const char* force = getenv("NVL_CRC32C_HOST");
    const int cap = force && !strcmp(force, "table") ? 0 : (force && !strcmp(force, "sse") ? 1 : 2);
    int t = 0;
#if defined(__x86_64__)
    // self-tests mirror util/crc32c.cc:290-297 ("TestCRCBuffer"), plus a
    // 4 KiB cross-check of every faster tier against slice-by-8
    static const char kTest[] = "TestCRCBuffer";
    if (cap >= 1 && have_sse42() &&
        (raw_sse42(0xffffffffu, reinterpret_cast<const uint8_t*>(kTest), 13) ^ 0xffffffffu) == 0xdcbc59fau)
      t = 1;
    if (t == 1 && cap >= 2 && have_vpclmul512()) {
      uint8_t buf[4096 + 77];
      uint64_t x = 0x9E3779B97F4A7C15ull;
      for (auto& b : buf) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        b = (uint8_t)(x >> 56);
      }
      bool ok = true;
      for (size_t n : {(size_t)256, (size_t)300, (size_t)1024, (size_t)4096 + 77})
        ok = ok && raw_vpclmul(0x12345678u, buf, n) == raw_slice8(0x12345678u, buf, n);
      if (ok) t = 2;
    }
#endif
    return t;
  }();
  return tier;
}
}  // namespace

uint32_t host_extend(uint32_t init, const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  const uint32_t l = init ^ 0xffffffffu;
#if defined(__x86_64__)
  const int t = host_tier();
  if (t == 2 && n >= 256) return raw_vpclmul(l, p, n) ^ 0xffffffffu;
  if (t >= 1) return raw_sse42(l, p, n) ^ 0xffffffffu;
#endif
  return raw_slice8(l, p, n) ^ 0xffffffffu;
}

int host_tier_id() { return host_tier(); }

const char* host_impl_name() {
  static const char* const kNames[] = {"slice-by-8", "sse4.2 crc32q x3", "avx512 vpclmulqdq fold + sse4.2"};
  return kNames[host_tier()];
}

}  // namespace nvl
