// nvlevelz_amd/csrc/crc32c_math.h -- GF(2) arithmetic for CRC32C, shared by
// host C++ and the HIP kernels.
//
// CRC32C (Castagnoli): reflected polynomial 0x82F63B78, register pre/post
// inverted, as defined by util/crc32c.cc:299-347 / port/port_posix_sse.cc:69-126
// of the reference.  Representation: a 32-bit register value is a polynomial
// of degree < 32 with bit 31 = x^0 and bit 0 = x^31 (the reflected convention);
// feeding one zero byte into the register multiplies it by x^8 mod P.
//
// Identities used throughout the engine (proved in tests/test_math.py against
// the oracle):
//   raw(s, D)         : register after feeding D starting from register s
//   raw(s, D)          = shift(s, |D|) ^ raw(0, D)
//   raw(0, A || B)     = shift(raw(0, A), |B|) ^ raw(0, B)
//   Extend(init, D)    = ~raw(~init, D)                      (crc32c.cc:307,346)
//   raw(s, w || rest)  = raw(0, (w ^ s) || rest)  for a 4-byte LE word w
//   shift(v, n)        = v * x^(8n) mod P         (gf_mul(xpow8(n), v))
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define NVL_HD __host__ __device__
#else
#define NVL_HD
#endif

namespace nvl {

constexpr uint32_t kPolyReflected = 0x82F63B78u;  // util/crc32c.cc tables' generator
constexpr uint32_t kMaskDelta = 0xa282ead8u;      // util/crc32c.h:24
constexpr uint32_t kOne = 0x80000000u;            // x^0 in reflected form

// util/crc32c.h:31-34
NVL_HD inline uint32_t mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + kMaskDelta;
}

// util/crc32c.h:37-40
NVL_HD inline uint32_t unmask(uint32_t masked) {
  const uint32_t rot = masked - kMaskDelta;
  return (rot >> 17) | (rot << 15);
}

// a * b mod P in the reflected representation (32 fixed iterations, no
// data-dependent trip count so it is cheap to run in a divergent lane).
NVL_HD inline uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 8
#endif
  for (int i = 0; i < 32; ++i) {
    p ^= (a & (kOne >> i)) ? b : 0u;
    b = (b >> 1) ^ ((b & 1u) ? kPolyReflected : 0u);
  }
  return p;
}

// One bit-serial step table entry: register after feeding byte b from 0.
NVL_HD inline uint32_t byte_table0(uint32_t b) {
  uint32_t c = b;
  for (int i = 0; i < 8; ++i) c = (c >> 1) ^ ((c & 1u) ? kPolyReflected : 0u);
  return c;
}

// Host-side constant tables.  x2n[k] = x^(2^k) mod P.  64 entries, so
// xpow8(n) covers every n < 2^61 without assuming anything about the order
// of x modulo P.
struct PowTable {
  uint32_t x2n[64];
};

inline void build_pow_table(PowTable* t) {
  uint32_t p = kOne >> 1;  // x^1
  for (int k = 0; k < 64; ++k) {
    t->x2n[k] = p;
    p = gf_mul(p, p);
  }
}

// x^(8n) mod P given the x2n table.
NVL_HD inline uint32_t xpow8(const uint32_t* x2n, uint64_t n) {
  uint32_t p = kOne;
  int k = 3;
  while (n) {
    if (n & 1u) p = gf_mul(x2n[k], p);
    n >>= 1;
    ++k;
  }
  return p;
}

// shift(v, nbytes): the register after feeding nbytes zero bytes.
NVL_HD inline uint32_t shift_bytes(const uint32_t* x2n, uint32_t v, uint64_t nbytes) {
  return gf_mul(xpow8(x2n, nbytes), v);
}

// Byte-sliced operator table for "shift by a fixed distance": op[j][b] =
// shift(b << 8j, dist), so shift(v, dist) = XOR_j op[j][byte_j(v)].
inline void build_shift_op(const uint32_t* x2n, uint64_t dist, uint32_t op[4][256]) {
  const uint32_t m = xpow8(x2n, dist);
  for (int j = 0; j < 4; ++j)
    for (uint32_t b = 0; b < 256; ++b) op[j][b] = gf_mul(m, b << (8 * j));
}

// Slice-by-4 tables (same contents as util/crc32c.cc:18-281's table0_..3_,
// regenerated from the polynomial): t[k][b] = register after byte b then k
// zero bytes.
inline void build_slice4(uint32_t t[4][256]) {
  for (uint32_t b = 0; b < 256; ++b) t[0][b] = byte_table0(b);
  for (int k = 1; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b)
      t[k][b] = (t[k - 1][b] >> 8) ^ t[0][t[k - 1][b] & 0xffu];
}

}  // namespace nvl
