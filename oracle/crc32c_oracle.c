/*
 * oracle/crc32c_oracle.c -- CPU restatement of the reference CRC32C path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (nvlevelz_amd/, include/)
 * may link, import or call this file.  Only tests/, __graft_entry__.smoke()
 * and bench.py's `cpu_baseline` leg use it, and only as the checker or as the
 * reported CPU baseline -- never as the thing measured or shipped.
 *
 * Parity pinning: every function here is checked (tests/test_oracle.py)
 * against the golden vectors in tests/golden/, which were produced by the
 * reference's own util/crc32c.cc + port/port_posix_sse.cc compiled from
 * /root/reference (oracle/Makefile -> oracle/_ref/, generator
 * oracle/gen_golden.py), and against util/crc32c_test.cc:13-65's RFC 3720
 * known answers.
 *
 * The restatement is clean-room: the lookup tables are regenerated from the
 * reflected Castagnoli polynomial 0x82F63B78 instead of copying the literal
 * tables at util/crc32c.cc:18-281.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>
#if defined(__x86_64__)
#include <nmmintrin.h>
#include <cpuid.h>
#endif

#define POLY_REFLECTED 0x82F63B78u

/* util/crc32c.cc:18-281 -- table0_..table3_ (slice-by-4).  table_k[b] is the
 * raw register after feeding byte b followed by k zero bytes. */
static uint32_t tab[4][256];
static int tab_ready = 0;

static void build_tables(void) {
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int i = 0; i < 8; ++i) c = (c >> 1) ^ ((c & 1u) ? POLY_REFLECTED : 0u);
    tab[0][b] = c;
  }
  for (int k = 1; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b)
      tab[k][b] = (tab[k - 1][b] >> 8) ^ tab[0][tab[k - 1][b] & 0xffu];
  tab_ready = 1;
}

static inline void ensure_tables(void) {
  if (!tab_ready) build_tables();  /* idempotent; benign race */
}

/* util/crc32c.cc:284-286 -> util/coding.h:58-70: little-endian 32-bit load */
static inline uint32_t le_load32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}

/* util/crc32c.cc:299-347 (the portable path, taken when the accelerator probe
 * fails): pre-invert, STEP1 to 4-byte alignment (324-331), 16 B as four STEP4
 * (333-335), STEP4 (337-339), STEP1 tail (341-343), post-invert (346). */
uint32_t oracle_crc32c_extend_table(uint32_t crc, const void* buf, size_t size) {
  ensure_tables();
  const uint8_t* p = (const uint8_t*)buf;
  const uint8_t* e = p + size;
  uint32_t l = crc ^ 0xffffffffu;
#define O_STEP1 do { int c_ = (int)((l & 0xffu) ^ *p++); l = tab[0][c_] ^ (l >> 8); } while (0)
#define O_STEP4 do { uint32_t c_ = l ^ le_load32(p); p += 4;                       \
    l = tab[3][c_ & 0xffu] ^ tab[2][(c_ >> 8) & 0xffu] ^ tab[1][(c_ >> 16) & 0xffu] \
        ^ tab[0][c_ >> 24]; } while (0)
  const uintptr_t pval = (uintptr_t)p;
  const uint8_t* x = (const uint8_t*)(((pval + 3) >> 2) << 2);
  if (x <= e) {
    while (p != x) O_STEP1;
  }
  while ((e - p) >= 16) { O_STEP4; O_STEP4; O_STEP4; O_STEP4; }
  while ((e - p) >= 4) O_STEP4;
  while (p != e) O_STEP1;
#undef O_STEP4
#undef O_STEP1
  return l ^ 0xffffffffu;
}

/* port/port_posix_sse.cc:51-63 -- CPUID.1:ECX bit 20 */
static int have_sse42(void) {
#if defined(__x86_64__)
  unsigned int eax, ebx, ecx, edx;
  if (!__get_cpuid(1, &eax, &ebx, &ecx, &edx)) return 0;
  return (ecx & (1u << 20)) != 0;
#else
  return 0;
#endif
}

/* port/port_posix_sse.cc:69-126.  Returns 0 when SSE4.2 is unavailable
 * (contract port/port_example.h:132-136).  For size > 16: a byte prologue of
 * (p % 8) steps (94-98; note: p%8, not 8-p%8, exactly as the reference), 8 B
 * crc32q steps (103-105), at most one 4 B step (107-109), then byte tail
 * (118-120). */
#if defined(__x86_64__)
__attribute__((target("sse4.2")))
#endif
uint32_t oracle_crc32c_extend_sse(uint32_t crc, const void* buf, size_t size) {
#if defined(__x86_64__)
  static int have = -1;
  if (have < 0) have = have_sse42();
  if (!have) return 0;
  const uint8_t* p = (const uint8_t*)buf;
  const uint8_t* e = p + size;
  uint32_t l = crc ^ 0xffffffffu;
  if (size > 16) {
    for (unsigned int i = (unsigned int)((uintptr_t)p % 8); i; --i) l = _mm_crc32_u8(l, *p++);
    while ((e - p) >= 8) {
      uint64_t w;
      memcpy(&w, p, 8);
      l = (uint32_t)_mm_crc32_u64(l, w);
      p += 8;
    }
    if ((e - p) >= 4) {
      uint32_t w;
      memcpy(&w, p, 4);
      l = _mm_crc32_u32(l, w);
      p += 4;
    }
  }
  while (p != e) l = _mm_crc32_u8(l, *p++);
  return l ^ 0xffffffffu;
#else
  (void)crc; (void)buf; (void)size;
  return 0;
#endif
}

/* util/crc32c.cc:290-297: the accelerator self-test "TestCRCBuffer" ->
 * 0xdcbc59fa, and util/crc32c.cc:299-303: dispatch on it. */
int oracle_can_accelerate(void) {
  static const char kTest[] = "TestCRCBuffer";
  return oracle_crc32c_extend_sse(0, kTest, sizeof(kTest) - 1) == 0xdcbc59fau;
}

uint32_t oracle_crc32c_extend(uint32_t crc, const void* buf, size_t size) {
  static int accel = -1;
  if (accel < 0) accel = oracle_can_accelerate();
  if (accel) return oracle_crc32c_extend_sse(crc, buf, size);
  return oracle_crc32c_extend_table(crc, buf, size);
}

/* util/crc32c.h:20-22 */
uint32_t oracle_crc32c_value(const void* buf, size_t size) {
  return oracle_crc32c_extend(0, buf, size);
}

/* util/crc32c.h:24,31-34 */
uint32_t oracle_crc32c_mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
}

/* util/crc32c.h:37-40 */
uint32_t oracle_crc32c_unmask(uint32_t masked) {
  uint32_t rot = masked - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}

/* ------------------------------------------------------------------------ */
/* Synthetic input generator: successive splitmix64 outputs,
 * little-endian, the final partial word truncated.  Buffer i of a fixed-stride
 * batch starts at byte i*stride of the stream, so a generator that only knows
 * (seed, byte offset) reproduces any slice. */
static inline uint64_t splitmix64_at(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Fill dst[0..n) with stream bytes [offset, offset+n). */
void oracle_fill_splitmix(uint64_t seed, uint64_t offset, uint8_t* dst, size_t n) {
  size_t i = 0;
  while (i < n && ((offset + i) & 7u)) {  /* head up to a word boundary */
    uint64_t pos = offset + i;
    dst[i++] = (uint8_t)(splitmix64_at(seed, pos >> 3) >> (8 * (pos & 7u)));
  }
  while (i + 8 <= n) {                     /* whole little-endian words */
    uint64_t w = splitmix64_at(seed, (offset + i) >> 3);
    for (int b = 0; b < 8; ++b) dst[i + b] = (uint8_t)(w >> (8 * b));
    i += 8;
  }
  while (i < n) {                          /* truncated final word */
    uint64_t pos = offset + i;
    dst[i++] = (uint8_t)(splitmix64_at(seed, pos >> 3) >> (8 * (pos & 7u)));
  }
}

/* Config-3 length stream: len_k = 512 + splitmix64_k(seed) %
 * 65025, packed back to back until `total` bytes, last one truncated.
 * Returns the number of buffers; writes at most `cap` lengths. */
uint64_t oracle_cfg3_lengths(uint64_t seed, uint64_t total, uint64_t* lens, uint64_t cap) {
  uint64_t used = 0, k = 0;
  while (used < total) {
    uint64_t len = 512 + splitmix64_at(seed, k) % 65025u;
    if (len > total - used) len = total - used;
    if (k < cap) lens[k] = len;
    used += len;
    ++k;
  }
  return k;
}

/* Batch helpers (used by tests and the CPU baseline). */
void oracle_crc32c_fixed(const uint8_t* base, uint64_t stride, uint64_t len,
                         uint64_t n, const uint32_t* init, uint32_t* out) {
  for (uint64_t i = 0; i < n; ++i)
    out[i] = oracle_crc32c_extend(init ? init[i] : 0u, base + i * stride, (size_t)len);
}

void oracle_crc32c_varlen(const uint8_t* base, const uint64_t* offsets,
                          const uint64_t* lengths, uint64_t n,
                          const uint32_t* init, uint32_t* out) {
  for (uint64_t i = 0; i < n; ++i)
    out[i] = oracle_crc32c_extend(init ? init[i] : 0u, base + offsets[i], (size_t)lengths[i]);
}

/* digest = Value() over the little-endian array of per-buffer CRCs (§8d). */
uint32_t oracle_digest(const uint32_t* crcs, uint64_t n) {
  uint32_t l = 0;
  /* stream the LE bytes of the u32 array through Extend in pieces */
  uint8_t buf[4096];
  uint64_t i = 0;
  while (i < n) {
    size_t m = 0;
    while (i < n && m + 4 <= sizeof(buf)) {
      uint32_t v = crcs[i++];
      buf[m++] = (uint8_t)v; buf[m++] = (uint8_t)(v >> 8);
      buf[m++] = (uint8_t)(v >> 16); buf[m++] = (uint8_t)(v >> 24);
    }
    l = oracle_crc32c_extend(l, buf, m);
  }
  return l;
}

/* Multi-threaded fixed-stride batch: contiguous partition per thread
 * (interleaving caused false sharing).  which: 0 = dispatching
 * Extend (SSE when available), 1 = table path. */
typedef struct {
  const uint8_t* base; uint64_t stride, len, lo, hi; uint32_t* out; int which; uint64_t reps;
} oracle_job_t;

static void* oracle_job(void* arg) {
  oracle_job_t* j = (oracle_job_t*)arg;
  for (uint64_t r = 0; r < j->reps; ++r)
    for (uint64_t i = j->lo; i < j->hi; ++i)
      j->out[i] = j->which ? oracle_crc32c_extend_table(0, j->base + i * j->stride, (size_t)j->len)
                           : oracle_crc32c_extend(0, j->base + i * j->stride, (size_t)j->len);
  return 0;
}

/* reps passes over each thread's share (a timed baseline pays the thread
 * start-up once). */
int oracle_crc32c_fixed_mt_reps(const uint8_t* base, uint64_t stride, uint64_t len,
                                uint64_t n, uint32_t* out, int threads, int which, uint64_t reps) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  oracle_job_t jobs[256];
  ensure_tables();
  (void)oracle_crc32c_extend(0, "", 0);  /* resolve the static dispatch once */
  for (int t = 0; t < threads; ++t) {
    jobs[t].base = base; jobs[t].stride = stride; jobs[t].len = len;
    jobs[t].lo = n * (uint64_t)t / (uint64_t)threads;
    jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
    jobs[t].out = out; jobs[t].which = which; jobs[t].reps = reps;
  }
  for (int t = 1; t < threads; ++t)
    if (pthread_create(&tid[t], 0, oracle_job, &jobs[t]) != 0) return -1;
  oracle_job(&jobs[0]);
  for (int t = 1; t < threads; ++t) pthread_join(tid[t], 0);
  return 0;
}

int oracle_crc32c_fixed_mt(const uint8_t* base, uint64_t stride, uint64_t len,
                           uint64_t n, uint32_t* out, int threads, int which) {
  return oracle_crc32c_fixed_mt_reps(base, stride, len, n, out, threads, which, 1);
}
