// oracle/ref_shim.cc -- C-ABI shim over the REFERENCE's own CRC32C objects.
//
// TEST INFRASTRUCTURE ONLY.  This file contains no reference code: it
// includes the reference header util/crc32c.h from /root/reference and is
// linked (oracle/Makefile) against util/crc32c.cc and port/port_posix_sse.cc
// compiled straight from /root/reference into oracle/_ref/.  Two builds:
//   oracle/_ref/libref_crc32c_sse.so   -- -msse4.2 -DLEVELDB_PLATFORM_POSIX_SSE
//                                         (port/port_posix_sse.cc:69-126 path)
//   oracle/_ref/libref_crc32c_table.so -- no SSE define: AcceleratedCRC32C
//                                         returns 0, the probe at
//                                         util/crc32c.cc:290-297 fails and
//                                         Extend runs the slice-by-4 table
//                                         path util/crc32c.cc:305-346.
// Used to (a) generate tests/golden/ fixtures (oracle/gen_golden.py) and
// (b) as bench.py's cpu_baseline (kind "reference").
#include <stddef.h>
#include <stdint.h>
#include <pthread.h>
#include <string.h>
#include <time.h>
#include "util/crc32c.h"

namespace leveldb {
namespace port {
uint32_t AcceleratedCRC32C(uint32_t crc, const char* buf, size_t size);
}
}  // namespace leveldb

extern "C" {

__attribute__((visibility("default")))
uint32_t ref_crc32c_extend(uint32_t init, const void* data, size_t n) {
  return leveldb::crc32c::Extend(init, static_cast<const char*>(data), n);
}

__attribute__((visibility("default")))
uint32_t ref_crc32c_value(const void* data, size_t n) {
  return leveldb::crc32c::Value(static_cast<const char*>(data), n);
}

__attribute__((visibility("default")))
uint32_t ref_crc32c_mask(uint32_t crc) { return leveldb::crc32c::Mask(crc); }

__attribute__((visibility("default")))
uint32_t ref_crc32c_unmask(uint32_t m) { return leveldb::crc32c::Unmask(m); }

__attribute__((visibility("default")))
uint32_t ref_accelerated_crc32c(uint32_t init, const void* data, size_t n) {
  return leveldb::port::AcceleratedCRC32C(init, static_cast<const char*>(data), n);
}

// Batch driver for baselines: buffer i = base + i*stride, len bytes, Value().
// `reps` passes over each thread's contiguous share, so a timed baseline
// pays the thread start-up once, not per pass.
struct RefJob {
  const uint8_t* base; uint64_t stride, len, lo, hi; uint32_t* out; uint64_t reps;
};

static void* ref_job(void* a) {
  RefJob* j = static_cast<RefJob*>(a);
  for (uint64_t r = 0; r < j->reps; ++r)
    for (uint64_t i = j->lo; i < j->hi; ++i)
      j->out[i] = leveldb::crc32c::Value(
          reinterpret_cast<const char*>(j->base + i * j->stride), j->len);
  return nullptr;
}

__attribute__((visibility("default")))
int ref_crc32c_fixed_mt_reps(const uint8_t* base, uint64_t stride, uint64_t len,
                             uint64_t n, uint32_t* out, int threads, uint64_t reps) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  RefJob jobs[256];
  (void)leveldb::crc32c::Value("", 0);  // resolve the static probe once
  for (int t = 0; t < threads; ++t) {
    jobs[t] = RefJob{base, stride, len, n * (uint64_t)t / (uint64_t)threads,
                     n * (uint64_t)(t + 1) / (uint64_t)threads, out, reps};
  }
  for (int t = 1; t < threads; ++t)
    if (pthread_create(&tid[t], nullptr, ref_job, &jobs[t]) != 0) return -1;
  ref_job(&jobs[0]);
  for (int t = 1; t < threads; ++t) pthread_join(tid[t], nullptr);
  return 0;
}

__attribute__((visibility("default")))
int ref_crc32c_fixed_mt(const uint8_t* base, uint64_t stride, uint64_t len,
                        uint64_t n, uint32_t* out, int threads) {
  return ref_crc32c_fixed_mt_reps(base, stride, len, n, out, threads, 1);
}

// db/db_bench.cc:729-746 Crc32c(): Value() of ONE 4096-byte buffer of 'x'
// until `total` bytes are checksummed, on the calling thread.  fn == NULL:
// the reference's own leveldb::crc32c::Value (util/crc32c.h:20-22 inline ->
// Extend, util/crc32c.cc:299-347 -> port::AcceleratedCRC32C); otherwise the
// same loop through fn (e.g. the drop-in's nvl_crc32c_value).  Returns the
// loop's wall time in ns (CLOCK_MONOTONIC); *crc = the last value.
__attribute__((visibility("default")))
uint64_t ref_dbbench_crc32c(uint32_t (*fn)(const void*, size_t), int64_t total, uint32_t* crc_out) {
  const int size = 4096;
  static char data[4096];
  memset(data, 'x', sizeof(data));
  (void)leveldb::crc32c::Value("", 0);  // resolve the static probe before timing
  timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  int64_t bytes = 0;
  uint32_t crc = 0;
  if (fn) {
    while (bytes < total) {
      crc = fn(data, size);
      bytes += size;
    }
  } else {
    while (bytes < total) {
      crc = leveldb::crc32c::Value(data, size);
      bytes += size;
    }
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (crc_out) *crc_out = crc;
  return (uint64_t)(t1.tv_sec - t0.tv_sec) * 1000000000ull + (uint64_t)(t1.tv_nsec - t0.tv_nsec);
}

}  // extern "C"
