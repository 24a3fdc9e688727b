// nvlevelz_amd/csrc/crc32c_capi.cpp -- the extern "C" boundary declared in
// include/nvl_crc32c.h.  Owns per-device lookup tables, the GPU known-answer
// probe (util/crc32c.cc:290-297 analogue), workspace carving and the
// host-resident staging paths.
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/nvl_crc32c.h"
#include "crc32c_internal.h"
#include "crc32c_math.h"

namespace nvl {

static_assert(kRegionMaxLen == NVL_CRC32C_REGION_MAX_LEN, "the route's length limit is the header's");

void build_device_tables(uint32_t* w) {
  uint32_t slice[4][256];
  build_slice4(slice);
  memcpy(w, slice, sizeof(slice));
  PowTable pw;
  build_pow_table(&pw);
  uint32_t op[4][256];
  for (int lev = 0; lev < 6; ++lev) {
    build_shift_op(pw.x2n, 64ull << lev, op);
    memcpy(w + 1024 + lev * 1024, op, sizeof(op));
  }
  build_shift_op(pw.x2n, 4096, op);
  memcpy(w + 7168, op, sizeof(op));
  memcpy(w + 8192, pw.x2n, sizeof(pw.x2n));
  // Powers of x^8 and of its inverse for the region fold.  Multiplying by x
  // in the reflected form is v >> 1 (^ P when bit 0 = x^31 overflows); its
  // inverse: bit 31 (x^0) set means P was added, so v = ((v ^ P) << 1) | 1.
  uint32_t p = kOne, q = kOne;
  for (uint32_t d = 0; d < kXp8Len; ++d) {
    w[kTabXp8 + d] = p;
    if (d < 4096) w[kTabXm8 + d] = q;
    for (int b = 0; b < 8; ++b) {
      p = (p >> 1) ^ ((p & 1u) ? kPolyReflected : 0u);
      q = (q & kOne) ? (((q ^ kPolyReflected) << 1) | 1u) : (q << 1);
    }
  }
  // the region kernel's per-lane shifts to the chunk end: T[n][v][j] = shift(v << 4n, 64(63 - j))
  for (uint32_t j = 0; j < 64; ++j) {
    const uint32_t m = w[kTabXp8 + 64u * (63u - j)];
    for (uint32_t n = 0; n < 8; ++n)
      for (uint32_t v = 0; v < 16; ++v) w[kTabNib + (n * 16u + v) * 64u + j] = gf_mul(m, v << (4u * n));
  }
  // the region fold's chunk shifts: by 4096, 8192, 12288 and 16384 bytes
  for (uint32_t d = 1; d <= 4; ++d) {
    build_shift_op(pw.x2n, 4096ull * d, op);
    memcpy(w + kTabShc + (d - 1u) * 1024u, op, sizeof(op));
  }
  // x^(8*4096*q): q chunks' worth of x^8 (the long fold's x^(8L) = x^(8 (L mod 4096)) x^(8*4096*q) ...)
  const uint32_t c4k = w[kTabXp8 + 4096];
  uint32_t a = kOne;
  for (uint32_t q = 0; q < 256; ++q) {
    w[kTabPw4k + q] = a;
    a = gf_mul(a, c4k);
  }
}

namespace {

constexpr int kMaxDevices = 64;

struct DeviceState {
  int device = -1;
  int num_cu = 0;
  uint32_t* tables = nullptr;
  int status = NVL_CRC32C_OK;  // OK, or why the backend is unusable
  std::mutex cmu;
  std::unordered_map<hipStream_t, uint32_t*> counters;  // per-stream counter blocks
};

std::mutex g_mu;
std::atomic<DeviceState*> g_state[kMaxDevices];
std::atomic<uint64_t> g_generation{1};  // bumped by shutdown: invalidates the per-thread cache

// Streams that get a counter block; launches on further streams run the
// unfused pipeline (plan, kernel, fix-up).
constexpr size_t kMaxCounterStreams = 4096;

// The counter block of `st` (LaunchCtx::counter), created zeroed on first
// use (a hipMemsetAsync on `st`, so it is ordered before the first launch);
// nullptr when unavailable.  Lock-free after a thread's first launch on a
// stream.
uint32_t* counters_for(DeviceState* s, hipStream_t st) {
  struct Cache {
    uint64_t gen = 0;
    DeviceState* s = nullptr;
    hipStream_t st = nullptr;
    uint32_t* c = nullptr;
  };
  thread_local Cache cache;
  const uint64_t gen = g_generation.load(std::memory_order_acquire);
  if (cache.gen == gen && cache.s == s && cache.st == st && cache.c) return cache.c;
  std::lock_guard<std::mutex> lk(s->cmu);
  auto it = s->counters.find(st);
  uint32_t* c = it == s->counters.end() ? nullptr : it->second;
  if (!c) {
    if (s->counters.size() >= kMaxCounterStreams) return nullptr;
    void* p = nullptr;
    if (hipMalloc(&p, kCounterBytes) != hipSuccess) return nullptr;
    if (hipMemsetAsync(p, 0, kCounterBytes, st) != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    c = static_cast<uint32_t*>(p);
    s->counters[st] = c;
  }
  cache = Cache{gen, s, st, c};
  return c;
}

// Drop the counter block of a stream that is about to be destroyed (a later
// stream may get the same handle value; the block is re-created zeroed).
void forget_counter(int device, hipStream_t st) {
  if (device < 0 || device >= kMaxDevices) return;
  DeviceState* s = g_state[device].load(std::memory_order_acquire);
  if (!s) return;
  std::lock_guard<std::mutex> lk(s->cmu);
  auto it = s->counters.find(st);
  if (it == s->counters.end()) return;
  (void)hipFree(it->second);
  s->counters.erase(it);
}

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// The device a stream belongs to (the null stream: the calling thread's
// current device).  Batch calls take their tables and self-test state from
// it, so a stream of device d always runs with device d's tables whatever
// the thread's current device is.
int stream_device(hipStream_t st, int* dev) {
  if (st) {
    hipDevice_t d = -1;
    if (hipStreamGetDevice(st, &d) == hipSuccess && d >= 0) {
      *dev = d;
      return NVL_CRC32C_OK;
    }
  }
  if (hipGetDevice(dev) != hipSuccess || *dev < 0) return NVL_CRC32C_ENODEV;
  return NVL_CRC32C_OK;
}

int run_self_test(DeviceState* s);

// Create (once) and return the state of `device`; nullptr on failure with *rc set.
DeviceState* state_for(int device, int* rc) {
  if (device < 0 || device >= kMaxDevices) {
    *rc = NVL_CRC32C_ENODEV;
    return nullptr;
  }
  DeviceState* s = g_state[device].load(std::memory_order_acquire);
  if (s) {
    *rc = s->status;
    return s->status == NVL_CRC32C_OK ? s : nullptr;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  s = g_state[device].load(std::memory_order_relaxed);
  if (!s) {
    s = new DeviceState;
    s->device = device;
    int prev = -1;
    (void)hipGetDevice(&prev);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) {
      s->status = NVL_CRC32C_ENODEV;
    } else if (hipSetDevice(device) != hipSuccess ||
               hipDeviceGetAttribute(&s->num_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
               s->num_cu <= 0) {
      s->status = NVL_CRC32C_EHIP;
    } else {
      std::vector<uint32_t> words(kTableWords);
      build_device_tables(words.data());
      if (hipMalloc(&s->tables, kTableWords * sizeof(uint32_t)) != hipSuccess ||
          hipMemcpy(s->tables, words.data(), kTableWords * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
        s->status = NVL_CRC32C_EHIP;
      } else {
        s->status = run_self_test(s);
      }
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    g_state[device].store(s, std::memory_order_release);
  }
  *rc = s->status;
  return s->status == NVL_CRC32C_OK ? s : nullptr;
}

DeviceState* current_state(int* rc) {
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) {
    *rc = NVL_CRC32C_ENODEV;
    return nullptr;
  }
  return state_for(dev, rc);
}

// Variable-batch workspace: [chunk counts n+1][chunk_start n+1 (fused: lpre)]
// [unit map (fused: tiles)][records][hc: n u32][flags: long_bufs][scan temp]
// then, for a routed call, [route partials][region workspace: `cap` chunk raws
// + 2 x n event records].
struct BatchWs {
  size_t cs, map, recs, hc, flags, tmp, parts, region, total;
  uint64_t cap;  // region chunk raws (0: no routed part)
};
BatchWs batch_ws(uint64_t n, int num_cu, uint64_t cap) {
  BatchWs w;
  const size_t cnt = align_up((n + 1) * sizeof(uint64_t), 256);
  w.cs = cnt;
  w.map = w.cs + cnt;
  w.recs = w.map + align_up(var_unit_map_bytes(num_cu), 256);
  w.hc = w.recs + align_up(var_recs_bytes(num_cu), 256);
  w.flags = w.hc + align_up(n * sizeof(uint32_t), 256);
  w.tmp = w.flags + 256;
  w.parts = w.tmp + align_up(scan_temp_bytes(n + 1), 256);
  w.region = w.parts + (cap ? route_parts_bytes() : 0);
  w.total = w.region + (cap ? region_ws_bytes_cap(cap, n) : 0);
  w.cap = cap;
  return w;
}

size_t fixed_ws_bytes(uint64_t len, uint64_t n, int num_cu) { return fixed_recs_bytes(num_cu, len, n); }

int hip_rc(hipError_t e) { return e == hipSuccess ? NVL_CRC32C_OK : NVL_CRC32C_EHIP; }

int do_fixed(DeviceState* s, const void* base, uint64_t stride, uint64_t len, uint64_t n, const uint32_t* init,
             uint32_t init_all, uint32_t* out, uint32_t flags, void* ws, size_t ws_bytes, hipStream_t st,
             hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr) {
  if (n == 0) return NVL_CRC32C_OK;
  if (!out || (!base && len)) return NVL_CRC32C_EINVAL;
  if (n > (1ull << 40) || len > (1ull << 40) || (n > 1 && stride > (1ull << 50))) return NVL_CRC32C_EINVAL;
  const size_t need = fixed_ws_bytes(len, n, s->num_cu);
  bool own = false;
  if (need && !ws) {
    if (hipMallocAsync(&ws, need, st) != hipSuccess) return NVL_CRC32C_EHIP;
    own = true;
  } else if (need && ws_bytes < need) {
    return NVL_CRC32C_ENOSPC;
  }
  LaunchCtx lc{st, s->num_cu, s->tables, nullptr, ev_start, ev_stop};
  hipError_t e = launch_fixed(lc, static_cast<const uint8_t*>(base), stride, len, n, init, init_all, out, flags,
                              static_cast<Rec*>(ws));
  if (own) (void)hipFreeAsync(ws, st);
  return hip_rc(e);
}

// A variable-length batch.  routed: the device decides (launch_routed: the
// region path for a region-shaped batch, else the head + body kernels) --
// for metadata only the device holds (nvl_crc32c_batch_dev); otherwise the
// head + body kernels, max_len a host-known bound on the lengths.
int do_batch(DeviceState* s, const void* base, const uint64_t* offsets, const uint64_t* lengths,
             const uint32_t* init, uint32_t init_all, uint32_t* out, uint64_t n, uint32_t flags, void* ws,
             size_t ws_bytes, hipStream_t st, uint64_t max_len = UINT64_MAX, bool routed = false) {
  if (n == 0) return NVL_CRC32C_OK;
  if (!offsets || !lengths || !out) return NVL_CRC32C_EINVAL;
  if (n >= (1ull << 31) - 2) return NVL_CRC32C_EINVAL;
  const BatchWs L = batch_ws(n, s->num_cu, routed ? route_cap_chunks(n) : 0);
  bool own = false;
  if (!ws) {
    if (hipMallocAsync(&ws, L.total, st) != hipSuccess) return NVL_CRC32C_EHIP;
    own = true;
  } else if (ws_bytes < L.total) {
    return NVL_CRC32C_ENOSPC;
  }
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint64_t* cnt = reinterpret_cast<uint64_t*>(w);
  uint64_t* cs = reinterpret_cast<uint64_t*>(w + L.cs);
  uint64_t* unit_first = reinterpret_cast<uint64_t*>(w + L.map);
  Rec* recs = reinterpret_cast<Rec*>(w + L.recs);
  uint32_t* hc = reinterpret_cast<uint32_t*>(w + L.hc);
  uint32_t* long_bufs = reinterpret_cast<uint32_t*>(w + L.flags);
  void* tmp = w + L.tmp;
  LaunchCtx lc{st, s->num_cu, s->tables, nullptr};
  const bool small = var_plan_small(n);
  if (s->num_cu <= 1023) lc.counter = counters_for(s, st);
  if (lc.counter) {  // (cs holds lpre, the unit map region the tiles)
    hipError_t ef =
        routed ? launch_routed(lc, static_cast<const uint8_t*>(base), 0, true, offsets, lengths, n, init, init_all, out,
                               flags, w + L.region, L.cap, w + L.parts, recs, hc, cs, unit_first)
               : launch_var_fused(lc, static_cast<const uint8_t*>(base), offsets, lengths, n, init, init_all, out,
                                  flags, recs, hc, cs, unit_first, max_len);
    if (own) (void)hipFreeAsync(ws, st);
    return hip_rc(ef);
  }
  hipError_t e;
  if (small) {
    e = launch_var_plan_small(lc, lengths, n, cs, unit_first, long_bufs);
  } else {
    e = launch_var_counts(lengths, n, cnt, long_bufs, st);
    if (e == hipSuccess) e = exclusive_scan_u64(tmp, L.parts - L.tmp, cnt, cs, n + 1, st);
  }
  if (e == hipSuccess)
    e = launch_var(lc, static_cast<const uint8_t*>(base), offsets, lengths, cs, unit_first, n, init, init_all, out,
                   flags, recs, hc, long_bufs, small);
  if (own) (void)hipFreeAsync(ws, st);
  return hip_rc(e);
}

// Workspace of a checked region call: the routed batch workspace with the
// caller's region as the region part.
size_t region_checked_ws_bytes(uint64_t region_len, uint64_t n, int num_cu) {
  return batch_ws(n, num_cu, region_cap_chunks(region_len)).total;
}

// Region batch.  checked (nvl_crc32c_region_dev: the layout is the device's
// to check): routed over the caller's region -- a batch that is not
// region-shaped (unsorted, overlapping, outside the region, a buffer longer
// than kRegionMaxLen) runs the batch path.  Unchecked (the host has checked
// the layout itself): the region kernel alone, one launch.
int do_region(DeviceState* s, const void* region, uint64_t region_len, const uint64_t* offsets,
              const uint64_t* lengths, const uint32_t* init, uint32_t init_all, uint32_t* out, uint64_t n,
              uint32_t flags, void* ws, size_t ws_bytes, hipStream_t st, hipEvent_t ev_start = nullptr,
              hipEvent_t ev_stop = nullptr, bool checked = true) {
  if (n == 0) return NVL_CRC32C_OK;
  if (!offsets || !lengths || !out || !region) return NVL_CRC32C_EINVAL;
  if (n >= (1ull << 31) - 2 || region_len > (1ull << 50)) return NVL_CRC32C_EINVAL;
  LaunchCtx lc{st, s->num_cu, s->tables, nullptr, ev_start, ev_stop};
  if (checked && s->num_cu <= 1023) lc.counter = counters_for(s, st);
  checked = checked && lc.counter;
  const BatchWs L = batch_ws(n, s->num_cu, region_cap_chunks(region_len));
  const size_t need = checked ? L.total : region_ws_bytes(region_len, n);
  bool own = false;
  if (!ws) {
    if (hipMallocAsync(&ws, need, st) != hipSuccess) return NVL_CRC32C_EHIP;
    own = true;
  } else if (ws_bytes < need) {
    return NVL_CRC32C_ENOSPC;
  }
  uint8_t* w = static_cast<uint8_t*>(ws);
  hipError_t e =
      checked ? launch_routed(lc, static_cast<const uint8_t*>(region), region_len, false, offsets, lengths, n, init,
                              init_all, out, flags, w + L.region, L.cap, w + L.parts, reinterpret_cast<Rec*>(w + L.recs),
                              reinterpret_cast<uint32_t*>(w + L.hc), reinterpret_cast<uint64_t*>(w + L.cs),
                              reinterpret_cast<uint64_t*>(w + L.map))
              : launch_region(lc, static_cast<const uint8_t*>(region), region_len, offsets, lengths, init, init_all,
                              out, n, flags, ws);
  if (own) (void)hipFreeAsync(ws, st);
  return hip_rc(e);
}

// Sorted by offset and non-overlapping (what the region pass is fast for).
bool region_sorted(const uint64_t* offsets, const uint64_t* lengths, uint64_t n) {
  for (uint64_t i = 1; i < n; ++i)
    if (offsets[i] < offsets[i - 1] + lengths[i - 1]) return false;
  return true;
}

// Known-answer probe on the GPU: "TestCRCBuffer" -> 0xdcbc59fa at every
// alignment 0..15 through the variable-length kernel, plus fixed-stride fast
// and general paths against the host implementation.
int run_self_test(DeviceState* s) {
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return NVL_CRC32C_EHIP;
  int rc = NVL_CRC32C_OK;
  const size_t kBytes = 3 * 4096 + 64;
  std::vector<uint8_t> h(kBytes);
  uint64_t x = 0x5EEDF00Dull;
  for (auto& b : h) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    b = (uint8_t)(x >> 56);
  }
  static const char kTest[] = "TestCRCBuffer";
  for (int o = 0; o < 16; ++o) memcpy(h.data() + 8192 + o * 32 + o, kTest, 13);
  uint8_t* d = nullptr;
  uint64_t* meta = nullptr;
  uint32_t* out = nullptr;
  const int nvar = 16;
  std::vector<uint64_t> hm(2 * nvar);
  for (int o = 0; o < nvar; ++o) {
    hm[o] = 8192 + o * 32 + o;
    hm[nvar + o] = 13;
  }
  std::vector<uint32_t> ho(nvar + 4, 0);
  if (hipMalloc(&d, kBytes) != hipSuccess || hipMalloc(&meta, hm.size() * 8) != hipSuccess ||
      hipMalloc(&out, ho.size() * 4) != hipSuccess) {
    rc = NVL_CRC32C_EHIP;
  } else if (hipMemcpy(d, h.data(), kBytes, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(meta, hm.data(), hm.size() * 8, hipMemcpyHostToDevice) != hipSuccess) {
    rc = NVL_CRC32C_EHIP;
  } else {
    rc = do_batch(s, d, meta, meta + nvar, nullptr, 0, out, nvar, 0, nullptr, 0, st);
    if (rc == NVL_CRC32C_OK)
      rc = do_fixed(s, d, 4096, 4096, 2, nullptr, 0, out + nvar, 0, nullptr, 0, st);  // fast path
    if (rc == NVL_CRC32C_OK)
      rc = do_fixed(s, d + 3, 4100, 4100, 2, nullptr, 0x1234567u, out + nvar + 2, 0, nullptr, 0, st);  // general
    if (rc == NVL_CRC32C_OK) rc = hip_rc(hipStreamSynchronize(st));
    if (rc == NVL_CRC32C_OK) rc = hip_rc(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
    if (rc == NVL_CRC32C_OK) {
      std::vector<uint32_t> want(ho.size());
      for (int o = 0; o < nvar; ++o) want[o] = 0xdcbc59fau;
      for (int k = 0; k < 2; ++k) {
        want[nvar + k] = host_extend(0, h.data() + 4096 * k, 4096);
        want[nvar + 2 + k] = host_extend(0x1234567u, h.data() + 3 + 4100 * k, 4100);
      }
      for (size_t k = 0; k < ho.size(); ++k) {
        if (ho[k] != want[k]) {
          rc = NVL_CRC32C_ESELFTEST;
          fprintf(stderr, "[nvl_crc32c] self-test case %zu: gpu 0x%08x want 0x%08x\n", k, ho[k], want[k]);
        }
      }
#if defined(NVL_DEV_TUNING)
      // Kernel-development builds only (-DNVL_DEV_TUNING, never the shipped
      // library): report but do not disable.
      const char* skip = getenv("NVL_CRC32C_SELFTEST_REPORT_ONLY");
      if (rc == NVL_CRC32C_ESELFTEST && skip && skip[0] == '1') rc = NVL_CRC32C_OK;
#endif
    }
  }
  if (d) (void)hipFree(d);
  if (meta) (void)hipFree(meta);
  if (out) (void)hipFree(out);
  (void)hipStreamDestroy(st);
  return rc;
}

// Per-thread buffers above this size are released when a call needs less
// than a quarter of them (DevSlab / table_pinned only grew).
constexpr size_t kSlabKeep = 64u << 20;

// Pinned host staging for the host-resident entry points (grown on demand,
// one per thread so concurrent callers never share it).
struct Staging {
  void* host = nullptr;
  size_t host_bytes = 0;
  void release() {
    if (host) (void)hipHostFree(host);
    host = nullptr;
    host_bytes = 0;
  }
  void* get(size_t bytes) {
    // grown on demand; a large buffer is given back when a call needs less
    // than a quarter of it (a thread that once verified a huge table does
    // not keep hundreds of MB pinned for good)
    if (bytes > host_bytes || (host_bytes > kSlabKeep && bytes < host_bytes / 4)) {
      if (host) (void)hipHostFree(host);
      host = nullptr;
      host_bytes = 0;
      if (hipHostMalloc(&host, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
      host_bytes = bytes;
    }
    return host;
  }
};
// Per-thread double-buffered device slabs + streams of nvl_crc32c_fixed_host,
// kept across calls (a hipMalloc of two 64 MiB slabs, a hipFree that
// synchronises the device and two stream creations per call were part of
// every host-resident call's latency).  Rebuilt when the device, the
// engine generation (nvl_crc32c_shutdown) or the needed size changes.
struct HostPipe {
  int device = -1;
  uint64_t gen = 0;
  hipStream_t st[2] = {nullptr, nullptr};
  uint8_t* buf[2] = {nullptr, nullptr};
  size_t cap = 0;
  void release() {
    for (int k = 0; k < 2; ++k) {
      if (st[k]) (void)hipStreamSynchronize(st[k]);
      if (buf[k]) (void)hipFree(buf[k]);
      if (st[k]) (void)hipStreamDestroy(st[k]);
      buf[k] = nullptr;
      st[k] = nullptr;
    }
    cap = 0;
  }
  bool get(int dev, size_t bytes) {
    const uint64_t g = g_generation.load(std::memory_order_acquire);
    if (dev == device && g == gen && bytes <= cap && st[0]) return true;
    release();  // nvl_crc32c_shutdown does not reset the device: the old slabs and streams are still valid
    device = dev;
    gen = g;
    for (int k = 0; k < 2; ++k) {
      if (hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking) != hipSuccess) return false;
      if (hipMalloc(&buf[k], bytes) != hipSuccess) return false;
    }
    cap = bytes;
    return true;
  }
};

// A per-thread device buffer (nvl_sstable_verify_table_dev's workspace),
// grown on demand; rebuilt when the device or the engine generation changes.
struct DevSlab {
  int device = -1;
  uint64_t gen = 0;
  void* p = nullptr;
  size_t cap = 0;
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    device = -1;
  }
  void* get(int dev, size_t bytes) {
    const uint64_t g = g_generation.load(std::memory_order_acquire);
    // (shrunk like Staging: a huge slab goes when a call needs < 1/4 of it)
    if (dev == device && g == gen && bytes <= cap && p && !(cap > kSlabKeep && bytes < cap / 4)) return p;
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (device >= 0 && device != prev) (void)hipSetDevice(device);
    release();
    (void)hipSetDevice(dev);
    if (hipMalloc(&p, bytes) != hipSuccess) p = nullptr;
    if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    if (!p) return nullptr;
    device = dev;
    gen = g;
    cap = bytes;
    return p;
  }
};

// Everything a thread acquires for the host-resident entry points: one
// non-blocking stream per device (a stream per call would also mean a
// counter block per call), the pinned staging buffer and the fixed_host
// pipe.  Registered globally so nvl_crc32c_shutdown can free what every
// thread holds; a thread's own resources are freed when it exits (the
// calling thread's thread_local destructors run before exit()'s atexit
// handlers and static destructors, so the HIP runtime is still up).
struct ThreadRes;
std::mutex g_tr_mu;
std::vector<ThreadRes*> g_tr;

struct ThreadRes {
  hipStream_t st[kMaxDevices] = {};
  Staging staging;
  Staging results;  // pinned landing area of the host entries' results (see wait_host_call)
  HostPipe pipe;
  DevSlab table_dev;      // nvl_sstable_verify_table_dev
  Staging table_pinned;
  hipEvent_t table_ev[kMaxDevices][2] = {};
  hipEvent_t wait_ev[kMaxDevices] = {};  // wait_host_call's events
  bool registered = false;

  void enroll() {
    if (registered) return;
    std::lock_guard<std::mutex> lk(g_tr_mu);
    g_tr.push_back(this);
    registered = true;
  }
  // Caller holds g_tr_mu or is the owning thread with no shutdown running.
  void release() {
    int prev = -1;
    (void)hipGetDevice(&prev);
    for (int d = 0; d < kMaxDevices; ++d) {
      for (hipEvent_t& e : table_ev[d]) {
        if (!e) continue;
        (void)hipSetDevice(d);
        (void)hipEventDestroy(e);
        e = nullptr;
      }
      if (wait_ev[d]) {
        (void)hipSetDevice(d);
        (void)hipEventDestroy(wait_ev[d]);
        wait_ev[d] = nullptr;
      }
      if (!st[d]) continue;
      (void)hipSetDevice(d);
      (void)hipStreamSynchronize(st[d]);
      forget_counter(d, st[d]);
      (void)hipStreamDestroy(st[d]);
      st[d] = nullptr;
    }
    if (pipe.device >= 0) (void)hipSetDevice(pipe.device);
    pipe.release();
    if (table_dev.device >= 0) (void)hipSetDevice(table_dev.device);
    table_dev.release();
    staging.release();
    results.release();
    table_pinned.release();
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  ~ThreadRes() {
    std::lock_guard<std::mutex> lk(g_tr_mu);
    if (registered) {
      g_tr.erase(std::find(g_tr.begin(), g_tr.end(), this));
      release();
    }
  }
  hipStream_t stream(int device) {
    if (device < 0 || device >= kMaxDevices) return nullptr;
    enroll();
    if (!st[device]) {
      int prev = -1;
      (void)hipGetDevice(&prev);
      if (prev != device) (void)hipSetDevice(device);
      if (hipStreamCreateWithFlags(&st[device], hipStreamNonBlocking) != hipSuccess) st[device] = nullptr;
      if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    }
    return st[device];
  }
};
thread_local ThreadRes t_res;

hipStream_t thread_stream(int device) { return t_res.stream(device); }

// The end of a synchronous host-resident call: wait for `st` (on `device`).
// hipStreamSynchronize (and, on this runtime, hipEventSynchronize of a
// blocking-sync event too: measured, profiles/r06/host_cpu_probe.jsonl) spins
// the calling core for the whole call -- the host CPU the GPU path is meant
// to give back (host CPU-seconds per GiB).  A call moving
// at least kBlockingWaitBytes sleeps instead: until `t0` (the call's start)
// + the least time its bytes need on the link (bytes / kSleepBytesPerSec;
// PCIe Gen5 x16 moves ~53 GB/s here, so this never oversleeps the transfer),
// then polls the stream's event every kPollUs.  Short calls keep the spin (their latency is
// the shims' per-call cost).
constexpr uint64_t kBlockingWaitBytes = 4ull << 20;
constexpr double kSleepBytesPerSec = 64e9;
constexpr int kPollUs = 20;
using Clock = std::chrono::steady_clock;
// The results of a host entry land here (pinned): a D2H into the caller's
// pageable `out` would have the runtime wait for the stream inside the copy
// call -- spinning the calling core for the whole call (measured,
// tools/host_cpu_probe.py: ~1 core per call, profiles/r06/host_cpu_probe.jsonl).
uint32_t* pinned_results(uint64_t n) { return static_cast<uint32_t*>(t_res.results.get(std::max<uint64_t>(n, 1) * 4)); }
hipError_t wait_host_call(int device, hipStream_t st, uint64_t bytes, Clock::time_point t0) {
  if (bytes >= kBlockingWaitBytes && device >= 0 && device < kMaxDevices) {
    hipEvent_t& e = t_res.wait_ev[device];
    if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
    if (e && hipEventRecord(e, st) == hipSuccess) {
      std::this_thread::sleep_until(t0 + std::chrono::microseconds((int64_t)((double)bytes / kSleepBytesPerSec * 1e6)));
      for (;;) {
        const hipError_t q = hipEventQuery(e);
        if (q != hipErrorNotReady) return q;
        std::this_thread::sleep_for(std::chrono::microseconds(kPollUs));
      }
    }
    (void)hipGetLastError();
  }
  return hipStreamSynchronize(st);
}

}  // namespace

void* thread_table_device(int device, size_t bytes) {
  t_res.enroll();
  return t_res.table_dev.get(device, bytes);
}

void* thread_table_pinned(size_t bytes) {
  t_res.enroll();
  return t_res.table_pinned.get(bytes);
}

bool thread_table_aux(int device, hipStream_t* side, hipEvent_t* ev_a, hipEvent_t* ev_b) {
  if (device < 0 || device >= kMaxDevices) return false;
  *side = t_res.stream(device);  // enrolls
  hipEvent_t* e = t_res.table_ev[device];
  if (!e[0] || !e[1]) {
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (prev != device) (void)hipSetDevice(device);
    for (int k = 0; k < 2; ++k)
      if (!e[k] && hipEventCreateWithFlags(&e[k], hipEventDisableTiming) != hipSuccess) e[k] = nullptr;
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
  }
  *ev_a = e[0];
  *ev_b = e[1];
  return *side && e[0] && e[1];
}

}  // namespace nvl

using namespace nvl;

extern "C" {

int nvl_crc32c_abi_version(void) { return NVL_CRC32C_ABI_VERSION; }

const char* nvl_crc32c_strerror(int status) {
  switch (status) {
    case NVL_CRC32C_OK: return "ok";
    case NVL_CRC32C_EINVAL: return "invalid argument";
    case NVL_CRC32C_EHIP: return "HIP runtime error";
    case NVL_CRC32C_ENODEV: return "no HIP device";
    case NVL_CRC32C_ESELFTEST: return "GPU CRC32C backend failed its known-answer self-test";
    case NVL_CRC32C_ENOSPC: return "workspace too small";
    default: return "unknown status";
  }
}

int nvl_crc32c_init(int device) {
  int rc = NVL_CRC32C_OK;
  state_for(device, &rc);
  return rc;
}

int nvl_crc32c_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_generation.fetch_add(1, std::memory_order_acq_rel);
  {  // every thread's streams, staging and slabs (threads re-create them on their next call)
    std::lock_guard<std::mutex> tk(g_tr_mu);
    for (ThreadRes* r : g_tr) {
      r->release();
      r->registered = false;
    }
    g_tr.clear();
  }
  for (int d = 0; d < kMaxDevices; ++d) {
    DeviceState* s = g_state[d].exchange(nullptr);
    if (s) {
      if (s->tables) {
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(d);
        (void)hipFree(s->tables);
        for (auto& kv : s->counters) (void)hipFree(kv.second);
        if (prev >= 0) (void)hipSetDevice(prev);
      }
      delete s;
    }
  }
  return NVL_CRC32C_OK;
}

int nvl_crc32c_gpu_accelerated(void) {
  int rc = NVL_CRC32C_OK;
  return current_state(&rc) != nullptr ? 1 : 0;
}

uint32_t nvl_crc32c_extend(uint32_t init_crc, const void* data, size_t n) {
  return host_extend(init_crc, data, n);
}

uint32_t nvl_crc32c_value(const void* data, size_t n) { return host_extend(0, data, n); }

const char* nvl_crc32c_host_impl(void) { return host_impl_name(); }

uint32_t nvl_crc32c_mask(uint32_t crc) { return nvl::mask(crc); }

uint32_t nvl_crc32c_unmask(uint32_t masked_crc) { return nvl::unmask(masked_crc); }

size_t nvl_crc32c_fixed_workspace_bytes(uint64_t stride, uint64_t len, uint64_t n) {
  (void)stride;
  int rc = NVL_CRC32C_OK;
  DeviceState* s = current_state(&rc);
  return fixed_ws_bytes(len, n, s ? s->num_cu : 256);
}

size_t nvl_crc32c_batch_workspace_bytes(uint64_t n) {
  int rc = NVL_CRC32C_OK;
  DeviceState* s = current_state(&rc);
  return batch_ws(n, s ? s->num_cu : 256, route_cap_chunks(n)).total;
}

int nvl_crc32c_fixed_dev(const void* base, uint64_t stride, uint64_t len, uint64_t n, const uint32_t* init,
                         uint32_t init_all, uint32_t* out, uint32_t flags, void* workspace, size_t workspace_bytes,
                         void* stream) {
  int dev = -1;
  int rc = stream_device(static_cast<hipStream_t>(stream), &dev);
  if (rc != NVL_CRC32C_OK) return rc;
  DeviceState* s = state_for(dev, &rc);
  if (!s) return rc;
  return do_fixed(s, base, stride, len, n, init, init_all, out, flags, workspace, workspace_bytes,
                  static_cast<hipStream_t>(stream));
}

int nvl_crc32c_fixed_dev_timed(const void* base, uint64_t stride, uint64_t len, uint64_t n, const uint32_t* init,
                               uint32_t init_all, uint32_t* out, uint32_t flags, void* workspace,
                               size_t workspace_bytes, void* stream, void* start_event, void* stop_event) {
  int dev = -1;
  int rc = stream_device(static_cast<hipStream_t>(stream), &dev);
  if (rc != NVL_CRC32C_OK) return rc;
  DeviceState* s = state_for(dev, &rc);
  if (!s) return rc;
  return do_fixed(s, base, stride, len, n, init, init_all, out, flags, workspace, workspace_bytes,
                  static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(start_event),
                  static_cast<hipEvent_t>(stop_event));
}

int nvl_crc32c_batch_dev(const void* base, const uint64_t* offsets, const uint64_t* lengths, const uint32_t* init,
                         uint32_t init_all, uint32_t* out, uint64_t n, uint32_t flags, void* workspace,
                         size_t workspace_bytes, void* stream) {
  int dev = -1;
  int rc = stream_device(static_cast<hipStream_t>(stream), &dev);
  if (rc != NVL_CRC32C_OK) return rc;
  DeviceState* s = state_for(dev, &rc);
  if (!s) return rc;
  return do_batch(s, base, offsets, lengths, init, init_all, out, n, flags, workspace, workspace_bytes,
                  static_cast<hipStream_t>(stream), UINT64_MAX, /*routed=*/true);
}

size_t nvl_crc32c_region_workspace_bytes(uint64_t region_len, uint64_t n) {
  int rc = NVL_CRC32C_OK;
  DeviceState* s = current_state(&rc);
  return region_checked_ws_bytes(region_len, n, s ? s->num_cu : 256);
}

int nvl_crc32c_region_dev(const void* region, uint64_t region_len, const uint64_t* offsets, const uint64_t* lengths,
                          const uint32_t* init, uint32_t init_all, uint32_t* out, uint64_t n, uint32_t flags,
                          void* workspace, size_t workspace_bytes, void* stream) {
  int dev = -1;
  int rc = stream_device(static_cast<hipStream_t>(stream), &dev);
  if (rc != NVL_CRC32C_OK) return rc;
  DeviceState* s = state_for(dev, &rc);
  if (!s) return rc;
  return do_region(s, region, region_len, offsets, lengths, init, init_all, out, n, flags & NVL_CRC32C_FLAG_MASK,
                   workspace, workspace_bytes, static_cast<hipStream_t>(stream), nullptr, nullptr,
                   !(flags & NVL_CRC32C_FLAG_REGION_SHAPED));
}

int nvl_crc32c_region_dev_timed(const void* region, uint64_t region_len, const uint64_t* offsets,
                                const uint64_t* lengths, const uint32_t* init, uint32_t init_all, uint32_t* out,
                                uint64_t n, uint32_t flags, void* workspace, size_t workspace_bytes, void* stream,
                                void* start_event, void* stop_event) {
  int dev = -1;
  int rc = stream_device(static_cast<hipStream_t>(stream), &dev);
  if (rc != NVL_CRC32C_OK) return rc;
  DeviceState* s = state_for(dev, &rc);
  if (!s) return rc;
  return do_region(s, region, region_len, offsets, lengths, init, init_all, out, n, flags & NVL_CRC32C_FLAG_MASK,
                   workspace, workspace_bytes, static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(start_event),
                   static_cast<hipEvent_t>(stop_event), !(flags & NVL_CRC32C_FLAG_REGION_SHAPED));
}

int nvl_crc32c_batch_host(const void* const* ptrs, const uint64_t* lengths, const uint32_t* init,
                          uint32_t init_all, uint32_t* out, uint64_t n, uint32_t flags) {
  const auto t_call = Clock::now();
  if (n == 0) return NVL_CRC32C_OK;
  if (!ptrs || !lengths || !out) return NVL_CRC32C_EINVAL;
  int rc = NVL_CRC32C_OK;
  DeviceState* s = current_state(&rc);
  if (!s) return rc;
  // host layout: [data (16-B aligned per buffer)] [offsets n] [lengths n] [init n]
  uint64_t data_bytes = 0, max_len = 0;  // (the lengths are on the host: a bound for the plan)
  for (uint64_t i = 0; i < n; ++i) {
    if (!ptrs[i] && lengths[i]) return NVL_CRC32C_EINVAL;
    data_bytes += align_up(lengths[i], 16);
    max_len = std::max(max_len, lengths[i]);
  }
  const size_t meta_off = align_up(data_bytes, 256);
  const size_t total = meta_off + n * 8 * 2 + n * 4 + 256;
  uint8_t* hst = static_cast<uint8_t*>(t_res.staging.get(total));
  if (!hst) return NVL_CRC32C_EHIP;
  uint64_t* hoff = reinterpret_cast<uint64_t*>(hst + meta_off);
  uint64_t* hlen = hoff + n;
  uint32_t* hini = reinterpret_cast<uint32_t*>(hlen + n);
  uint64_t pos = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (lengths[i]) memcpy(hst + pos, ptrs[i], lengths[i]);
    hoff[i] = pos;
    hlen[i] = lengths[i];
    hini[i] = init ? init[i] : init_all;
    pos += align_up(lengths[i], 16);
  }
  hipStream_t st = thread_stream(s->device);
  if (!st) return NVL_CRC32C_EHIP;
  uint8_t* d = nullptr;
  const size_t ws = batch_ws(n, s->num_cu, 0).total;
  const size_t dbytes = total + n * 4 + ws + 512;
  if (hipMallocAsync(&d, dbytes, st) != hipSuccess) return NVL_CRC32C_EHIP;
  uint32_t* dout = reinterpret_cast<uint32_t*>(d + align_up(total, 256));
  void* dws = d + align_up(total, 256) + align_up(n * 4, 256);
  hipError_t e = hipMemcpyAsync(d, hst, total, hipMemcpyHostToDevice, st);
  if (e == hipSuccess)
    rc = do_batch(s, d, reinterpret_cast<uint64_t*>(d + meta_off), reinterpret_cast<uint64_t*>(d + meta_off) + n,
                  reinterpret_cast<uint32_t*>(d + meta_off + n * 16), 0, dout, n, flags, dws, ws, st, max_len);
  else
    rc = NVL_CRC32C_EHIP;
  uint32_t* hres = pinned_results(n);
  if (!hres && rc == NVL_CRC32C_OK) rc = NVL_CRC32C_EHIP;
  if (rc == NVL_CRC32C_OK) rc = hip_rc(hipMemcpyAsync(hres, dout, n * 4, hipMemcpyDeviceToHost, st));
  (void)hipFreeAsync(d, st);
  if (wait_host_call(s->device, st, data_bytes, t_call) != hipSuccess && rc == NVL_CRC32C_OK) rc = NVL_CRC32C_EHIP;
  if (rc == NVL_CRC32C_OK) memcpy(out, hres, n * 4);
  return rc;
}

// Copy src[0, bytes) to dst (device) through the pinned staging buffer hst,
// slice by slice: workers fill hst slices in order while this thread queues
// each finished slice's H2D on st.  Returns the first HIP error.
static hipError_t stage_h2d(uint8_t* dst, uint8_t* hst, const uint8_t* src, uint64_t bytes, hipStream_t st) {
  constexpr uint64_t kSlice = 8ull << 20;
  const uint64_t ns = (bytes + kSlice - 1) / kSlice;
  if (ns <= 1) {
    memcpy(hst, src, bytes);
    return bytes ? hipMemcpyAsync(dst, hst, bytes, hipMemcpyHostToDevice, st) : hipSuccess;
  }
  const unsigned nw = bytes >= (64ull << 20) ? 4u : 1u;
  std::vector<std::atomic<uint8_t>> done(ns);
  for (auto& f : done) f.store(0, std::memory_order_relaxed);
  std::atomic<uint64_t> next{0};
  auto work = [&] {
    for (uint64_t k; (k = next.fetch_add(1, std::memory_order_relaxed)) < ns;) {
      const uint64_t o = k * kSlice, m = std::min(kSlice, bytes - o);
      memcpy(hst + o, src + o, m);
      done[k].store(1, std::memory_order_release);
    }
  };
  std::vector<std::thread> th;
  for (unsigned w = 0; w < nw; ++w) th.emplace_back(work);
  hipError_t e = hipSuccess;
  for (uint64_t k = 0; k < ns; ++k) {
    while (!done[k].load(std::memory_order_acquire)) std::this_thread::yield();
    const uint64_t o = k * kSlice, m = std::min(kSlice, bytes - o);
    if (e == hipSuccess) e = hipMemcpyAsync(dst + o, hst + o, m, hipMemcpyHostToDevice, st);
  }
  for (auto& t : th) t.join();
  return e;
}

// ---- registered host ranges (nvl_crc32c_host_register) ---------------------
// base -> bytes of every live registration (hipHostRegister, portable |
// mapped: every device may DMA from it and map it).
namespace {
std::mutex g_reg_mu;
std::map<uintptr_t, uint64_t> g_reg;

// The registration holding [p, p + bytes), or g_reg.end(); caller holds g_reg_mu.
std::map<uintptr_t, uint64_t>::const_iterator reg_find(uintptr_t p, uint64_t bytes) {
  auto it = g_reg.upper_bound(p);
  if (it == g_reg.begin()) return g_reg.end();
  --it;
  return (p >= it->first && bytes <= it->second && p - it->first <= it->second - bytes) ? it : g_reg.end();
}
}  // namespace

int nvl_crc32c_host_register(const void* ptr, size_t bytes) {
  if (!ptr || bytes == 0 || bytes > (1ull << 50)) return NVL_CRC32C_EINVAL;
  const uintptr_t p = reinterpret_cast<uintptr_t>(ptr);
  if (p + bytes < p) return NVL_CRC32C_EINVAL;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto nx = g_reg.lower_bound(p);
  if (nx != g_reg.end() && nx->first < p + bytes) return NVL_CRC32C_EINVAL;  // overlaps a later one
  if (nx != g_reg.begin()) {
    auto pv = std::prev(nx);
    if (pv->first + pv->second > p) return NVL_CRC32C_EINVAL;  // overlaps an earlier one
  }
  int rc = NVL_CRC32C_OK;
  if (!current_state(&rc)) return rc;  // (a device and its runtime first: no GPU -> ENODEV)
  if (hipHostRegister(const_cast<void*>(ptr), bytes, hipHostRegisterPortable | hipHostRegisterMapped) !=
      hipSuccess) {
    (void)hipGetLastError();
    return NVL_CRC32C_EHIP;
  }
  g_reg.emplace(p, (uint64_t)bytes);
  return NVL_CRC32C_OK;
}

int nvl_crc32c_host_unregister(const void* ptr) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg.find(reinterpret_cast<uintptr_t>(ptr));
  if (!ptr || it == g_reg.end()) return NVL_CRC32C_EINVAL;
  if (hipHostUnregister(const_cast<void*>(ptr)) != hipSuccess) {  // (still registered: the entry stays)
    (void)hipGetLastError();
    return NVL_CRC32C_EHIP;
  }
  g_reg.erase(it);
  return NVL_CRC32C_OK;
}

int nvl_crc32c_host_registered(const void* ptr, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  return ptr && reg_find(reinterpret_cast<uintptr_t>(ptr), bytes) != g_reg.end() ? 1 : 0;
}

int nvl_crc32c_batch_region_host(const void* region, uint64_t region_len, const uint64_t* offsets,
                                 const uint64_t* lengths, const uint32_t* init, uint32_t init_all, uint32_t* out,
                                 uint64_t n, uint32_t flags) {
  const auto t_call = Clock::now();
  if (n == 0) return NVL_CRC32C_OK;
  if (!offsets || !lengths || !out || (!region && region_len)) return NVL_CRC32C_EINVAL;
  if (flags & ~(NVL_CRC32C_FLAG_MASK | NVL_CRC32C_FLAG_HOST_ZERO_COPY)) return NVL_CRC32C_EINVAL;
  uint64_t lo = UINT64_MAX, hi = 0, max_len = 0;  // staged window [lo, hi)
  for (uint64_t i = 0; i < n; ++i) {
    if (lengths[i] > region_len || offsets[i] > region_len - lengths[i]) return NVL_CRC32C_EINVAL;
    if (offsets[i] < lo) lo = offsets[i];
    if (offsets[i] + lengths[i] > hi) hi = offsets[i] + lengths[i];
    max_len = std::max(max_len, lengths[i]);
  }
  const uint64_t wbytes = hi - lo;
  const uint8_t* src = static_cast<const uint8_t*>(region) + lo;
  // A window inside one registration (nvl_crc32c_host_register): DMA from the
  // caller's pages (no staging copy), or with ZERO_COPY no copy at all.
  const bool reg = nvl_crc32c_host_registered(src, wbytes) == 1;
  const bool zero_copy = (flags & NVL_CRC32C_FLAG_HOST_ZERO_COPY) != 0;
  if (zero_copy && !reg) return NVL_CRC32C_EINVAL;
  flags &= NVL_CRC32C_FLAG_MASK;
  int rc = NVL_CRC32C_OK;
  DeviceState* s = current_state(&rc);
  if (!s) return rc;
  const uint8_t* dsrc = nullptr;  // the kernels' view of the window (zero copy)
  if (zero_copy) {
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, const_cast<uint8_t*>(src), 0) != hipSuccess || !dp) {
      (void)hipGetLastError();
      return NVL_CRC32C_EHIP;
    }
    dsrc = static_cast<const uint8_t*>(dp);
    // The kernels read whole 4 KiB pages of the window (the region grid from
    // the page below its start; the batch kernels within the buffers' own
    // pages): safe only if the device view keeps the host page offsets, so
    // that every page read holds a registered byte.
    if (((uintptr_t)dsrc & 4095u) != ((uintptr_t)src & 4095u)) return NVL_CRC32C_EHIP;
  }
  // host layout: [window bytes (staged calls only)] [offsets n (rebased to the window)] [lengths n] [init n]
  const size_t meta_off = reg ? 0 : align_up(wbytes, 256);
  const size_t total = meta_off + n * 8 * 2 + n * 4 + 256;
  uint8_t* hst = static_cast<uint8_t*>(t_res.staging.get(total));
  if (!hst) return NVL_CRC32C_EHIP;
  hipStream_t st = thread_stream(s->device);
  if (!st) return NVL_CRC32C_EHIP;
  uint8_t* d = nullptr;
  // region-shaped (checked here, on the host): the region kernel alone;
  // otherwise the batch path with the host's bound on the lengths
  const bool as_region = max_len <= kRegionMaxLen && region_sorted(offsets, lengths, n);
  const size_t ws = as_region ? region_ws_bytes(wbytes, n) : batch_ws(n, s->num_cu, 0).total;
  // device layout: [window (not for zero copy)] [metadata] [out] [workspace]
  const size_t win_dev = zero_copy ? 0 : align_up(wbytes, 256);
  const size_t dbytes = win_dev + align_up(total - meta_off, 256) + align_up(n * 4, 256) + ws + 256;
  if (hipMallocAsync(&d, dbytes, st) != hipSuccess) return NVL_CRC32C_EHIP;
  uint8_t* dmeta = d + win_dev;
  uint32_t* dout = reinterpret_cast<uint32_t*>(dmeta + align_up(total - meta_off, 256));
  void* dws = reinterpret_cast<uint8_t*>(dout) + align_up(n * 4, 256);
  const uint8_t* dwin = zero_copy ? dsrc : d;
  hipError_t e = hipSuccess;
  if (reg && !zero_copy && wbytes) {
    e = hipMemcpyAsync(d, src, wbytes, hipMemcpyHostToDevice, st);  // DMA from the registered pages
  } else if (!reg) {
    // The window goes to the GPU in slices: the staging copy of slice k+1 (a
    // few host threads for large windows) overlaps the H2D DMA of slice k, so
    // the call costs max(copy, PCIe) instead of their sum.
    e = stage_h2d(d, hst, src, wbytes, st);
  }
  uint64_t* hoff = reinterpret_cast<uint64_t*>(hst + meta_off);
  uint64_t* hlen = hoff + n;
  uint32_t* hini = reinterpret_cast<uint32_t*>(hlen + n);
  for (uint64_t i = 0; i < n; ++i) {
    hoff[i] = offsets[i] - lo;
    hlen[i] = lengths[i];
    hini[i] = init ? init[i] : init_all;
  }
  if (e == hipSuccess) e = hipMemcpyAsync(dmeta, hst + meta_off, total - meta_off, hipMemcpyHostToDevice, st);
  if (e == hipSuccess && as_region)
    rc = do_region(s, dwin, wbytes, reinterpret_cast<uint64_t*>(dmeta), reinterpret_cast<uint64_t*>(dmeta) + n,
                   reinterpret_cast<uint32_t*>(dmeta + n * 16), 0, dout, n, flags, dws, ws, st, nullptr, nullptr,
                   /*checked=*/false);
  else if (e == hipSuccess)
    rc = do_batch(s, dwin, reinterpret_cast<uint64_t*>(dmeta), reinterpret_cast<uint64_t*>(dmeta) + n,
                  reinterpret_cast<uint32_t*>(dmeta + n * 16), 0, dout, n, flags, dws, ws, st, max_len);
  else
    rc = NVL_CRC32C_EHIP;
  uint32_t* hres = pinned_results(n);
  if (!hres && rc == NVL_CRC32C_OK) rc = NVL_CRC32C_EHIP;
  if (rc == NVL_CRC32C_OK) rc = hip_rc(hipMemcpyAsync(hres, dout, n * 4, hipMemcpyDeviceToHost, st));
  (void)hipFreeAsync(d, st);
  if (wait_host_call(s->device, st, wbytes, t_call) != hipSuccess && rc == NVL_CRC32C_OK) rc = NVL_CRC32C_EHIP;
  if (rc == NVL_CRC32C_OK) memcpy(out, hres, n * 4);
  return rc;
}

// ---- several devices, host-resident ----------------------------------------
// nvl_crc32c_batch_region_host_multi: the batch in contiguous index ranges of
// about equal covered bytes, one per device, each staged and checksummed by
// nvl_crc32c_batch_region_host on its device from its own thread (its own
// pinned staging, stream and PCIe link), results straight into out.  Part 0
// runs on the calling thread; the others on a pool of persistent worker
// threads (their staging survives between calls).  Multi calls are
// serialised on the pool.

int nvl_crc32c_multi_plan(const uint64_t* offsets, const uint64_t* lengths, uint64_t n, int ndev,
                          uint64_t min_bytes, uint64_t* part_first) {
  if (!offsets || !lengths || !part_first || ndev <= 0) return NVL_CRC32C_EINVAL;
  if (min_bytes == 0) min_bytes = NVL_CRC32C_MULTI_MIN_BYTES;
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) total += lengths[i];
  uint64_t parts = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)ndev, total / min_bytes));
  if (parts > n) parts = std::max<uint64_t>(1, n);
  // cut where the running byte count crosses k * total / parts
  part_first[0] = 0;
  uint64_t k = 1, acc = 0;
  for (uint64_t i = 0; i < n && k < parts; ++i) {
    acc += lengths[i];
    while (k < parts && acc >= (total / parts) * k && i + 1 < n) part_first[k++] = i + 1;
  }
  while (k < parts) part_first[k++] = n;  // (degenerate: fewer cuts than parts)
  part_first[parts] = n;
  return (int)parts;
}

namespace {
struct MultiPool {
  struct Worker {
    std::mutex m;
    std::condition_variable cv;
    std::function<void()> job;
    bool busy = false;
  };
  std::mutex call_mu;  // one multi call at a time
  std::mutex mu;
  std::vector<Worker*> workers;
  Worker* get(size_t k) {
    std::lock_guard<std::mutex> lk(mu);
    while (workers.size() <= k) {
      Worker* w = new Worker;
      std::thread([w] {
        for (;;) {
          std::function<void()> j;
          {
            std::unique_lock<std::mutex> lk2(w->m);
            w->cv.wait(lk2, [w] { return w->busy && w->job; });
            j = std::move(w->job);
            w->job = nullptr;
          }
          j();
          {
            std::lock_guard<std::mutex> lk2(w->m);
            w->busy = false;
          }
          w->cv.notify_all();
        }
      }).detach();  // (idle at exit; never joined: the HIP runtime may already be gone)
      workers.push_back(w);
    }
    return workers[k];
  }
  void run(Worker* w, std::function<void()> j) {
    std::lock_guard<std::mutex> lk(w->m);
    w->job = std::move(j);
    w->busy = true;
    w->cv.notify_all();
  }
  void wait(Worker* w) {
    std::unique_lock<std::mutex> lk(w->m);
    w->cv.wait(lk, [w] { return !w->busy; });
  }
};
MultiPool& multi_pool() {
  static MultiPool* p = new MultiPool;  // (leaked on purpose: detached workers hold it)
  return *p;
}
}  // namespace

int nvl_crc32c_batch_region_host_multi(const void* region, uint64_t region_len, const uint64_t* offsets,
                                       const uint64_t* lengths, const uint32_t* init, uint32_t init_all,
                                       uint32_t* out, uint64_t n, uint32_t flags, const int* devices, int ndev,
                                       uint64_t min_bytes_per_device) {
  if (n == 0) return NVL_CRC32C_OK;
  if (!devices || ndev <= 0 || ndev > 64) return NVL_CRC32C_EINVAL;
  if (!offsets || !lengths || !out || (!region && region_len)) return NVL_CRC32C_EINVAL;
  std::vector<uint64_t> first((size_t)ndev + 1);
  const int parts = nvl_crc32c_multi_plan(offsets, lengths, n, ndev, min_bytes_per_device, first.data());
  if (parts < 0) return parts;
  int prev = -1;
  (void)hipGetDevice(&prev);
  auto part = [&](int k) -> int {
    if (hipSetDevice(devices[k]) != hipSuccess) return NVL_CRC32C_ENODEV;
    const uint64_t a = first[k], b = first[k + 1];
    return nvl_crc32c_batch_region_host(region, region_len, offsets + a, lengths + a, init ? init + a : nullptr,
                                        init_all, out + a, b - a, flags);
  };
  if (parts == 1) {
    const int rc = part(0);
    if (prev >= 0) (void)hipSetDevice(prev);
    return rc;
  }
  MultiPool& pool = multi_pool();
  std::lock_guard<std::mutex> call(pool.call_mu);
  std::vector<int> rc((size_t)parts, NVL_CRC32C_OK);
  std::vector<MultiPool::Worker*> ws((size_t)parts, nullptr);
  for (int k = 1; k < parts; ++k) {
    ws[k] = pool.get((size_t)k - 1);
    pool.run(ws[k], [&, k] { rc[k] = part(k); });
  }
  rc[0] = part(0);
  for (int k = 1; k < parts; ++k) pool.wait(ws[k]);
  if (prev >= 0) (void)hipSetDevice(prev);
  for (int k = 0; k < parts; ++k)
    if (rc[k] != NVL_CRC32C_OK) return rc[k];
  return NVL_CRC32C_OK;
}

// ---- several devices, device-resident ---------------------------------------

// The stream a shard runs on (NULL: its device's null stream), checked to
// belong to the shard's device.
static int shard_stream(const nvl_crc32c_shard& sh, hipStream_t* st) {
  *st = static_cast<hipStream_t>(sh.stream);
  if (*st) {
    int d = -1;
    if (stream_device(*st, &d) != NVL_CRC32C_OK || d != sh.device) return NVL_CRC32C_EINVAL;
  }
  return NVL_CRC32C_OK;
}

int nvl_crc32c_fixed_dev_multi(const nvl_crc32c_shard* shards, int nshards, uint32_t init_all, uint32_t flags) {
  if (!shards || nshards <= 0 || nshards > 4096) return NVL_CRC32C_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    (void)hipGetLastError();
    ndev = 0;
  }
  for (int k = 0; k < nshards; ++k) {  // every argument first: nothing is enqueued for a bad call
    const nvl_crc32c_shard& sh = shards[k];
    if (sh.device < 0 || sh.n > (1ull << 40)) return NVL_CRC32C_EINVAL;
    if (sh.n && (!sh.out || (!sh.base && sh.len))) return NVL_CRC32C_EINVAL;
    if (sh.device >= ndev) return NVL_CRC32C_ENODEV;
  }
  int prev = -1;
  (void)hipGetDevice(&prev);
  int rc = NVL_CRC32C_OK;
  for (int k = 0; k < nshards && rc == NVL_CRC32C_OK; ++k) {
    const nvl_crc32c_shard& sh = shards[k];
    if (sh.n == 0) continue;
    DeviceState* s = state_for(sh.device, &rc);
    if (!s) break;
    hipStream_t st = nullptr;
    if ((rc = shard_stream(sh, &st)) != NVL_CRC32C_OK) break;
    if (hipSetDevice(sh.device) != hipSuccess) {
      rc = NVL_CRC32C_ENODEV;
      break;
    }
    rc = do_fixed(s, sh.base, sh.stride, sh.len, sh.n, nullptr, init_all, sh.out, flags, nullptr, 0, st);
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  return rc;
}

// `st` (on dst_device, current) waits for the work enqueued so far on the
// shard's stream, unless that is `st` itself.
static hipError_t after_shard(const nvl_crc32c_shard& sh, int dst_device, hipStream_t st) {
  hipStream_t ss = nullptr;
  if (shard_stream(sh, &ss) != NVL_CRC32C_OK) return hipErrorInvalidValue;
  if (ss == st && sh.device == dst_device) return hipSuccess;
  hipError_t e;
  hipEvent_t ev = nullptr;
  if ((e = hipSetDevice(sh.device)) == hipSuccess &&
      (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) == hipSuccess &&
      (e = hipEventRecord(ev, ss)) == hipSuccess && (e = hipSetDevice(dst_device)) == hipSuccess)
    e = hipStreamWaitEvent(st, ev, 0);
  if (ev) (void)hipEventDestroy(ev);  // (released once the recorded work is done)
  (void)hipSetDevice(dst_device);
  return e;
}

// Whether kernels on `dev` may read memory of `peer` (peer access enabled
// once per pair, process-wide; a pair that cannot gathers by peer copies).
static bool peer_mapped(int dev, int peer) {
  if (dev < 0 || peer < 0 || dev >= kMaxDevices || peer >= kMaxDevices) return false;
  static std::atomic<int8_t> s_state[kMaxDevices][kMaxDevices];  // 0 unknown, 1 mapped, -1 not
  std::atomic<int8_t>& s = s_state[dev][peer];
  int8_t v = s.load(std::memory_order_acquire);
  if (v) return v > 0;
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  if ((v = s.load(std::memory_order_relaxed))) return v > 0;
  int can = 0;
  bool ok = hipDeviceCanAccessPeer(&can, dev, peer) == hipSuccess && can;
  if (ok) {
    int cur = -1;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(dev);
    const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    ok = e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled;
    if (cur >= 0) (void)hipSetDevice(cur);
  }
  (void)hipGetLastError();
  s.store(ok ? 1 : -1, std::memory_order_release);
  return ok;
}

int nvl_crc32c_gather_dev(uint32_t* dst, int dst_device, const nvl_crc32c_shard* shards, int nshards,
                          uint32_t layout, void* stream) {
  if (!dst || !shards || nshards <= 0 || nshards > 4096 || layout > NVL_CRC32C_GATHER_ROUND_ROBIN)
    return NVL_CRC32C_EINVAL;
  uint64_t N = 0;
  for (int k = 0; k < nshards; ++k) {
    if (shards[k].n && !shards[k].out) return NVL_CRC32C_EINVAL;
    N += shards[k].n;
  }
  if (layout == NVL_CRC32C_GATHER_ROUND_ROBIN)
    for (int k = 0; k < nshards; ++k)
      if (shards[k].n != (N > (uint64_t)k ? (N - (uint64_t)k + nshards - 1) / (uint64_t)nshards : 0))
        return NVL_CRC32C_EINVAL;
  int rc = NVL_CRC32C_OK;
  if (!state_for(dst_device, &rc)) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);  // (NULL: dst_device's null stream)
  if (st) {
    int d = -1;
    if (stream_device(st, &d) != NVL_CRC32C_OK || d != dst_device) return NVL_CRC32C_EINVAL;
  }
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(dst_device) != hipSuccess) return NVL_CRC32C_ENODEV;
  // One launch when every shard's results are on dst_device or peer-mapped
  // to it (up to kGatherMax shards): the kernel reads each result where its
  // shard wrote it (over xGMI for a peer) after the shards' streams.
  bool direct = nshards <= (int)dev::kGatherMax;
  for (int k = 0; k < nshards && direct; ++k)
    if (shards[k].n && shards[k].device != dst_device) direct = peer_mapped(dst_device, shards[k].device);
  if (direct) {
    dev::GatherSrc gs{};
    gs.G = (uint32_t)nshards;
    gs.rr = layout == NVL_CRC32C_GATHER_ROUND_ROBIN ? 1u : 0u;
    uint64_t pos = 0;
    hipError_t e = hipSuccess;
    for (int k = 0; k < nshards && e == hipSuccess; ++k) {
      const nvl_crc32c_shard& sh = shards[k];
      gs.src[k] = sh.out;
      gs.pos[k] = pos;
      pos += sh.n;
      if (sh.n) e = after_shard(sh, dst_device, st);
    }
    gs.pos[nshards] = pos;
    if (e == hipSuccess) e = launch_gather(gs, N, dst, st);
    if (prev >= 0) (void)hipSetDevice(prev);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return NVL_CRC32C_EHIP;
    }
    return NVL_CRC32C_OK;
  }
  uint32_t* tmp = nullptr;
  const bool rr = layout == NVL_CRC32C_GATHER_ROUND_ROBIN && nshards > 1;
  hipError_t e = rr ? hipMallocAsync(reinterpret_cast<void**>(&tmp), std::max<uint64_t>(N, 1) * 4, st) : hipSuccess;
  uint32_t* to = rr ? tmp : dst;
  uint64_t pos = 0;
  for (int k = 0; k < nshards && e == hipSuccess; ++k) {
    const nvl_crc32c_shard& sh = shards[k];
    if (sh.n) {
      // after the shard's own stream (its results), then the copy: a peer
      // copy over xGMI for another device, a device copy for the same one
      e = after_shard(sh, dst_device, st);
      if (e == hipSuccess)
        e = sh.device == dst_device
                ? hipMemcpyAsync(to + pos, sh.out, sh.n * 4, hipMemcpyDeviceToDevice, st)
                : hipMemcpyPeerAsync(to + pos, dst_device, sh.out, sh.device, sh.n * 4, st);
    }
    pos += sh.n;
  }
  if (e == hipSuccess && rr) e = launch_interleave_rr(tmp, N, (uint32_t)nshards, dst, st);
  if (tmp) (void)hipFreeAsync(tmp, st);
  if (prev >= 0) (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return NVL_CRC32C_EHIP;
  }
  return NVL_CRC32C_OK;
}

int nvl_crc32c_fixed_host(const void* base, uint64_t stride, uint64_t len, uint64_t n, const uint32_t* init,
                          uint32_t init_all, uint32_t* out, uint32_t flags) {
  const auto t_call = Clock::now();
  if (n == 0) return NVL_CRC32C_OK;
  if (!base || !out) return NVL_CRC32C_EINVAL;
  int rc = NVL_CRC32C_OK;
  DeviceState* s = current_state(&rc);
  if (!s) return rc;
  // Slabs of whole buffers, ~64 MiB each, double-buffered over two streams:
  // H2D(k+1) overlaps kernel(k) and D2H(k-1).
  const uint64_t span = stride;  // bytes between buffer starts
  uint64_t per = span ? std::max<uint64_t>(1, (64ull << 20) / std::max<uint64_t>(span, 1)) : n;
  per = std::min<uint64_t>(per, n);
  const uint64_t slab_bytes = (per - 1) * stride + len;
  const size_t ws = fixed_ws_bytes(len, per, s->num_cu);
  if (!t_res.pipe.get(s->device, align_up(slab_bytes, 256) + per * 8 + ws + 512)) {
    t_res.pipe.release();
    return NVL_CRC32C_EHIP;
  }
  hipStream_t* st = t_res.pipe.st;
  uint8_t* dbuf[2] = {t_res.pipe.buf[0], t_res.pipe.buf[1]};
  uint32_t* dout[2] = {nullptr, nullptr};
  uint32_t* dini[2] = {nullptr, nullptr};
  void* dws[2] = {nullptr, nullptr};
  for (int k = 0; k < 2; ++k) {
    dout[k] = reinterpret_cast<uint32_t*>(dbuf[k] + align_up(slab_bytes, 256));
    dini[k] = dout[k] + per;
    dws[k] = reinterpret_cast<uint8_t*>(dini[k] + per) + 256 - ((uintptr_t)(dini[k] + per) & 255);
  }
  const uint8_t* hb = static_cast<const uint8_t*>(base);
  uint32_t* hres = pinned_results(n);
  if (!hres) return NVL_CRC32C_EHIP;
  for (uint64_t i0 = 0, k = 0; rc == NVL_CRC32C_OK && i0 < n; i0 += per, k ^= 1) {
    const uint64_t m = std::min<uint64_t>(per, n - i0);
    const uint64_t bytes = (m - 1) * stride + len;
    hipError_t e = hipMemcpyAsync(dbuf[k], hb + i0 * stride, bytes, hipMemcpyHostToDevice, st[k]);
    if (e == hipSuccess && init) e = hipMemcpyAsync(dini[k], init + i0, m * 4, hipMemcpyHostToDevice, st[k]);
    if (e != hipSuccess) { rc = NVL_CRC32C_EHIP; break; }
    rc = do_fixed(s, dbuf[k], stride, len, m, init ? dini[k] : nullptr, init_all, dout[k], flags, dws[k], ws,
                  st[k]);
    if (rc == NVL_CRC32C_OK) rc = hip_rc(hipMemcpyAsync(hres + i0, dout[k], m * 4, hipMemcpyDeviceToHost, st[k]));
  }
  for (int k = 0; k < 2; ++k)
    if (wait_host_call(s->device, st[k], n * stride, t_call) != hipSuccess && rc == NVL_CRC32C_OK) rc = NVL_CRC32C_EHIP;
  if (rc == NVL_CRC32C_OK) memcpy(out, hres, n * 4);
  return rc;
}

int nvl_crc32c_fill_splitmix(void* dst, uint64_t nblocks, uint64_t block_bytes, uint64_t first_block,
                             uint64_t block_step, uint64_t seed, void* stream) {
  if (nblocks == 0) return NVL_CRC32C_OK;
  if (!dst || block_bytes == 0 || (block_bytes % 8) != 0) return NVL_CRC32C_EINVAL;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return NVL_CRC32C_ENODEV;
  return hip_rc(launch_fill(dst, nblocks, block_bytes, first_block, block_step, seed,
                            static_cast<hipStream_t>(stream)));
}

int nvl_crc32c_read_probe(const void* src, uint64_t bytes, uint32_t* sink, void* stream) {
  if (bytes == 0) return NVL_CRC32C_OK;
  if (!src || !sink || (bytes % 16) != 0 || (reinterpret_cast<uintptr_t>(src) % 16) != 0) return NVL_CRC32C_EINVAL;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return NVL_CRC32C_ENODEV;
  return hip_rc(launch_read_probe(src, bytes, sink, static_cast<hipStream_t>(stream)));
}

}  // extern "C"
