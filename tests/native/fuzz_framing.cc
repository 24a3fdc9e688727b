// tests/native/fuzz_framing.cc -- AddressSanitizer/UBSan fuzz driver for the
// host-side parsers of the call-site shims (nvlevelz_amd/csrc/crc32c_framing.cpp):
// nvl_sstable_verify_table (footer, index/metaindex Block::Iter walk),
// nvl_sstable_verify_blocks (handle bounds) and nvl_log_scan (log block
// parse).  Built by tests/native/Makefile with -fsanitize=address,undefined
// against the framing and host-CRC sources only; the CRCs run on the host
// (NVL_FRAMING_HOST), the GPU batch entry point is a stub that must never be
// reached.  Every image lives in a heap allocation of exactly its length, so
// any read past it is reported.  Test infrastructure (tests/test_fuzz_framing.py).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "nvl_framing.h"

extern "C" int nvl_crc32c_batch_region_host(const void*, uint64_t, const uint64_t*, const uint64_t*,
                                            const uint32_t*, uint32_t, uint32_t*, uint64_t, uint32_t) {
  fprintf(stderr, "device path reached in a host-mode fuzz run\n");
  abort();
}

namespace {

uint64_t g_rng = 0x9E3779B97F4A7C15ull;
uint64_t rnd() {  // splitmix64
  uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
uint64_t rnd(uint64_t n) { return n ? rnd() % n : 0; }

void varint(std::string* s, uint64_t v) {
  while (v >= 128) {
    s->push_back((char)((v & 127) | 128));
    v >>= 7;
  }
  s->push_back((char)v);
}
void fixed32(std::string* s, uint32_t v) {
  for (int i = 0; i < 4; ++i) s->push_back((char)(v >> (8 * i)));
}

// a block of (key, value) entries with restart interval `ri`, sealed in the image
std::pair<uint64_t, uint64_t> put_block(std::string* img, const std::vector<std::pair<std::string, std::string>>& e,
                                        int ri) {
  std::string b;
  std::vector<uint32_t> restarts;
  for (size_t i = 0; i < e.size(); ++i) {
    if (i % ri == 0) restarts.push_back((uint32_t)b.size());
    varint(&b, 0);
    varint(&b, e[i].first.size());
    varint(&b, e[i].second.size());
    b += e[i].first + e[i].second;
  }
  if (restarts.empty()) restarts.push_back(0);
  for (uint32_t r : restarts) fixed32(&b, r);
  fixed32(&b, (uint32_t)restarts.size());
  const uint64_t off = img->size();
  *img += b;
  img->push_back(0);
  fixed32(img, 0);
  nvl_block_handle h{off, b.size()};
  if (nvl_sstable_seal_trailers(&(*img)[0], img->size(), &h, 1, NVL_FRAMING_HOST) != 0) abort();
  return {off, b.size()};
}

std::pair<uint64_t, uint64_t> g_index;  // the last table's index block handle

std::string make_table() {
  std::string img;
  std::vector<std::pair<std::string, std::string>> index, meta;
  const int nb = (int)rnd(12);
  for (int i = 0; i < nb; ++i) {
    std::vector<std::pair<std::string, std::string>> d;
    for (int k = (int)rnd(5); k >= 0; --k) d.push_back({"key" + std::to_string(rnd(1000)), std::string(rnd(300), 'v')});
    auto h = put_block(&img, d, 16);
    std::string v;
    varint(&v, h.first);
    varint(&v, h.second);
    index.push_back({"k" + std::to_string(i), v});
  }
  for (int m = (int)rnd(3); m > 0; --m) {
    auto h = put_block(&img, {{"f", std::string(rnd(100), 'f')}}, 16);
    std::string v;
    varint(&v, h.first);
    varint(&v, h.second);
    meta.push_back({"filter." + std::to_string(m), v});
  }
  auto mh = put_block(&img, meta, 16);
  auto ih = put_block(&img, index, 1);
  g_index = ih;
  std::string foot;
  varint(&foot, mh.first);
  varint(&foot, mh.second);
  varint(&foot, ih.first);
  varint(&foot, ih.second);
  foot.resize(40, '\0');
  fixed32(&foot, 0x8b80fb57u);
  fixed32(&foot, 0xdb477524u);
  return img + foot;
}

void mutate(std::string* s, uint64_t tail_bias) {
  const int k = 1 + (int)rnd(6);
  for (int i = 0; i < k && !s->empty(); ++i) {
    const uint64_t n = s->size();
    const uint64_t pos = rnd(2) && tail_bias ? n - 1 - rnd(tail_bias < n ? tail_bias : n) : rnd(n);
    switch (rnd(5)) {
      case 0: (*s)[pos] ^= (char)(1u << rnd(8)); break;
      case 1: (*s)[pos] = (char)rnd(256); break;
      case 2: (*s)[pos] = (char)0xFF; break;
      case 3: s->resize(n - rnd(n < 64 ? n : 64)); break;
      default: s->append(rnd(40), (char)rnd(256)); break;
    }
  }
}

// an exact-size heap copy so ASan sees reads past the end
struct Exact {
  uint8_t* p;
  size_t n;
  explicit Exact(const std::string& s) : p((uint8_t*)malloc(s.size() ? s.size() : 1)), n(s.size()) {
    memcpy(p, s.data(), s.size());
  }
  ~Exact() { free(p); }
};

uint64_t g_status[8];  // table outcomes seen (coverage check)

void fuzz_table(int iters) {
  std::vector<nvl_table_block> out(4096);
  for (int it = 0; it < iters; ++it) {
    std::string img = make_table();
    if (rnd(2)) {
      mutate(&img, 400);
    } else if (g_index.second) {  // corrupt the index entries but keep its CRC valid: the walk must cope
      for (int k = 1 + (int)rnd(4); k > 0; --k) {
        const uint64_t pos = g_index.first + rnd(g_index.second);
        img[pos] = rnd(3) ? (char)rnd(256) : (char)(img[pos] ^ (1 << rnd(8)));
      }
      nvl_block_handle h{g_index.first, g_index.second};
      if (nvl_sstable_seal_trailers(&img[0], img.size(), &h, 1, NVL_FRAMING_HOST) != 0) abort();
    }
    Exact e(img);
    size_t n = 0;
    uint32_t st = 0;
    uint64_t bad = 0;
    int rc = nvl_sstable_verify_table(e.p, e.n, nullptr, 0, &n, &st, &bad, NVL_FRAMING_HOST);
    if (rc != 0 || st > NVL_TABLE_COMPRESSED_INDEX) abort();
    ++g_status[st];
    if (n <= out.size()) {
      rc = nvl_sstable_verify_table(e.p, e.n, out.data(), out.size(), &n, &st, &bad, NVL_FRAMING_HOST);
      if (rc != 0) abort();
      for (size_t i = 0; i < n; ++i)
        if (out[i].verdict > NVL_BLOCK_BAD_HANDLE || out[i].role > NVL_TBLOCK_DATA) abort();
    }
    // random handles, including ones that overflow offset + size
    nvl_block_handle h[4];
    uint8_t v[4];
    for (auto& x : h) x = nvl_block_handle{rnd(2) ? rnd(e.n + 8) : ~rnd(16), rnd(2) ? rnd(e.n + 8) : ~rnd(16)};
    if (nvl_sstable_verify_blocks(e.p, e.n, h, 4, v, &bad, NVL_FRAMING_HOST) != 0) abort();
  }
}

std::string make_log() {
  std::string img;
  const int nr = (int)rnd(40);
  std::vector<uint64_t> hdrs;
  for (int r = 0; r < nr; ++r) {
    uint64_t left = NVL_LOG_BLOCK_SIZE - img.size() % NVL_LOG_BLOCK_SIZE;
    if (left < NVL_LOG_HEADER_SIZE) img.append(left, '\0'), left = NVL_LOG_BLOCK_SIZE;
    uint64_t len = rnd(3) ? rnd(200) : rnd(40000);
    if (len > left - NVL_LOG_HEADER_SIZE) len = left - NVL_LOG_HEADER_SIZE;
    hdrs.push_back(img.size());
    fixed32(&img, 0);
    img.push_back((char)(len & 0xFF));
    img.push_back((char)(len >> 8));
    img.push_back((char)(1 + rnd(4)));
    img.append(len, (char)rnd(256));
  }
  if (!hdrs.empty() && nvl_log_seal(&img[0], img.size(), hdrs.data(), hdrs.size(), NVL_FRAMING_HOST) != 0) abort();
  return img;
}

void fuzz_log(int iters) {
  std::vector<nvl_log_event> ev(1 << 16);
  for (int it = 0; it < iters; ++it) {
    std::string img = make_log();
    mutate(&img, 0);
    Exact e(img);
    size_t n = 0;
    const int checksum = (int)rnd(2);
    int rc = nvl_log_scan(e.p, e.n, 0, checksum, nullptr, 0, &n, NVL_FRAMING_HOST);
    if (rc != 0 || n == 0) abort();
    rc = nvl_log_scan(e.p, e.n, 0, checksum, ev.data(), ev.size(), &n, NVL_FRAMING_HOST);
    if (rc != 0 || ev[n - 1].kind != NVL_LOG_EOF) abort();
    for (size_t i = 0; i < n; ++i)
      if (ev[i].kind == NVL_LOG_RECORD && ev[i].offset + NVL_LOG_HEADER_SIZE + ev[i].length > e.n) abort();
  }
}

}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  if (argc > 2) g_rng = strtoull(argv[2], nullptr, 0);
  fuzz_table(iters);
  fuzz_log(iters / 4);
  printf("fuzz ok: %d tables, %d logs; table outcomes", iters, iters / 4);
  for (int k = 0; k < 8; ++k) printf(" %llu", (unsigned long long)g_status[k]);
  printf("\n");
  return 0;
}
