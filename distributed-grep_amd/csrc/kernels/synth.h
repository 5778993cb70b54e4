// synth.h — deterministic synthetic log corpus, identical on
// the host and the device (the same __host__ __device__ code runs in both).
//
// The split is cut into independent 8 KiB pages; page p is filled with lines
// generated from splitmix64(seed, p, line). Every line is
//   "YYYY-MM-DDTHH:MM:SS.mmm LEVEL component_name: msg words...\n"
// with a total length (incl. '\n') uniform in [40, 200]; LEVEL is INFO 70 %,
// DEBUG 15 %, WARN 10 %, ERROR 5 %; the lowercase word "error" is planted in
// 2 % of messages and the phrase "timeout while waiting for lock" in 0.5 %.
// kind 1 additionally plants one of the seed's 1,000 keywords (a-z, 5-12
// letters, random letter case) in 1 % of messages (config 4). kind 2 is a
// long-line corpus: a page is a "boundary" page (normal log lines, as kind 0)
// with probability 1/512, else filler -- space-separated words, no '\n', the
// word "error" in 1 page of 2048 -- so lines of consecutive filler pages,
// 4 MiB long on average (geometric), alternate with a page of short lines;
// kind 3 is kind 2 whose first 1 GiB holds no boundary page (one newline-free
// line of 1 GiB plus the head of the next boundary page); kind 4 is kind 2 for
// config 4: its boundary pages are kind-1 lines and a filler page plants one
// of the seed's keywords (random case) instead of "error". Bytes are printable
// ASCII plus '\n'. Any page can be regenerated alone, so a window of a 16 GiB
// split can be checked on the CPU.
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define DG_HD __host__ __device__ __forceinline__
#else
#define DG_HD static inline
#endif

namespace dgrep {
namespace synth {

constexpr uint32_t kPage = 8192;
constexpr uint32_t kMinLine = 40, kMaxLine = 200;
constexpr int kKeywords = 1000;

DG_HD uint64_t mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct Rng {
  uint64_t s;
  DG_HD uint64_t next() { s += 0x9e3779b97f4a7c15ull; uint64_t z = s; z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull; z = (z ^ (z >> 27)) * 0x94d049bb133111ebull; return z ^ (z >> 31); }
  DG_HD uint32_t below(uint32_t n) { return uint32_t((next() >> 32) * uint64_t(n) >> 32); }
};

// keyword i of `seed` (lowercase a-z, 5..12 letters); returns its length.
// The set depends on seed % 1000 only, so the splits of a multi-GPU run
// (seed + 1000 * rank) plant the same keywords.
DG_HD int keyword(uint64_t seed, int i, char* out) {
  Rng r{mix((seed % 1000) ^ 0x6b6579776f726473ull) ^ mix(uint64_t(i) + 0x1234)};
  int len = 5 + int(r.below(8));
  for (int k = 0; k < len; ++k) out[k] = char('a' + r.below(26));
  return len;
}

// fixed vocabularies (no word contains "error")
DG_HD const char* word(uint32_t i, int* len) {
  static const char* const kWords[32] = {
      "request", "user", "cache", "miss", "hit", "latency", "ms", "session", "token", "refresh",
      "queue", "depth", "retry", "worker", "shard", "replica", "commit", "offset", "bytes", "read",
      "write", "open", "close", "handle", "ok", "done", "start", "stop", "value", "key",
      "disk", "node"};
  static const unsigned char kLen[32] = {7, 4, 5, 4, 3, 7, 2, 7, 5, 7, 5, 5, 5, 6, 5, 7,
                                         6, 6, 5, 4, 5, 4, 5, 6, 2, 4, 5, 4, 5, 3, 4, 4};
  *len = kLen[i & 31];
  return kWords[i & 31];
}
DG_HD const char* component(uint32_t i, int* len) {
  static const char* const kComp[16] = {
      "auth_service", "db_pool", "http_server", "scheduler", "cache_layer", "rpc_client", "storage_engine",
      "gc_worker", "metrics", "config_loader", "net_io", "query_planner", "log_shipper", "lease_manager",
      "kv_store", "raft_node"};
  static const unsigned char kLen[16] = {12, 7, 11, 9, 11, 10, 14, 9, 7, 13, 6, 13, 11, 13, 8, 9};
  *len = kLen[i & 15];
  return kComp[i & 15];
}

// Writes one line of exactly `len` bytes (len in [40, 200], last byte '\n').
DG_HD void line(uint64_t seed, uint64_t page, uint32_t li, int kind, char* o, uint32_t len) {
  Rng r{mix(seed) ^ mix(page * 0x100000001b3ull + li)};
  const uint32_t end = len - 1;
  uint32_t p = 0;
  auto put = [&](char ch) {
    if (p < end) o[p++] = ch;
  };
  // timestamp (23 bytes)
  uint32_t mo = 1 + r.below(12), d = 1 + r.below(28), h = r.below(24), mi = r.below(60), se = r.below(60),
           ms = r.below(1000);
  put('2'); put('0'); put('2'); put('4'); put('-');
  put(char('0' + mo / 10)); put(char('0' + mo % 10)); put('-');
  put(char('0' + d / 10)); put(char('0' + d % 10)); put('T');
  put(char('0' + h / 10)); put(char('0' + h % 10)); put(':');
  put(char('0' + mi / 10)); put(char('0' + mi % 10)); put(':');
  put(char('0' + se / 10)); put(char('0' + se % 10)); put('.');
  put(char('0' + ms / 100)); put(char('0' + (ms / 10) % 10)); put(char('0' + ms % 10));
  put(' ');
  uint32_t lv = r.below(100);
  const char* L = lv < 70 ? "INFO" : (lv < 85 ? "DEBUG" : (lv < 95 ? "WARN" : "ERROR"));
  for (int k = 0; L[k]; ++k) put(L[k]);
  put(' ');
  int cl;
  const char* c = component(r.below(16), &cl);
  for (int k = 0; k < cl; ++k) put(c[k]);
  put(':');
  const bool plant_err = r.below(1000) < 20;
  const bool plant_lock = r.below(1000) < 5;
  const bool plant_kw = kind == 1 && r.below(1000) < 10;
  char kw[16];
  int kwl = 0;
  if (plant_kw) {
    kwl = keyword(seed, int(r.below(kKeywords)), kw);
    for (int k = 0; k < kwl; ++k)
      if (r.below(2)) kw[k] = char(kw[k] - 32);
  }
  const char* lock = "timeout while waiting for lock";
  int wi = 0;
  while (p < end) {
    put(' ');
    const char* wd;
    int wl;
    if (plant_err && wi == 0) { wd = "error"; wl = 5; }
    else if (plant_lock && wi == 1) { wd = lock; wl = 30; }
    else if (plant_kw && wi == 2) { wd = kw; wl = kwl; }
    else wd = word(r.below(32), &wl);
    for (int k = 0; k < wl; ++k) put(wd[k]);
    ++wi;
  }
  o[end] = '\n';
}

// kinds 2 / 3 / 4: a filler page of a long line (no '\n'); kw: plant a keyword
DG_HD void filler_page(uint64_t seed, uint64_t page, char* o, uint32_t bytes, bool kw = false) {
  Rng r{mix(seed + 0xf111) ^ mix(page)};
  const bool plant = r.below(2048) == 0;
  // a keyword (kind 4) is up to 12 bytes: planted 16 bytes before the page end;
  // 'error' 8 before (kinds 2 / 3 as in round 3; round 4's long / long1g lines
  // used the 16-byte placement for them too)
  const uint32_t back = kw ? 16u : 8u;
  const uint32_t at = r.below(bytes > back ? bytes - back : 1);
  uint32_t p = 0;
  while (p < bytes) {
    int wl;
    const char* wd = word(r.below(32), &wl);
    for (int k = 0; k < wl && p < bytes; ++k) o[p++] = wd[k];
    if (p < bytes) o[p++] = ' ';
  }
  if (plant && kw) {
    Rng q{mix(seed + 0x6b77) ^ mix(page)};  // its own stream: kinds 2 / 3 unchanged
    char w[16];
    const int wl = keyword(seed, int(q.below(kKeywords)), w);
    for (int k = 0; k < wl && at + uint32_t(k) < bytes; ++k) o[at + k] = q.below(2) ? char(w[k] - 32) : w[k];
  } else if (plant) {
    for (int k = 0; k < 5 && at + uint32_t(k) < bytes; ++k) o[at + k] = "error"[k];
  }
}
constexpr uint32_t kLongBoundary = 512;          // 1 page in 512 ends a long line
constexpr uint64_t kLongFirstPages = (1u << 30) / kPage;  // kind 3: first 1 GiB

// Fills page `page` (kPage bytes, or fewer for the split's last page: `bytes`).
DG_HD void page_fill(uint64_t seed, uint64_t page, int kind, char* o, uint32_t bytes) {
  if (kind == 2 || kind == 3 || kind == 4) {
    const bool boundary = (mix(seed ^ 0xb0b0) ^ mix(page + 7)) % kLongBoundary == 0 &&
                          !(kind == 3 && page < kLongFirstPages);
    if (!boundary) {
      filler_page(seed, page, o, bytes, kind == 4);
      return;
    }
    kind = kind == 4 ? 1 : 0;
  }
  Rng r{mix(seed + 0x5151) ^ mix(page)};
  uint32_t p = 0, li = 0;
  while (p < bytes) {
    uint32_t rem = bytes - p;
    uint32_t len;
    if (rem < kMinLine) {
      // short remainder of a truncated last page: a line of '.' ending in '\n'
      for (uint32_t k = 0; k + 1 < rem; ++k) o[p + k] = '.';
      o[p + rem - 1] = '\n';
      return;
    }
    if (rem <= kMaxLine) len = rem;
    else if (rem < kMaxLine + kMinLine) len = rem / 2;
    else len = kMinLine + r.below(kMaxLine - kMinLine + 1);
    line(seed, page, li++, kind, o + p, len);
    p += len;
  }
}

}  // namespace synth
}  // namespace dgrep
