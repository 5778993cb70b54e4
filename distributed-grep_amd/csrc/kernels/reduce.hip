// reduce.hip — the grep reduce task on the GPU.
//
// Reference (map_reduce/worker.go):
//   readReduceInput (44-68): json.NewDecoder over each mr-<map>-<r> file, one
//     KeyValue per line (the lines encode.hip / writeMapOutput produced);
//   reduceDistinctKeys (22-42): sort.Sort(ByKey) -- NOT stable -- then one
//     reducef(key, values) per distinct key; the grep plugin's Reduce is
//     values[0] (application/grep.go:38-40), so the result is ONE of the
//     key's values (which one is unspecified for duplicate keys);
//   161-165: fmt.Sprintf("%v %v\n", k, v) per entry of a Go map, i.e. in
//     random order.
// Here: the concatenated input bytes sit in HBM; a newline select gives the
// lines; one thread per line decodes {"Key":"..","Value":".."} (JSON string
// escapes, \uXXXX incl. surrogate pairs -> UTF-8) to measure the raw key and
// value and hash the raw key (FNV-1a 64); a radix sort of (hash, line) groups
// equal keys and an exact byte compare inside each equal-hash run keeps the
// first line of every distinct key; a scan of the kept lines' output lengths
// places "key value\n"; one thread per kept line writes it. Output order = input
// line order of the kept lines (one of the orders the reference can produce).
// Input must be json.Encoder KeyValue lines (what writeMapOutput writes); any
// other line is reported as malformed (DGREP_E_INVALID), never guessed.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "reduce.h"

namespace dgrep {
namespace {
constexpr int kRT = 256;

__device__ inline int hexval(uint32_t c) {
  if (c >= '0' && c <= '9') return int(c - '0');
  if (c >= 'a' && c <= 'f') return int(c - 'a' + 10);
  if (c >= 'A' && c <= 'F') return int(c - 'A' + 10);
  return -1;
}

// Decodes the JSON string starting after its opening quote at s[i]; returns
// the index after the closing quote (or UINT64_MAX if malformed). WRITE:
// raw bytes go to out. *olen: raw length; *h: FNV-1a 64 of the raw bytes.
template <bool WRITE>
__device__ uint64_t json_string(const uint8_t* s, uint64_t i, uint64_t end, uint8_t* out, uint64_t* olen,
                                uint64_t* h) {
  uint64_t o = 0, hh = 1469598103934665603ull;
  auto put = [&](uint32_t b) {
    if (WRITE) out[o] = uint8_t(b);
    ++o;
    hh = (hh ^ b) * 1099511628211ull;
  };
  auto put_rune = [&](uint32_t r) {
    if (r < 0x80) put(r);
    else if (r < 0x800) { put(0xC0 | (r >> 6)); put(0x80 | (r & 0x3F)); }
    else if (r < 0x10000) { put(0xE0 | (r >> 12)); put(0x80 | ((r >> 6) & 0x3F)); put(0x80 | (r & 0x3F)); }
    else { put(0xF0 | (r >> 18)); put(0x80 | ((r >> 12) & 0x3F)); put(0x80 | ((r >> 6) & 0x3F)); put(0x80 | (r & 0x3F)); }
  };
  auto hex4 = [&](uint64_t p, uint32_t* r) -> bool {
    if (p + 4 > end) return false;
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      const int d = hexval(s[p + k]);
      if (d < 0) return false;
      v = (v << 4) | uint32_t(d);
    }
    *r = v;
    return true;
  };
  while (i < end) {
    const uint32_t b = s[i];
    if (b == '"') {
      *olen = o;
      *h = hh;
      return i + 1;
    }
    if (b < 0x20) return UINT64_MAX;
    if (b != '\\') {
      put(b);
      ++i;
      continue;
    }
    if (i + 1 >= end) return UINT64_MAX;
    const uint32_t e = s[i + 1];
    i += 2;
    switch (e) {
      case '"': case '\\': case '/': put(e); break;
      case 'b': put(8); break;
      case 'f': put(12); break;
      case 'n': put(10); break;
      case 'r': put(13); break;
      case 't': put(9); break;
      case 'u': {
        uint32_t r;
        if (!hex4(i, &r)) return UINT64_MAX;
        i += 4;
        if (r >= 0xD800 && r < 0xDC00) {
          // encoding/json: a high surrogate followed by \u low surrogate pairs up;
          // any other lone surrogate decodes to U+FFFD
          uint32_t r2;
          if (i + 1 < end && s[i] == '\\' && s[i + 1] == 'u' && hex4(i + 2, &r2) && r2 >= 0xDC00 && r2 < 0xE000) {
            i += 6;
            r = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00);
          } else {
            r = 0xFFFD;
          }
        } else if (r >= 0xDC00 && r < 0xE000) {
          r = 0xFFFD;
        }
        put_rune(r);
        break;
      }
      default: return UINT64_MAX;
    }
  }
  return UINT64_MAX;
}

__device__ inline bool lit(const uint8_t* s, uint64_t i, uint64_t end, const char* t) {
  for (; *t; ++t, ++i)
    if (i >= end || s[i] != uint8_t(*t)) return false;
  return true;
}

// Parses line [a, e) (e = its '\n'). Fills key/value raw extents in the
// decoded sense: returns false if malformed.
template <bool WRITE>
__device__ bool parse_line(const uint8_t* s, uint64_t a, uint64_t e, uint8_t* out, uint64_t* klen, uint64_t* vlen,
                           uint64_t* kh) {
  if (!lit(s, a, e, "{\"Key\":\"")) return false;
  uint64_t vh;
  uint64_t i = json_string<WRITE>(s, a + 8, e, out, klen, kh);
  if (i == UINT64_MAX || !lit(s, i, e, ",\"Value\":\"")) return false;
  if (WRITE) out[*klen] = ' ';
  i = json_string<WRITE>(s, i + 10, e, WRITE ? out + *klen + 1 : nullptr, vlen, &vh);
  if (i == UINT64_MAX || !lit(s, i, e, "}") || i + 1 != e) return false;
  if (WRITE) out[*klen + 1 + *vlen] = '\n';
  return true;
}

struct IsNewline {
  const uint8_t* s;
  __host__ __device__ bool operator()(const uint64_t& i) const { return s[i] == '\n'; }
};

__global__ __launch_bounds__(kRT) void measure_kernel(const uint8_t* s, const uint64_t* nl, uint64_t nlines,
                                                      uint64_t* klen, uint64_t* vlen, uint64_t* kh, uint32_t* idx,
                                                      unsigned long long* bad) {
  for (uint64_t j = uint64_t(blockIdx.x) * kRT + threadIdx.x; j < nlines; j += uint64_t(gridDim.x) * kRT) {
    const uint64_t a = j ? nl[j - 1] + 1 : 0, e = nl[j];
    if (!parse_line<false>(s, a, e, nullptr, &klen[j], &vlen[j], &kh[j])) {
      atomicMin(bad, (unsigned long long)j);
      klen[j] = vlen[j] = 0;
      kh[j] = 0;
    }
    idx[j] = uint32_t(j);
  }
}

// keep[line] = 1 unless an earlier line of the same equal-hash run has the
// identical raw key (compared by decoding both); sorted order by (hash, line)
__global__ __launch_bounds__(kRT) void dedupe_kernel(const uint8_t* s, const uint64_t* nl, const uint64_t* h_sorted,
                                                     const uint32_t* idx_sorted, uint64_t nlines, const uint64_t* klen,
                                                     uint64_t* out_len, const uint64_t* vlen) {
  for (uint64_t q = uint64_t(blockIdx.x) * kRT + threadIdx.x; q < nlines; q += uint64_t(gridDim.x) * kRT) {
    const uint32_t j = idx_sorted[q];
    bool keep = true;
    for (uint64_t p = q; keep && p-- > 0 && h_sorted[p] == h_sorted[q];) {
      const uint32_t k = idx_sorted[p];
      if (klen[k] != klen[j]) continue;
      // byte compare of the two raw keys: decode both a byte at a time
      const uint64_t aj = j ? nl[j - 1] + 1 : 0, ak = k ? nl[k - 1] + 1 : 0;
      uint8_t bj[64], bk[64];
      uint64_t lj, lk, hj, hk;
      // keys longer than 64 raw bytes: compare the escaped forms instead --
      // json.Encoder output is canonical, so equal raw keys have equal escapes
      if (klen[j] <= 64) {
        json_string<true>(s, aj + 8, nl[j], bj, &lj, &hj);
        json_string<true>(s, ak + 8, nl[k], bk, &lk, &hk);
        bool same = true;
        for (uint64_t t = 0; t < lj && same; ++t) same = bj[t] == bk[t];
        if (same) keep = false;
      } else {
        bool same = true;
        for (uint64_t t = 8;; ++t) {
          const uint8_t x = s[aj + t], y = s[ak + t];
          if (x != y) { same = false; break; }
          if (x == '"') break;  // the closing quote (escaped ones are skipped below)
          if (x == '\\') {
            ++t;
            if (s[aj + t] != s[ak + t]) { same = false; break; }
          }
        }
        if (same) keep = false;
      }
    }
    out_len[j] = keep ? klen[j] + 1 + vlen[j] + 1 : 0;
  }
}

__global__ __launch_bounds__(kRT) void write_kernel(const uint8_t* s, const uint64_t* nl, uint64_t nlines,
                                                    const uint64_t* out_len, const uint64_t* pos, uint8_t* out,
                                                    uint64_t out_cap) {
  for (uint64_t j = uint64_t(blockIdx.x) * kRT + threadIdx.x; j < nlines; j += uint64_t(gridDim.x) * kRT) {
    if (!out_len[j] || pos[j] + out_len[j] > out_cap) continue;
    uint64_t kl, vl, kh;
    parse_line<true>(s, j ? nl[j - 1] + 1 : 0, nl[j], out + pos[j], &kl, &vl, &kh);
  }
}

__global__ __launch_bounds__(kRT) void count_kernel(const uint8_t* s, uint64_t n, unsigned long long* count) {
  uint64_t c = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * kRT + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kRT) c += s[i] == '\n';
  if (c) atomicAdd(count, (unsigned long long)c);
}

__global__ void total_kernel(const uint64_t* pos, const uint64_t* out_len, uint64_t nlines, uint64_t* total) {
  *total = pos[nlines - 1] + out_len[nlines - 1];
}

inline size_t a256(size_t x) { return (x + 255) & ~size_t(255); }
inline int grid_of(uint64_t n) { return int(std::min<uint64_t>((n + kRT - 1) / kRT, 8192)); }
}  // namespace

hipError_t reduce_count_lines(const uint8_t* d_in, uint64_t n, uint64_t* d_count, hipStream_t s) {
  hipError_t e = hipMemsetAsync(d_count, 0, 8, s);
  if (e != hipSuccess || n == 0) return e;
  hipLaunchKernelGGL(count_kernel, dim3(grid_of(n)), dim3(kRT), 0, s, d_in, n,
                     reinterpret_cast<unsigned long long*>(d_count));
  return hipGetLastError();
}

hipError_t reduce_lines(const uint8_t* d_in, uint64_t n, uint64_t nlines, void* scratch, size_t* scratch_bytes,
                        uint8_t* out, uint64_t out_cap, uint64_t* d_info, hipStream_t s) {
  const uint64_t L = std::max<uint64_t>(nlines, 1);
  size_t sel_tmp = 0, sort_tmp = 0, scan_tmp = 0;
  hipcub::CountingInputIterator<uint64_t> it(0);
  hipError_t e = hipcub::DeviceSelect::If(nullptr, sel_tmp, it, (uint64_t*)nullptr, (uint64_t*)nullptr, n,
                                          IsNewline{d_in}, s);
  if (e != hipSuccess) return e;
  if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                              (uint32_t*)nullptr, (uint32_t*)nullptr, L, 0, 64, s)) != hipSuccess)
    return e;
  if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (uint64_t*)nullptr, (uint64_t*)nullptr, L, s)) !=
      hipSuccess)
    return e;
  const size_t tmp = std::max({sel_tmp, sort_tmp, scan_tmp});
  const size_t need = a256(L * 8) * 7 + a256(L * 4) * 2 + a256(tmp);
  if (!scratch || *scratch_bytes < need) {
    *scratch_bytes = need;
    return hipSuccess;
  }
  uint8_t* p = static_cast<uint8_t*>(scratch);
  auto take = [&](size_t b) {
    uint8_t* q = p;
    p += a256(b);
    return q;
  };
  uint64_t* nl = reinterpret_cast<uint64_t*>(take(L * 8));
  uint64_t* klen = reinterpret_cast<uint64_t*>(take(L * 8));
  uint64_t* vlen = reinterpret_cast<uint64_t*>(take(L * 8));
  uint64_t* kh = reinterpret_cast<uint64_t*>(take(L * 8));
  uint64_t* kh_sorted = reinterpret_cast<uint64_t*>(take(L * 8));
  uint64_t* out_len = reinterpret_cast<uint64_t*>(take(L * 8));
  uint64_t* pos = reinterpret_cast<uint64_t*>(take(L * 8));
  uint32_t* idx = reinterpret_cast<uint32_t*>(take(L * 4));
  uint32_t* idx_sorted = reinterpret_cast<uint32_t*>(take(L * 4));
  void* t = take(tmp);

  // d_info: [0] lines found, [1] first malformed line (all ones: none), [2] output bytes
  if ((e = hipMemsetAsync(d_info, 0, 8, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(d_info + 1, 0xff, 8, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(d_info + 2, 0, 8, s)) != hipSuccess) return e;
  if (n == 0 || nlines == 0) return hipSuccess;
  size_t tb = tmp;
  if ((e = hipcub::DeviceSelect::If(t, tb, it, nl, d_info, n, IsNewline{d_in}, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(measure_kernel, dim3(grid_of(nlines)), dim3(kRT), 0, s, d_in, nl, nlines, klen, vlen, kh, idx,
                     reinterpret_cast<unsigned long long*>(d_info + 1));
  if ((e = hipGetLastError()) != hipSuccess) return e;
  tb = tmp;
  if ((e = hipcub::DeviceRadixSort::SortPairs(t, tb, kh, kh_sorted, idx, idx_sorted, nlines, 0, 64, s)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(dedupe_kernel, dim3(grid_of(nlines)), dim3(kRT), 0, s, d_in, nl, kh_sorted, idx_sorted, nlines,
                     klen, out_len, vlen);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  tb = tmp;
  if ((e = hipcub::DeviceScan::ExclusiveSum(t, tb, out_len, pos, nlines, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(write_kernel, dim3(grid_of(nlines)), dim3(kRT), 0, s, d_in, nl, nlines, out_len, pos, out,
                     out_cap);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(total_kernel, dim3(1), dim3(1), 0, s, pos, out_len, nlines, d_info + 2);
  return hipGetLastError();
}

}  // namespace dgrep
