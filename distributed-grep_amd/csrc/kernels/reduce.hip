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

// ---- newline positions: two coalesced passes over the input ------------
// (replaces a generic select over every byte). Block b owns bytes
// [b * kSeg, (b + 1) * kSeg); pass 1 counts its '\n' (16 B per thread and
// round, SWAR), an exclusive scan of the block counts gives each block's first
// index, pass 2 writes the positions in order (block-wide scan per round).
constexpr uint64_t kSeg = 256u << 10;

__device__ __forceinline__ uint32_t nl_bits4(uint32_t w) {  // bit k: byte k of w is '\n'
  const uint32_t x = w ^ 0x0a0a0a0au;
  const uint32_t m = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
  return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u);
}
// bit k: byte q + k is a '\n' inside [lo, hi) (q 16-B aligned)
__device__ __forceinline__ uint32_t nl_piece(const uint8_t* s, uint64_t n, uint64_t q, uint64_t hi) {
  if (q >= hi) return 0;
  uint32_t m = 0;
  if (q + 16 <= n) {
    const uint4 v = *reinterpret_cast<const uint4*>(s + q);
    m = nl_bits4(v.x) | (nl_bits4(v.y) << 4) | (nl_bits4(v.z) << 8) | (nl_bits4(v.w) << 12);
  } else {
    for (uint32_t k = 0; q + k < n; ++k) m |= uint32_t(s[q + k] == '\n') << k;
  }
  if (q + 16 > hi) m &= (1u << uint32_t(hi - q)) - 1u;
  return m;
}

// block-wide exclusive scan of v (kRT threads); *total = the block's sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum[kRT / 64];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(x, d, 64);
    if (lane >= uint32_t(d)) x += t;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int k = 0; k < kRT / 64; ++k) {
    before += uint32_t(k) < w ? wsum[k] : 0u;
    all += wsum[k];
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

__global__ __launch_bounds__(kRT) void nl_count_kernel(const uint8_t* s, uint64_t n, uint64_t* counts) {
  const uint64_t lo = uint64_t(blockIdx.x) * kSeg, hi = min(n, lo + kSeg);
  uint32_t c = 0;
  for (uint64_t q = lo + 16u * threadIdx.x; q < hi; q += 16u * kRT) c += uint32_t(__popc(nl_piece(s, n, q, hi)));
  uint32_t total;
  (void)block_excl_scan(c, &total);
  if (threadIdx.x == 0) counts[blockIdx.x] = total;
}

__global__ __launch_bounds__(kRT) void nl_write_kernel(const uint8_t* s, uint64_t n, const uint64_t* offs,
                                                       uint64_t* nl) {
  const uint64_t lo = uint64_t(blockIdx.x) * kSeg, hi = min(n, lo + kSeg);
  uint64_t base = offs[blockIdx.x];
  for (uint64_t q0 = lo; q0 < hi; q0 += 16u * kRT) {
    const uint64_t q = q0 + 16u * threadIdx.x;
    uint32_t m = nl_piece(s, n, q, hi), total;
    const uint32_t ex = block_excl_scan(uint32_t(__popc(m)), &total);
    for (uint32_t k = 0; m; ++k) {
      const uint32_t b = uint32_t(__builtin_ctz(m));
      m &= m - 1u;
      nl[base + ex + k] = q + b;
    }
    base += total;
  }
}

__global__ void nl_total_kernel(const uint64_t* offs, const uint64_t* counts, uint64_t nblk, uint64_t* total) {
  *total = offs[nblk - 1] + counts[nblk - 1];
}

// ---- writer: one WAVE per 64 kept lines ----------------------------------
// Lane l fetches line j0 + l's extents, then the wave walks the 64 lines and
// lane l builds output dwords (pos >> 2) + l + 64k of `key value\n`. A line
// with no escape in it (encoded length == 21 + raw key + raw value: the
// `{"Key":"`, `","Value":"`, `"}` frame) is a copy of two byte ranges: a dword
// wholly inside one range is one unaligned read (two aligned dwords +
// v_alignbyte); a line with escapes is decoded by its own lane (parse_line).
__global__ __launch_bounds__(kRT) void write_kernel(const uint8_t* s, uint64_t n, const uint64_t* nl, uint64_t nlines,
                                                    const uint64_t* klen, const uint64_t* vlen,
                                                    const uint64_t* out_len, const uint64_t* pos, uint8_t* out,
                                                    uint64_t out_cap) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nwaves = uint64_t(gridDim.x) * (kRT / 64);
  for (uint64_t j0 = (uint64_t(blockIdx.x) * (kRT / 64) + (threadIdx.x >> 6)) * 64u; j0 < nlines; j0 += nwaves * 64u) {
    const uint64_t jm = j0 + lane;
    uint64_t a = 0, e = 0, kl = 0, vl = 0, ol = 0, P = 0;
    if (jm < nlines) {
      a = jm ? nl[jm - 1] + 1 : 0;
      e = nl[jm];
      ol = out_len[jm];
      P = pos[jm];
      kl = klen[jm];
      vl = vlen[jm];
    }
    const uint32_t cnt = uint32_t(min(uint64_t(64), nlines - j0));
    for (uint32_t r = 0; r < cnt; ++r) {
      const uint64_t olr = __shfl(ol, int(r), 64), Pr = __shfl(P, int(r), 64);
      if (!olr || Pr + olr > out_cap) continue;
      const uint64_t ar = __shfl(a, int(r), 64), er = __shfl(e, int(r), 64);
      const uint64_t klr = __shfl(kl, int(r), 64), vlr = __shfl(vl, int(r), 64);
      if (er - ar != 21u + klr + vlr) {  // escapes inside: decoded by the line's lane
        if (lane == r) {
          uint64_t x, y, h;
          parse_line<true>(s, a, e, out + P, &x, &y, &h);
        }
        continue;
      }
      const uint64_t ks = ar + 8u, vs = ar + 19u + klr;  // raw key / value starts in the input
      for (uint64_t d = (Pr >> 2) + lane; d < ((Pr + olr + 3) >> 2); d += 64) {
        const uint64_t q0 = 4u * d;
        const int64_t o0 = int64_t(q0) - int64_t(Pr);
        uint64_t src = UINT64_MAX;
        if (o0 >= 0 && uint64_t(o0) + 4u <= klr) src = ks + uint64_t(o0);
        else if (o0 >= int64_t(klr) + 1 && uint64_t(o0) + 4u <= klr + 1u + vlr) src = vs + uint64_t(o0) - klr - 1u;
        if (src != UINT64_MAX && ((src + 3) | 3u) < n) {
          const uint32_t sh = uint32_t(src & 3u);
          const uint32_t* w = reinterpret_cast<const uint32_t*>(s + (src & ~uint64_t(3)));
          const uint32_t lo = w[0], hi = sh ? w[1] : 0u;
          *reinterpret_cast<uint32_t*>(out + q0) = __builtin_amdgcn_alignbyte(hi, lo, sh);
          continue;
        }
        uint32_t word = 0, have = 0;
#pragma unroll
        for (uint32_t b = 0; b < 4; ++b) {
          const int64_t ob = o0 + int64_t(b);
          if (ob < 0 || uint64_t(ob) >= olr) continue;
          const uint64_t o = uint64_t(ob);
          const uint32_t ch = o < klr ? s[ks + o] : o == klr ? uint32_t(' ') : o < klr + 1u + vlr ? s[vs + o - klr - 1u] : uint32_t('\n');
          word |= ch << (8 * b);
          have |= 1u << b;
        }
        if (have == 15u) {
          *reinterpret_cast<uint32_t*>(out + q0) = word;
        } else {
          for (uint32_t b = 0; b < 4; ++b)
            if (have & (1u << b)) out[q0 + b] = uint8_t(word >> (8 * b));
        }
      }
    }
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
  const uint64_t nblk = std::max<uint64_t>((n + kSeg - 1) / kSeg, 1);
  size_t sel_tmp = 0, sort_tmp = 0, scan_tmp = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, sel_tmp, (uint64_t*)nullptr, (uint64_t*)nullptr, nblk, s);
  if (e != hipSuccess) return e;
  if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                              (uint32_t*)nullptr, (uint32_t*)nullptr, L, 0, 64, s)) != hipSuccess)
    return e;
  if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (uint64_t*)nullptr, (uint64_t*)nullptr, L, s)) !=
      hipSuccess)
    return e;
  const size_t tmp = std::max({sel_tmp, sort_tmp, scan_tmp});
  const size_t need = a256(L * 8) * 7 + a256(L * 4) * 2 + a256(tmp) + 2 * a256(nblk * 8);
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
  uint64_t* blk_cnt = reinterpret_cast<uint64_t*>(take(nblk * 8));
  uint64_t* blk_off = reinterpret_cast<uint64_t*>(take(nblk * 8));

  // d_info: [0] lines found, [1] first malformed line (all ones: none), [2] output bytes
  if ((e = hipMemsetAsync(d_info, 0, 8, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(d_info + 1, 0xff, 8, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(d_info + 2, 0, 8, s)) != hipSuccess) return e;
  if (n == 0 || nlines == 0) return hipSuccess;
  size_t tb = tmp;
  hipLaunchKernelGGL(nl_count_kernel, dim3(nblk), dim3(kRT), 0, s, d_in, n, blk_cnt);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = hipcub::DeviceScan::ExclusiveSum(t, tb, blk_cnt, blk_off, nblk, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(nl_write_kernel, dim3(nblk), dim3(kRT), 0, s, d_in, n, blk_off, nl);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(nl_total_kernel, dim3(1), dim3(1), 0, s, blk_off, blk_cnt, nblk, d_info);
  if ((e = hipGetLastError()) != hipSuccess) return e;
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
  hipLaunchKernelGGL(write_kernel, dim3(std::min<uint64_t>((nlines + 255) / 256, 4096)), dim3(kRT), 0, s, d_in, n, nl,
                     nlines, klen, vlen, out_len, pos, out, out_cap);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(total_kernel, dim3(1), dim3(1), 0, s, pos, out_len, nlines, d_info + 2);
  return hipGetLastError();
}

}  // namespace dgrep
