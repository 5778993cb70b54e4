// encode.hip — the worker's partition + intermediate writer on the GPU.
//
// Reference (map_reduce/worker.go:78-109, writeMapOutput): for each reduce
// partition i, every KeyValue of the Map output with ihash(kv.Key) % nReduce
// == i is appended, in Map output order, to mr-<task>-<i> as the line
// json.NewEncoder(f).Encode(&kv) writes:
//     {"Key":<json string>,"Value":<json string>}\n
// ihash (worker.go:13-17) = FNV-1a 32 of the key & 0x7fffffff; the grep
// plugin's key is Sprintf("%s (line number #%v)", filename, line)
// (application/grep.go:25). Here the Map output is the scan's compacted
// records (line_no, start, len) over the HBM-resident split, so a partition's
// bytes are produced without ever building the KeyValue slice:
//   1. measure: per record, the key's partition (FNV-1a continued from the
//      host-hashed prefix "filename (line number #" over the decimal digits
//      and ')') and the encoded line's length (Go's JSON string escaping of the
//      value bytes, read from the split);
//   2. a stable radix sort of (partition, record) keeps line order inside a
//      partition; an exclusive scan of the sorted lengths gives each line's
//      byte offset; partition boundaries give each partition's byte range;
//   3. write: one thread per record emits its line at its offset.
// Algorithmic bytes: the matched lines' bytes read twice (measure, write) +
// the encoded output written once + ~40 B per record of sort/scan traffic.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "encode.h"

namespace dgrep {

__host__ __device__ inline uint32_t fnv_step(uint32_t h, uint32_t b) { return (h ^ b) * 16777619u; }

// Go encoding/json string escaping (encode.go encodeState.string, HTML escape
// on, as json.NewEncoder sets it): '"' '\\' get a backslash; \n \r \t their
// short forms; other bytes < 0x20 and < > & become \u00XX; invalid UTF-8 (as
// utf8.DecodeRuneInString: each bad byte on its own) becomes �;
// U+2028/U+2029 become  / ; every other byte passes unchanged.
// OUT = nullptr measures. Returns the bytes written (quotes excluded).
template <bool WRITE>
__host__ __device__ inline uint64_t json_body(const uint8_t* s, uint64_t n, uint8_t* out) {
  const char* hex = "0123456789abcdef";
  uint64_t o = 0, i = 0;
  auto put = [&](uint8_t ch) {
    if (WRITE) out[o] = ch;
    ++o;
  };
  while (i < n) {
    const uint32_t b = s[i];
    if (b < 0x80) {
      if (b >= 0x20 && b != '"' && b != '\\' && b != '<' && b != '>' && b != '&') {
        put(uint8_t(b));
      } else {
        put('\\');
        if (b == '\\' || b == '"') put(uint8_t(b));
        else if (b == '\n') put('n');
        else if (b == '\r') put('r');
        else if (b == '\t') put('t');
        else { put('u'); put('0'); put('0'); put(uint8_t(hex[b >> 4])); put(uint8_t(hex[b & 15])); }
      }
      ++i;
      continue;
    }
    uint32_t need = 0, lo = 0x80, hi = 0xBF, r = 0;
    bool ok = true;
    if (b >= 0xC2 && b <= 0xDF) { need = 2; r = b & 0x1F; }
    else if (b >= 0xE0 && b <= 0xEF) { need = 3; r = b & 0x0F; if (b == 0xE0) lo = 0xA0; if (b == 0xED) hi = 0x9F; }
    else if (b >= 0xF0 && b <= 0xF4) { need = 4; r = b & 7; if (b == 0xF0) lo = 0x90; if (b == 0xF4) hi = 0x8F; }
    else ok = false;
    if (ok && i + need > n) ok = false;
    if (ok && (s[i + 1] < lo || s[i + 1] > hi)) ok = false;
    for (uint32_t k = 1; ok && k < need; ++k) {
      if (k > 1 && (s[i + k] < 0x80 || s[i + k] > 0xBF)) ok = false;
      r = (r << 6) | (s[i + k] & 0x3Fu);
    }
    if (!ok) {
      put('\\'); put('u'); put('f'); put('f'); put('f'); put('d');
      ++i;
      continue;
    }
    if (r == 0x2028 || r == 0x2029) {
      put('\\'); put('u'); put('2'); put('0'); put('2'); put(uint8_t(hex[r & 15]));
    } else {
      for (uint32_t k = 0; k < need; ++k) put(s[i + k]);
    }
    i += need;
  }
  return o;
}

uint64_t json_escape_host(const uint8_t* s, uint64_t n, uint8_t* out) {
  return out ? json_body<true>(s, n, out) : json_body<false>(s, n, nullptr);
}

uint32_t key_prefix_hash(const uint8_t* filename, uint64_t fn) {
  uint32_t h = 2166136261u;
  for (uint64_t i = 0; i < fn; ++i) h = fnv_step(h, filename[i]);
  const char* mid = " (line number #";
  for (int i = 0; mid[i]; ++i) h = fnv_step(h, uint8_t(mid[i]));
  return h;
}

namespace {
constexpr int kEncThreads = 256;

// bit 7 of byte k set iff byte k of x is zero (exact)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) { return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u; }
// bit 7 of byte k set iff byte k of x needs JSON escaping or is not ASCII:
// < 0x20, >= 0x80, '"', '\\', '<', '>', '&'
__device__ __forceinline__ uint32_t special_bytes(uint32_t x) {
  return zero_bytes(x & 0xe0e0e0e0u) | (x & 0x80808080u) | zero_bytes(x ^ 0x22222222u) | zero_bytes(x ^ 0x5c5c5c5cu) |
         zero_bytes(x ^ 0x3c3c3c3cu) | zero_bytes(x ^ 0x3e3e3e3eu) | zero_bytes(x ^ 0x26262626u);
}
// byte mask (bit 7 of each byte) of the bytes at absolute positions [lo, hi)
// within the aligned word at position w
__device__ __forceinline__ uint32_t range_mask(uint64_t w, uint64_t lo, uint64_t hi) {
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (w + uint64_t(k) >= lo && w + uint64_t(k) < hi) m |= 0x80u << (8 * k);
  return m;
}

// true iff the value bytes [st, st + L) encode as themselves (plain printable
// ASCII, nothing to escape): aligned 16-byte reads + SWAR tests, no per-byte
// loads. The common case of text logs; otherwise json_body's byte loop.
__device__ __forceinline__ bool plain_value(const uint8_t* data, uint64_t n, uint64_t st, uint64_t L) {
  const uint64_t e = st + L;
  for (uint64_t q = st & ~uint64_t(15); q < e; q += 16) {
    if (q + 16 > n) {
      for (uint64_t i = q > st ? q : st; i < e; ++i) {
        const uint32_t b = data[i];
        if (b < 0x20 || b >= 0x80 || b == '"' || b == '\\' || b == '<' || b == '>' || b == '&') return false;
      }
      return true;
    }
    const uint4 v = *reinterpret_cast<const uint4*>(data + q);
    const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
    uint32_t bad = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t w = q + 4u * uint32_t(k);
      const uint32_t in = (w >= st && w + 4 <= e) ? 0x80808080u : range_mask(w, st, e);
      bad |= special_bytes(ws[k]) & in;
    }
    if (bad) return false;
  }
  return true;
}

// dst[0:L) = src[0:L) with 4-byte stores after the head: the source is read in
// aligned dwords and realigned with v_alignbyte (whole-dword reads never pass
// the source's last dword, which lies inside the 16-B-aligned split).
__device__ __forceinline__ void copy_bytes(uint8_t* dst, const uint8_t* src, uint64_t L) {
  uint64_t i = 0;
  while (i < L && (reinterpret_cast<uintptr_t>(dst + i) & 3)) {
    dst[i] = src[i];
    ++i;
  }
  if (L - i >= 8) {
    const uint8_t* s = src + i;
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(s) & 3);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(s - sh);
    uint32_t* dw = reinterpret_cast<uint32_t*>(dst + i);
    const uint64_t nd = (L - i) / 4 - 1;  // the last dword needs sw[k + 1], which may lie past the value: leave it
    uint32_t lo = sw[0];
    for (uint64_t k = 0; k < nd; ++k) {
      const uint32_t hi = sw[k + 1];
      // v_alignbyte_b32 takes the shift in BYTES: ({hi, lo} >> 8 * sh)[31:0]
      dw[k] = __builtin_amdgcn_alignbyte(hi, lo, sh);
      lo = hi;
    }
    i += nd * 4;
  }
  for (; i < L; ++i) dst[i] = src[i];
}
// {"Key":" + name + " (line number #" + digits + ")" + ,"Value":" + value + "}\n
constexpr uint32_t kFixedBytes = 8 + 15 + 2 + 10 + 3;

__device__ inline uint32_t ndigits(uint64_t v) {
  uint32_t d = 1;
  while (v >= 10) { v /= 10; ++d; }
  return d;
}

__global__ __launch_bounds__(kEncThreads) void encode_measure_kernel(EncodeArgs a, uint16_t* part, uint32_t* idx,
                                                                     uint64_t* enc_len) {
  for (uint64_t i = uint64_t(blockIdx.x) * kEncThreads + threadIdx.x; i < a.count;
       i += uint64_t(gridDim.x) * kEncThreads) {
    const uint64_t ln = a.line_no[i];
    const uint32_t nd = ndigits(ln);
    uint64_t p10 = 1;
    for (uint32_t k = 1; k < nd; ++k) p10 *= 10;
    uint32_t h = a.key_hash0;
    for (uint64_t v = ln; p10; p10 /= 10) {
      h = fnv_step(h, uint32_t('0' + v / p10));
      v %= p10;
    }
    h = fnv_step(h, uint32_t(')'));
    part[i] = uint16_t((h & 0x7fffffffu) % a.nreduce);
    idx[i] = uint32_t(i);
    const uint64_t st = a.start[i], L = a.len[i];
    const uint64_t body = plain_value(a.data, a.n, st, L) ? L : json_body<false>(a.data + st, L, nullptr);
    enc_len[i] = kFixedBytes + a.fname_json_len + nd + body;
  }
}

__global__ __launch_bounds__(kEncThreads) void gather_len_kernel(const uint32_t* idx, const uint64_t* enc_len,
                                                                 uint64_t* len_sorted, uint64_t count) {
  for (uint64_t j = uint64_t(blockIdx.x) * kEncThreads + threadIdx.x; j < count; j += uint64_t(gridDim.x) * kEncThreads)
    len_sorted[j] = enc_len[idx[j]];
}

// bounds[p] / bounds[nreduce + p]: byte range of partition p (both 0 when
// empty; zeroed beforehand); bounds[2 * nreduce]: total bytes
__global__ __launch_bounds__(kEncThreads) void bounds_kernel(const uint16_t* part, const uint64_t* pos,
                                                             const uint64_t* len_sorted, uint64_t count,
                                                             uint32_t nreduce, uint64_t* bounds) {
  for (uint64_t j = uint64_t(blockIdx.x) * kEncThreads + threadIdx.x; j < count; j += uint64_t(gridDim.x) * kEncThreads) {
    const uint32_t p = part[j];
    if (j == 0 || part[j - 1] != p) bounds[p] = pos[j];
    if (j + 1 == count || part[j + 1] != p) bounds[nreduce + p] = pos[j] + len_sorted[j];
    if (j + 1 == count) bounds[2 * nreduce] = pos[j] + len_sorted[j];
  }
}

__device__ inline void put_str(uint8_t*& o, const char* s) {
  while (*s) *o++ = uint8_t(*s++);
}

__global__ __launch_bounds__(kEncThreads) void encode_write_kernel(EncodeArgs a, const uint32_t* idx,
                                                                   const uint64_t* pos, const uint64_t* len_sorted,
                                                                   uint8_t* out, uint64_t out_cap) {
  for (uint64_t j = uint64_t(blockIdx.x) * kEncThreads + threadIdx.x; j < a.count;
       j += uint64_t(gridDim.x) * kEncThreads) {
    if (pos[j] + len_sorted[j] > out_cap) continue;
    const uint64_t i = idx[j];
    uint8_t* o = out + pos[j];
    put_str(o, "{\"Key\":\"");
    for (uint32_t k = 0; k < a.fname_json_len; ++k) *o++ = a.fname_json[k];
    put_str(o, " (line number #");
    const uint64_t ln = a.line_no[i];
    const uint32_t nd = ndigits(ln);
    uint64_t v = ln;
    for (uint32_t k = nd; k-- > 0;) {
      o[k] = uint8_t('0' + v % 10);
      v /= 10;
    }
    o += nd;
    put_str(o, ")\",\"Value\":\"");
    const uint64_t L = a.len[i];
    if (len_sorted[j] == kFixedBytes + a.fname_json_len + nd + L) {
      // the measure pass found nothing to escape: the value is copied as is
      copy_bytes(o, a.data + a.start[i], L);
      o += L;
    } else {
      o += json_body<true>(a.data + a.start[i], L, o);
    }
    put_str(o, "\"}\n");
  }
}

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }
inline int grid_for(uint64_t n) { return int(std::min<uint64_t>((n + kEncThreads - 1) / kEncThreads, 8192)); }
}  // namespace

hipError_t encode_partitions(const EncodeArgs& a, void* scratch, size_t* scratch_bytes, uint8_t* out,
                             uint64_t out_cap, uint64_t* d_bounds, hipStream_t s) {
  const uint64_t n = a.count;
  int end_bit = 1;
  while ((1u << end_bit) < a.nreduce) ++end_bit;
  size_t sort_tmp = 0, scan_tmp = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (uint16_t*)nullptr, (uint16_t*)nullptr,
                                                    (uint32_t*)nullptr, (uint32_t*)nullptr, n, 0, end_bit, s);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (uint64_t*)nullptr, (uint64_t*)nullptr, n, s);
  if (e != hipSuccess) return e;
  const size_t tmp = std::max(sort_tmp, scan_tmp);
  const size_t need = 2 * align256(n * 2) + 2 * align256(n * 4) + 3 * align256(n * 8) + align256(tmp);
  if (!scratch || *scratch_bytes < need) {
    *scratch_bytes = need;
    return hipSuccess;
  }
  uint8_t* p = static_cast<uint8_t*>(scratch);
  auto take = [&](size_t bytes) {
    uint8_t* q = p;
    p += align256(bytes);
    return q;
  };
  uint16_t* part_in = reinterpret_cast<uint16_t*>(take(n * 2));
  uint16_t* part_out = reinterpret_cast<uint16_t*>(take(n * 2));
  uint32_t* idx_in = reinterpret_cast<uint32_t*>(take(n * 4));
  uint32_t* idx_out = reinterpret_cast<uint32_t*>(take(n * 4));
  uint64_t* enc_len = reinterpret_cast<uint64_t*>(take(n * 8));
  uint64_t* len_sorted = reinterpret_cast<uint64_t*>(take(n * 8));
  uint64_t* pos = reinterpret_cast<uint64_t*>(take(n * 8));
  void* t = take(tmp);

  e = hipMemsetAsync(d_bounds, 0, (2 * size_t(a.nreduce) + 1) * 8, s);
  if (e != hipSuccess || n == 0) return e;
  hipLaunchKernelGGL(encode_measure_kernel, dim3(grid_for(n)), dim3(kEncThreads), 0, s, a, part_in, idx_in, enc_len);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  size_t tb = tmp;
  if ((e = hipcub::DeviceRadixSort::SortPairs(t, tb, part_in, part_out, idx_in, idx_out, n, 0, end_bit, s)) !=
      hipSuccess)
    return e;
  hipLaunchKernelGGL(gather_len_kernel, dim3(grid_for(n)), dim3(kEncThreads), 0, s, idx_out, enc_len, len_sorted, n);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  tb = tmp;
  if ((e = hipcub::DeviceScan::ExclusiveSum(t, tb, len_sorted, pos, n, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(bounds_kernel, dim3(grid_for(n)), dim3(kEncThreads), 0, s, part_out, pos, len_sorted, n,
                     a.nreduce, d_bounds);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(encode_write_kernel, dim3(grid_for(n)), dim3(kEncThreads), 0, s, a, idx_out, pos, len_sorted, out,
                     out_cap);
  return hipGetLastError();
}

}  // namespace dgrep
