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


// decimal digits of v (most significant first) into d[20]; returns their count.
// Line numbers below 2^32 (every split under 4 G lines) take the 32-bit path,
// whose division by 10 is a multiply-high (the 64-bit one is a library loop).
__device__ __forceinline__ uint32_t digits_of(uint64_t v, uint8_t (&d)[20]) {
  uint8_t t[20];
  uint32_t nd = 0;
  if (v < (1ull << 32)) {
    uint32_t x = uint32_t(v);
    do { t[nd++] = uint8_t(x % 10u); x /= 10u; } while (x);
  } else {
    do { t[nd++] = uint8_t(v % 10u); v /= 10u; } while (v);
  }
  for (uint32_t k = 0; k < nd; ++k) d[k] = t[nd - 1 - k];
  return nd;
}

// Per record (one thread each): the key's partition and the encoded line's
// length ASSUMING a plain value (nothing to escape); encode_values_kernel
// corrects the length of the rare values that need escaping.
__global__ __launch_bounds__(kEncThreads) void encode_measure_kernel(EncodeArgs a, uint16_t* part, uint32_t* idx,
                                                                     uint64_t* enc_len) {
  for (uint64_t i = uint64_t(blockIdx.x) * kEncThreads + threadIdx.x; i < a.count;
       i += uint64_t(gridDim.x) * kEncThreads) {
    uint8_t d[20];
    const uint32_t nd = digits_of(a.line_no[i], d);
    uint32_t h = a.key_hash0;
    for (uint32_t k = 0; k < nd; ++k) h = fnv_step(h, uint32_t('0') + d[k]);
    h = fnv_step(h, uint32_t(')'));
    part[i] = uint16_t((h & 0x7fffffffu) % a.nreduce);
    idx[i] = uint32_t(i);
    enc_len[i] = kFixedBytes + a.fname_json_len + nd + a.len[i];
  }
}

// One WAVE per record: the value's bytes are tested 4 per lane (aligned
// dwords, SWAR) and a ballot decides; a value with anything to escape gets its
// exact encoded length from json_body (lane 0). Consecutive lanes read
// consecutive dwords, so a record's value is one coalesced sweep.
__global__ __launch_bounds__(kEncThreads) void encode_values_kernel(EncodeArgs a, uint64_t* enc_len) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t waves = uint64_t(gridDim.x) * (kEncThreads / 64);
  for (uint64_t i = uint64_t(blockIdx.x) * (kEncThreads / 64) + (threadIdx.x >> 6); i < a.count; i += waves) {
    const uint64_t st = a.start[i], e = st + a.len[i];
    bool bad = false;
    for (uint64_t w = (st & ~uint64_t(3)) + 4u * lane; w < e; w += 256) {
      uint32_t x;
      if (w + 4 <= a.n) {
        x = *reinterpret_cast<const uint32_t*>(a.data + w);
      } else {  // the split's last partial dword: no read past n
        x = 0x20202020u;
        for (uint32_t k = 0; w + k < a.n; ++k) x = (x & ~(0xffu << (8 * k))) | (uint32_t(a.data[w + k]) << (8 * k));
      }
      const uint32_t in = (w >= st && w + 4 <= e) ? 0x80808080u : range_mask(w, st, e);
      bad = bad || (special_bytes(x) & in) != 0u;
    }
    if (__ballot(bad) == 0ull) continue;  // wave-uniform: plain value
    if (lane == 0) enc_len[i] += json_body<false>(a.data + st, e - st, nullptr) - (e - st);
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

// Per-thread writer of one record's line (values that need escaping).
__device__ void write_line_thread(const EncodeArgs& a, uint64_t i, uint8_t* o, uint64_t enc) {
  put_str(o, "{\"Key\":\"");
  for (uint32_t k = 0; k < a.fname_json_len; ++k) *o++ = a.fname_json[k];
  put_str(o, " (line number #");
  uint8_t d[20];
  const uint32_t nd = digits_of(a.line_no[i], d);
  for (uint32_t k = 0; k < nd; ++k) *o++ = uint8_t('0' + d[k]);
  put_str(o, ")\",\"Value\":\"");
  const uint64_t L = a.len[i];
  if (enc == kFixedBytes + a.fname_json_len + nd + L) {
    copy_bytes(o, a.data + a.start[i], L);
    o += L;
  } else {
    o += json_body<true>(a.data + a.start[i], L, o);
  }
  put_str(o, "\"}\n");
}

// One WAVE per 64 output lines (sorted order j0 .. j0 + 63). Lane l first
// fetches line j0 + l's record (coalesced: idx, pos, length, then the record)
// and writes its line number's digits to the wave's LDS row; then the wave
// walks the 64 lines, each broadcast from its lane, and lane l builds the
// line's output dwords (pos >> 2) + l + 64k from its five pieces -- the
// constant head `{"Key":"<file> (line number #` (LDS), the digits (LDS),
// `)","Value":"`, the value bytes, `"}\n`. A dword wholly inside the value is
// one unaligned read of the split (two aligned dwords + v_alignbyte); the
// first and last dwords of a line, shared with its neighbours, are stored byte
// by byte. A value that needs escaping is written by its own lane alone
// (write_line_thread).
constexpr uint32_t kHeadMax = 2048;
constexpr int kEncWaves = kEncThreads / 64;
__global__ __launch_bounds__(kEncThreads) void encode_write_kernel(EncodeArgs a, const uint32_t* idx,
                                                                   const uint64_t* pos, const uint64_t* len_sorted,
                                                                   uint8_t* out, uint64_t out_cap) {
  __shared__ uint8_t head[kHeadMax];
  __shared__ uint8_t dig[kEncWaves][64][20];
  const uint32_t F = a.fname_json_len, A = 8u + F + 15u;  // head bytes (host guarantees A <= kHeadMax)
  for (uint32_t k = threadIdx.x; k < A; k += kEncThreads)
    head[k] = k < 8u ? uint8_t("{\"Key\":\""[k]) : k < 8u + F ? a.fname_json[k - 8u] : uint8_t(" (line number #"[k - 8u - F]);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t nwaves = uint64_t(gridDim.x) * kEncWaves;
  for (uint64_t j0 = (uint64_t(blockIdx.x) * kEncWaves + wv) * 64u; j0 < a.count; j0 += nwaves * 64u) {
    const uint64_t jm = j0 + lane;
    uint64_t P = 0, T = 0, st = 0, L = 0, i = 0;
    uint32_t nd = 0;
    if (jm < a.count) {
      i = idx[jm];
      P = pos[jm];
      T = len_sorted[jm];
      st = a.start[i];
      L = a.len[i];
      uint8_t d[20];
      nd = digits_of(a.line_no[i], d);
      for (uint32_t k = 0; k < nd; ++k) dig[wv][lane][k] = d[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t cnt = uint32_t(min(uint64_t(64), a.count - j0));
    for (uint32_t r = 0; r < cnt; ++r) {
      const uint64_t Pr = __shfl(P, int(r), 64), Tr = __shfl(T, int(r), 64);
      const uint64_t str = __shfl(st, int(r), 64), Lr = __shfl(L, int(r), 64);
      const uint32_t ndr = uint32_t(__shfl(int(nd), int(r), 64));
      if (Pr + Tr > out_cap) continue;
      if (Tr != kFixedBytes + F + ndr + Lr) {  // escaped value: wave-uniform, rare
        if (lane == r) write_line_thread(a, i, out + P, T);
        continue;
      }
      const uint64_t V0 = uint64_t(A) + ndr + 12u;  // line offset of the first value byte
      const uint64_t d0 = Pr >> 2, d1 = (Pr + Tr + 3) >> 2;
      for (uint64_t d = d0 + lane; d < d1; d += 64) {
        const uint64_t q0 = 4u * d;
        const int64_t o0 = int64_t(q0) - int64_t(Pr);  // line offset of the dword's byte 0
        const uint64_t src = str + uint64_t(o0 - int64_t(V0));  // split position of byte 0 if it were value
        if (o0 >= int64_t(V0) && uint64_t(o0) + 4u <= V0 + Lr && ((src + 3) | 3u) < a.n) {
          const uint32_t sh = uint32_t(src & 3u);
          const uint32_t* w = reinterpret_cast<const uint32_t*>(a.data + (src & ~uint64_t(3)));
          const uint32_t lo = w[0], hi = sh ? w[1] : 0u;
          *reinterpret_cast<uint32_t*>(out + q0) = __builtin_amdgcn_alignbyte(hi, lo, sh);
          continue;
        }
        uint32_t word = 0, have = 0;
#pragma unroll
        for (uint32_t b = 0; b < 4; ++b) {
          const int64_t ob = o0 + int64_t(b);
          if (ob < 0 || uint64_t(ob) >= Tr) continue;
          const uint64_t o = uint64_t(ob);
          uint32_t ch;
          if (o < A) ch = head[o];
          else if (o < uint64_t(A) + ndr) ch = uint32_t('0') + dig[wv][r][o - A];
          else if (o < V0) ch = uint8_t(")\",\"Value\":\""[o - A - ndr]);
          else if (o < V0 + Lr) ch = a.data[str + (o - V0)];
          else ch = uint8_t("\"}\n"[o - V0 - Lr]);
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
    __builtin_amdgcn_wave_barrier();  // the LDS digit row is rewritten next round
  }
}

// the per-thread writer for file names whose head does not fit kHeadMax
__global__ __launch_bounds__(kEncThreads) void encode_write_thread_kernel(EncodeArgs a, const uint32_t* idx,
                                                                          const uint64_t* pos,
                                                                          const uint64_t* len_sorted, uint8_t* out,
                                                                          uint64_t out_cap) {
  for (uint64_t j = uint64_t(blockIdx.x) * kEncThreads + threadIdx.x; j < a.count;
       j += uint64_t(gridDim.x) * kEncThreads) {
    if (pos[j] + len_sorted[j] > out_cap) continue;
    write_line_thread(a, idx[j], out + pos[j], len_sorted[j]);
  }
}

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }
inline int grid_for(uint64_t n) { return int(std::min<uint64_t>((n + kEncThreads - 1) / kEncThreads, 8192)); }
// one wave per record: 4 records per workgroup, at most 8 resident-sized rounds of the chip
inline int wave_grid_for(uint64_t n) { return int(std::min<uint64_t>((n + 3) / 4, 16384)); }
// one wave per 64 records
inline int wave64_grid_for(uint64_t n) { return int(std::min<uint64_t>((n + 255) / 256, 4096)); }
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
  hipLaunchKernelGGL(encode_values_kernel, dim3(wave_grid_for(n)), dim3(kEncThreads), 0, s, a, enc_len);
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
  if (8u + a.fname_json_len + 15u <= kHeadMax)
    hipLaunchKernelGGL(encode_write_kernel, dim3(wave64_grid_for(n)), dim3(kEncThreads), 0, s, a, idx_out, pos,
                       len_sorted, out, out_cap);
  else
    hipLaunchKernelGGL(encode_write_thread_kernel, dim3(grid_for(n)), dim3(kEncThreads), 0, s, a, idx_out, pos,
                       len_sorted, out, out_cap);
  return hipGetLastError();
}

}  // namespace dgrep
