// scan_dfa.hip — CDNA4 (gfx950) kernels for the distributed-grep Map hot path.
//
// Reference path (application/grep.go:17-29):
//     lines := strings.Split(contents, "\n")
//     for line_number, line := range lines {
//         matched, _ := regexp.Match(pattern, []byte(line))
//         if matched { emit(line_number+1, line) }
// Here the pattern is a byte DFA (dgrep_blob.h) that restarts at every '\n'
// and enters START_M on the '\n' of a matching line, so a single streaming
// pass over the split evaluates every line.
//
// Work decomposition (HBM-bound: every input byte is read once):
//   * tile = 256 lanes x C bytes; lane i owns chunk i of its tile.
//   * A lane OWNS the lines that start inside its chunk after its first '\n'
//     (the very first line of the split is owned by global lane 0). It runs the
//     DFA from its chunk start -- the bytes before its first '\n' are run with a
//     don't-care state, which the first '\n' resets -- through its chunk and on
//     past the chunk end until the first '\n' at or after the end (the last
//     owned line's terminator) or the end of the split. No lane ever waits for
//     another lane's state; a line longer than a chunk is simply run to its end
//     by the lane that owns it.
//   * Per 4-byte word: 4 x (v_perm_b32 + ds_read_u8) DFA steps from an
//     LDS-resident u8 table [state][byte]; newline bookkeeping by SWAR on the
//     word; a matching line is detected by "state == START_M" (rare path).
//   * Matching lines are parked in per-lane LDS slots, counted, then the tile's
//     lines are appended to a staging buffer with ONE atomic per tile, in
//     ascending order inside the tile. A second pass (dgrep_order_lines)
//     turns tile-relative line numbers into global ones and lays the tiles out
//     in split order.
#include <hip/hip_runtime.h>

#include "scan_common.h"

namespace dgrep {

__device__ __forceinline__ uint32_t nl_mask(uint32_t w) {
  // exact per-byte zero test of w ^ '\n\n\n\n': bit 7 of byte k set iff byte k == '\n'
  uint32_t x = w ^ 0x0a0a0a0au;
  uint32_t t = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;
  return ~t & 0x80808080u;
}
__device__ __forceinline__ uint32_t hi_byte(uint32_t m) { return (31u - __clz(m)) >> 3; }

// Per-lane run state. `pos` and every position below are relative to the
// lane's chunk start `cs`.
struct LaneRun {
  uint32_t s;        // DFA state
  uint32_t nl;       // '\n' bytes consumed so far
  int64_t prev_nl;   // position of the last consumed '\n' (-1: none / split start)
  bool seen;         // a line boundary has been crossed (owned lines begin)
  bool term;         // the terminating '\n' at or after the chunk end was consumed
  uint32_t nev;      // matching lines emitted
};

template <int C, int E, bool DIRECT>
struct Emitter {
  const ScanArgs* a;
  uint32_t* slots;       // LDS [E][3] of this lane (slot mode)
  uint64_t cs;
  uint64_t out_base;     // first staging index of this lane (direct mode)
  uint32_t nl_prefix;    // '\n' between tile start and chunk start (direct mode)

  __device__ __forceinline__ void operator()(LaneRun& r, uint64_t q, int64_t start, uint32_t rel) const {
    uint64_t len = q - uint64_t(start);
    if (DIRECT) {
      uint64_t o = out_base + r.nev;
      if (o < a->capacity) {
        StagedLine L;
        L.start = cs + uint64_t(start);
        L.len = uint32_t(len);
        L.rel = nl_prefix + rel;
        a->staging[o] = L;
      }
    } else if (r.nev < uint32_t(E)) {
      slots[r.nev * 3 + 0] = uint32_t(start);
      slots[r.nev * 3 + 1] = uint32_t(len);
      slots[r.nev * 3 + 2] = rel;
    }
    if (len > 0xffffffffull || q > 0xffffffffull) atomicOr(a->status, kStatusLineTooLong);
    ++r.nev;
  }
};

// Runs one lane (see file comment). Returns the number of '\n' inside the
// lane's own chunk [cs, cs + C).
template <int C, int E, bool DIRECT>
__device__ uint32_t run_lane(const ScanArgs& a, const uint8_t* __restrict__ tbl, uint64_t cs, LaneRun& r,
                             const Emitter<C, E, DIRECT>& emit) {
  const uint32_t M = a.start_m;
  const uint64_t avail = cs < a.n ? a.n - cs : 0;
  r.s = a.start;
  r.nl = 0;
  r.prev_nl = -1;
  r.seen = (cs == 0);
  r.term = false;
  r.nev = 0;
  if (avail == 0) return 0;
  const uint8_t* __restrict__ p = a.data + cs;
  uint32_t nl_chunk = 0;
  bool snap = false;
  uint64_t pos = 0;
  for (;;) {
    if (pos == uint64_t(C)) { nl_chunk = r.nl; snap = true; }
    if (pos >= uint64_t(C) && r.term) break;
    if (pos + 64 <= avail) {
      const uint4* b = reinterpret_cast<const uint4*>(p + pos);
      const uint4 v0 = b[0], v1 = b[1], v2 = b[2], v3 = b[3];
      const uint32_t w[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                              v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
      const bool past = pos >= uint64_t(C);
      uint32_t s = r.s;
      // block-entry bookkeeping; per word we only track the last word with a '\n'
      const uint32_t nl0 = r.nl;
      uint32_t nlrun = 0;
      uint32_t lastm = 0;
      int lastj = -1;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint32_t x = w[j];
        const uint32_t m = nl_mask(x);
        const uint32_t s0 = tbl[__builtin_amdgcn_perm(s, x, 0x0c0c0400u)];
        const uint32_t s1 = tbl[__builtin_amdgcn_perm(s0, x, 0x0c0c0401u)];
        const uint32_t s2 = tbl[__builtin_amdgcn_perm(s1, x, 0x0c0c0402u)];
        const uint32_t s3 = tbl[__builtin_amdgcn_perm(s2, x, 0x0c0c0403u)];
        if (__builtin_expect((s0 == M) | (s1 == M) | (s2 == M) | (s3 == M), 0)) {
          // a '\n' in this word ends a matching line: resolve exactly
          const uint64_t q0 = pos + 4u * uint32_t(j);
          const bool seen_w = r.seen || lastm != 0;
          const bool term_w = r.term || (past && lastm != 0);
          const int64_t prev_w = lastm ? int64_t(pos + 4u * uint32_t(lastj) + hi_byte(lastm)) : r.prev_nl;
          const uint32_t st[4] = {s0, s1, s2, s3};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (st[k] != M) continue;
            const uint32_t below = m & ((1u << (8 * k)) - 1u);
            bool ok = seen_w || below != 0;
            if (past) ok = ok && !term_w && below == 0;
            if (!ok) continue;
            const int64_t start = below ? int64_t(q0 + hi_byte(below)) + 1 : prev_w + 1;
            emit(r, q0 + uint32_t(k), start, nl0 + nlrun + uint32_t(__popc(below)));
          }
        }
        nlrun += uint32_t(__popc(m));
        if (m) { lastm = m; lastj = j; }
        s = s3;
      }
      r.s = s;
      r.nl = nl0 + nlrun;
      if (lastm) {
        r.seen = true;
        r.prev_nl = int64_t(pos + 4u * uint32_t(lastj) + hi_byte(lastm));
        if (past) r.term = true;
      }
      pos += 64;
    } else {
      // tail of the split: byte at a time up to the end
      for (; pos < avail; ++pos) {
        if (pos == uint64_t(C)) { nl_chunk = r.nl; snap = true; }
        if (pos >= uint64_t(C) && r.term) break;
        const uint32_t b = p[pos];
        const uint32_t s1 = tbl[(r.s << 8) | b];
        if (b == '\n') {
          if (s1 == M && r.seen && !(pos >= uint64_t(C) && r.term)) emit(r, pos, r.prev_nl + 1, r.nl);
          r.seen = true;
          ++r.nl;
          r.prev_nl = int64_t(pos);
          if (pos >= uint64_t(C)) r.term = true;
        }
        r.s = s1;
      }
      if (!r.term) {
        // end of the split ends the last owned line (strings.Split's final piece)
        if (r.seen && tbl[(r.s << 8) | uint32_t('\n')] == M) emit(r, avail, r.prev_nl + 1, r.nl);
      }
      break;
    }
  }
  if (!snap) nl_chunk = r.nl;
  return nl_chunk;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = int(threadIdx.x & 63);
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

template <int C, int E>
__global__ __launch_bounds__(kScanThreads) void scan_dfa8_kernel(ScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // [table (padded to 16)] [slots: 256 x E x 3 u32] [scan scratch]
  const uint32_t tpad = (a.table_bytes + 15u) & ~15u;
  uint8_t* tbl = smem;
  uint32_t* slots_all = reinterpret_cast<uint32_t*>(smem + tpad);
  uint32_t* scratch = slots_all + kScanThreads * E * 3;  // [0..3] nl wave sums, [4..7] ev wave sums, [8..9] base

  const int tid = int(threadIdx.x);
  for (uint32_t i = uint32_t(tid) * 16u; i < tpad; i += kScanThreads * 16u)
    *reinterpret_cast<uint4*>(tbl + i) = *reinterpret_cast<const uint4*>(a.table + i);
  __syncthreads();

  uint32_t* slots = slots_all + tid * E * 3;
  const int wave = tid >> 6;
  const int lane = tid & 63;

  for (uint64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    const uint64_t tile0 = t * uint64_t(kScanThreads) * uint64_t(C);
    const uint64_t cs = tile0 + uint64_t(tid) * uint64_t(C);
    LaneRun r;
    Emitter<C, E, false> em{&a, slots, cs, 0, 0};
    const uint32_t nlc = run_lane<C, E, false>(a, tbl, cs, r, em);
    const uint32_t nev = r.nev;

    // tile-wide exclusive scans of (newlines, matching lines)
    const uint32_t nl_inc = wave_incl_scan(nlc);
    const uint32_t ev_inc = wave_incl_scan(nev);
    if (lane == 63) {
      scratch[wave] = nl_inc;
      scratch[4 + wave] = ev_inc;
    }
    __syncthreads();
    uint32_t nl_off = nl_inc - nlc, ev_off = ev_inc - nev;
    uint32_t nl_tot = 0, ev_tot = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; ++w) {
      const uint32_t a_nl = scratch[w], a_ev = scratch[4 + w];
      if (w < wave) { nl_off += a_nl; ev_off += a_ev; }
      nl_tot += a_nl;
      ev_tot += a_ev;
    }
    if (tid == 0) {
      unsigned long long base = 0;
      if (ev_tot) base = atomicAdd(a.counter, (unsigned long long)ev_tot);
      TileInfo ti;
      ti.base = base;
      ti.count = ev_tot;
      ti.nl = nl_tot;
      a.tiles[t] = ti;
      scratch[8] = uint32_t(base);
      scratch[9] = uint32_t(base >> 32);
    }
    __syncthreads();
    if (ev_tot) {
      const uint64_t base = (uint64_t(scratch[9]) << 32) | scratch[8];
      const uint64_t o0 = base + ev_off;
      if (nev <= uint32_t(E)) {
        for (uint32_t k = 0; k < nev; ++k) {
          const uint64_t o = o0 + k;
          if (o < a.capacity) {
            StagedLine L;
            L.start = cs + slots[k * 3 + 0];
            L.len = slots[k * 3 + 1];
            L.rel = nl_off + slots[k * 3 + 2];
            a.staging[o] = L;
          }
        }
      } else {
        // this lane owned more matching lines than LDS slots: run it again
        // writing straight to its final staging positions
        LaneRun r2;
        Emitter<C, E, true> ed{&a, nullptr, cs, o0, nl_off};
        run_lane<C, E, true>(a, tbl, cs, r2, ed);
      }
    }
    __syncthreads();  // scratch/slots reuse by the next tile
  }
}

// Exclusive scans over the tiles (one workgroup): out_off = sum of counts of
// earlier tiles, line_base = 1 + newlines of earlier tiles.
__global__ __launch_bounds__(1024) void tile_scan_kernel(TileInfo* tiles, uint64_t ntiles, uint64_t* out_off,
                                                         uint64_t* line_base) {
  __shared__ uint64_t s_cnt[1024], s_nl[1024];
  const uint64_t per = (ntiles + 1023) / 1024;
  const uint64_t b = uint64_t(threadIdx.x) * per;
  const uint64_t e = b + per < ntiles ? b + per : ntiles;
  uint64_t c = 0, l = 0;
  for (uint64_t i = b; i < e; ++i) { c += tiles[i].count; l += tiles[i].nl; }
  s_cnt[threadIdx.x] = c;
  s_nl[threadIdx.x] = l;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    uint64_t tc = 0, tl = 0;
    if (int(threadIdx.x) >= d) { tc = s_cnt[threadIdx.x - d]; tl = s_nl[threadIdx.x - d]; }
    __syncthreads();
    s_cnt[threadIdx.x] += tc;
    s_nl[threadIdx.x] += tl;
    __syncthreads();
  }
  c = s_cnt[threadIdx.x] - c;
  l = s_nl[threadIdx.x] - l;
  for (uint64_t i = b; i < e; ++i) {
    out_off[i] = c;
    line_base[i] = l + 1;
    c += tiles[i].count;
    l += tiles[i].nl;
  }
  if (threadIdx.x == 1023) {
    out_off[ntiles] = s_cnt[1023];
    line_base[ntiles] = s_nl[1023] + 1;
  }
}

// Tile-ordered copy of the staged lines into the result arrays (SoA).
__global__ __launch_bounds__(256) void order_lines_kernel(const TileInfo* tiles, const StagedLine* staging,
                                                          uint64_t ntiles, const uint64_t* out_off,
                                                          const uint64_t* line_base, uint64_t capacity,
                                                          uint64_t* line_no, uint64_t* start, uint32_t* len) {
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const TileInfo ti = tiles[t];
    const uint64_t o = out_off[t], lb = line_base[t];
    for (uint32_t k = threadIdx.x; k < ti.count; k += blockDim.x) {
      const uint64_t src = ti.base + k, dst = o + k;
      if (src < capacity && dst < capacity) {
        const StagedLine L = staging[src];
        line_no[dst] = lb + L.rel;
        start[dst] = L.start;
        len[dst] = L.len;
      }
    }
  }
}

// ---- host-side launchers (called from dgrep_runtime.cpp) ----------------

template <int C, int E>
static hipError_t launch_scan_dfa8(const ScanArgs& a, int grid, hipStream_t stream) {
  const uint32_t tpad = (a.table_bytes + 15u) & ~15u;
  const size_t lds = tpad + size_t(kScanThreads) * E * 3 * 4 + 16 * 4;
  hipLaunchKernelGGL((scan_dfa8_kernel<C, E>), dim3(grid), dim3(kScanThreads), lds, stream, a);
  return hipGetLastError();
}

constexpr int kChunk = 1024;
constexpr int kSlots = 12;

uint64_t scan_tile_bytes() { return uint64_t(kScanThreads) * kChunk; }

size_t scan_dfa8_lds_bytes(uint32_t table_bytes) {
  return ((table_bytes + 15u) & ~15u) + size_t(kScanThreads) * kSlots * 3 * 4 + 16 * 4;
}

hipError_t scan_dfa8_occupancy(uint32_t table_bytes, int* blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, scan_dfa8_kernel<kChunk, kSlots>,
                                                      kScanThreads, scan_dfa8_lds_bytes(table_bytes));
}

hipError_t scan_dfa8(const ScanArgs& a, int grid, hipStream_t stream) {
  return launch_scan_dfa8<kChunk, kSlots>(a, grid, stream);
}

hipError_t tile_scan(TileInfo* tiles, uint64_t ntiles, uint64_t* out_off, uint64_t* line_base, hipStream_t stream) {
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, stream, tiles, ntiles, out_off, line_base);
  return hipGetLastError();
}

hipError_t order_lines(const TileInfo* tiles, const StagedLine* staging, uint64_t ntiles, const uint64_t* out_off,
                       const uint64_t* line_base, uint64_t capacity, uint64_t* line_no, uint64_t* start,
                       uint32_t* len, hipStream_t stream) {
  int grid = int(ntiles < 4096 ? ntiles : 4096);
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(order_lines_kernel, dim3(grid), dim3(256), 0, stream, tiles, staging, ntiles, out_off,
                     line_base, capacity, line_no, start, len);
  return hipGetLastError();
}

}  // namespace dgrep
