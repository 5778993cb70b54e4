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

// LDS row stride of the u8 transition table: 256 bytes + 4. Row s starts at
// s*260, so byte b of state s sits in bank (s + b/4) mod 32: lanes in
// different states that read the same input byte hit different banks.
constexpr uint32_t kRow = 260;

template <int TBL, int E>
struct ScanSmem {
  uint8_t tbl[TBL];  // first member: the table sits at LDS address 0
  uint32_t slots[kScanThreads * E * 2];
  uint32_t scratch[16];
};

__device__ __forceinline__ uint32_t dfa_step(const uint8_t* tbl, uint32_t s, uint32_t w, uint32_t sel) {
  // v_perm builds (s << 8) | byte(w); + 4s staggers the row: tbl[s*260 + byte]
  return tbl[__builtin_amdgcn_perm(s, w, sel) + (s << 2)];
}

// Per-lane run state. Positions are relative to the lane's chunk start `cs`.
struct LaneRun {
  uint32_t s;        // DFA state
  uint32_t nl;       // '\n' bytes consumed so far
  int64_t prev_nl;   // position of the last consumed '\n' (-1: none / split start)
  bool seen;         // a line boundary has been crossed (owned lines begin)
  bool term;         // the terminating '\n' at or after the chunk end was consumed
  uint32_t nev;      // matching lines emitted
};

template <int E, bool DIRECT>
struct Emitter {
  const ScanArgs* a;
  uint32_t* slots;       // LDS [E][2] of this lane (slot mode)
  uint64_t cs;
  uint64_t out_base;     // first staging index of this lane (direct mode)
  uint32_t nl_prefix;    // '\n' between tile start and chunk start (direct mode)

  __device__ __forceinline__ void operator()(LaneRun& r, uint64_t q, int64_t start, uint32_t rel) const {
    const uint64_t len = q - uint64_t(start);
    if (DIRECT) {
      const uint64_t o = out_base + r.nev;
      if (o < a->capacity) {
        StagedLine L;
        L.start = cs + uint64_t(start);
        L.len = uint32_t(len);
        L.rel = nl_prefix + rel;
        a->staging[o] = L;
      }
    } else if (r.nev < uint32_t(E)) {
      // start <= C and rel <= C fit 16 bits each
      slots[r.nev * 2 + 0] = uint32_t(start) | (rel << 16);
      slots[r.nev * 2 + 1] = uint32_t(len);
    }
    if (len > 0xffffffffull) atomicOr(a->status, kStatusLineTooLong);
    ++r.nev;
  }
};

// Block-local bookkeeping shared by the 16 word steps of one 64-byte block.
struct Blk {
  uint64_t pos;     // block start
  bool past;        // block lies at or beyond the chunk end
  uint32_t nl0;     // r.nl at block start
  uint32_t nlrun;   // '\n' in the words processed so far
  uint32_t lastm;   // newline mask of the last word with a '\n' (0: none yet)
  int lastj;        // its index
};

template <int J, int E, bool DIRECT>
__device__ __forceinline__ void word_step(const uint8_t* tbl, uint32_t M, uint32_t x, uint32_t& s, Blk& b,
                                          LaneRun& r, const Emitter<E, DIRECT>& emit) {
  // keep each word's work in place: hoisting the (chain-independent) newline
  // masks of a whole block ahead of the DFA chain costs ~100 VGPRs
  __builtin_amdgcn_sched_barrier(0);
  const uint32_t m = nl_mask(x);
  const uint32_t s0 = dfa_step(tbl, s, x, 0x0c0c0400u);
  const uint32_t s1 = dfa_step(tbl, s0, x, 0x0c0c0401u);
  const uint32_t s2 = dfa_step(tbl, s1, x, 0x0c0c0402u);
  const uint32_t s3 = dfa_step(tbl, s2, x, 0x0c0c0403u);
  if (__builtin_expect((s0 == M) | (s1 == M) | (s2 == M) | (s3 == M), 0)) {
    // a '\n' in this word ends a matching line: resolve it exactly
    const uint64_t q0 = b.pos + 4u * J;
    const bool seen_w = r.seen || b.lastm != 0;
    const bool term_w = r.term || (b.past && b.lastm != 0);
    const int64_t prev_w = b.lastm ? int64_t(b.pos + 4u * uint32_t(b.lastj) + hi_byte(b.lastm)) : r.prev_nl;
    uint32_t evm = uint32_t(s0 == M) | (uint32_t(s1 == M) << 1) | (uint32_t(s2 == M) << 2) | (uint32_t(s3 == M) << 3);
    while (evm) {
      const uint32_t k = uint32_t(__builtin_ctz(evm));
      evm &= evm - 1;
      const uint32_t below = m & ((1u << (8 * k)) - 1u);
      bool ok = seen_w || below != 0;
      if (b.past) ok = ok && !term_w && below == 0;  // only the first '\n' past the chunk end
      if (!ok) continue;
      const int64_t start = below ? int64_t(q0 + hi_byte(below)) + 1 : prev_w + 1;
      emit(r, q0 + k, start, b.nl0 + b.nlrun + uint32_t(__popc(below)));
    }
  }
  b.nlrun += uint32_t(__popc(m));
  if (m) { b.lastm = m; b.lastj = J; }
  s = s3;
}

template <int E, bool DIRECT>
__device__ __forceinline__ void run_block(const uint8_t* tbl, uint32_t M, const uint4 (&v)[4], uint64_t pos,
                                          uint64_t C, LaneRun& r, const Emitter<E, DIRECT>& emit) {
  Blk b;
  b.pos = pos;
  b.past = pos >= C;
  b.nl0 = r.nl;
  b.nlrun = 0;
  b.lastm = 0;
  b.lastj = -1;
  uint32_t s = r.s;
#define DG_W4(I)                                                           \
  word_step<4 * I + 0, E, DIRECT>(tbl, M, v[I].x, s, b, r, emit);          \
  word_step<4 * I + 1, E, DIRECT>(tbl, M, v[I].y, s, b, r, emit);          \
  word_step<4 * I + 2, E, DIRECT>(tbl, M, v[I].z, s, b, r, emit);          \
  word_step<4 * I + 3, E, DIRECT>(tbl, M, v[I].w, s, b, r, emit);
  DG_W4(0) DG_W4(1) DG_W4(2) DG_W4(3)
#undef DG_W4
  r.s = s;
  r.nl = b.nl0 + b.nlrun;
  if (b.lastm) {
    r.seen = true;
    r.prev_nl = int64_t(pos + 4u * uint32_t(b.lastj) + hi_byte(b.lastm));
    if (b.past) r.term = true;
  }
}

__device__ __forceinline__ void load_block(uint4 (&v)[4], const uint8_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = q[i];
}

// The last < 64 bytes of the split, one byte at a time, then the end of the
// split closes the last owned line (strings.Split's final piece).
template <int E, bool DIRECT>
__device__ __forceinline__ void run_tail(const uint8_t* tbl, uint32_t M, const uint8_t* p, uint64_t pos, uint64_t avail, uint64_t C,
                         LaneRun& r, uint32_t& nl_chunk, bool& snap, const Emitter<E, DIRECT>& emit) {
  for (; pos < avail; ++pos) {
    if (pos == C) { nl_chunk = r.nl; snap = true; }
    if (pos >= C && r.term) return;
    const uint32_t b = p[pos];
    const uint32_t s1 = tbl[r.s * kRow + b];
    if (b == '\n') {
      if (s1 == M && r.seen && !(pos >= C && r.term)) emit(r, pos, r.prev_nl + 1, r.nl);
      r.seen = true;
      ++r.nl;
      r.prev_nl = int64_t(pos);
      if (pos >= C) r.term = true;
    }
    r.s = s1;
  }
  if (!r.term && r.seen && tbl[r.s * kRow + uint32_t('\n')] == M) emit(r, avail, r.prev_nl + 1, r.nl);
}

// Runs one lane (see file comment) over 64-byte blocks, prefetching the next
// block while the current one is stepped (two register buffers, ping-pong).
// Returns the number of '\n' inside the lane's own chunk [cs, cs + C).
template <int C, int E, bool DIRECT>
__device__ __forceinline__ uint32_t run_lane(const ScanArgs& a, const uint8_t* tbl, uint64_t cs, LaneRun& r,
                                             const Emitter<E, DIRECT>& emit) {
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
  uint4 A[4], B[4];
  if (avail >= 64) load_block(A, p);
  for (;;) {
    if (pos == uint64_t(C)) { nl_chunk = r.nl; snap = true; }
    if (pos >= uint64_t(C) && r.term) break;
    if (pos + 64 > avail) { run_tail<E, DIRECT>(tbl, M, p, pos, avail, C, r, nl_chunk, snap, emit); break; }
    load_block(B, p + (pos + 128 <= avail ? pos + 64 : pos));  // prefetch (or a harmless re-read)
    run_block<E, DIRECT>(tbl, M, A, pos, C, r, emit);
    pos += 64;

    if (pos == uint64_t(C)) { nl_chunk = r.nl; snap = true; }
    if (pos >= uint64_t(C) && r.term) break;
    if (pos + 64 > avail) { run_tail<E, DIRECT>(tbl, M, p, pos, avail, C, r, nl_chunk, snap, emit); break; }
    load_block(A, p + (pos + 128 <= avail ? pos + 64 : pos));
    run_block<E, DIRECT>(tbl, M, B, pos, C, r, emit);
    pos += 64;
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

template <int C, int E, int TBL>
__global__ __launch_bounds__(kScanThreads) void scan_dfa8_kernel(ScanArgs a) {
  __shared__ ScanSmem<TBL, E> sm;
  const int tid = int(threadIdx.x);
  for (uint32_t i = uint32_t(tid) * 16u; i < a.table_bytes; i += kScanThreads * 16u)
    *reinterpret_cast<uint4*>(sm.tbl + i) = *reinterpret_cast<const uint4*>(a.table + i);
  __syncthreads();

  uint32_t* slots = sm.slots + tid * E * 2;
  uint32_t* scratch = sm.scratch;  // [0..3] nl wave sums, [4..7] match wave sums, [8..9] staging base
  const int wave = tid >> 6;
  const int lane = tid & 63;

  for (uint64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    const uint64_t tile0 = t * uint64_t(kScanThreads) * uint64_t(C);
    const uint64_t cs = tile0 + uint64_t(tid) * uint64_t(C);
    LaneRun r;
    Emitter<E, false> em{&a, slots, cs, 0, 0};
    const uint32_t nlc = run_lane<C, E, false>(a, sm.tbl, cs, r, em);
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
            const uint32_t w0 = slots[k * 2 + 0];
            StagedLine L;
            L.start = cs + (w0 & 0xffffu);
            L.len = slots[k * 2 + 1];
            L.rel = nl_off + (w0 >> 16);
            a.staging[o] = L;
          }
        }
      } else {
        // more matching lines than LDS slots: scan_overflow_kernel re-runs
        // this lane and writes straight to its final staging positions
        const unsigned long long k = atomicAdd(a.overflow_count, 1ull);
        if (k < a.overflow_cap) {
          OverflowLane ol;
          ol.cs = cs;
          ol.out_base = o0;
          ol.nl_prefix = nl_off;
          ol.pad = 0;
          a.overflow[k] = ol;
        }
      }
    }
    __syncthreads();  // scratch/slots reuse by the next tile
  }
}

// Lanes that owned more matching lines than their LDS slots: one thread per
// such lane runs it again in direct-write mode (rare: dense short matches).
template <int C, int E, int TBL>
__global__ __launch_bounds__(64) void scan_overflow_kernel(ScanArgs a, uint64_t nover) {
  __shared__ ScanSmem<TBL, 1> sm;
  for (uint32_t i = threadIdx.x * 16u; i < a.table_bytes; i += 64 * 16u)
    *reinterpret_cast<uint4*>(sm.tbl + i) = *reinterpret_cast<const uint4*>(a.table + i);
  __syncthreads();
  for (uint64_t k = uint64_t(blockIdx.x) * 64 + threadIdx.x; k < nover; k += uint64_t(gridDim.x) * 64) {
    const OverflowLane ol = a.overflow[k];
    LaneRun r;
    Emitter<E, true> ed{&a, nullptr, ol.cs, ol.out_base, ol.nl_prefix};
    run_lane<C, E, true>(a, sm.tbl, ol.cs, r, ed);
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

constexpr int kChunk = 1024;  // bytes per lane chunk (multiple of 128)
constexpr int kSlots = 8;     // LDS slots per lane for matching lines

uint64_t scan_tile_bytes() { return uint64_t(kScanThreads) * kChunk; }
uint32_t scan_table_row() { return kRow; }

namespace {
template <int TBL>
hipError_t launch_t(const ScanArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL((scan_dfa8_kernel<kChunk, kSlots, TBL>), dim3(grid), dim3(kScanThreads), 0, stream, a);
  return hipGetLastError();
}
template <int TBL>
hipError_t overflow_t(const ScanArgs& a, uint64_t nover, hipStream_t stream) {
  int grid = int((nover + 63) / 64);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL((scan_overflow_kernel<kChunk, kSlots, TBL>), dim3(grid), dim3(64), 0, stream, a, nover);
  return hipGetLastError();
}
template <int TBL>
hipError_t occ_t(int* b) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(b, scan_dfa8_kernel<kChunk, kSlots, TBL>, kScanThreads, 0);
}
}  // namespace

// variants by table size: up to 16, 32, 64, 128, 256 states
hipError_t scan_dfa8_occupancy(uint32_t table_bytes, int* b) {
  if (table_bytes <= 16 * kRow) return occ_t<16 * kRow>(b);
  if (table_bytes <= 32 * kRow) return occ_t<32 * kRow>(b);
  if (table_bytes <= 64 * kRow) return occ_t<64 * kRow>(b);
  if (table_bytes <= 128 * kRow) return occ_t<128 * kRow>(b);
  return occ_t<256 * kRow>(b);
}

hipError_t scan_dfa8(const ScanArgs& a, int grid, hipStream_t stream) {
  if (a.table_bytes <= 16 * kRow) return launch_t<16 * kRow>(a, grid, stream);
  if (a.table_bytes <= 32 * kRow) return launch_t<32 * kRow>(a, grid, stream);
  if (a.table_bytes <= 64 * kRow) return launch_t<64 * kRow>(a, grid, stream);
  if (a.table_bytes <= 128 * kRow) return launch_t<128 * kRow>(a, grid, stream);
  return launch_t<256 * kRow>(a, grid, stream);
}

hipError_t scan_dfa8_overflow(const ScanArgs& a, uint64_t nover, hipStream_t stream) {
  if (a.table_bytes <= 16 * kRow) return overflow_t<16 * kRow>(a, nover, stream);
  if (a.table_bytes <= 32 * kRow) return overflow_t<32 * kRow>(a, nover, stream);
  if (a.table_bytes <= 64 * kRow) return overflow_t<64 * kRow>(a, nover, stream);
  if (a.table_bytes <= 128 * kRow) return overflow_t<128 * kRow>(a, nover, stream);
  return overflow_t<256 * kRow>(a, nover, stream);
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
