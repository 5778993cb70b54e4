// dgrep_runtime.hip — device contexts, DFA upload, split scanning (C ABI).
//
// This is the native runtime under the grep plugin's Map (application/grep.go:13-36):
// dgrep_scan replaces the strings.Split + per-line regexp.Match loop
// (grep.go:17-29) for one split. Everything here is fail-stop: a HIP error is
// returned as DGREP_E_HIP with its message in dgrep_last_error; there is no
// CPU fallback path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "../../../include/dgrep.h"
#include "../../../include/dgrep_blob.h"
#include "../kernels/encode.h"
#include "../kernels/reduce.h"
#include "../kernels/scan_common.h"
#include "../kernels/synth.h"

// DFAs of at most this many states use the Sheng stepper (8 = its limit; 0
// sends every DFA of <= 256 states to the table stepper)
#ifndef DGREP_SHENG_MAX_STATES
#define DGREP_SHENG_MAX_STATES 8
#endif
// DFAs above the Sheng limit whose two-byte table fits in LDS use the pair
// stepper (0: they use the u8 table stepper)
#ifndef DGREP_PAIR_ENABLE
#define DGREP_PAIR_ENABLE 1
#endif
// matching-line records per resident thread of the HBM spill area the
// one-chunk-per-lane steppers move full LDS slots to (0: no spilling)
#ifndef DGREP_SPILL_RECORDS
#define DGREP_SPILL_RECORDS 240
#endif
// A/B knobs (shipped: 1, 1): park long lines at all (0: a lane reads its last
// line to its end), and the Sheng stepper's chunk maps (0: Sheng parks at 2 C
// and resolves through the per-chunk '\n' counts like the other steppers)
#ifndef DGREP_PARK
#define DGREP_PARK 1
#endif
// A/B knob: cap on the scan's resident workgroups per CU (the grid)
#ifndef DGREP_MAX_WG_PER_CU
#define DGREP_MAX_WG_PER_CU 64
#endif
#ifndef DGREP_SHENG_MAPS
#define DGREP_SHENG_MAPS 1
#endif
namespace dgrep {
// scan_dfa.hip
uint64_t scan_tile_bytes(int kind, uint32_t table_bytes, uint64_t n, uint64_t resident_blocks, uint32_t force,
                         double density, uint32_t spill_per_lane, uint32_t* chunk, uint32_t* waves_per_block,
                         uint32_t* slots, uint32_t* threads, bool* spills);
uint32_t scan_table_row();
uint32_t scan_max_lane_chunk();
hipError_t scan_dfa_occupancy(int kind, uint32_t table_bytes, int* blocks_per_cu);
hipError_t scan_dfa(int kind, const ScanArgs& a, int grid, hipStream_t stream);
hipError_t scan_dfa_overflow(int kind, const ScanArgs& a, uint64_t nover, hipStream_t stream);
hipError_t order_lines(const TileInfo* tiles, const StagedLine* staging, uint64_t ntiles, uint64_t* out_off,
                       uint64_t* line_base, uint64_t staging_cap, uint64_t capacity, uint64_t* line_no,
                       uint64_t* start, uint64_t* len, hipStream_t stream);
hipError_t verify_candidates(const VerifyArgs& v, bool candidates, hipStream_t stream);
hipError_t long_lines_end(const LongArgs& la, hipStream_t stream);
hipError_t long_lines_resolve(const LongArgs& la, hipStream_t stream);
hipError_t long_lines_sheng(const LongArgs& la, hipStream_t stream);
hipError_t long_lines_dfa(const LongDfaArgs& la, bool u32, hipStream_t stream);
uint32_t long_lookback();
uint32_t long_dfa_hot_bytes();
uint32_t long_dfa_lds_bytes();
uint32_t long_guesses();
uint32_t long_seeds();
uint32_t verify_hot_bytes();
}  // namespace dgrep

using namespace dgrep;

constexpr size_t kCounters = 8;

// StepPair image offsets and thresholds (see StepPair in scan_dfa.hip)
struct PairArgs {
  uint32_t t1 = 0, thr = 0, div = 0, w32 = 0;
};

struct dgrep_ctx {
  int device = 0;
  int num_cus = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;

  // loaded pattern
  bool loaded = false;
  uint32_t flags = 0, nstates = 0, start = 0, start_m = 0;
  bool empty_line_matches = false;
  uint8_t* d_table = nullptr;  // stepper image (see dgrep_load_dfa)
  uint32_t table_bytes = 0;
  uint32_t nclasses = 0;
  // dgrep_set_stepper: force a stepper (0 auto, 2 u8 table, 3 pair, 4 filter) /
  // cap the filter stepper's LDS rows (tests, tuning)
  int force_stepper = 0;
  uint32_t filter_rows_cap = UINT32_MAX;
  uint32_t lane_chunk = 0;  // dgrep_set_lane_chunk (0 = adaptive)
  int step_kind = kStepTable;
  PairArgs pair_args;
  // kStepFilter: CAND_END (premultiplied), and the whole DFA for verify_kernel
  uint32_t cand_end = UINT32_MAX;
  void* d_full = nullptr;      // [nstates][nclasses], the blob's ids: u16, or u32 above 65535 states
  bool full_u32 = false;
  uint8_t* d_cls = nullptr;    // [256]
  uint32_t blob_start = 0, blob_start_m = 0;  // start / start_m in d_full's (breadth-first) ids
  uint32_t blob_matched = UINT32_MAX;          // the absorbing accepting state in d_full's ids (none: UINT32_MAX)
  uint32_t blob_dead = UINT32_MAX;             // the absorbing rejecting state (none: UINT32_MAX)
  std::vector<uint32_t> long_seed;             // lookback start states of long_dfa_seg1_kernel (d_full's ids)
  uint32_t verify_hot = 0;                     // leading entries of d_full verify_kernel keeps in LDS
  uint8_t* d_ximg = nullptr;                   // the whole-DFA LDS image (build_ximg; u16 DFAs that fit)
  uint32_t ximg_bytes = 0, x_hot = 0, x_rec = 0, xr_off = 0;
  uint32_t* d_nfa = nullptr;                   // DGREP_DFA_PARTIAL: the NFA program (verify_nfa_kernel)
  uint32_t nfa_words = 0;                      // its position-set words
  int blocks_per_cu = 1;

  // per-scan scratch (grown on demand, reused)
  TileInfo* d_tiles = nullptr;
  uint64_t* d_out_off = nullptr;
  uint64_t* d_line_base = nullptr;
  uint64_t tiles_cap = 0, off_cap = 0, lb_cap = 0;
  StagedLine* d_staging = nullptr;
  uint64_t staging_cap = 0;
  // device counters: [0] staging append counter, [1] overflow lanes, [2] parked
  // lines, [3] dropped candidates, [4] claimed tiles
  unsigned long long* d_counters = nullptr;
  OverflowLane* d_overflow = nullptr;
  uint64_t overflow_cap = 0;
  uint2* d_spill = nullptr;  // HBM spill areas of the resident threads (ScanArgs::spill)
  uint64_t spill_cap = 0;
  uint64_t* d_tails = nullptr;     // ScanArgs::tails (resident threads x streams)
  uint64_t tails_cap = 0;
  uint32_t* d_chunk_nl = nullptr;  // '\n' per chunk (ScanArgs::chunk_nl)
  uint64_t chunk_nl_cap = 0;
  ChunkMap* d_chunk_map = nullptr;  // Sheng: per-chunk maps (ScanArgs::chunk_map)
  uint64_t chunk_map_cap = 0;
  uint32_t sheng_nl_lo = 0, sheng_nl_hi = 0;  // Sheng: V['\n']
  PendingLine* d_pend = nullptr;   // parked long lines
  uint64_t pend_cap = 0;
  // long lines: the blob's u8 [S][256] table and stepper state -> blob state
  // (only for <= 256-state DFAs on the Sheng / pair / table steppers)
  uint8_t* d_long_tbl = nullptr;
  uint32_t* d_st2id = nullptr;
  uint32_t long_start_m = 0, long_states = 0;
  LongSeg* d_seg = nullptr;
  uint64_t seg_cap = 0;
  uint64_t* d_seg_off = nullptr;
  uint64_t seg_off_cap = 0;
  uint8_t* d_segmap = nullptr;
  uint64_t segmap_cap = 0;
  // filter stepper: parked lines on the whole DFA (long_dfa_* kernels)
  uint64_t* d_seg_from = nullptr;
  uint64_t seg_from_cap = 0;
  uint32_t* d_seg_state = nullptr;  // [2][guesses][nseg]: guesses, exits
  uint64_t seg_state_cap = 0;

  // dgrep_scan (host data) buffers
  uint8_t* d_data = nullptr;
  size_t data_cap = 0;
  uint64_t* d_res_line = nullptr;
  uint64_t* d_res_start = nullptr;
  uint64_t* d_res_len = nullptr;
  uint64_t res_cap = 0;

  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr, ev4 = nullptr, ev5 = nullptr;
  uint64_t staged_hint = 0;  // kStepFilter: staged lines (candidates included) of the last scan
  float last_ms = 0.f;
  double ms_sum = 0.0;  // last_ms summed over the dgrep_scan_device calls since dgrep_take_kernel_ms
  uint64_t ms_scans = 0;
  dgrep_scan_stats stats{};
  // matching lines per byte of the last scan of the loaded pattern (0 after
  // dgrep_load_dfa): caps the adaptive lane chunk (scan_tile_bytes)
  double density = 0.0;

  // dgrep_scan ingest (worker split -> HBM): host bytes are copied by
  // `ingest_threads` CPU threads into one of `ingest_bufs` pinned staging
  // buffers of `ingest_chunk` bytes while the copy engine DMAs the previous
  // one to HBM on `copy_stream` (dgrep_set_ingest; chunk 0 = one direct
  // pageable hipMemcpyAsync)
  size_t ingest_chunk = size_t(64) << 20;
  int ingest_bufs = 4;
  int ingest_threads = 4;
  std::vector<uint8_t*> h_stage;
  std::vector<hipEvent_t> ev_stage;
  size_t stage_bytes = 0;
  hipStream_t copy_stream = nullptr;
  float last_ingest_ms = 0.f;

  // partition + intermediate writer (dgrep_encode_device / dgrep_map_partitions)
  uint8_t* d_enc_scratch = nullptr;
  uint64_t enc_scratch_cap = 0;
  uint8_t* d_fname = nullptr;
  uint64_t fname_cap = 0;
  uint64_t* d_bounds = nullptr;
  uint64_t bounds_cap = 0;
  uint8_t* d_enc_out = nullptr;
  uint64_t enc_out_cap = 0;
  float last_encode_ms = 0.f;

  // reduce task (dgrep_reduce)
  uint8_t* d_red_scratch = nullptr;
  uint64_t red_scratch_cap = 0;
  uint8_t* d_red_out = nullptr;
  uint64_t red_out_cap = 0;
};

// the kind handed to the scan entry points: the stepper, with kKindW32 for the
// pair stepper's u32-entry image
static int launch_kind(const dgrep_ctx* c) {
  return c->step_kind | (c->step_kind == kStepPair && c->pair_args.w32 ? kKindW32 : 0);
}

namespace {

int hip_fail(dgrep_ctx* c, hipError_t e, const char* what) {
  c->err = std::string(what) + ": " + hipGetErrorString(e);
  return DGREP_E_HIP;
}
#define HIPCHK(expr)                                   \
  do {                                                 \
    hipError_t e_ = (expr);                            \
    if (e_ != hipSuccess) return hip_fail(c, e_, #expr); \
  } while (0)

template <class T>
int grow(dgrep_ctx* c, T** p, uint64_t* cap, uint64_t need) {
  if (*cap >= need && *p) return DGREP_OK;
  if (*p) HIPCHK(hipFree(*p));
  *p = nullptr;
  uint64_t n = std::max<uint64_t>(need, 1);
  HIPCHK(hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T)));
  *cap = n;
  return DGREP_OK;
}

// Host wait per scan (scan_resident): block on the scan kernel's end event,
// then poll the stream for the short tail (ordering passes, the 32-B count
// copy) for at most DGREP_SYNC_SPIN_US microseconds before a blocking wait.
// The poll holds one host core per rank busy for that tail (C3: ~0.16 ms per
// scan, C2: ~0.05 ms); the blocking wait alone returned tens of µs after the
// copy (profiles/r05/ablation/sync_spin.txt). 0: always the blocking wait.
#ifndef DGREP_SYNC_SPIN_US
#define DGREP_SYNC_SPIN_US 1000
#endif

// The LDS image through which long_dfa_seg1_kernel and verify_kernel read a
// whole u16 DFA F ([S][K], breadth-first ids) with no HBM access on the chain:
// rows [0, H) whole; then one DfaXRec (scan_common.h) for each state in
// [H, S) -- its default = the resident row differing from its own in the
// fewest classes (exhaustive, stopping at one difference; config 4: 30 ms),
// with the <= 2 differing classes as exceptions; a state no resident row
// comes within two classes of gets its own row after the first H (an EXTRA
// row, its record's default, no exceptions). Layout: rows (H + X) * K u16,
// records at *xr_off (8-aligned). H is the most rows that leave room for
// everything within `budget`; false if even 64 rows do not (the kernels then
// keep the first rows and read the rest from HBM).
#ifndef DGREP_LONG_XREC
#define DGREP_LONG_XREC 1
#endif
// verify_kernel on the same LDS image (one 1024-thread workgroup per CU)
#ifndef DGREP_VERIFY_XREC
#define DGREP_VERIFY_XREC 1
#endif
static bool build_ximg(const uint16_t* F, uint32_t S, uint32_t K, uint32_t budget, std::vector<uint8_t>* img,
                       uint32_t* hot, uint32_t* xr_off) {
  const uint64_t row = 2ull * K;
  if (K >= kXNone || row <= 8 || budget < 8ull * S + 64 * row + 8) return false;
  uint64_t H = std::min<uint64_t>(S, (budget - 8 - 8ull * S) / (row - 8));
  for (int attempt = 0; attempt < 8 && H >= 64; ++attempt) {
    const uint64_t R = S - H;
    std::vector<uint2> rec(R);
    std::vector<uint32_t> extra;
    for (uint64_t j = 0; j < R; ++j) {
      const uint16_t* f = F + (H + j) * K;
      uint32_t best = 3, bd = 0;
      for (uint64_t d = 0; d < H && best > 1; ++d) {
        const uint16_t* g = F + d * K;
        uint32_t diff = 0;
        for (uint32_t k = 0; k < K && diff < best; ++k) diff += f[k] != g[k];
        if (diff < best) { best = diff; bd = uint32_t(d); }
      }
      if (best > 2) {
        rec[j] = make_uint2(uint32_t(H + extra.size()) | (kXNone << 16) | (kXNone << 24), 0u);
        extra.push_back(uint32_t(H + j));
        continue;
      }
      uint32_t cl[2] = {kXNone, kXNone}, nx[2] = {0, 0}, e = 0;
      const uint16_t* g = F + uint64_t(bd) * K;
      for (uint32_t k = 0; k < K; ++k)
        if (f[k] != g[k]) { cl[e] = k; nx[e] = f[k]; ++e; }
      rec[j] = make_uint2(bd | (cl[0] << 16) | (cl[1] << 24), nx[0] | (nx[1] << 16));
    }
    const uint64_t off = ((H + extra.size()) * row + 7) & ~7ull, bytes = (off + 8 * R + 15) & ~15ull;
    if (bytes > budget || H + extra.size() > 0xffffu) {
      H -= std::min<uint64_t>(H, (bytes - budget) / (row - 8) + 1 + extra.size());
      continue;
    }
    img->assign(bytes, 0);
    memcpy(img->data(), F, H * row);
    for (size_t x = 0; x < extra.size(); ++x) memcpy(img->data() + (H + x) * row, F + uint64_t(extra[x]) * K, row);
    memcpy(img->data() + off, rec.data(), 8 * R);
    *hot = uint32_t(H);
    *xr_off = uint32_t(off);
    return true;
  }
  return false;
}

// The pair stepper's LDS image (StepPair, scan_dfa.hip) from the blob's DFA:
// C u8 [256] (byte -> esz class), T2 u32 (u16 if the image exceeds 16 KiB) [S'][K][K] at kPairT2 (two
// bytes per lookup), T1 u16 [S'][K] (single bytes); states premultiplied to
// their T2 row's LDS address (kPairT2 + id * 2K^2). S' = S + shadows: a pair whose FIRST byte is a '\n'
// entering start_m hides that event in the state between its bytes, so it
// leads to shadow(y) -- a copy of y = T[start_m][c2] -- instead of y. Ids:
// the states other than start_m, then the shadows of y != start_m, then
// start_m, then shadow(start_m): a pair-end id >= first shadow holds an
// event. Returns false if the DFA does not fit (T2 > kPairMaxT2 bytes).
bool build_pair_image(const dgrep_blob_header& h, const uint32_t* trans, std::vector<uint8_t>* img, uint32_t* start,
                      uint32_t* start_m, PairArgs* pa, std::vector<uint32_t>* orig_out) {
  const uint32_t S = h.nstates, K = h.nclasses, M = h.start_m;
  const uint32_t cn = h.byte_class[uint8_t('\n')];
  auto T = [&](uint32_t s, uint32_t c) { return trans[size_t(s) * K + c]; };
  // shadow targets, in class order
  std::vector<uint32_t> shadow_of(S, UINT32_MAX);  // original state -> shadow id
  std::vector<uint32_t> targets;
  bool any_flag = false;
  for (uint32_t s = 0; s < S; ++s) any_flag = any_flag || T(s, cn) == M;
  if (any_flag)
    for (uint32_t c = 0; c < K; ++c) {
      const uint32_t y = T(M, c);
      if (std::find(targets.begin(), targets.end(), y) == targets.end()) targets.push_back(y);
    }
  const uint32_t Sp = S + uint32_t(targets.size());
  // T2 entry: u32 when the image fits kPairW32MaxImage, else u16. Bytes per T2
  // row: esz K^2, padded to an ODD number of dwords so that the same column of
  // different rows falls in different LDS banks
  auto row_of = [&](uint64_t esz) { return ((esz * K * K + 3) & ~3ull) | 4ull; };
  auto end_of = [&](uint64_t r) {
    const uint64_t t1 = (kPairT2 + r * Sp + 15) & ~15ull;
    return std::make_pair(t1, (t1 + 2ull * Sp * K + 15) & ~15ull);
  };
  uint32_t esz = DGREP_PAIR_T2_U32 && end_of(row_of(4)).second <= kPairW32MaxImage ? 4u : 2u;
  const uint64_t row = row_of(esz);
  if (row * Sp > kPairMaxT2) return false;
  const uint64_t t1_off = end_of(row).first, end = end_of(row).second;
  if (end > kPairMaxImage) return false;
  std::vector<uint32_t> id(S), orig(Sp);
  uint32_t next = 0;
  for (uint32_t s = 0; s < S; ++s)
    if (s != M) { id[s] = next; orig[next++] = s; }
  const bool m_shadow = std::find(targets.begin(), targets.end(), M) != targets.end();
  for (uint32_t y : targets)
    if (y != M) { shadow_of[y] = next; orig[next++] = y; }
  id[M] = next;
  orig[next++] = M;
  if (m_shadow) { shadow_of[M] = next; orig[next++] = M; }
  // ids S-1 .. S'-1: the shadows of y != start_m, start_m, shadow(start_m)
  const uint32_t thr_id = S - 1;
  auto premul = [&](uint32_t i) { return uint16_t(kPairT2 + uint64_t(i) * row); };
  img->assign(end, 0);
  uint8_t* const t2 = img->data() + kPairT2;
  uint16_t* t1 = reinterpret_cast<uint16_t*>(img->data() + t1_off);
  for (uint32_t i = 0; i < Sp; ++i) {
    const uint32_t x = orig[i];
    for (uint32_t c1 = 0; c1 < K; ++c1) {
      const uint32_t a = T(x, c1);
      const bool flagged = c1 == cn && a == M;
      t1[size_t(i) * K + c1] = premul(id[a]);
      for (uint32_t c2 = 0; c2 < K; ++c2) {
        const uint32_t y = T(a, c2);
        const uint16_t v = premul(flagged ? shadow_of[y] : id[y]);
        uint8_t* const e = t2 + size_t(i) * row + esz * (size_t(c1) * K + c2);
        if (esz == 4) {
          const uint32_t v32 = v;
          memcpy(e, &v32, 4);
        } else {
          memcpy(e, &v, 2);
        }
      }
    }
  }
  // one u8 table C[b] = esz class(b) at LDS 0; esz (K - 1) < 256; and (for
  // the pair's first byte) CK[b] = esz K class(b), u16 at kPairCK
  if (esz * (K - 1u) > 255u) return false;
  for (int b = 0; b < 256; ++b) {
    img->data()[b] = uint8_t(esz * h.byte_class[b]);
    const uint16_t ck = uint16_t(esz * K * h.byte_class[b]);
    memcpy(img->data() + kPairCK + 2 * b, &ck, 2);
  }
  *start = premul(id[h.start]);
  *start_m = premul(id[M]);
  *orig_out = orig;  // pair state index -> blob state (a shadow -> the state it copies)
  pa->t1 = uint32_t(t1_off);
  pa->thr = premul(thr_id);
  pa->div = uint32_t(row);
  pa->w32 = esz == 4 ? 1u : 0u;
  return true;
}

#ifndef DGREP_FILTER_PITCH
#define DGREP_FILTER_PITCH 1
#endif
// The filter stepper's LDS image (StepFilter, scan_dfa.hip): byte classes (kFilterClassBytes),
// then u16 rows of the DFA's first
// R - 2 states in breadth-first order from start (start_m at depth 0), as many
// rows as kFilterImageBytes holds, plus CAND (every transition out of them;
// '\n' -> CAND_END) and CAND_END (start's row). Ids: kept states other than
// start_m, CAND, start_m, CAND_END; entries premultiplied by K. Returns false
// if not even start, start_m and their successors fit.
// `excluded`: a partial blob's CAND state (never kept, so every transition
// into it is a filter CAND too).
bool build_filter_image(const dgrep_blob_header& h, const uint32_t* trans, uint32_t row_cap, std::vector<uint8_t>* img,
                        uint32_t* start, uint32_t* start_m, uint32_t* cand_end, uint32_t excluded = UINT32_MAX) {
  const uint32_t S = h.nstates, K = h.nclasses, M = h.start_m;
  const uint32_t cn = h.byte_class[uint8_t('\n')];
  // row pitch P >= K entries with P / 2 odd (DGREP_FILTER_PITCH): consecutive
  // rows start an odd number of dwords apart, so the rows a wave's lanes sit in
  // cover the 32 banks in turn (a CPU model of config 4's chain reads: 5.8 ->
  // 5.6 LDS cycles per read)
  const uint32_t P = DGREP_FILTER_PITCH ? ((K + 1) & ~1u) + (((K + 1) & 2u) ? 0u : 2u) : K;
  // rows that fit (row_cap: dgrep_set_stepper's test knob)
  const uint32_t R = std::min<uint32_t>((kFilterImageBytes - kFilterClassBytes) / (2 * P), row_cap);
  if (R < 4 || uint64_t(R) * P > 65535) return false;
  std::vector<uint32_t> order;
  std::vector<uint8_t> seen(S, 0);
  auto visit = [&](uint32_t x) {
    if (!seen[x] && x != excluded) { seen[x] = 1; order.push_back(x); }
  };
  visit(h.start);
  visit(M);
  for (size_t q = 0; q < order.size(); ++q)
    for (uint32_t k = 0; k < K; ++k) visit(trans[size_t(order[q]) * K + k]);
  const bool part = excluded != UINT32_MAX;
  const uint32_t keep = std::min<uint32_t>(uint32_t(order.size()), S <= R && !part ? S : R - 2);
  if (keep < 2) return false;
  std::vector<uint32_t> id(S, UINT32_MAX);
  uint32_t next = 0;
  for (uint32_t i = 0; i < keep; ++i)
    if (order[i] != M) id[order[i]] = next++;
  const bool exact = keep == S && !part;  // the whole DFA fits: no candidates
  const uint32_t CAND = exact ? UINT32_MAX : next++;
  id[M] = next++;
  const uint32_t CEND = exact ? UINT32_MAX : next++;
  const uint32_t Sf = next;
  auto to = [&](uint32_t x) { return uint16_t((id[x] == UINT32_MAX ? CAND : id[x]) * P); };
  img->assign((kFilterClassBytes + size_t(Sf) * P * 2 + 15) & ~size_t(15), 0);
  for (int b = 0; b < 256; ++b) img->data()[b] = h.byte_class[b];
  uint16_t* rows = reinterpret_cast<uint16_t*>(img->data() + kFilterClassBytes);
  for (uint32_t i = 0; i < keep; ++i) {
    const uint32_t x = order[i];
    for (uint32_t k = 0; k < K; ++k) rows[size_t(id[x]) * P + k] = to(trans[size_t(x) * K + k]);
  }
  if (!exact) {
    for (uint32_t k = 0; k < K; ++k) {
      rows[size_t(CAND) * P + k] = uint16_t((k == cn ? CEND : CAND) * P);
      rows[size_t(CEND) * P + k] = to(trans[size_t(h.start) * K + k]);
    }
  }
  *start = id[h.start] * P;
  *start_m = id[M] * P;
  *cand_end = exact ? UINT32_MAX : CEND * P;
  return true;
}

}  // namespace

extern "C" int dgrep_pick_device(int worker_id, int* device) {
  if (!device) return DGREP_E_INVALID;
  *device = -1;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return DGREP_E_HIP;
  long dev;
  if (const char* e = getenv("DGREP_DEVICE")) {
    char* end = nullptr;
    dev = strtol(e, &end, 10);
    if (!*e || *end || dev < 0) return DGREP_E_INVALID;
    if (dev >= count) return DGREP_E_HIP;
  } else {
    long id = worker_id;
    if (id < 0) {
      const char* w = getenv("DGREP_WORKER_ID");
      char* end = nullptr;
      id = w && *w ? strtol(w, &end, 10) : -1;
      if (id < 0 || (end && *end)) id = long(getpid());
    }
    dev = id % count;
  }
  *device = int(dev);
  return DGREP_OK;
}

extern "C" int dgrep_open(int device, dgrep_ctx** out) {
  if (!out) return DGREP_E_INVALID;
  *out = nullptr;
  dgrep_ctx* c = new dgrep_ctx();
  c->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&c->num_cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&c->ev0);
  if (e == hipSuccess) e = hipEventCreate(&c->ev1);
  if (e == hipSuccess) e = hipEventCreate(&c->ev2);
  if (e == hipSuccess) e = hipEventCreate(&c->ev3);
  if (e == hipSuccess) e = hipEventCreate(&c->ev4);
  if (e == hipSuccess) e = hipEventCreate(&c->ev5);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&c->d_counters), kCounters * sizeof(unsigned long long));
  if (e != hipSuccess) {
    // keep the context so the caller can read the message
    c->err = std::string("dgrep_open: ") + hipGetErrorString(e);
    *out = c;
    return DGREP_E_HIP;
  }
  c->stream = c->own_stream;
  *out = c;
  return DGREP_OK;
}

extern "C" void dgrep_close(dgrep_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void* bufs[] = {c->d_table, c->d_full, c->d_ximg, c->d_nfa, c->d_cls, c->d_spill, c->d_tails, c->d_chunk_nl, c->d_chunk_map,
                  c->d_pend, c->d_long_tbl, c->d_st2id, c->d_seg, c->d_seg_off, c->d_segmap, c->d_seg_from, c->d_seg_state, c->d_tiles, c->d_out_off, c->d_line_base, c->d_staging, c->d_counters,
                  c->d_overflow, c->d_data, c->d_res_line, c->d_res_start, c->d_res_len, c->d_enc_scratch,
                  c->d_fname, c->d_bounds, c->d_enc_out, c->d_red_scratch, c->d_red_out};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
  for (uint8_t* h : c->h_stage)
    if (h) (void)hipHostFree(h);
  for (hipEvent_t e : c->ev_stage)
    if (e) (void)hipEventDestroy(e);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev2) (void)hipEventDestroy(c->ev2);
  if (c->ev3) (void)hipEventDestroy(c->ev3);
  if (c->ev4) (void)hipEventDestroy(c->ev4);
  if (c->ev5) (void)hipEventDestroy(c->ev5);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
}

extern "C" const char* dgrep_last_error(dgrep_ctx* c) { return c ? c->err.c_str() : "null context"; }

// for exchange.hip (the communicator runs on its context's device and stream)
namespace dgrep {
int ctx_device(const dgrep_ctx* c) { return c->device; }
hipStream_t ctx_stream(const dgrep_ctx* c) { return c->stream; }
}  // namespace dgrep

extern "C" int dgrep_set_stream(dgrep_ctx* c, void* s) {
  if (!c) return DGREP_E_INVALID;
  c->stream = s ? static_cast<hipStream_t>(s) : c->own_stream;
  return DGREP_OK;
}

extern "C" int dgrep_set_lane_chunk(dgrep_ctx* c, uint32_t chunk_bytes) {
  if (!c) return DGREP_E_INVALID;
  if (chunk_bytes && (chunk_bytes % 128 || chunk_bytes < 4096 || chunk_bytes > scan_max_lane_chunk())) {
    c->err = "lane chunk must be 0 or a multiple of 128 in [4096, " + std::to_string(scan_max_lane_chunk()) + "]";
    return DGREP_E_INVALID;
  }
  c->lane_chunk = chunk_bytes;
  return DGREP_OK;
}

extern "C" int dgrep_set_stepper(dgrep_ctx* c, int force, uint32_t filter_rows) {
  // 1 (the r01 wide stepper) and 5 (the r05 word stepper) were removed in round 6
  if (!c || force < 0 || force > 4 || force == 1) return DGREP_E_INVALID;
  c->force_stepper = force;
  c->filter_rows_cap = filter_rows ? filter_rows : UINT32_MAX;
  return DGREP_OK;
}

extern "C" int dgrep_load_dfa(dgrep_ctx* c, const void* blob, size_t n) {
  if (!c) return DGREP_E_INVALID;
  dgrep_blob_info info;
  if (dgrep_blob_info_get(blob, n, &info) != DGREP_OK) {
    c->err = "dgrep_load_dfa: malformed blob";
    return DGREP_E_INVALID;
  }
  HIPCHK(hipSetDevice(c->device));
  dgrep_blob_header h;
  memcpy(&h, blob, sizeof h);
  const uint32_t* trans = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(blob) + sizeof h);
  for (size_t i = 0; i < size_t(h.nstates) * h.nclasses; ++i)
    if (trans[i] >= h.nstates) {
      c->err = "dgrep_load_dfa: transition out of range";
      return DGREP_E_INVALID;
    }
  // expand byte classes into the kernel's LDS image
  std::vector<uint8_t> t;
  uint32_t start = h.start, start_m = h.start_m;
  const int force = c->force_stepper;
  // a partial DFA (DGREP_DFA_PARTIAL) runs only as a filter: its last state is
  // CAND, and the NFA program after `trans` verifies the lines that reach it
  const bool partial = (h.flags & DGREP_DFA_PARTIAL) != 0;
  if (partial && force != 0 && force != 4) {
    c->err = "dgrep_load_dfa: a partial DFA (over the compiler's state budget) runs on the filter stepper only";
    return DGREP_E_UNSUPPORTED;
  }
  std::vector<uint8_t> pair_img;
  uint32_t pair_start = 0, pair_m = 0;
  std::vector<uint32_t> st2id;  // stepper state index -> blob state (long lines, see resolve_long_lines)
  const bool want_pair =
      !partial && ((force == 0 && h.nstates > DGREP_SHENG_MAX_STATES && DGREP_PAIR_ENABLE) || force == 3);
  const bool pair_ok = want_pair && build_pair_image(h, trans, &pair_img, &pair_start, &pair_m, &c->pair_args, &st2id);
  if (force == 3 && !pair_ok) {
    c->err = "dgrep_load_dfa: the pair stepper's two-byte table does not fit this DFA";
    return DGREP_E_UNSUPPORTED;
  }
  std::vector<uint8_t> filter_img;
  uint32_t f_start = 0, f_m = 0, f_cend = UINT32_MAX;
  const bool filter_ok = !pair_ok && ((force == 0 && (h.nstates > 256 || partial)) || force == 4) &&
                         build_filter_image(h, trans, c->filter_rows_cap, &filter_img, &f_start, &f_m, &f_cend,
                                            partial ? h.nstates - 1 : UINT32_MAX);
  if ((force == 4 || partial) && !filter_ok) {
    c->err = "dgrep_load_dfa: the filter stepper cannot hold this DFA's first states";
    return DGREP_E_UNSUPPORTED;
  }
  if (pair_ok) {
    c->step_kind = kStepPair;
    c->nclasses = h.nclasses;
    t.swap(pair_img);
    start = pair_start;
    start_m = pair_m;
  } else if (filter_ok) {
    c->step_kind = kStepFilter;
    c->nclasses = h.nclasses;
    c->cand_end = f_cend;
    t.swap(filter_img);
    start = f_start;
    start_m = f_m;
  }
  c->loaded = false;  // the previous pattern's verification tables go now
  if (c->d_nfa) HIPCHK(hipFree(c->d_nfa));
  c->d_nfa = nullptr;
  if (c->d_full) HIPCHK(hipFree(c->d_full));
  c->d_full = nullptr;
  if (c->d_ximg) HIPCHK(hipFree(c->d_ximg));
  c->d_ximg = nullptr;
  c->ximg_bytes = c->x_hot = c->x_rec = c->xr_off = 0;
  if (pair_ok) {
    // image built above
  } else if (filter_ok && partial) {
    const uint32_t* prog = trans + size_t(h.nstates) * h.nclasses;
    if (h.nfa_bytes < 32 || prog[0] != DGREP_NFA_MAGIC || prog[1] > DGREP_NFA_MAX_POS) {
      c->err = "dgrep_load_dfa: malformed NFA program";
      return DGREP_E_INVALID;
    }
    c->nfa_words = prog[2];
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&c->d_nfa), h.nfa_bytes));
    HIPCHK(hipMemcpy(c->d_nfa, prog, h.nfa_bytes, hipMemcpyHostToDevice));
  } else if (filter_ok) {
    // the whole DFA for verify_kernel, renumbered breadth-first from start
    // (start, start_m, then BFS) so its hot rows lead; u16 entries while the
    // ids fit, u32 above 65535 states (up to the compiler's budget)
    const uint32_t S = h.nstates, K = h.nclasses;
    std::vector<uint32_t> order, bid(S, UINT32_MAX);
    order.reserve(S);
    auto visit = [&](uint32_t x) {
      if (bid[x] == UINT32_MAX) { bid[x] = uint32_t(order.size()); order.push_back(x); }
    };
    visit(h.start);
    visit(h.start_m);
    for (size_t q = 0; q < order.size(); ++q)
      for (uint32_t k = 0; k < K; ++k) visit(trans[size_t(order[q]) * K + k]);
    for (uint32_t x = 0; x < S; ++x) visit(x);
    const size_t ne = size_t(S) * K;
    c->full_u32 = S > 65535;
    const size_t esz = c->full_u32 ? 4 : 2;
    std::vector<uint8_t> full(ne * esz);
    for (uint32_t n = 0; n < S; ++n)
      for (uint32_t k = 0; k < K; ++k) {
        const uint32_t x = bid[trans[size_t(order[n]) * K + k]];
        if (c->full_u32) reinterpret_cast<uint32_t*>(full.data())[size_t(n) * K + k] = x;
        else reinterpret_cast<uint16_t*>(full.data())[size_t(n) * K + k] = uint16_t(x);
      }
    HIPCHK(hipMalloc(&c->d_full, full.size()));
    HIPCHK(hipMemcpy(c->d_full, full.data(), full.size(), hipMemcpyHostToDevice));
    c->verify_hot = uint32_t(std::min<size_t>(ne, verify_hot_bytes() / esz)) / K * K;
    std::vector<uint8_t> ximg;
    if (!c->full_u32 &&
        build_ximg(reinterpret_cast<const uint16_t*>(full.data()), S, K, long_dfa_lds_bytes(), &ximg, &c->x_hot,
                   &c->xr_off)) {
      c->x_rec = S - c->x_hot;
      c->ximg_bytes = uint32_t(ximg.size());
      HIPCHK(hipMalloc(reinterpret_cast<void**>(&c->d_ximg), ximg.size()));
      HIPCHK(hipMemcpy(c->d_ximg, ximg.data(), ximg.size(), hipMemcpyHostToDevice));
    }
    if (!c->d_cls) HIPCHK(hipMalloc(reinterpret_cast<void**>(&c->d_cls), 256));
    HIPCHK(hipMemcpy(c->d_cls, h.byte_class, 256, hipMemcpyHostToDevice));
    c->blob_start = bid[h.start];
    c->blob_start_m = bid[h.start_m];
    // the absorbing states: MATCHED (every byte but '\n' loops, '\n' ->
    // start_m; verification stops there) and DEAD (the same with '\n' ->
    // start: a line there never matches)
    c->blob_matched = c->blob_dead = UINT32_MAX;
    const uint32_t cn = h.byte_class[uint8_t('\n')];
    for (uint32_t x = 0; x < S; ++x) {
      bool absorbing = true;
      for (uint32_t k = 0; k < K && absorbing; ++k)
        if (k != cn && trans[size_t(x) * K + k] != x) absorbing = false;
      if (!absorbing) continue;
      if (trans[size_t(x) * K + cn] == h.start_m && c->blob_matched == UINT32_MAX) c->blob_matched = bid[x];
      if (trans[size_t(x) * K + cn] == h.start && c->blob_dead == UINT32_MAX) c->blob_dead = bid[x];
    }
    // long lines' lookback seeds: start, then states spread over the first
    // breadth-first ids -- the rows the seg kernel holds in LDS, so a seed's
    // first steps do not take the cold path -- never an absorbing one: a DFA
    // keeping a finite memory of the whole line (a parity, a flag) has seeds
    // in each memory class with high probability, so a segment's guesses cover
    // its true entry state (long_c4p: 4.7 -> 485 GB/s)
    const uint32_t NS = long_seeds();
    const uint32_t H = std::min<uint32_t>(S, std::max<uint32_t>(
                                                 64, c->x_hot ? c->x_hot : long_dfa_hot_bytes() / (esz * K)));
    c->long_seed.assign(NS, c->blob_start);
    for (uint32_t i = 1; i < NS && H > 2; ++i) {
      uint32_t x = uint32_t(uint64_t(i) * (H - 1) / NS);
      for (uint32_t t = 0; t < S && (x == c->blob_matched || x == c->blob_dead || x == c->blob_start); ++t)
        x = (x + 1) % S;
      c->long_seed[i] = x;
    }
  } else if (h.nstates > 256) {
    // the filter holds any DFA's first states (build_filter_image): only its
    // forced row cap (dgrep_set_stepper) can leave a large DFA here
    c->err = "dgrep_load_dfa: a DFA of " + std::to_string(h.nstates) + " states needs the filter stepper";
    return DGREP_E_UNSUPPORTED;
  } else if (h.nstates <= DGREP_SHENG_MAX_STATES && force != 2) {
    // StepSheng8: V[b] = 8 bytes, byte s = next state of s on input byte b
    c->step_kind = kStepSheng8;
    // renumber so start_m is the highest state (the kernel tests a word's four
    // states for start_m with one max), and carry the start state replicated
    // in all four bytes: v_perm keeps a replicated selector replicated, so
    // every state on the chain is a clean 0x01010101 multiple
    const uint32_t S = h.nstates, top = S - 1;
    std::vector<uint32_t> id(S);
    for (uint32_t x = 0; x < S; ++x) id[x] = x;
    std::swap(id[h.start_m], id[top]);
    t.assign(256 * 8, 0);
    for (int b = 0; b < 256; ++b)
      for (uint32_t s = 0; s < S; ++s)
        t[size_t(b) * 8 + id[s]] = uint8_t(id[trans[size_t(s) * h.nclasses + h.byte_class[b]]]);
    start = id[h.start] * 0x01010101u;
    // V['\n'] for the long-line kernel (a line the split's end closes)
    c->sheng_nl_lo = c->sheng_nl_hi = 0;
    for (int k = 0; k < 4; ++k) {
      c->sheng_nl_lo |= uint32_t(t[size_t('\n') * 8 + k]) << (8 * k);
      c->sheng_nl_hi |= uint32_t(t[size_t('\n') * 8 + 4 + k]) << (8 * k);
    }
    start_m = top;
    st2id.assign(S, 0);
    for (uint32_t x = 0; x < S; ++x) st2id[id[x]] = x;
  } else {
    // StepTable: row s (stride scan_table_row() = 260, bank-staggered) holds
    // trans[s][class(b)] at byte b
    c->step_kind = kStepTable;
    st2id.resize(h.nstates);
    for (uint32_t x = 0; x < h.nstates; ++x) st2id[x] = x;
    const size_t row = scan_table_row();
    t.assign((size_t(h.nstates) * row + 15) & ~size_t(15), 0);
    for (uint32_t s = 0; s < h.nstates; ++s)
      for (int b = 0; b < 256; ++b) t[size_t(s) * row + size_t(b)] = uint8_t(trans[size_t(s) * h.nclasses + h.byte_class[b]]);
  }
  if (c->d_table) HIPCHK(hipFree(c->d_table));
  c->d_table = nullptr;
  c->table_bytes = uint32_t(t.size());
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&c->d_table), (t.size() + 15) & ~size_t(15)));
  HIPCHK(hipMemcpy(c->d_table, t.data(), t.size(), hipMemcpyHostToDevice));
  c->flags = h.flags;
  c->nstates = h.nstates;
  c->start = start;
  c->start_m = start_m;
  // long lines: the blob's u8 [S][256] table for the long-line kernels
  if (c->d_long_tbl) HIPCHK(hipFree(c->d_long_tbl));
  if (c->d_st2id) HIPCHK(hipFree(c->d_st2id));
  c->d_long_tbl = nullptr;
  c->d_st2id = nullptr;
  c->long_states = 0;
  if ((c->step_kind == kStepSheng8 || c->step_kind == kStepPair || c->step_kind == kStepTable) &&
      h.nstates <= 256 &&
      !st2id.empty()) {
    std::vector<uint8_t> lt(size_t(h.nstates) * 256);
    for (uint32_t s = 0; s < h.nstates; ++s)
      for (int b = 0; b < 256; ++b) lt[size_t(s) * 256 + b] = uint8_t(trans[size_t(s) * h.nclasses + h.byte_class[b]]);
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&c->d_long_tbl), lt.size()));
    HIPCHK(hipMemcpy(c->d_long_tbl, lt.data(), lt.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&c->d_st2id), st2id.size() * 4));
    HIPCHK(hipMemcpy(c->d_st2id, st2id.data(), st2id.size() * 4, hipMemcpyHostToDevice));
    c->long_states = h.nstates;
    c->long_start_m = h.start_m;
  }
  c->empty_line_matches = trans[size_t(h.start) * h.nclasses + h.byte_class[uint8_t('\n')]] == h.start_m;
  int bpc = 0;
  HIPCHK(scan_dfa_occupancy(launch_kind(c), c->table_bytes, &bpc));
  c->blocks_per_cu = std::max(1, std::min(bpc, DGREP_MAX_WG_PER_CU));
  c->density = 0.0;
  c->staged_hint = 0;
  c->loaded = true;
  return DGREP_OK;
}

// The lines the scan parked (npend > 0): their ends, then their segments'
// maps, then each line's verdict and length (long_* kernels in scan_dfa.hip).
// The segment cut is made on the host from the ends (one small readback).
static int resolve_long_lines(dgrep_ctx* c, const uint8_t* d_data, uint64_t n, uint64_t chunk, uint64_t nchunks,
                              uint64_t npend) {
  int rc;
  LongArgs la;
  memset(&la, 0, sizeof la);
  la.data = d_data;
  la.n = n;
  la.chunk = chunk;
  la.nchunks = nchunks;
  la.chunk_nl = c->d_chunk_nl;
  la.pend = c->d_pend;
  la.npend = npend;
  la.st2id = c->d_st2id;
  la.tbl = c->d_long_tbl;
  la.nstates = c->long_states;
  la.start_m = c->long_start_m;
  HIPCHK(long_lines_end(la, c->stream));
  std::vector<PendingLine> P(npend);
  HIPCHK(hipMemcpyAsync(P.data(), c->d_pend, npend * sizeof(PendingLine), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  // segments of about 1/4096 of the parked bytes (so the GPU fills), at least
  // 256 KiB (a wave's 64 pieces of 4 KiB) and 64-B aligned
  uint64_t total = 0;
  for (const PendingLine& p : P) total += p.end > p.resume ? p.end - p.resume : 0;
  uint64_t seg = std::max<uint64_t>(uint64_t(256) << 10, (total / 4096 + 63) & ~uint64_t(63));
  std::vector<LongSeg> segs;
  std::vector<uint64_t> off(npend + 1, 0);
  for (uint64_t i = 0; i < npend; ++i) {
    for (uint64_t b = P[i].resume; b < P[i].end; b += seg) segs.push_back(LongSeg{b, std::min(P[i].end, b + seg)});
    off[i + 1] = segs.size();
  }
  if ((rc = grow(c, &c->d_seg, &c->seg_cap, std::max<uint64_t>(segs.size(), 1))) != DGREP_OK) return rc;
  if ((rc = grow(c, &c->d_seg_off, &c->seg_off_cap, npend + 1)) != DGREP_OK) return rc;
  if ((rc = grow(c, &c->d_segmap, &c->segmap_cap, std::max<uint64_t>(segs.size(), 1) * 256)) != DGREP_OK) return rc;
  if (!segs.empty())
    HIPCHK(hipMemcpyAsync(c->d_seg, segs.data(), segs.size() * sizeof(LongSeg), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_seg_off, off.data(), off.size() * 8, hipMemcpyHostToDevice, c->stream));
  la.seg = c->d_seg;
  la.nseg = segs.size();
  la.seg_off = c->d_seg_off;
  la.segmap = c->d_segmap;
  HIPCHK(long_lines_resolve(la, c->stream));
  // the host vectors are read by the async copies above: wait before they go
  HIPCHK(hipStreamSynchronize(c->stream));
  return DGREP_OK;
}

// The filter stepper's parked lines (> 256 states): their ends from the chunk
// '\n' counts, then each line decided on the whole DFA from its start, in
// segments run in parallel from guessed entry states and checked in order
// (long_dfa_* kernels in scan_dfa.hip). Segments sized so that every resident
// lane gets about four (two at a time, stepped in lockstep), >= 16 KiB.
static int resolve_long_filter(dgrep_ctx* c, const uint8_t* d_data, uint64_t n, uint64_t chunk, uint64_t nchunks,
                               uint64_t npend) {
  int rc;
  LongArgs le;
  memset(&le, 0, sizeof le);
  le.data = d_data;
  le.n = n;
  le.chunk = chunk;
  le.nchunks = nchunks;
  le.chunk_nl = c->d_chunk_nl;
  le.pend = c->d_pend;
  le.npend = npend;
  HIPCHK(long_lines_end(le, c->stream));
  std::vector<PendingLine> P(npend);
  HIPCHK(hipMemcpyAsync(P.data(), c->d_pend, npend * sizeof(PendingLine), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  uint64_t total = 0;
  for (const PendingLine& p : P) total += p.end - p.line_start;
  // one segment per lane of ONE round of long_dfa_seg1_kernel (one
  // 1024-thread workgroup per CU): a second, partly filled round held half the
  // CUs idle for a whole segment (long_c4: 384 workgroups over 256 CUs). Each
  // line adds at most one partial segment, hence the npend in the divisor.
  // >= 16 KiB.
  const uint64_t lanes2 = uint64_t(c->num_cus) * 1024;
  const uint64_t div = npend < lanes2 / 2 ? lanes2 - npend : uint64_t(c->num_cus) * 1536;
  const uint64_t seg = std::max<uint64_t>(uint64_t(16) << 10, (total / div + 16) & ~uint64_t(15));
  std::vector<LongSeg> segs;
  std::vector<uint64_t> from, off(npend + 1, 0);
  const uint64_t lb = long_lookback();
  for (uint64_t i = 0; i < npend; ++i) {
    for (uint64_t b = P[i].line_start; b < P[i].end; b += seg) {
      segs.push_back(LongSeg{b, std::min(P[i].end, b + seg)});
      from.push_back(b - std::min(lb, b - P[i].line_start));
    }
    off[i + 1] = segs.size();
  }
  const uint64_t ns = std::max<uint64_t>(segs.size(), 1);
  if ((rc = grow(c, &c->d_seg, &c->seg_cap, ns)) != DGREP_OK) return rc;
  if ((rc = grow(c, &c->d_seg_from, &c->seg_from_cap, ns)) != DGREP_OK) return rc;
  const uint64_t ng = long_guesses();
  if ((rc = grow(c, &c->d_seg_state, &c->seg_state_cap, 2 * ng * ns)) != DGREP_OK) return rc;
  if ((rc = grow(c, &c->d_seg_off, &c->seg_off_cap, npend + 1)) != DGREP_OK) return rc;
  if (!segs.empty()) {
    HIPCHK(hipMemcpyAsync(c->d_seg, segs.data(), segs.size() * sizeof(LongSeg), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_seg_from, from.data(), from.size() * 8, hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(hipMemcpyAsync(c->d_seg_off, off.data(), off.size() * 8, hipMemcpyHostToDevice, c->stream));
  LongDfaArgs la;
  memset(&la, 0, sizeof la);
  la.data = d_data;
  la.full = c->d_full;
  la.hot_entries = c->verify_hot;
  {
    const size_t esz = c->full_u32 ? 4 : 2, ne = size_t(c->nstates) * c->nclasses;
    la.seg_hot_entries = uint32_t(std::min<size_t>(ne, long_dfa_hot_bytes() / esz)) / c->nclasses * c->nclasses;
  }
  la.nclasses = c->nclasses;
  la.cls = c->d_cls;
  la.start = c->blob_start;
  la.start_m = c->blob_start_m;
  la.matched = c->blob_matched;
  la.dead = c->blob_dead;
  for (uint32_t i = 0; i < long_seeds() && i < uint32_t(kLongSeeds); ++i) la.seed[i] = c->long_seed[i];
  la.seg = c->d_seg;
  la.seg_from = c->d_seg_from;
  la.nseg = segs.size();
  la.seg_guess = c->d_seg_state;
  la.seg_exit = c->d_seg_state + ng * ns;
  la.seg_off = c->d_seg_off;
  la.pend = c->d_pend;
  la.npend = npend;
  la.ximg = DGREP_LONG_XREC ? c->d_ximg : nullptr;
  la.ximg_bytes = c->ximg_bytes;
  la.x_hot = c->x_hot;
  la.xr_off = c->xr_off;
  HIPCHK(long_lines_dfa(la, c->full_u32, c->stream));
  // the host vectors are read by the async copies above: wait before they go
  HIPCHK(hipStreamSynchronize(c->stream));
  return DGREP_OK;
}

// Core of every scan: the split is resident at d_data (n bytes). Results go to
// device arrays of `capacity` lines; *count receives the number of matches.
static int scan_resident(dgrep_ctx* c, const uint8_t* d_data, uint64_t n, uint64_t* d_line, uint64_t* d_start,
                         uint64_t* d_len, uint64_t capacity, uint64_t* count) {
  *count = 0;
  dgrep_scan_stats& S = c->stats;
  S = dgrep_scan_stats{};
  S.stepper = uint32_t(c->step_kind);
  c->last_ms = 0.f;
  if (c->flags & DGREP_DFA_MATCH_NONE) return DGREP_OK;
  if (n == 0) {
    // strings.Split("", "\n") == [""]: one empty line, line 1
    if (!c->empty_line_matches) return DGREP_OK;
    *count = 1;
    S.matches = 1;
    if (capacity >= 1) {
      const uint64_t one = 1, zero = 0;
      HIPCHK(hipMemcpyAsync(d_line, &one, 8, hipMemcpyHostToDevice, c->stream));
      HIPCHK(hipMemcpyAsync(d_start, &zero, 8, hipMemcpyHostToDevice, c->stream));
      HIPCHK(hipMemcpyAsync(d_len, &zero, 8, hipMemcpyHostToDevice, c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
    }
    return DGREP_OK;
  }
  if (reinterpret_cast<uintptr_t>(d_data) & 15) {
    c->err = "device split must be 16-byte aligned";
    return DGREP_E_INVALID;
  }
  const uint64_t resident = uint64_t(c->num_cus) * uint64_t(c->blocks_per_cu);
  uint32_t chunk = 0, wpb = 1, slots = 0, threads = 0;
  bool spills = false;
  const uint64_t tile = scan_tile_bytes(launch_kind(c), c->table_bytes, n, resident, c->lane_chunk, c->density,
                                        DGREP_SPILL_RECORDS, &chunk, &wpb, &slots, &threads, &spills);
  const uint64_t ntiles = (n + tile - 1) / tile;
  int rc;
  if ((rc = grow(c, &c->d_tiles, &c->tiles_cap, ntiles)) != DGREP_OK) return rc;
  if ((rc = grow(c, &c->d_out_off, &c->off_cap, ntiles + 1)) != DGREP_OK) return rc;
  if ((rc = grow(c, &c->d_line_base, &c->lb_cap, ntiles + 1)) != DGREP_OK) return rc;
  // kStepFilter stages its candidates too: the staging buffer holds at least
  // the previous scan's staged lines, and grows (one re-scan) if they overflow
  const bool filt = c->step_kind == kStepFilter && c->cand_end != UINT32_MAX;
  if ((rc = grow(c, &c->d_staging, &c->staging_cap, filt ? std::max(capacity, c->staged_hint) : capacity)) != DGREP_OK)
    return rc;

  if (!c->d_overflow && (rc = grow(c, &c->d_overflow, &c->overflow_cap, 1u << 16)) != DGREP_OK) return rc;
  const int grid = int(std::min<uint64_t>(ntiles, resident));
  // chunks per lane (the two-stream steppers step two in lockstep)
  const uint32_t streams = tile / (uint64_t(kTileLanes) * chunk);
  const bool use_spill = spills && DGREP_SPILL_RECORDS > 0;
  if (use_spill && (rc = grow(c, &c->d_spill, &c->spill_cap,
                              uint64_t(grid) * threads * streams * DGREP_SPILL_RECORDS)) != DGREP_OK)
    return rc;
  // long lines: the lanes' tail entries, '\n' per chunk and the pending list
  // (parking needs the blob's table: <= 256-state DFAs on the Sheng / pair /
  // table steppers)
  if ((rc = grow(c, &c->d_tails, &c->tails_cap, uint64_t(grid) * threads * streams)) != DGREP_OK) return rc;
  // the filter parks too when the whole DFA is at hand (not a partial blob, whose
  // candidates an NFA program decides: its lanes read a long line on)
  const bool park_filter = DGREP_PARK && c->step_kind == kStepFilter && c->d_full != nullptr;
  const bool park = (DGREP_PARK && c->d_long_tbl != nullptr) || park_filter;
  const uint64_t nchunks = (n + chunk - 1) / chunk;
  // Sheng: the chunk maps replace the '\n' counts (long_sheng_kernel)
  const bool park_maps = park && c->step_kind == kStepSheng8 && DGREP_SHENG_MAPS;
  if (park) {
    if (park_maps) {
      if ((rc = grow(c, &c->d_chunk_map, &c->chunk_map_cap, nchunks)) != DGREP_OK) return rc;
    } else if ((rc = grow(c, &c->d_chunk_nl, &c->chunk_nl_cap, nchunks)) != DGREP_OK) {
      return rc;
    }
    if (!c->d_pend && (rc = grow(c, &c->d_pend, &c->pend_cap, 1024)) != DGREP_OK) return rc;
  }

  ScanArgs a;
  memset(&a, 0, sizeof a);
  a.data = d_data;
  a.n = n;
  a.table = c->d_table;
  a.table_bytes = c->table_bytes;
  a.start = c->start;
  a.start_m = c->start_m;
  a.chunk = chunk;
  a.ntiles = ntiles;
  a.counter = c->d_counters;
  a.tiles = c->d_tiles;
  a.overflow_count = c->d_counters + 1;
  a.pend_count = c->d_counters + 2;
  a.tile_next = c->d_counters + 4;
  a.tails = c->d_tails;
  a.chunk_nl = park && !park_maps ? c->d_chunk_nl : nullptr;
  a.chunk_map = park_maps ? c->d_chunk_map : nullptr;
  a.nclasses = c->nclasses;
  a.pair_t1 = c->pair_args.t1;
  a.pair_thr = c->pair_args.thr;
  a.pair_div = c->pair_args.div;
  a.cand_end = c->cand_end;
  a.spill = use_spill ? c->d_spill : nullptr;
  a.spill_per_lane = use_spill ? DGREP_SPILL_RECORDS : 0;
  // every resident workgroup is launched even when the last round of tiles is
  // part-empty: trimming the grid so that every wave runs the same number of
  // tiles leaves some CUs with 2 workgroups and others with 3, and the time
  // follows the fullest CU (C2 16 KiB chunks: 4.13 TB/s trimmed, 4.74 full)
  (void)wpb;
  unsigned long long ctr[4] = {0, 0, 0, 0};
  S.lane_chunk = chunk;
  S.lane_slots = slots;
  S.tiles = ntiles;
  // The common case -- no overflowing lane, no parked line, no filter
  // candidates -- takes ONE host synchronisation per scan: the ordering passes
  // are queued right behind the scan (they read the tiles' counts on the device
  // and never write past `capacity`) and the counters are read back after them.
  // Anything else shows in the counters, and the ordering is queued again once
  // the extra passes have run.
  const bool speculate = !filt && capacity != 0;
  // Each buffer a scan can outgrow (overflow list, pending list, the filter's
  // staging) is grown to what the scan counted and the scan re-run, so every
  // grow is followed by a scan that fits: at most three grows, four scans. (A
  // loop that could end on a grow left the filter's candidates unverified but
  // counted.)
  bool settled = false;
  for (int attempt = 0; attempt < 4 && !settled; ++attempt) {
    a.staging = c->d_staging;
    a.capacity = c->staging_cap;
    a.overflow = c->d_overflow;
    a.overflow_cap = c->overflow_cap;
    a.pend = park ? c->d_pend : nullptr;
    a.pend_cap = park ? c->pend_cap : 0;
    HIPCHK(hipMemsetAsync(c->d_counters, 0, kCounters * sizeof(unsigned long long), c->stream));
    HIPCHK(hipEventRecord(c->ev0, c->stream));
    HIPCHK(scan_dfa(launch_kind(c), a, grid, c->stream));
    HIPCHK(hipEventRecord(c->ev1, c->stream));
    if (speculate)
      HIPCHK(order_lines(c->d_tiles, c->d_staging, ntiles, c->d_out_off, c->d_line_base, c->staging_cap, capacity,
                         d_line, d_start, d_len, c->stream));
    HIPCHK(hipMemcpyAsync(ctr, c->d_counters, sizeof ctr, hipMemcpyDeviceToHost, c->stream));
    if (DGREP_SYNC_SPIN_US > 0) {
      // block until the scan kernel is done (its wake-up latency overlaps the
      // ordering passes), then poll the short tail, bounded (see DGREP_SYNC_SPIN_US)
      HIPCHK(hipEventSynchronize(c->ev1));
      const auto t0 = std::chrono::steady_clock::now();
      hipError_t q;
      while ((q = hipStreamQuery(c->stream)) == hipErrorNotReady &&
             std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(DGREP_SYNC_SPIN_US)) {
      }
      if (q == hipErrorNotReady) q = hipStreamSynchronize(c->stream);
      HIPCHK(q);
    } else {
      HIPCHK(hipStreamSynchronize(c->stream));
    }
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    S.scan_ms += ms;  // a re-run scan is counted: it is part of this call's device time
    ++S.scan_attempts;
    if (ctr[1] > c->overflow_cap) {
      // more overflowing lanes than recorded: grow the list and scan again
      if ((rc = grow(c, &c->d_overflow, &c->overflow_cap, ctr[1])) != DGREP_OK) return rc;
    } else if (park && ctr[2] > c->pend_cap) {
      // more parked long lines than the pending list holds
      if ((rc = grow(c, &c->d_pend, &c->pend_cap, ctr[2])) != DGREP_OK) return rc;
    } else if (filt && ctr[0] > c->staging_cap) {
      // candidates included, more staged lines than the staging buffer holds
      if ((rc = grow(c, &c->d_staging, &c->staging_cap, ctr[0] + ctr[0] / 8)) != DGREP_OK) return rc;
    } else {
      settled = true;
    }
  }
  if (!settled) {
    c->err = "scan buffers still too small after three grows";
    return DGREP_E_HIP;
  }
  const uint64_t staged = ctr[0];
  const uint64_t npend = park ? ctr[2] : 0;
  S.overflow_lanes = ctr[1];
  S.pending = npend;
  c->last_ms = S.scan_ms;
  // matching (and candidate) lines per byte: caps the next scan's lane chunk
  c->density = double(staged) / double(n);
  const bool over = ctr[1] && staged <= a.capacity;
  if (over) {
    HIPCHK(hipEventRecord(c->ev2, c->stream));
    HIPCHK(scan_dfa_overflow(launch_kind(c), a, ctr[1], c->stream));
    HIPCHK(hipEventRecord(c->ev3, c->stream));
  }
  uint64_t total = staged;
  // verification pass: the filter's candidates, parked long lines
  const bool verify = filt || npend;
  bool ordered = false;  // the verification branch queued the ordering already
  if (verify && staged && staged <= a.capacity) {
    VerifyArgs v;
    memset(&v, 0, sizeof v);
    v.data = d_data;
    v.full = c->d_full;
    v.full_u32 = c->full_u32 ? 1u : 0u;
    v.hot_entries = c->verify_hot;
    v.cls = c->d_cls;
    v.nclasses = c->nclasses;
    v.start = c->blob_start;
    v.start_m = c->blob_start_m;
    v.tiles = c->d_tiles;
    v.ntiles = ntiles;
    v.staging = c->d_staging;
    v.staging_cap = c->staging_cap;
    v.removed = c->d_counters + 3;  // zeroed before the scan
    v.nfa = c->d_nfa;
    v.nfa_words = c->nfa_words;
    v.matched = c->d_nfa ? UINT32_MAX : c->blob_matched;
    v.pend = c->d_pend;
    v.ximg = DGREP_VERIFY_XREC ? c->d_ximg : nullptr;
    v.ximg_bytes = c->ximg_bytes;
    v.x_hot = c->x_hot;
    v.xr_off = c->xr_off;
    v.num_cus = uint32_t(c->num_cus);
    HIPCHK(hipEventRecord(c->ev4, c->stream));
    if (npend && park_maps) {
      LongArgs la;
      memset(&la, 0, sizeof la);
      la.n = n;
      la.chunk = chunk;
      la.nchunks = nchunks;
      la.pend = c->d_pend;
      la.npend = npend;
      la.chunk_map = c->d_chunk_map;
      la.sheng_m = c->start_m;
      la.nl_lo = c->sheng_nl_lo;
      la.nl_hi = c->sheng_nl_hi;
      la.sheng_v = reinterpret_cast<const uint2*>(c->d_table);
      la.data = d_data;
      HIPCHK(long_lines_sheng(la, c->stream));
    } else if (npend && park_filter) {
      if ((rc = resolve_long_filter(c, d_data, n, chunk, nchunks, npend)) != DGREP_OK) return rc;
    } else if (npend && (rc = resolve_long_lines(c, d_data, n, chunk, nchunks, npend)) != DGREP_OK) {
      return rc;
    }
    HIPCHK(verify_candidates(v, filt, c->stream));
    HIPCHK(hipEventRecord(c->ev5, c->stream));
    unsigned long long removed = 0;
    HIPCHK(hipMemcpyAsync(&removed, c->d_counters + 3, 8, hipMemcpyDeviceToHost, c->stream));
    // nothing changes the staged lines after the verification: when every
    // staged line fits the output, order them before the one host wait (the
    // kept lines are fewer still; a separate wait cost C4 ~30 us a scan)
    if (capacity != 0 && staged <= capacity) {
      HIPCHK(order_lines(c->d_tiles, c->d_staging, ntiles, c->d_out_off, c->d_line_base, c->staging_cap, capacity,
                         d_line, d_start, d_len, c->stream));
      ordered = true;
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipEventElapsedTime(&S.verify_ms, c->ev4, c->ev5));
    c->last_ms += S.verify_ms;
    total = staged - removed;
    S.candidates = removed;  // dropped ones; kept candidates count as matches
  } else if (npend && staged > a.capacity) {
    // The staged lines did not fit (a size query, or too small a capacity), so
    // no record is resolved -- but the count must still be exact: every parked
    // line was counted as one staged record, so resolve the pending list (it
    // does not depend on staging) and subtract the parked lines that do not
    // match. (Overflow lanes were counted in full by the scan: no pass needed.)
    HIPCHK(hipEventRecord(c->ev4, c->stream));
    if (park_maps) {
      LongArgs la;
      memset(&la, 0, sizeof la);
      la.n = n;
      la.chunk = chunk;
      la.nchunks = nchunks;
      la.pend = c->d_pend;
      la.npend = npend;
      la.chunk_map = c->d_chunk_map;
      la.sheng_m = c->start_m;
      la.nl_lo = c->sheng_nl_lo;
      la.nl_hi = c->sheng_nl_hi;
      la.sheng_v = reinterpret_cast<const uint2*>(c->d_table);
      la.data = d_data;
      HIPCHK(long_lines_sheng(la, c->stream));
    } else if ((rc = park_filter ? resolve_long_filter(c, d_data, n, chunk, nchunks, npend)
                                 : resolve_long_lines(c, d_data, n, chunk, nchunks, npend)) != DGREP_OK) {
      return rc;
    }
    HIPCHK(hipEventRecord(c->ev5, c->stream));
    std::vector<PendingLine> P(npend);
    HIPCHK(hipMemcpyAsync(P.data(), c->d_pend, npend * sizeof(PendingLine), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipEventElapsedTime(&S.verify_ms, c->ev4, c->ev5));
    c->last_ms += S.verify_ms;
    uint64_t unmatched = 0;
    for (const PendingLine& p : P) unmatched += p.matched ? 0u : 1u;
    total = staged - unmatched;
  }
  if (filt) c->staged_hint = staged;
  S.matches = total;
  *count = total;
  // the speculative ordering stands unless the overflow pass, the long-line
  // resolution or the verification changed the staged lines since
  const bool order = total != 0 && total <= capacity && (!speculate || over || verify) && !ordered;
  if (order)
    HIPCHK(order_lines(c->d_tiles, c->d_staging, ntiles, c->d_out_off, c->d_line_base, c->staging_cap, capacity,
                       d_line, d_start, d_len, c->stream));
  if (over || order) HIPCHK(hipStreamSynchronize(c->stream));
  if (over) {
    HIPCHK(hipEventElapsedTime(&S.overflow_ms, c->ev2, c->ev3));
    c->last_ms += S.overflow_ms;
  }
  return DGREP_OK;
}

extern "C" int dgrep_scan_device(dgrep_ctx* c, const void* d_data, size_t n, uint64_t* d_line_no, uint64_t* d_start,
                                 uint64_t* d_len, uint64_t capacity, uint64_t* count) {
  if (!c || !count || (n && !d_data)) return DGREP_E_INVALID;
  if (!c->loaded) { c->err = "no DFA loaded"; return DGREP_E_NO_DFA; }
  HIPCHK(hipSetDevice(c->device));
  const int rc = scan_resident(c, static_cast<const uint8_t*>(d_data), n, d_line_no, d_start, d_len, capacity, count);
  if (rc == DGREP_OK) {
    c->ms_sum += c->last_ms;
    ++c->ms_scans;
  }
  return rc;
}

// Worker-side ingest of one split (the bytes map_reduce/worker.go:72-76
// read with os.ReadFile and hand to Map): host -> pinned staging -> HBM.
// Piece k is memcpy'd by the CPU threads into staging buffer k % B once the
// DMA that last read that buffer has finished, then DMA'd on the copy stream;
// so the CPU copy of piece k+1 overlaps the DMA of piece k. The scan stream
// waits on the last DMA. A split of at most one piece below 4 MiB, or chunk
// 0, takes one pageable hipMemcpyAsync instead.
static int ingest(dgrep_ctx* c, const uint8_t* data, size_t n) {
  const auto t0 = std::chrono::steady_clock::now();
  if (c->ingest_chunk == 0 || n < (size_t(4) << 20)) {
    HIPCHK(hipMemcpyAsync(c->d_data, data, n, hipMemcpyHostToDevice, c->stream));
    c->last_ingest_ms = 0.f;
    return DGREP_OK;
  }
  const size_t S = c->ingest_chunk;
  const int B = std::max(2, c->ingest_bufs);
  if (c->stage_bytes != S || int(c->h_stage.size()) != B) {
    if (c->copy_stream) HIPCHK(hipStreamSynchronize(c->copy_stream));
    for (uint8_t* h : c->h_stage)
      if (h) HIPCHK(hipHostFree(h));
    for (hipEvent_t e : c->ev_stage)
      if (e) HIPCHK(hipEventDestroy(e));
    c->h_stage.assign(B, nullptr);
    c->ev_stage.assign(B, nullptr);
    c->stage_bytes = 0;
    for (int b = 0; b < B; ++b) {
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->h_stage[b]), S, hipHostMallocDefault));
      HIPCHK(hipEventCreateWithFlags(&c->ev_stage[b], hipEventDisableTiming));
    }
    c->stage_bytes = S;
  }
  if (!c->copy_stream) HIPCHK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
  // the previous scan may still read d_data: the first DMA waits for it
  HIPCHK(hipEventRecord(c->ev1, c->stream));
  HIPCHK(hipStreamWaitEvent(c->copy_stream, c->ev1, 0));
  const int T = std::max(1, c->ingest_threads);
  std::vector<bool> used(B, false);
  const size_t pieces = (n + S - 1) / S;
  for (size_t k = 0; k < pieces; ++k) {
    const int b = int(k % size_t(B));
    const size_t off = k * S, len = std::min(S, n - off);
    if (used[b]) HIPCHK(hipEventSynchronize(c->ev_stage[b]));  // buffer b's last DMA is done
    uint8_t* dst = c->h_stage[b];
    const uint8_t* src = data + off;
    if (T == 1 || len < (size_t(1) << 20)) {
      memcpy(dst, src, len);
    } else {
      std::vector<std::thread> th;
      const size_t part = ((len + T - 1) / T + 4095) & ~size_t(4095);
      for (int t = 0; t < T; ++t) {
        const size_t a = size_t(t) * part;
        if (a >= len) break;
        const size_t m = std::min(part, len - a);
        th.emplace_back([=] { memcpy(dst + a, src + a, m); });
      }
      for (auto& x : th) x.join();
    }
    HIPCHK(hipMemcpyAsync(c->d_data + off, dst, len, hipMemcpyHostToDevice, c->copy_stream));
    HIPCHK(hipEventRecord(c->ev_stage[b], c->copy_stream));
    used[b] = true;
  }
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_stage[int((pieces - 1) % size_t(B))], 0));
  HIPCHK(hipStreamSynchronize(c->copy_stream));
  c->last_ingest_ms =
      std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return DGREP_OK;
}

extern "C" int dgrep_set_ingest(dgrep_ctx* c, size_t chunk_bytes, int nbufs, int threads) {
  if (!c || nbufs < 0 || threads < 0 || nbufs > 64 || threads > 256) return DGREP_E_INVALID;
  c->ingest_chunk = chunk_bytes;
  if (nbufs) c->ingest_bufs = nbufs;
  if (threads) c->ingest_threads = threads;
  return DGREP_OK;
}

extern "C" int dgrep_last_ingest_ms(dgrep_ctx* c, float* ms) {
  if (!c || !ms) return DGREP_E_INVALID;
  *ms = c->last_ingest_ms;
  return DGREP_OK;
}

// Host split -> HBM (ingest) -> scan into the context's result arrays.
static int scan_host(dgrep_ctx* c, const uint8_t* data, size_t n, uint64_t* count) {
  int rc;
  if (n) {
    uint64_t cap = c->data_cap;
    if ((rc = grow(c, &c->d_data, &cap, (n + 63) & ~uint64_t(63))) != DGREP_OK) return rc;
    c->data_cap = cap;
    if ((rc = ingest(c, data, n)) != DGREP_OK) return rc;
  }
  uint64_t want = std::max<uint64_t>(c->res_cap, std::max<uint64_t>(1024, n / 512));
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (want > c->res_cap) {
      uint64_t c1 = 0, c2 = 0, c3 = 0;
      if (c->d_res_line) { HIPCHK(hipFree(c->d_res_line)); c->d_res_line = nullptr; }
      if (c->d_res_start) { HIPCHK(hipFree(c->d_res_start)); c->d_res_start = nullptr; }
      if (c->d_res_len) { HIPCHK(hipFree(c->d_res_len)); c->d_res_len = nullptr; }
      if ((rc = grow(c, &c->d_res_line, &c1, want)) != DGREP_OK) return rc;
      if ((rc = grow(c, &c->d_res_start, &c2, want)) != DGREP_OK) return rc;
      if ((rc = grow(c, &c->d_res_len, &c3, want)) != DGREP_OK) return rc;
      c->res_cap = want;
    }
    if ((rc = scan_resident(c, c->d_data, n, c->d_res_line, c->d_res_start, c->d_res_len, c->res_cap, count)) !=
        DGREP_OK)
      return rc;
    if (*count <= c->res_cap) break;
    want = *count;
  }
  return DGREP_OK;
}

extern "C" int dgrep_scan(dgrep_ctx* c, const uint8_t* data, size_t n, dgrep_result* out) {
  if (!c || !out || (n && !data)) return DGREP_E_INVALID;
  memset(out, 0, sizeof *out);
  if (!c->loaded) { c->err = "no DFA loaded"; return DGREP_E_NO_DFA; }
  HIPCHK(hipSetDevice(c->device));
  uint64_t count = 0;
  int rc;
  if ((rc = scan_host(c, data, n, &count)) != DGREP_OK) return rc;
  out->count = count;
  if (count == 0) return DGREP_OK;
  out->line_no = static_cast<uint64_t*>(malloc(count * 8));
  out->start = static_cast<uint64_t*>(malloc(count * 8));
  out->len = static_cast<uint64_t*>(malloc(count * 8));
  if (!out->line_no || !out->start || !out->len) {
    dgrep_result_free(out);
    return DGREP_E_NOMEM;
  }
  HIPCHK(hipMemcpyAsync(out->line_no, c->d_res_line, count * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(out->start, c->d_res_start, count * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(out->len, c->d_res_len, count * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return DGREP_OK;
}

// ---- partition + intermediate writer (map_reduce/worker.go:13-17,78-109) ----
static int encode_resident(dgrep_ctx* c, const uint8_t* d_data, uint64_t n, const uint64_t* d_line, const uint64_t* d_start,
                           const uint64_t* d_len, uint64_t count, const char* filename, size_t fn, uint32_t nreduce,
                           uint8_t* d_out, uint64_t out_cap, uint64_t* begin, uint64_t* end, uint64_t* total) {
  if (nreduce == 0 || nreduce > 65535) { c->err = "nreduce must be 1..65535"; return DGREP_E_INVALID; }
  if (count >= (uint64_t(1) << 32)) { c->err = "more than 2^32-1 records"; return DGREP_E_UNSUPPORTED; }
  int rc;
  const uint8_t* fname = reinterpret_cast<const uint8_t*>(filename);
  const uint64_t fj = json_escape_host(fname, fn, nullptr);
  if (fj >= (uint64_t(1) << 31)) { c->err = "filename too long"; return DGREP_E_INVALID; }
  std::vector<uint8_t> fjson(fj + 1);
  json_escape_host(fname, fn, fjson.data());
  if ((rc = grow(c, &c->d_fname, &c->fname_cap, fj + 1)) != DGREP_OK) return rc;
  HIPCHK(hipMemcpyAsync(c->d_fname, fjson.data(), fj + 1, hipMemcpyHostToDevice, c->stream));
  if ((rc = grow(c, &c->d_bounds, &c->bounds_cap, 2 * uint64_t(nreduce) + 1)) != DGREP_OK) return rc;
  EncodeArgs a;
  a.data = d_data;
  a.n = n;
  a.line_no = d_line;
  a.start = d_start;
  a.len = d_len;
  a.count = count;
  a.fname_json = c->d_fname;
  a.fname_json_len = uint32_t(fj);
  a.key_hash0 = key_prefix_hash(fname, fn);
  a.nreduce = nreduce;
  size_t need = 0;
  HIPCHK(encode_partitions(a, nullptr, &need, nullptr, 0, nullptr, c->stream));
  if ((rc = grow(c, &c->d_enc_scratch, &c->enc_scratch_cap, need)) != DGREP_OK) return rc;
  size_t have = c->enc_scratch_cap;
  HIPCHK(hipEventRecord(c->ev0, c->stream));
  HIPCHK(encode_partitions(a, c->d_enc_scratch, &have, d_out, out_cap, c->d_bounds, c->stream));
  HIPCHK(hipEventRecord(c->ev1, c->stream));
  std::vector<uint64_t> b(2 * size_t(nreduce) + 1);
  HIPCHK(hipMemcpyAsync(b.data(), c->d_bounds, b.size() * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipEventElapsedTime(&c->last_encode_ms, c->ev0, c->ev1));
  for (uint32_t p = 0; p < nreduce; ++p) {
    begin[p] = b[p];
    end[p] = b[nreduce + p];
  }
  *total = b[2 * size_t(nreduce)];
  return DGREP_OK;
}

extern "C" int dgrep_encode_device(dgrep_ctx* c, const void* d_data, size_t n, const uint64_t* d_line_no,
                                   const uint64_t* d_start, const uint64_t* d_len, uint64_t count,
                                   const char* filename, size_t fn, uint32_t nreduce, void* d_out, uint64_t out_cap,
                                   uint64_t* part_begin, uint64_t* part_end, uint64_t* total) {
  if (!c || !part_begin || !part_end || !total || (fn && !filename) || (count && (!d_line_no || !d_start || !d_len)) ||
      (n && !d_data) || (out_cap && !d_out))
    return DGREP_E_INVALID;
  HIPCHK(hipSetDevice(c->device));
  return encode_resident(c, static_cast<const uint8_t*>(d_data), n, d_line_no, d_start, d_len, count, filename, fn,
                         nreduce, static_cast<uint8_t*>(d_out), out_cap, part_begin, part_end, total);
}

extern "C" int dgrep_map_partitions(dgrep_ctx* c, const uint8_t* data, size_t n, const char* filename, size_t fn,
                                    uint32_t nreduce, dgrep_partitions* out) {
  if (!c || !out || (n && !data) || (fn && !filename) || nreduce == 0) return DGREP_E_INVALID;
  memset(out, 0, sizeof *out);
  if (!c->loaded) { c->err = "no DFA loaded"; return DGREP_E_NO_DFA; }
  HIPCHK(hipSetDevice(c->device));
  uint64_t count = 0;
  int rc;
  if ((rc = scan_host(c, data, n, &count)) != DGREP_OK) return rc;
  out->nreduce = nreduce;
  out->begin = static_cast<uint64_t*>(calloc(nreduce, 8));
  out->end = static_cast<uint64_t*>(calloc(nreduce, 8));
  if (!out->begin || !out->end) { dgrep_partitions_free(out); return DGREP_E_NOMEM; }
  const uint8_t* dd = c->d_data ? c->d_data : reinterpret_cast<const uint8_t*>(c->d_counters);
  uint64_t total = 0;
  for (int attempt = 0; attempt < 2; ++attempt) {
    if ((rc = encode_resident(c, dd, c->d_data ? n : 0, c->d_res_line, c->d_res_start, c->d_res_len, count, filename,
                              fn, nreduce,
                              c->d_enc_out, c->enc_out_cap, out->begin, out->end, &total)) != DGREP_OK) {
      dgrep_partitions_free(out);
      return rc;
    }
    if (total <= c->enc_out_cap) break;
    if ((rc = grow(c, &c->d_enc_out, &c->enc_out_cap, total + total / 16)) != DGREP_OK) {
      dgrep_partitions_free(out);
      return rc;
    }
  }
  out->total = total;
  if (total) {
    out->bytes = static_cast<uint8_t*>(malloc(total));
    if (!out->bytes) { dgrep_partitions_free(out); return DGREP_E_NOMEM; }
    HIPCHK(hipMemcpyAsync(out->bytes, c->d_enc_out, total, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  return DGREP_OK;
}

extern "C" void dgrep_partitions_free(dgrep_partitions* p) {
  if (!p) return;
  free(p->begin);
  free(p->end);
  free(p->bytes);
  memset(p, 0, sizeof *p);
}

// ---- reduce task (map_reduce/worker.go:22-68,161-165 + grep.go:38-40) -------
extern "C" int dgrep_reduce(dgrep_ctx* c, const uint8_t* data, size_t n, dgrep_reduce_out* out) {
  if (!c || !out || (n && !data)) return DGREP_E_INVALID;
  memset(out, 0, sizeof *out);
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return DGREP_OK;
  int rc;
  uint64_t cap = c->data_cap;
  if ((rc = grow(c, &c->d_data, &cap, (n + 63) & ~uint64_t(63))) != DGREP_OK) return rc;
  c->data_cap = cap;
  if ((rc = ingest(c, data, n)) != DGREP_OK) return rc;
  uint64_t* d_info = reinterpret_cast<uint64_t*>(c->d_counters);  // 3 of its 4 u64
  HIPCHK(reduce_count_lines(c->d_data, n, d_info, c->stream));
  uint64_t nlines = 0;
  HIPCHK(hipMemcpyAsync(&nlines, d_info, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (data[n - 1] != '\n') {
    c->err = "reduce input must be whole json.Encoder lines (the last byte is not '\\n')";
    return DGREP_E_INVALID;
  }
  size_t need = 0;
  HIPCHK(reduce_lines(c->d_data, n, nlines, nullptr, &need, nullptr, 0, d_info, c->stream));
  if ((rc = grow(c, &c->d_red_scratch, &c->red_scratch_cap, need)) != DGREP_OK) return rc;
  uint64_t info[3] = {0, 0, 0};
  for (int attempt = 0; attempt < 2; ++attempt) {
    size_t have = c->red_scratch_cap;
    HIPCHK(hipEventRecord(c->ev0, c->stream));
    HIPCHK(reduce_lines(c->d_data, n, nlines, c->d_red_scratch, &have, c->d_red_out, c->red_out_cap, d_info,
                        c->stream));
    HIPCHK(hipEventRecord(c->ev1, c->stream));
    HIPCHK(hipMemcpyAsync(info, d_info, sizeof info, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (info[1] != UINT64_MAX) {
      c->err = "reduce input line " + std::to_string(info[1] + 1) + " is not a json.Encoder KeyValue line";
      return DGREP_E_INVALID;
    }
    if (info[2] <= c->red_out_cap) break;
    if ((rc = grow(c, &c->d_red_out, &c->red_out_cap, info[2])) != DGREP_OK) return rc;
  }
  HIPCHK(hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
  out->lines_in = info[0];
  out->total = info[2];
  if (info[2]) {
    out->bytes = static_cast<uint8_t*>(malloc(info[2]));
    if (!out->bytes) return DGREP_E_NOMEM;
    HIPCHK(hipMemcpyAsync(out->bytes, c->d_red_out, info[2], hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  return DGREP_OK;
}

extern "C" void dgrep_reduce_free(dgrep_reduce_out* r) {
  if (!r) return;
  free(r->bytes);
  memset(r, 0, sizeof *r);
}

extern "C" int dgrep_last_encode_ms(dgrep_ctx* c, float* ms) {
  if (!c || !ms) return DGREP_E_INVALID;
  *ms = c->last_encode_ms;
  return DGREP_OK;
}

extern "C" void dgrep_result_free(dgrep_result* r) {
  if (!r) return;
  free(r->line_no);
  free(r->start);
  free(r->len);
  memset(r, 0, sizeof *r);
}

extern "C" int dgrep_last_kernel_ms(dgrep_ctx* c, float* ms) {
  if (!c || !ms) return DGREP_E_INVALID;
  *ms = c->last_ms;
  return DGREP_OK;
}

extern "C" int dgrep_take_kernel_ms(dgrep_ctx* c, double* sum_ms, uint64_t* scans) {
  if (!c || !sum_ms || !scans) return DGREP_E_INVALID;
  *sum_ms = c->ms_sum;
  *scans = c->ms_scans;
  c->ms_sum = 0.0;
  c->ms_scans = 0;
  return DGREP_OK;
}

extern "C" int dgrep_last_scan_stats(dgrep_ctx* c, dgrep_scan_stats* out, size_t out_size) {
  if (!c || !out || out_size == 0) return DGREP_E_INVALID;
  // a shorter (older) caller layout gets its own size; a longer one a zeroed tail
  const size_t k = std::min(out_size, sizeof(dgrep_scan_stats));
  memcpy(out, &c->stats, k);
  if (out_size > k) memset(reinterpret_cast<uint8_t*>(out) + k, 0, out_size - k);
  return DGREP_OK;
}


// ---- synthetic corpus ------------------------------------------------------
__global__ void synth_kernel(char* out, uint64_t n, uint64_t seed, int kind) {
  const uint64_t pages = (n + synth::kPage - 1) / synth::kPage;
  for (uint64_t p = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; p < pages; p += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t off = p * synth::kPage;
    const uint32_t bytes = uint32_t(std::min<uint64_t>(synth::kPage, n - off));
    synth::page_fill(seed, p, kind, out + off, bytes);
  }
}

extern "C" int dgrep_synth_corpus(dgrep_ctx* c, void* d_out, size_t n, uint64_t seed, int kind) {
  if (!c || (n && !d_out)) return DGREP_E_INVALID;
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return DGREP_OK;
  const uint64_t pages = (n + synth::kPage - 1) / synth::kPage;
  const int block = 256;
  const int grid = int(std::min<uint64_t>((pages + block - 1) / block, 65536));
  hipLaunchKernelGGL(synth_kernel, dim3(grid), dim3(block), 0, c->stream, static_cast<char*>(d_out), uint64_t(n),
                     seed, kind);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return DGREP_OK;
}

// Host twin of dgrep_synth_corpus (same code path, synth.h): used by tests to
// regenerate any window of a device corpus on the CPU.
extern "C" int dgrep_synth_corpus_host(void* out, size_t n, uint64_t seed, int kind) {
  if (n && !out) return DGREP_E_INVALID;
  const uint64_t pages = (n + synth::kPage - 1) / synth::kPage;
  for (uint64_t p = 0; p < pages; ++p) {
    const uint64_t off = p * synth::kPage;
    const uint32_t bytes = uint32_t(std::min<uint64_t>(synth::kPage, n - off));
    synth::page_fill(seed, p, kind, static_cast<char*>(out) + off, bytes);
  }
  return DGREP_OK;
}

extern "C" int dgrep_synth_keyword(uint64_t seed, int i, char* out16) {
  if (!out16 || i < 0 || i >= synth::kKeywords) return -1;
  return synth::keyword(seed, i, out16);
}
