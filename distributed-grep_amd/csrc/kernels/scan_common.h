// scan_common.h — types shared by the scan kernels and the host runtime.
#pragma once
#include <stdint.h>

namespace dgrep {

// One matching line as produced by a tile, before global ordering.
// meta = rel | flags | len_hi: `rel` (bits 0-22) = number of '\n' between the
// tile start and the line start, so the 1-based line number
// (application/grep.go:25 `line_number+1`) is newlines_before_tile + rel + 1.
// A tile is at most 64 x 64 KiB = 2^22 bytes, and its last lane's last line
// can start right after a tile made of nothing but '\n': rel <= 2^22 needs 23
// bits (round 4 had 22, enough for 32 KiB chunks only). Bit 23 = filter
// CANDIDATE (verified afterwards); bit 24 = PENDING long line (len_lo = its
// index in the pending list, resolved afterwards); bits 25-31 = bits 32-38 of
// the length (lines up to 512 GiB: more than the 288 GB of HBM hold).
struct StagedLine {
  uint64_t start;  // absolute byte offset of the line in the split
  uint32_t len_lo; // bytes, '\n' excluded (low 32 bits)
  uint32_t meta;
};
constexpr uint32_t kRelBits = 23;
constexpr uint32_t kMetaCand = 1u << 23;
constexpr uint32_t kMetaPend = 1u << 24;
constexpr uint32_t kLenHiShift = 25;
__host__ __device__ inline uint32_t meta_of(uint32_t rel, uint64_t len, bool cand) {
  return rel | (cand ? kMetaCand : 0u) | (uint32_t(len >> 32) << kLenHiShift);
}
__host__ __device__ inline uint64_t staged_len(const StagedLine& L) {
  return uint64_t(L.len_lo) | (uint64_t(L.meta >> kLenHiShift) << 32);
}
__host__ __device__ inline uint32_t staged_rel(const StagedLine& L) { return L.meta & ((1u << kRelBits) - 1u); }

// Per-tile bookkeeping written by the scan kernel.
struct TileInfo {
  uint64_t base;   // first StagedLine of this tile in the staging buffer
  uint32_t count;  // matching lines owned by the tile
  uint32_t nl;     // '\n' bytes inside the tile
};

// A lane whose matching lines overflowed its LDS slots (re-run by
// scan_overflow_kernel in direct-write mode).
struct OverflowLane {
  uint64_t cs;         // chunk start
  uint64_t out_base;   // its first staging index
  uint32_t nl_prefix;  // '\n' between the tile start and cs
  uint32_t pend;       // the lane's parked last line: pending index + 1 (0: none)
};

// A long line the scan parked (see park_pending): its start, the chunk boundary
// where the lane stopped and its state there (as an index of the stepper's
// state -> blob state table); the long-line kernels fill end, len, matched.
struct PendingLine {
  uint64_t line_start;
  uint64_t resume;
  uint32_t state;
  uint32_t matched;
  uint64_t end;
  uint64_t len;
};
// Sheng stepper (<= 8 states): per lane chunk, the transition map of its bytes
// up to and including its first '\n' (first = that byte's chunk-relative
// offset), or of the whole chunk (first = kNoNewline). Map byte s (lo: states
// 0-3, hi: 4-7) = the stepper state reached from state s. A parked long line
// is finished by composing the maps of the chunks it crosses (long_sheng_kernel).
struct ChunkMap {
  uint32_t lo, hi;
  uint32_t first;
  uint32_t pad;
};
constexpr uint32_t kNoNewline = 0xffffffffu;
// LAZY record: the chunk's first '\n' lies in its first kLazyMapBytes, where
// the scan computes no map (nearly every chunk of text): the resolution runs
// the DFA over those bytes itself, from the state the earlier maps give.
constexpr uint32_t kLazyNewline = 0xfffffffeu;
#ifndef DGREP_LAZY_MAP_BYTES
#define DGREP_LAZY_MAP_BYTES 256
#endif
constexpr uint32_t kLazyMapBytes = DGREP_LAZY_MAP_BYTES;  // a multiple of the Sheng block (0: maps from byte 0)

// a segment of a parked line's remaining bytes (long_map_kernel)
struct LongSeg {
  uint64_t begin, end;
};

struct ScanArgs {
  const uint8_t* data;
  uint64_t n;
  const uint8_t* table;   // u8 transition table, [state][byte] (nstates*256 bytes)
  uint32_t table_bytes;
  uint32_t start, start_m;
  uint32_t chunk;         // lane chunk bytes of the adaptive (Sheng) stepper, from scan_tile_bytes
  uint64_t ntiles;
  StagedLine* staging;
  uint64_t capacity;      // staging/output capacity in lines
  unsigned long long* counter;  // staging append counter
  TileInfo* tiles;
  OverflowLane* overflow;
  uint64_t overflow_cap;
  unsigned long long* overflow_count;
  uint32_t nclasses;
  // kStepPair only (byte offsets into the LDS image, see StepPair)
  uint32_t pair_t1;   // single-byte table T1
  uint32_t pair_thr;  // lowest premultiplied shadow state: a pair ending at >= thr holds an event
  uint32_t pair_div;  // bytes per T2 row (esz * nclasses^2, padded): premultiplied state / pair_div = state id
  // kStepFilter only: the premultiplied CAND_END state (a '\n' ends a line that
  // left the LDS-resident part of the DFA: a candidate, verified afterwards)
  uint32_t cand_end;
  // one-chunk-per-lane steppers: per resident thread, spill_per_lane records of
  // HBM the lane moves its full LDS slots to (nullptr: no spilling)
  uint2* spill;
  uint32_t spill_per_lane;
  // slot mode: per resident thread and stream, the real length of the lane's
  // last record when its LDS slot holds kSlotLong (or its pending index)
  uint64_t* tails;
  // <= 256-state steppers: '\n' count per chunk, and the pending list of parked
  // long lines (pend nullptr: a long line is read to its end by its lane)
  uint32_t* chunk_nl;
  PendingLine* pend;
  uint64_t pend_cap;
  unsigned long long* pend_count;
  // Sheng stepper: the chunk maps instead of chunk_nl (nullptr: none)
  ChunkMap* chunk_map;
  // tiles claimed after each wave's first (zeroed per launch)
  unsigned long long* tile_next;
};

// the long-line kernels' arguments (long_end / long_map / long_fin)
struct LongArgs {
  const uint8_t* data;
  uint64_t n;
  uint64_t chunk;    // lane chunk bytes of the scan
  uint64_t nchunks;
  const uint32_t* chunk_nl;
  PendingLine* pend;
  uint64_t npend;
  const uint32_t* st2id;  // PendingLine::state -> blob state
  const uint8_t* tbl;     // u8 [S][256]: blob state x byte -> blob state
  uint32_t nstates;       // S <= 256
  uint32_t start_m;       // blob id
  const LongSeg* seg;
  uint64_t nseg;
  const uint64_t* seg_off;  // [npend + 1]: line i's segments
  uint8_t* segmap;          // [nseg][256]
  // Sheng stepper (long_sheng_kernel): the scan's chunk maps, stepper state
  // ids, start_m as a stepper id and V['\n'] (the 8 next states of '\n');
  // the whole V table (LAZY records are finished byte by byte)
  const ChunkMap* chunk_map;
  uint32_t sheng_m;
  uint32_t nl_lo, nl_hi;
  const uint2* sheng_v;
};

// the filter stepper's parked lines on the whole DFA (long_dfa_* kernels):
// each segment is run from up to kLongGuesses distinct entry guesses, the
// states its lookback leads to from kLongSeeds start states
constexpr int kLongSeeds = 8;
constexpr int kLongGuesses = 4;
constexpr uint32_t kNoGuess = 0xffffffffu;
struct LongDfaArgs {
  const uint8_t* data;
  const void* full;       // [nstates][nclasses] breadth-first ids: u16, or u32 above 65535 states
  uint32_t hot_entries;   // leading entries of `full` in LDS (long_dfa_fix_kernel)
  uint32_t seg_hot_entries;  // the same for long_dfa_seg1_kernel (a larger LDS copy)
  uint32_t nclasses;
  const uint8_t* cls;     // [256] byte classes (HBM)
  uint32_t start, start_m;
  uint32_t matched;       // the absorbing accepting state (UINT32_MAX: none)
  uint32_t dead;          // the absorbing rejecting state (UINT32_MAX: none)
  uint32_t seed[kLongSeeds];  // lookback start states: start, then states spread over the ids
  const LongSeg* seg;     // segments of the parked lines, line by line
  const uint64_t* seg_from;  // [nseg] where each segment's lookback starts
  uint64_t nseg;
  uint32_t* seg_guess;    // [kLongGuesses][nseg] distinct states after the lookback (kNoGuess: unused)
  uint32_t* seg_exit;     // [kLongGuesses][nseg] state after the segment from each guess
  const uint64_t* seg_off;  // [npend + 1]
  PendingLine* pend;
  uint64_t npend;
  // the whole-DFA LDS image of a u16 DFA (runtime build_ximg; nullptr: the
  // first rows in LDS, the rest read from `full`): x_hot rows (plus extra
  // rows), then a DfaXRec per state >= x_hot at byte xr_off
  const uint8_t* ximg;
  uint32_t ximg_bytes, x_hot, xr_off;
};
// DfaXRec: a state past the LDS image's first rows reads the row of a resident
// DEFAULT state except in at most two classes (keyword automata: 4,608 of
// config 4's 4,978 such states differ in one class, 367 in two; the 2 left
// get an extra row of their own as default): x = default row | class 1 << 16
// | class 2 << 24 (0xff: unused), y = next state on class 1 | on class 2 << 16.
constexpr uint32_t kXNone = 0xffu;

// verify_kernel's arguments (kStepFilter): the whole DFA with the blob's ids
struct VerifyArgs {
  const uint8_t* data;
  const void* full;      // [nstates][nclasses] breadth-first ids, HBM: u16 entries, or u32 if full_u32
  uint32_t full_u32;
  uint32_t hot_entries;  // leading entries of `full` verify_kernel copies to LDS
  const uint8_t* cls;    // [256] byte classes, HBM
  uint32_t nclasses, start, start_m;
  TileInfo* tiles;
  uint64_t ntiles;
  StagedLine* staging;
  uint64_t staging_cap;
  unsigned long long* removed;
  // DGREP_DFA_PARTIAL blobs: the NFA program (dgrep_blob.h) decides the
  // candidates instead of `full` (verify_nfa_kernel)
  const uint32_t* nfa;
  // `full` id of the absorbing accepting state (every byte but '\n' loops,
  // '\n' -> start_m; UINT32_MAX: none): a candidate that reaches it matches,
  // so verify_kernel stops reading the line there
  uint32_t matched;
  // resolved pending long lines (StagedLine kMetaPend: len_lo = index)
  const PendingLine* pend;
  uint32_t nfa_words;  // the NFA program's position-set words (nw)
  // u16 DFAs: the whole-DFA LDS image (see LongDfaArgs); nullptr: the first
  // hot_entries of `full` in LDS, the rest from HBM
  const uint8_t* ximg;
  uint32_t ximg_bytes, x_hot, xr_off;
  uint32_t num_cus;
};

// LDS slot records (8 B: start16 | rel16, then w1): w1 = the line's length with
// bit 31 the filter CANDIDATE flag; a length of kSlotLong or more (only a
// lane's LAST owned line can reach past its <= 64 KiB chunk) is stored as
// kSlotLong and the lane keeps the real length (or its pending index) in
// its ScanArgs::tails entry. The same holds for a last line that starts
// exactly AT the chunk end (its '\n' predecessor is the chunk's last byte):
// start = C = 65,536 does not fit 16 bits, so it is flagged in the tail
// (kTailAtEnd) and read back as start C, rel = the chunk's '\n' count.
constexpr uint32_t kCandidateBit = 0x80000000u;
constexpr uint32_t kSlotLong = 0x7fffffffu;

constexpr int kScanThreads = 256;  // 4 waves per workgroup
constexpr int kTileLanes = 64;     // a tile is one wave's 64 chunks

// DFA stepper selected by dgrep_load_dfa from the state count.
enum : int {
  kStepTable = 0,   // <= 256 states: u8 [state][byte] table, 260-byte rows
  kStepSheng8 = 1,  // <= 8 states: per-byte 8-state vectors (v_perm stepping)
  // 2: the r01 wide stepper (u16 rows, cold ones from HBM on the chain), removed in round 6
  kStepPair = 3,    // 2 * states * classes^2 <= kPairMaxT2 bytes: two input bytes per table lookup
  kStepFilter = 4,  // > 256 states: the DFA's shallow part in LDS, lines that leave it verified afterwards
  // 5: the r05 word stepper (one lookup per 4-byte word), measured slower than pair; removed in round 6
};

// LDS image of kStepFilter: byte classes [256] (u8), then u16 [state][class]
// rows of the filter DFA (its states premultiplied by the class count), at
// most this many bytes in all -- with 1024 threads x 4 slots x 8 B the
// workgroup stays within the CU's 160 KiB.
#ifndef DGREP_FILTER_KIB
#define DGREP_FILTER_KIB 124
#endif
constexpr uint32_t kFilterImageBytes = DGREP_FILTER_KIB * 1024;
// u8 classes: four byte values share a dword, so printable ASCII (0x20-0x7f)
// spans 24 dwords in 24 distinct banks and a wave's class reads of text never
// conflict (tools/lds_bank_bench.hip on the log corpus: u8 table 0 % conflict
// cycles, u32 entries at 4*b 52 %, u64 at 8*b 55 %). C4 kernel 3.18 -> 3.38 TB/s.
constexpr uint32_t kFilterClassBytes = 256;

// StepPair's T2 entries are u32 (ds_read_b32) when the whole image fits
// kPairW32MaxImage, else u16 (DGREP_PAIR_T2_U32=0: always u16). A u16 chain
// value carried across the previous word's event branch is re-masked by one
// v_and per word (LLVM keeps the phi as i16); a u32 entry has nothing to mask.
#ifndef DGREP_PAIR_T2_U32
#define DGREP_PAIR_T2_U32 1
#endif
constexpr uint32_t kPairW32MaxImage = 16384;
// StepPair's two-byte table T2 ([state][class][class], premultiplied states)
// addresses itself with 16-bit values: at most kPairMaxT2 bytes, the whole LDS
// image (class table, T2, T1) at most kPairMaxImage bytes.
constexpr uint32_t kPairMaxT2 = 32768;
// OR-ed into the stepper kind handed to the scan entry points (scan_dfa,
// scan_tile_bytes, ...): the pair stepper's u32-entry build
constexpr int kKindW32 = 0x100;
constexpr uint32_t kPairMaxImage = 40960;
constexpr uint32_t kPairT2 = 2048;  // LDS address of T2 (after the byte tables)
// DGREP_PAIR_CK: a second byte table CK[b] = esz K class(b) (u16 at kPairCK) for
// the first byte of each pair, so a pair's column needs no v_mul_u32_u24
#ifndef DGREP_PAIR_CK
#define DGREP_PAIR_CK 1
#endif
constexpr uint32_t kPairCK = 256;
// The filter's one workgroup per CU: 1024 threads (4 waves per SIMD) with
// 128-byte load blocks. With 64-byte blocks it fetched 1.82x the split from
// HBM (each lane's half-read 128-byte lines are evicted before their second
// half is read; tools/fetch_calib.hip measures 1.8x for the bare 64-byte
// per-lane pattern and 1.0x for 128-byte blocks). C4 kernel GB/s: 1024 / 128 B
// 3,163; 1024 / 64 B 2,900; 768 / 128 B 2,743; 512 / 128 B 2,449.
#ifndef DGREP_FILTER_THREADS
#define DGREP_FILTER_THREADS 1024
#endif
constexpr int kFilterThreads = DGREP_FILTER_THREADS;

}  // namespace dgrep
