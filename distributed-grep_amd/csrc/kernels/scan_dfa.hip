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
//   * tile = one wave = 64 lanes x C bytes; lane i owns chunk i of its tile.
//   * A lane OWNS the lines that start inside its chunk after its first '\n'
//     (the very first line of the split is owned by global lane 0). It runs the
//     DFA from its chunk start -- the bytes before its first '\n' are run with a
//     don't-care state, which the first '\n' resets -- through its chunk and on
//     past the chunk end until the first '\n' at or after the end (the last
//     owned line's terminator) or the end of the split. No lane ever waits for
//     another lane's state. A lane whose chunk holds no '\n' owns no line and
//     stops at its chunk end. Long lines: on the <= 256-state steppers a lane
//     whose last line is still open two chunks past its chunk start parks it
//     as PENDING (state + position); the long-line kernels (long_end_kernel,
//     long_map_kernel, long_fin_kernel) then find its end from the per-chunk
//     '\n' counts and run the DFA over it in parallel -- per-piece transition
//     maps, composed in order -- instead of one lane reading on alone.
//   * Per 4-byte word: 4 DFA steps by one of the steppers (StepSheng8,
//     StepPair, StepTable, StepFilter: see each struct), newline
//     bookkeeping by SWAR on the word, and a matching line is detected by
//     "state == START_M" (rare path).
//       StepSheng8 (DFA <= 8 states): LDS holds, per input byte b, the 8-byte
//         vector V[b][s] = next state; a step is ONE v_perm_b32 selecting byte
//         s of V[b] (SDWA does the byte extract for the ds_read_b64 address).
//         The dependent chain is a single VALU op per byte; the LDS reads do
//         not depend on the state, so their latency overlaps.
//       StepTable (DFA <= 256 states): u8 table [state][byte] with 260-byte
//         rows (bank-staggered); a step is v_perm (row|byte) + v_lshl_add +
//         ds_read_u8 on the dependent chain.
//       StepPair: one two-byte table lookup per two bytes; StepFilter: the
//         shallow states of a large DFA, lines leaving them verified after.
//   * Matching lines are parked in per-lane LDS slots, counted, then the tile's
//     lines are appended to a staging buffer with ONE atomic per tile, in
//     ascending order inside the tile (no workgroup barrier anywhere: waves
//     are independent). Two small passes (tile_block_sum_kernel: sums per
//     64 tiles; order_lines_kernel: a wave per tile adds the sums before it)
//     turn tile-relative line numbers into global ones and lay the tiles out
//     in split order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "scan_common.h"
#include "../../../include/dgrep_blob.h"

// Build parts: the Makefile compiles this file once per DGREP_SCAN_PART -- 0:
// the kernels that take no stepper (verification, long lines, ordering) and
// the host glue; 1: Sheng; 2: pair; 3: table; 4: filter -- so the
// stepper instantiations compile in parallel. Without the macro one
// translation unit holds everything (tools/build_commit_variant.sh).
#ifdef DGREP_SCAN_PART
#define DG_PART(k) (DGREP_SCAN_PART == (k))
#else
#define DG_PART(k) 1
#endif

// Build-time tuning knobs, per stepper (defaults are the shipped configuration,
// measured on MI355X; DESIGN.md §3 lists the variants that lost and were removed):
//   CHUNK    bytes per lane chunk (multiple of BLOCK; the adaptive steppers
//            start here and double, see adaptive_chunk_bytes)
//   SLOTS    LDS slots per lane for matching lines
//   BLOCK    bytes per lane per register load block (64 or 128)
//   WAVES    waves per SIMD the register allocation must allow
#ifndef DGREP_SHENG_CHUNK
#define DGREP_SHENG_CHUNK 4096
#endif
#ifndef DGREP_SHENG_SLOTS
#define DGREP_SHENG_SLOTS 23  // + the dummy slot + the chunk-map slot: 3 workgroups per CU (159,744 B of LDS)
#endif
#ifndef DGREP_SHENG_BLOCK
#define DGREP_SHENG_BLOCK 128
#endif
#ifndef DGREP_SHENG_WAVES
#define DGREP_SHENG_WAVES 3
#endif
// Table (<= 256 states not fitting Pair): two 2 KiB chunks per lane stepped in
// lockstep while the table is small (<= 64 states)
#ifndef DGREP_TABLE_CHUNK
#define DGREP_TABLE_CHUNK 2048
#endif
#ifndef DGREP_TABLE_SLOTS
#define DGREP_TABLE_SLOTS 6
#endif
#ifndef DGREP_TABLE_BLOCK
#define DGREP_TABLE_BLOCK 64
#endif
#ifndef DGREP_TABLE_WAVES
#define DGREP_TABLE_WAVES 3
#endif
// Pair (C3, 20 states): one chunk per lane, runtime (adaptive) chunk from 4.5 KiB
#ifndef DGREP_PAIR_CHUNK
#define DGREP_PAIR_CHUNK 4608
#endif
#ifndef DGREP_PAIR_SLOTS
#define DGREP_PAIR_SLOTS 16
#endif
#ifndef DGREP_PAIR_BLOCK
#define DGREP_PAIR_BLOCK 128
#endif
#ifndef DGREP_PAIR_WAVES
#define DGREP_PAIR_WAVES 3
#endif
// Filter (C4, > 256 states): one 1024-thread workgroup per CU shares one LDS image
#ifndef DGREP_FILTER_CHUNK
#define DGREP_FILTER_CHUNK 4096
#endif
#ifndef DGREP_FILTER_SLOTS
#define DGREP_FILTER_SLOTS 4
#endif
#ifndef DGREP_FILTER_BLOCK
#define DGREP_FILTER_BLOCK 128
#endif

namespace dgrep {

// nl_mask: the last op as inline asm, so the compiler neither re-derives
// "m != 0" from the mask's inputs (it canonicalised that test into v_bitop3 +
// v_cmp instead of one v_cmp on m) nor splits popcount + sum into v_bcnt +
// v_add (v_bcnt_u32_b32 accumulates): two VALU fewer per word on the per-word
// steppers, which are VALU-issue-bound.
__device__ __forceinline__ uint32_t nl_mask(uint32_t w) {
  // exact per-byte zero test of w ^ '\n\n\n\n': bit 7 of byte k set iff byte k == '\n'
  const uint32_t x = w ^ 0x0a0a0a0au;
  const uint32_t t = (x & 0x7f7f7f7fu) + 0x7f7f7f7fu;
  uint32_t m;
  // m = ~(t | w) & 0x80808080 (bit 7 of w equals bit 7 of x); truth table
  // index = (S0 << 2) | (S1 << 1) | S2: true only at S0 = S1 = 0, S2 = 1
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:2" : "=v"(m) : "v"(t), "v"(w), "s"(0x80808080u));
  return m;
}
// acc + popcount(m) in one v_bcnt_u32_b32
__device__ __forceinline__ uint32_t add_popc(uint32_t acc, uint32_t m) {
  uint32_t r;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(m), "v"(acc));
  return r;
}
__device__ __forceinline__ uint32_t hi_byte(uint32_t m) { return (31u - __clz(m)) >> 3; }

// LDS row stride of the u8 transition table: 256 bytes + 4. Row s starts at
// s*260, so byte b of state s sits in bank (s + b/4) mod 32: lanes in
// different states that read the same input byte hit different banks.
constexpr uint32_t kRow = 260;

template <int TBL, int E, int NT, bool MAPS = false>
struct ScanSmem {
  alignas(16) uint8_t tbl[TBL];  // first member: the table sits at LDS address 0
  uint32_t slots[NT * E * 2];
  uint2 maps[MAPS ? NT : 1];     // Sheng: each lane's chunk map between map-mode blocks
};

// DFA of at most 256 states: u8 transition table, row s at LDS s*260.
struct StepTable {
  static constexpr int kKind = kStepTable;
  const uint8_t* tbl;
  __device__ __forceinline__ uint32_t one(uint32_t s, uint32_t w, uint32_t sel) const {
    // v_perm builds (s << 8) | byte(w); + 4s staggers the row: tbl[s*260 + byte]
    return tbl[__builtin_amdgcn_perm(s, w, sel) + (s << 2)];
  }
  // the whole step depends on the state: nothing to issue ahead
  struct Pre {
    uint32_t x;
  };
  __device__ __forceinline__ Pre prep(uint32_t x) const { return Pre{x}; }
  __device__ __forceinline__ void apply(const Pre& p, uint32_t s, uint32_t& s0, uint32_t& s1, uint32_t& s2,
                                        uint32_t& s3) const {
    s0 = one(s, p.x, 0x0c0c0400u);
    s1 = one(s0, p.x, 0x0c0c0401u);
    s2 = one(s1, p.x, 0x0c0c0402u);
    s3 = one(s2, p.x, 0x0c0c0403u);
  }
  __device__ __forceinline__ uint32_t byte(uint32_t s, uint32_t b) const { return tbl[s * kRow + b]; }
  __device__ __forceinline__ static bool is(uint32_t s, uint32_t M) { return s == M; }
};

// DFA of at most 8 states (Sheng-style): V[b] = 8 next-state bytes. Only byte
// 0 of the carried state is meaningful; v_perm fills bytes 1-3 with other
// (valid, < 8) states, which never reach byte 0 of a later result.
struct StepSheng8 {
  static constexpr int kKind = kStepSheng8;
  const uint2* V;
  __device__ __forceinline__ static uint32_t sel(const uint2 v, uint32_t s) {
    return __builtin_amdgcn_perm(v.y, v.x, s);
  }
  // the four LDS reads depend only on the input word: issued a word ahead
  struct Pre {
    uint2 m0, m1, m2, m3;
  };
  __device__ __forceinline__ Pre prep(uint32_t x) const {
    return Pre{V[x & 0xffu], V[(x >> 8) & 0xffu], V[(x >> 16) & 0xffu], V[x >> 24]};
  }
  __device__ __forceinline__ void apply(const Pre& p, uint32_t s, uint32_t& s0, uint32_t& s1, uint32_t& s2,
                                        uint32_t& s3) const {
    s0 = sel(p.m0, s);
    s1 = sel(p.m1, s0);
    s2 = sel(p.m2, s1);
    s3 = sel(p.m3, s2);
  }
  __device__ __forceinline__ uint32_t byte(uint32_t s, uint32_t b) const { return sel(V[b], s); }
  __device__ __forceinline__ static bool is(uint32_t s, uint32_t M) { return (s & 0xffu) == M; }
  // states are replicated bytes and start_m is the highest state (host
  // renumbering): one max over the word's four states replaces four compares
  __device__ __forceinline__ static bool any4(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, uint32_t M) {
    return max(max(s0, s1), max(s2, s3)) >= M * 0x01010101u;
  }
  // map <- bytes 0..lim of the word applied to the 8-state map (lo: states 0-3,
  // hi: states 4-7; byte s = the state reached from state s); one v_perm per
  // byte and half
  __device__ __forceinline__ void compose(const Pre& p, uint32_t lim, uint32_t& lo, uint32_t& hi) const {
    lo = sel(p.m0, lo);
    hi = sel(p.m0, hi);
    const uint32_t l1 = sel(p.m1, lo), h1 = sel(p.m1, hi);
    lo = lim >= 1 ? l1 : lo;
    hi = lim >= 1 ? h1 : hi;
    const uint32_t l2 = sel(p.m2, lo), h2 = sel(p.m2, hi);
    lo = lim >= 2 ? l2 : lo;
    hi = lim >= 2 ? h2 : hi;
    const uint32_t l3 = sel(p.m3, lo), h3 = sel(p.m3, hi);
    lo = lim >= 3 ? l3 : lo;
    hi = lim >= 3 ? h3 : hi;
  }
  __device__ __forceinline__ void compose_byte(uint32_t b, uint32_t& lo, uint32_t& hi) const {
    lo = sel(V[b], lo);
    hi = sel(V[b], hi);
  }
};

// DFA whose two-byte table fits in LDS (esz * S' * K^2 <= kPairMaxT2 bytes;
// C3's 20-state, 12-class regex: 15.6 KiB with u32 entries): ONE table lookup
// per TWO input bytes. LDS image:
//   C (u8 [256] at LDS 0): C[b] = esz class(b); four byte values share a
//      dword, so ASCII's class reads never conflict. The pair's column offset
//      esz (c1 K + c2) = C[b0] K + C[b1] is one v_mad_u32_u24; the four class
//      reads of a word depend only on the input and are issued a word ahead.
//      (u32 byte tables UA[b] + UB[b], rounds 2-4, conflicted on text: 4.1 LDS
//      cycles per read on C3's corpus, tools/lds_bank_sim.py.)
//   T2 (at kPairT2): [S'][K][K] entries (u32, or u16 when the image exceeds
//      16 KiB), entry = next state after the pair, PREMULTIPLIED to its row's
//      LDS address (kPairT2 + id * row), so the dependent chain per pair is
//      one v_add3 + one ds_read;
//   T1: u16 [S'][K] premultiplied single-byte steps (split tail, last-line check).
// A pair hides the state between its two bytes, so a '\n' FIRST in a pair that
// ends a matching line (the byte enters start_m) leads to a SHADOW state: a copy
// of the state the second byte reaches, with its rows. The host numbers the
// states so that shadows, start_m and shadow(start_m) are the highest: a
// pair-end state >= thr means an event -- at its first byte if it is a shadow
// other than start_m, at its second byte if it is >= M (start_m or its shadow).
template <uint32_t ESZ>
struct StepPairT {
  static constexpr int kKind = kStepPair;
  static constexpr uint32_t kEsz = ESZ;  // bytes per T2 entry (u16 / u32)
  static constexpr uint32_t kT2 = kPairT2;
  const uint8_t* lds;
  const uint16_t* T1;
  uint32_t thr, M, div, K;
  // a0 = esz (c0 K + c1), a2 = esz (c2 K + c3): the word's two pair columns
  struct Pre {
    uint32_t a0, a2;
  };
  __device__ __forceinline__ Pre prep(uint32_t x) const {
    if constexpr (DGREP_PAIR_CK) {
      // bytes 0 and 2 from the u16 table CK[b] = esz K class(b) at kPairCK, bytes
      // 1 and 3 from C: a pair's column is CK[b0] + C[b1], no v_mul. The CK
      // addresses 2 b as ONE v_lshlrev_b32_sdwa each (byte select in the shift)
      uint32_t o0, o2;
      asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
          : "=v"(o0)
          : "v"(1u), "v"(x));
      asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
          : "=v"(o2)
          : "v"(1u), "v"(x));
      uint32_t k0 = *reinterpret_cast<const uint16_t*>(lds + kPairCK + o0), c1 = lds[(x >> 8) & 0xffu],
               k2 = *reinterpret_cast<const uint16_t*>(lds + kPairCK + o2), c3 = lds[x >> 24];
      asm("" : "+v"(k0), "+v"(c1), "+v"(k2), "+v"(c3));
      return Pre{k0 + c1, k2 + c3};
    }
    uint32_t c0 = lds[x & 0xffu], c1 = lds[(x >> 8) & 0xffu], c2 = lds[(x >> 16) & 0xffu], c3 = lds[x >> 24];
    // pinned as 32-bit values: carried across a branch as i8 they are re-masked
    asm("" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3));
    return Pre{__umul24(c0, K) + c1, __umul24(c2, K) + c3};
  }
  __device__ __forceinline__ uint32_t t2(uint32_t off) const {
    if constexpr (ESZ == 4) return *reinterpret_cast<const uint32_t*>(lds + off);
    return *reinterpret_cast<const uint16_t*>(lds + off);
  }
  __device__ __forceinline__ uint32_t first(const Pre& p, uint32_t s) const { return t2(s + p.a0); }
  __device__ __forceinline__ uint32_t second(const Pre& p, uint32_t s1) const { return t2(s1 + p.a2); }
  __device__ __forceinline__ void apply(const Pre& p, uint32_t s, uint32_t& s0, uint32_t& s1, uint32_t& s2,
                                        uint32_t& s3) const {
    s1 = first(p, s);
    s3 = second(p, s1);
    s0 = s1;
    s2 = s3;
  }
  // apply() in two parts: the word's first chain read (f), then the rest
  __device__ __forceinline__ void rest(const Pre& p, uint32_t f, uint32_t& s0, uint32_t& s1, uint32_t& s2,
                                       uint32_t& s3) const {
    s1 = f;
    s3 = second(p, s1);
    s0 = s1;
    s2 = s3;
  }
  // single-byte step (rare paths): state id = (premultiplied state - T2 base) / row bytes
  __device__ __forceinline__ uint32_t byte(uint32_t s, uint32_t b) const {
    return T1[((s - kT2) / div) * K + uint32_t(lds[b]) / ESZ];
  }
  __device__ __forceinline__ static bool is(uint32_t s, uint32_t M) { return s == M; }
  __device__ __forceinline__ bool any2(uint32_t s1, uint32_t s3) const { return max(s1, s3) >= thr; }
  // event bytes of a word whose pairs end in s1 (bytes 0-1) and s3 (bytes 2-3)
  __device__ __forceinline__ uint32_t evm(uint32_t s1, uint32_t s3) const {
    return uint32_t(s1 >= thr && s1 != M) | (uint32_t(s1 >= M) << 1) | (uint32_t(s3 >= thr && s3 != M) << 2) |
           (uint32_t(s3 >= M) << 3);
  }
};
// T2 entries: u32 when the image fits 16 KiB (a u16 chain value carried
// across the previous word's event branch is re-masked by one v_and per word:
// LLVM keeps the phi as i16), else u16 (twice the states per image)
using StepPair = StepPairT<4>;
using StepPair16 = StepPairT<2>;

// DFA of more than 256 states (large alternations, SURVEY config 4) as a
// FILTER that lives wholly in LDS: the runtime keeps the DFA's shallowest
// states (breadth-first from start, as many as kFilterImageBytes holds) and
// sends every transition that leaves them to CAND, which on '\n' enters
// CAND_END (a start-like state, like start_m). A line that never leaves the
// shallow part is decided exactly (start_m on its '\n' iff it matches); a line
// that does is emitted as a CANDIDATE (kCandidateBit) and verify_kernel re-runs
// it on the whole DFA. For C4's 1,000 keywords the shallow part is depth <= 3
// of the Aho-Corasick-like DFA and 0.8 % of the lines are candidates.
// LDS: the byte classes as u8 [256] (four byte values per dword: text's class
// reads never conflict, see kFilterClassBytes), then u16 [state][class] rows, entries premultiplied by the class count (entry
// index of the next state's row): the dependent chain per byte is one
// v_add_lshl + one ds_read_u16; the class lookups depend only on the input and
// are issued a word ahead. Ids: shallow states, CAND, start_m, CAND_END -- an
// event is a state >= start_m.
struct StepFilter {
  static constexpr int kKind = kStepFilter;
  const uint8_t* lds;
  uint32_t C;  // premultiplied CAND_END
  struct Pre {
    uint32_t c0, c1, c2, c3;
  };
  __device__ __forceinline__ uint32_t cls(uint32_t b) const { return lds[b]; }  // u8: see kFilterClassBytes
  __device__ __forceinline__ Pre prep(uint32_t x) const {
    Pre p{cls(x & 0xffu), cls((x >> 8) & 0xffu), cls((x >> 16) & 0xffu), cls(x >> 24)};
    // pin the zero-extended loads as 32-bit values: carried across the event
    // branch as i8, they cost a v_and_b32 0xff each per word
    asm("" : "+v"(p.c0), "+v"(p.c1), "+v"(p.c2), "+v"(p.c3));
    return p;
  }
  __device__ __forceinline__ uint32_t one(uint32_t s, uint32_t c) const {
    return *reinterpret_cast<const uint16_t*>(lds + kFilterClassBytes + 2u * (s + c));
  }
  __device__ __forceinline__ void apply(const Pre& p, uint32_t s, uint32_t& s0, uint32_t& s1, uint32_t& s2,
                                        uint32_t& s3) const {
    s0 = one(s, p.c0);
    s1 = one(s0, p.c1);
    s2 = one(s1, p.c2);
    s3 = one(s2, p.c3);
  }
  __device__ __forceinline__ uint32_t first(const Pre& p, uint32_t s) const { return one(s, p.c0); }
  __device__ __forceinline__ void rest(const Pre& p, uint32_t f, uint32_t& s0, uint32_t& s1, uint32_t& s2,
                                       uint32_t& s3) const {
    s0 = f;
    s1 = one(s0, p.c1);
    s2 = one(s1, p.c2);
    s3 = one(s2, p.c3);
  }
  __device__ __forceinline__ uint32_t byte(uint32_t s, uint32_t b) const { return one(s, cls(b)); }
  __device__ __forceinline__ static bool is(uint32_t s, uint32_t M) { return s >= M; }
};

// the candidate flag of an event state (kStepFilter: CAND_END)
template <class Step>
__device__ __forceinline__ bool cand_of(const Step& st, uint32_t s) {
  if constexpr (Step::kKind == kStepFilter) return s == st.C;
  return false;
}

template <class Step>
__device__ __forceinline__ Step make_step(const uint8_t* lds, const ScanArgs& a);
template <>
__device__ __forceinline__ StepFilter make_step<StepFilter>(const uint8_t* lds, const ScanArgs& a) {
  return StepFilter{lds, a.cand_end};
}
template <class P>
__device__ __forceinline__ P make_pair_step(const uint8_t* lds, const ScanArgs& a) {
  return P{lds, reinterpret_cast<const uint16_t*>(lds + a.pair_t1), a.pair_thr, a.start_m, a.pair_div, a.nclasses};
}
template <>
__device__ __forceinline__ StepPair make_step<StepPair>(const uint8_t* lds, const ScanArgs& a) {
  return make_pair_step<StepPair>(lds, a);
}
template <>
__device__ __forceinline__ StepPair16 make_step<StepPair16>(const uint8_t* lds, const ScanArgs& a) {
  return make_pair_step<StepPair16>(lds, a);
}

template <>
__device__ __forceinline__ StepTable make_step<StepTable>(const uint8_t* lds, const ScanArgs&) { return StepTable{lds}; }
template <>
__device__ __forceinline__ StepSheng8 make_step<StepSheng8>(const uint8_t* lds, const ScanArgs&) {
  return StepSheng8{reinterpret_cast<const uint2*>(lds)};
}

template <class Step>
struct Tune;
// S = chunks per lane (1, or 2 stepped in lockstep by run_lane2)
template <>
struct Tune<StepSheng8> {
  static constexpr int C = DGREP_SHENG_CHUNK, E = DGREP_SHENG_SLOTS, B = DGREP_SHENG_BLOCK, S = 1;
};
template <>
struct Tune<StepTable> {
  static constexpr int C = DGREP_TABLE_CHUNK, E = DGREP_TABLE_SLOTS, B = DGREP_TABLE_BLOCK, S = 2;
};
template <>
struct Tune<StepFilter> {
  static constexpr int C = DGREP_FILTER_CHUNK, E = DGREP_FILTER_SLOTS, B = DGREP_FILTER_BLOCK, S = 1;
};
static_assert(Tune<StepFilter>::C % Tune<StepFilter>::B == 0 && Tune<StepFilter>::C <= 32768, "bad filter chunk");
template <uint32_t ESZ>
struct Tune<StepPairT<ESZ>> {
  static constexpr int C = DGREP_PAIR_CHUNK, E = DGREP_PAIR_SLOTS, B = DGREP_PAIR_BLOCK, S = 1;
};
static_assert(Tune<StepPair>::B == 64 || Tune<StepPair>::B == 128, "block must be 64 or 128 bytes");
static_assert(Tune<StepPair>::C % Tune<StepPair>::B == 0 && Tune<StepPair>::C <= 32768, "bad pair chunk");
static_assert(Tune<StepSheng8>::B == 64 || Tune<StepSheng8>::B == 128, "block must be 64 or 128 bytes");
static_assert(Tune<StepTable>::B == 64 || Tune<StepTable>::B == 128, "block must be 64 or 128 bytes");
static_assert(Tune<StepSheng8>::C % Tune<StepSheng8>::B == 0 && Tune<StepTable>::C % Tune<StepTable>::B == 0,
              "chunk must be a multiple of the block");
// the LDS slots pack a matching line's chunk-relative start and '\n' index in
// 16 bits each (Emitter): a start below 65,536 and rel <= start fit, and the
// one start that does not -- a lane's last line starting exactly AT its chunk
// end C = 65,536 -- is flagged in the lane's tail (kTailAtEnd). Round 4's 64 KiB
// build packed that start as 0 and ORed bit 16 into rel, which failed the
// 32 GiB C5 full-split parity.
#ifndef DGREP_MAX_LANE_CHUNK
#define DGREP_MAX_LANE_CHUNK 65536
#endif
constexpr int kMaxLaneChunk = DGREP_MAX_LANE_CHUNK;
static_assert(kMaxLaneChunk <= 65536, "16-bit slot offsets and 23-bit tile-relative line indices");
static_assert(Tune<StepSheng8>::C <= kMaxLaneChunk && Tune<StepTable>::C <= kMaxLaneChunk,
              "lane chunk above 64 KiB overflows the 16-bit LDS slot offsets");

// chunks per lane: the table stepper runs two in lockstep while its table is
// small (<= 64 states); a bigger table would lose more occupancy (the LDS
// slots double) than the second dependency chain gains
template <class Step, int TBL>
constexpr int streams_of() {
  return Step::kKind == kStepTable ? (TBL <= 64 * int(kRow) ? Tune<Step>::S : 1) : Tune<Step>::S;
}

// Per-lane run state. Positions are relative to the lane's chunk start `cs`.
struct LaneRun {
  uint32_t s;        // DFA state
  uint32_t nl;       // '\n' bytes consumed so far
  int64_t prev_nl;   // position of the last consumed '\n' (-1: none / split start)
  bool seen;         // a line boundary has been crossed (owned lines begin)
  bool term;         // the terminating '\n' at or after the chunk end was consumed
  bool parked;       // the last owned line was parked (park_pending) in this tile
  uint32_t nev;      // matching lines emitted
};
// ScanArgs::tails entry of a lane whose last record's slot holds kSlotLong: the
// real length, or (bit 63) a PENDING line's index in the pending list; bit 62
// (either case): the line starts exactly at the chunk end, see kSlotLong
constexpr uint64_t kTailPending = 1ull << 63;
constexpr uint64_t kTailAtEnd = 1ull << 62;
// slot word 0 of a line starting at chunk-relative `start` (<= C <= 64 KiB)
// with `rel` '\n' of the chunk before it; a start of 65,536 (= C, the lane's
// last line) is flagged in the tail instead (returns kTailAtEnd)
__device__ __forceinline__ uint64_t slot_at_end(int64_t start) {
  return uint64_t(start) > 0xffffu ? kTailAtEnd : 0u;
}

template <int E, bool DIRECT>
struct Emitter {
  const ScanArgs* a;
  uint32_t* slots;       // LDS [E][2] of this lane (slot mode)
  uint64_t cs;
  uint64_t out_base;     // first staging index of this lane (direct mode)
  uint32_t nl_prefix;    // '\n' between tile start and chunk start (direct mode)
  uint2* spill = nullptr;    // slot mode: this lane's HBM spill area (nullptr: none)
  uint32_t spill_cap = 0;    // its records
  uint64_t* tail = nullptr;  // slot mode: this lane's ScanArgs::tails entry
  // Sheng chunk maps (nullptr: none): this lane's ChunkMap record, and its LDS
  // copy of the map while the chunk has shown no '\n' (kept out of registers:
  // only the map-mode blocks hold it)
  uint4* cmap = nullptr;
  uint2* mapsl = nullptr;
  // direct mode (overflow pass): the lane this sub-lane re-runs parked its last
  // line at chunk-relative `park_at` (0: it did not) as pending entry park_idx;
  // the sub-lane that reaches that point stages the same PENDING record instead
  // of reading the long line on alone
  uint64_t park_at = 0;
  uint32_t park_idx = 0;

  // cand: a filter candidate (verified afterwards)
  __device__ __forceinline__ void operator()(LaneRun& r, uint64_t q, int64_t start, uint32_t rel,
                                             bool cand = false) const {
    const uint64_t len = q - uint64_t(start);
    if (DIRECT) {
      const uint64_t o = out_base + r.nev;
      if (o < a->capacity) {
        StagedLine L;
        L.start = cs + uint64_t(start);
        L.len_lo = uint32_t(len);
        L.meta = meta_of(nl_prefix + rel, len, cand);
        a->staging[o] = L;
      }
    } else {
      // only the lane's last owned line can reach past its <= 64 KiB chunk
      // or start at its end
      const uint64_t ae = slot_at_end(start);
      uint32_t lw = uint32_t(len) | (cand ? kCandidateBit : 0u);
      if (len >= kSlotLong || ae) {
        lw = kSlotLong | (cand ? kCandidateBit : 0u);
        *tail = len | ae;
      }
      // start < 65,536 and rel <= start fit 16 bits each
      const uint32_t w0 = ae ? 0u : uint32_t(start) | (rel << 16);
      if (r.nev < uint32_t(E)) {
        slots[r.nev * 2 + 0] = w0;
        slots[r.nev * 2 + 1] = lw;
      } else if (r.nev - uint32_t(E) < spill_cap) {
        // LDS slots full: the lane's further records go to its spill area in
        // HBM (read back at the tile's end), so a dense pattern neither caps
        // the lane chunk nor sends the lane to the overflow pass
        spill[r.nev - uint32_t(E)] = make_uint2(w0, lw);
      }
    }
    ++r.nev;
  }
  // slot mode: the lane's last owned line is left PENDING (pending-list index
  // idx), resolved after the scan (long_end / long_map / long_fin kernels)
  __device__ __forceinline__ void pending(LaneRun& r, int64_t start, uint32_t rel, uint64_t idx) const {
    const uint64_t ae = slot_at_end(start);
    const uint32_t w0 = ae ? 0u : uint32_t(start) | (rel << 16);
    *tail = kTailPending | ae | idx;
    if (r.nev < uint32_t(E)) {
      slots[r.nev * 2 + 0] = w0;
      slots[r.nev * 2 + 1] = kSlotLong;
    } else if (r.nev - uint32_t(E) < spill_cap) {
      spill[r.nev - uint32_t(E)] = make_uint2(w0, kSlotLong);
    }
    ++r.nev;
  }
  // direct mode: the PENDING record of the line parked at park_at (see above)
  __device__ __forceinline__ void pending_direct(LaneRun& r, int64_t start, uint32_t rel) const {
    const uint64_t o = out_base + r.nev;
    if (o < a->capacity) {
      StagedLine L;
      L.start = cs + uint64_t(start);
      L.len_lo = park_idx;
      L.meta = (nl_prefix + rel) | kMetaPend;
      a->staging[o] = L;
    }
    ++r.nev;
  }
  // The same for a line wholly inside the lane's chunk (start < q < C <= 64 KiB):
  // 32-bit chunk-relative positions, no length checks.
  // inner() for the slot mode with a dummy slot E (flat_emit()): own = the
  // lane owns the line. A write for a line it does not own lands in a slot (or
  // spill entry) no record has claimed yet, so it is never read.
  __device__ __forceinline__ void inner_flat(LaneRun& r, uint32_t q, uint32_t start, uint32_t rel, bool cand,
                                             bool own) const {
    const uint32_t lw = (q - start) | (cand ? kCandidateBit : 0u);
    const uint32_t w0 = start | (rel << 16);
    const uint32_t i = min(r.nev, uint32_t(E));
    *reinterpret_cast<uint2*>(slots + 2u * i) = make_uint2(w0, lw);
    if (r.nev - uint32_t(E) < spill_cap) spill[r.nev - uint32_t(E)] = make_uint2(w0, lw);  // wraps below E
    r.nev += own ? 1u : 0u;
  }
  __device__ __forceinline__ void inner(LaneRun& r, uint32_t q, uint32_t start, uint32_t rel, bool cand) const {
    const uint32_t lw = (q - start) | (cand ? kCandidateBit : 0u);
    if (DIRECT) {
      const uint64_t o = out_base + r.nev;
      if (o < a->capacity) {
        StagedLine L;
        L.start = cs + uint64_t(start);
        L.len_lo = q - start;
        L.meta = meta_of(nl_prefix + rel, 0, cand);
        a->staging[o] = L;
      }
    } else {
      const uint32_t w0 = start | (rel << 16);
      if (r.nev < uint32_t(E)) {
        slots[r.nev * 2 + 0] = w0;
        slots[r.nev * 2 + 1] = lw;
      } else if (r.nev - uint32_t(E) < spill_cap) {
        spill[r.nev - uint32_t(E)] = make_uint2(w0, lw);
      }
    }
    ++r.nev;
  }
};

// Block-local bookkeeping shared by the 16 word steps of one 64-byte block.
struct Blk {
  uint64_t pos;     // block start
  bool past;        // block lies at or beyond the chunk end
  uint32_t nlrun;   // '\n' consumed by the lane so far (r.nl at block start + this block's)
  uint32_t lnl;     // the line the next byte belongs to, encoded (lnl_update); 0: not owned
};
// Where the current line started, as ONE register per block: lnl = 8 * (q + 3 +
// kLnlOff) for the last '\n' seen at block offset q. Word J with newline mask m
// gives f = sat(K_J - ffbh(m)), K_J = 32 J + 48 + 8 kLnlOff: 8 * (4 J + k + 3 +
// kLnlOff) for its last '\n' at byte k (ffbh = 24 - 8 k), 0 for a word without
// one (ffbh(0) = ~0u saturates); lnl = max(lnl, f) -- three VALU per word. A
// block inside the chunk starts from the lane's previous '\n' (q < 0, a value
// below every in-block one), so the matching-line path reads the line start
// with one shift and "the lane owns the line" is lnl != 0 (0: the lane has not
// crossed a '\n' yet). Blocks past the chunk end start from kLnlSeen (owned,
// previous '\n' in r.prev_nl: q there may lie further back than kLnlOff).
constexpr uint32_t kLnlOff = 1u << 17;  // > C + 1 for any C <= 64 KiB: any q >= -(C + 1) inside the chunk
constexpr uint32_t kLnlBase = 8u * (3u + kLnlOff);  // lnl >= kLnlBase: a '\n' inside this block
constexpr uint32_t kLnlSeen = 8u;
template <int J>
__device__ __forceinline__ uint32_t lnl_update(uint32_t lnl, uint32_t m) {
  uint32_t t;
  asm("v_ffbh_u32 %0, %1" : "=v"(t) : "v"(m));
  return max(lnl, __builtin_elementwise_sub_sat(uint32_t(32 * J + 48) + 8u * kLnlOff, t));
}
// block offset of the '\n' that lnl (>= kLnlBase) records
__device__ __forceinline__ uint32_t lnl_pos(uint32_t lnl) { return (lnl >> 3) - (3u + kLnlOff); }

// Steppers whose blocks start lnl from the lane's previous '\n' (the sentinel
// start above); the others start every block at 0 and take the line start
// from r.prev_nl with a select. Bit k = stepper kind k. Same-box A/B: the
// sentinel wins on the pair stepper (C3 kernel 4,116 -> 4,282 GB/s), whose
// event path runs in ~27 % of words, and costs the Sheng stepper 1.8 % (C2,
// profiles/r03/ablation/sentinel_c2.txt): a per-block init for a rare path.
#ifndef DGREP_SENTINEL_KINDS
#define DGREP_SENTINEL_KINDS ((1 << kStepPair) | (1 << kStepFilter) | (1 << kStepTable))
#endif
template <class Step>
constexpr bool sentinel() {
  return ((DGREP_SENTINEL_KINDS) >> Step::kKind) & 1;
}

// the steppers whose lanes carry the dummy slot (slot_stride): one stream per lane
template <class Step, bool DIRECT>
constexpr bool flat_emit() {
  // (not Filter: its 1024 threads x 8 B dummy would not fit beside its 124 KiB image)
  return !DIRECT && (Step::kKind == kStepSheng8 || Step::kKind == kStepPair) && Tune<Step>::S == 1;
}

// Everything a word step does after its four DFA steps s0..s3 (newline mask
// m): matching-line events, newline bookkeeping.
template <int J, class Step, int E, bool DIRECT>
__device__ __forceinline__ void word_events(const Step& st, uint32_t M, uint32_t m, uint32_t s0, uint32_t s1,
                                            uint32_t s2, uint32_t s3, Blk& b, LaneRun& r,
                                            const Emitter<E, DIRECT>& emit);

// Filter (four dependent LDS reads per word): issue the word's first chain
// read BEFORE the next word's class reads (`pf`). LDS reads complete in order,
// so a chain read issued after them also waits for them. Same-box A/B: C4
// kernel 3,678 -> 3,773 GB/s; the pair stepper (C3) lost 2.6 % with it.
#ifndef DGREP_CHAIN_FIRST_KINDS
#define DGREP_CHAIN_FIRST_KINDS (1 << kStepFilter)
#endif
template <class Step>
constexpr bool chain_first() {
  return ((DGREP_CHAIN_FIRST_KINDS) >> Step::kKind) & 1;
}
// sched_barrier mask: everything but LDS instructions may cross
constexpr int kSchedNoDs = 0x7f;

template <int J, bool MAP, class Step, int E, bool DIRECT, class PF>
__device__ __forceinline__ void word_step(const Step& st, uint32_t M, uint32_t x, const typename Step::Pre& pre,
                                          uint32_t& s, Blk& b, LaneRun& r, const Emitter<E, DIRECT>& emit,
                                          uint32_t& mlo, uint32_t& mhi, PF&& pf) {
  if constexpr (!chain_first<Step>()) pf();
  // StepTable: keep each word's work in place (hoisting the chain-independent
  // newline masks of a whole block costs ~100 VGPRs). StepSheng8 wants the
  // opposite: its state-independent LDS reads should run ahead of the chain.
  if (Step::kKind != kStepSheng8 && Step::kKind != kStepPair) __builtin_amdgcn_sched_barrier(0);
  const uint32_t m = nl_mask(x);
  uint32_t s0, s1, s2, s3;
  if constexpr (chain_first<Step>()) {
    const uint32_t f = st.first(pre, s);
    __builtin_amdgcn_sched_barrier(kSchedNoDs);
    pf();
    __builtin_amdgcn_sched_barrier(kSchedNoDs);
    st.rest(pre, f, s0, s1, s2, s3);
  } else {
    st.apply(pre, s, s0, s1, s2, s3);
  }
  if constexpr (MAP) {
    // Sheng chunk map: every state at once (two v_perm per byte), up to and
    // including the chunk's first '\n', whose offset completes the record
    if (!b.past && b.nlrun == 0u) {
      const uint32_t k = m ? uint32_t(__builtin_ctz(m)) >> 3 : 3u;
      st.compose(pre, k, mlo, mhi);
      if (m) *emit.cmap = make_uint4(mlo, mhi, uint32_t(b.pos) + 4u * J + k, 0u);
    }
  }
  word_events<J>(st, M, m, s0, s1, s2, s3, b, r, emit);
  s = s3;
}

// Two independent chunks per lane stepped in lockstep: both dependency chains
// are in one basic block (events come after both), so their latencies overlap.
template <int J, class Step, int E, bool DIRECT>
__device__ __forceinline__ void word_step2(const Step& st, uint32_t M, uint32_t xa, uint32_t xb,
                                           const typename Step::Pre& pa, const typename Step::Pre& pb, uint32_t& sa,
                                           uint32_t& sb, Blk& ba, Blk& bb, LaneRun& ra, LaneRun& rb,
                                           const Emitter<E, DIRECT>& ea, const Emitter<E, DIRECT>& eb) {
  __builtin_amdgcn_sched_barrier(0);
  const uint32_t ma = nl_mask(xa), mb = nl_mask(xb);
  uint32_t a0, a1, a2, a3, b0, b1, b2, b3;
  st.apply(pa, sa, a0, a1, a2, a3);
  st.apply(pb, sb, b0, b1, b2, b3);
  word_events<J>(st, M, ma, a0, a1, a2, a3, ba, ra, ea);
  word_events<J>(st, M, mb, b0, b1, b2, b3, bb, rb, eb);
  sa = a3;
  sb = b3;
}

// Does a word whose four DFA steps end in s0..s3 hold an event (a '\n' that
// ends a matching line)?
template <class Step>
__device__ __forceinline__ bool word_any(const Step& st, uint32_t M, uint32_t s0, uint32_t s1, uint32_t s2,
                                         uint32_t s3) {
  if constexpr (Step::kKind == kStepSheng8)
    return StepSheng8::any4(s0, s1, s2, s3, M);
  else if constexpr (Step::kKind == kStepPair)
    return st.any2(s1, s3);
  else if constexpr (Step::kKind == kStepFilter)
    return max(max(s0, s1), max(s2, s3)) >= M;
  else
    return bool(int(Step::is(s0, M)) | int(Step::is(s1, M)) | int(Step::is(s2, M)) | int(Step::is(s3, M)));
}

// The events of word J (newline mask m, states s0..s3), with `b` holding the
// block's bookkeeping of the words before J. Common case (a single '\n' in
// the word, inside the chunk): that byte is the event, the line started after
// the previous '\n' (an earlier word of the block, or r.prev_nl), all positions
// are chunk-relative 32-bit values. Anything else (several '\n' in one word,
// the part past the chunk end) takes the general loop.
template <class Step, int E, bool DIRECT>
__device__ __forceinline__ void word_emit_loop(const Step& st, uint32_t M, uint32_t J, uint32_t m, uint32_t s0,
                                               uint32_t s1, uint32_t s2, uint32_t s3, const Blk& b, LaneRun& r,
                                               const Emitter<E, DIRECT>& emit);
template <class Step, int E, bool DIRECT>
__device__ __forceinline__ void word_emit(const Step& st, uint32_t M, uint32_t J, uint32_t m, uint32_t s0,
                                          uint32_t s1, uint32_t s2, uint32_t s3, const Blk& b, LaneRun& r,
                                          const Emitter<E, DIRECT>& emit) {
  if (!b.past && (m & (m - 1u)) == 0u) {
    // branch-free operands (selects, no nested exec-mask regions)
    const uint32_t k = uint32_t(__builtin_ctz(m)) >> 3;
    // the line starts one byte after the '\n' lnl records (sentinel steppers:
    // inside the chunk lnl also encodes r.prev_nl, see lnl_update)
    uint32_t start;
    bool own;
    if constexpr (sentinel<Step>()) {
      start = uint32_t(b.pos) + (b.lnl >> 3) - (2u + kLnlOff);
      own = b.lnl != 0;
    } else {
      start = b.lnl ? uint32_t(b.pos) + (b.lnl >> 3) - (2u + kLnlOff) : uint32_t(r.prev_nl) + 1u;
      own = r.seen | (b.lnl != 0);
    }
    const uint32_t sk = k == 0 ? s0 : k == 1 ? s1 : k == 2 ? s2 : s3;
    if constexpr (flat_emit<Step, DIRECT>())
      emit.inner_flat(r, uint32_t(b.pos) + 4u * J + k, start, b.nlrun, cand_of(st, sk), own);
    else if (own)
      emit.inner(r, uint32_t(b.pos) + 4u * J + k, start, b.nlrun, cand_of(st, sk));
    return;
  }
  word_emit_loop(st, M, J, m, s0, s1, s2, s3, b, r, emit);
}

// word_emit's general loop: several '\n' in the word, or past the chunk end
template <class Step, int E, bool DIRECT>
__device__ __forceinline__ void word_emit_loop(const Step& st, uint32_t M, uint32_t J, uint32_t m, uint32_t s0,
                                               uint32_t s1, uint32_t s2, uint32_t s3, const Blk& b, LaneRun& r,
                                               const Emitter<E, DIRECT>& emit) {
  const uint64_t q0 = b.pos + 4u * J;
  const bool nl_w = b.lnl >= kLnlBase;  // a '\n' in an earlier word of this block
  const bool seen_w = sentinel<Step>() ? b.lnl != 0 : (r.seen || b.lnl != 0);
  const bool term_w = r.term || (b.past && nl_w);
  const int64_t prev_w = nl_w ? int64_t(b.pos + lnl_pos(b.lnl)) : r.prev_nl;
  uint32_t evm;
  if constexpr (Step::kKind == kStepPair)
    evm = st.evm(s1, s3);
  else
    evm = uint32_t(Step::is(s0, M)) | (uint32_t(Step::is(s1, M)) << 1) | (uint32_t(Step::is(s2, M)) << 2) |
          (uint32_t(Step::is(s3, M)) << 3);
  while (evm) {
    const uint32_t k = uint32_t(__builtin_ctz(evm));
    evm &= evm - 1;
    const uint32_t below = m & ((1u << (8 * k)) - 1u);
    bool ok = seen_w || below != 0;
    if (b.past) ok = ok && !term_w && below == 0;  // only the first '\n' past the chunk end
    if (!ok) continue;
    const int64_t start = below ? int64_t(q0 + hi_byte(below)) + 1 : prev_w + 1;
    const uint32_t sk = k == 0 ? s0 : k == 1 ? s1 : k == 2 ? s2 : s3;
    emit(r, q0 + k, start, b.nlrun + uint32_t(__popc(below)), cand_of(st, sk));
  }
}

// newline bookkeeping of word J
template <int J>
__device__ __forceinline__ void word_nl(uint32_t m, Blk& b) {
  b.nlrun = add_popc(b.nlrun, m);
  b.lnl = lnl_update<J>(b.lnl, m);
}

// Steppers whose per-word event test is a wave-uniform branch on the ballot
// (v_cmp, s_cbranch_vccnz when no lane has an event) instead of an exec-mask
// region (s_and_saveexec, s_cbranch_execnz, s_or_b64 exec on every word: pair
// hot path 4.3 -> 2.4 SALU per word). Bit k = stepper kind k. Same-box A/B,
// C3 kernel (with the uniform in-chunk loop): 0.581-0.584 -> 0.582-0.589; C4
// (filter) 0.475-0.477 -> 0.470-0.484 (two runs +1.5 %, one -1 %); on the
// Sheng stepper (round 3, before the pipelined pair chain) C2 lost 2 %.
#ifndef DGREP_EV_BALLOT
#define DGREP_EV_BALLOT ((1 << kStepPair) | (1 << kStepFilter))
#endif
template <int J, class Step, int E, bool DIRECT>
__device__ __forceinline__ void word_events(const Step& st, uint32_t M, uint32_t m, uint32_t s0, uint32_t s1,
                                            uint32_t s2, uint32_t s3, Blk& b, LaneRun& r,
                                            const Emitter<E, DIRECT>& emit) {
  const bool ev = word_any(st, M, s0, s1, s2, s3);
  if constexpr (((DGREP_EV_BALLOT) >> Step::kKind) & 1) {
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(ev) != 0, 0)) {
      if (ev) word_emit(st, M, J, m, s0, s1, s2, s3, b, r, emit);
    }
  } else {
    if (__builtin_expect(ev, 0)) word_emit(st, M, J, m, s0, s1, s2, s3, b, r, emit);
  }
  word_nl<J>(m, b);
}

// Deferred events (pair stepper, in-chunk blocks; DGREP_DEFER_EVENTS). The
// per-word event path ran for the whole wave whenever ANY of its 64 lanes
// ended a matching line in the word -- 27 % of C3's words for 1.2 lanes each,
// ~30 instructions a time, 14 % of the kernel (no-event probes, same box:
// 0.667 -> 0.572 of HBM peak). Instead, an event word only CAPTURES what its
// record needs in four registers per lane (the line-start encoding lnl and the
// '\n' count before the word, its newline mask, the two pair states) and the
// block's end emits every lane's captured line at once, one pass for the whole
// wave. A lane's second event in one block first emits the pending capture
// (records stay in line order): rare, as lines are >= 40 bytes in text.
struct EvCap {
  uint64_t lanes;  // wave-uniform: the lanes holding a capture
  uint32_t a;  // lnl | (J + 1) << 26 (lnl < 2^21)
  uint32_t n;  // '\n' of the chunk before word J (Blk::nlrun)
  uint32_t m;  // word J's newline mask (nl_mask)
  uint32_t s;  // s1 | s3 << 16 (premultiplied pair states < 64 KiB)
};
template <class Step, int E, bool DIRECT>
__device__ __forceinline__ void emit_cap(const Step& st, uint32_t M, const EvCap& c, const Blk& b, LaneRun& r,
                                         const Emitter<E, DIRECT>& emit) {
  Blk w = b;
  w.lnl = c.a & ((1u << 26) - 1u);
  w.nlrun = c.n;
  const uint32_t s1 = c.s & 0xffffu, s3 = c.s >> 16;
  word_emit(st, M, (c.a >> 26) - 1u, c.m, s1, s1, s3, s3, w, r, emit);
}
template <int J, class Step, int E, bool DIRECT>
__device__ __forceinline__ void word_events_defer(const Step& st, uint32_t M, uint32_t m, uint32_t s1,
                                                  uint32_t s3, Blk& b, LaneRun& r, const Emitter<E, DIRECT>& emit,
                                                  EvCap& c) {
  const bool ev = st.any2(s1, s3);
  const uint64_t em = __builtin_amdgcn_ballot_w64(ev);
  if (__builtin_expect(em != 0, 0)) {
    // lanes with an event and a capture pending from earlier in the block
    const uint64_t fl = em & c.lanes;
    if (__builtin_expect(fl != 0, 0)) {
      if ((fl >> (threadIdx.x & 63u)) & 1u) emit_cap(st, M, c, b, r, emit);
    }
    c.lanes |= em;
    if (ev) {
      c.a = b.lnl | uint32_t(J + 1) << 26;
      c.n = b.nlrun;
      c.m = m;
      c.s = s1 | s3 << 16;
    }
  }
  word_nl<J>(m, b);
}
// the block's captured lines, by the whole wave
template <class Step, int E, bool DIRECT>
__device__ __forceinline__ void flush_caps(const Step& st, uint32_t M, const EvCap& c, const Blk& b, LaneRun& r,
                                           const Emitter<E, DIRECT>& emit) {
  if (c.lanes != 0) {
    if ((c.lanes >> (threadIdx.x & 63u)) & 1u) emit_cap(st, M, c, b, r, emit);
  }
}
#ifndef DGREP_DEFER_EVENTS
#define DGREP_DEFER_EVENTS 1
#endif
template <class Step, bool DIRECT>
constexpr bool defer_events() {
  return DGREP_DEFER_EVENTS && Step::kKind == kStepPair && !DIRECT;
}

template <bool SENT>
__device__ __forceinline__ void blk_init(Blk& b, uint64_t pos, uint64_t C, const LaneRun& r) {
  b.pos = pos;
  b.past = pos >= C;
  b.nlrun = r.nl;
  // inside the chunk: r.prev_nl - pos >= -(C + 1) > -kLnlOff
  if constexpr (SENT)
    b.lnl = !r.seen ? 0u : b.past ? kLnlSeen : 8u * uint32_t(int32_t(r.prev_nl - int64_t(pos)) + int32_t(3u + kLnlOff));
  else
    b.lnl = 0u;
}

__device__ __forceinline__ void blk_finish(const Blk& b, uint32_t s, LaneRun& r) {
  r.s = s;
  r.nl = b.nlrun;
  if (b.lnl >= kLnlBase) {
    r.seen = true;
    r.prev_nl = int64_t(b.pos + lnl_pos(b.lnl));
    if (b.past) r.term = true;
  }
}

// One BK-byte block of each of a lane's two chunks (see word_step2).
template <int BK, class Step, int E, bool DIRECT>
__device__ __forceinline__ void run_block2(const Step& st, uint32_t M, const uint4 (&va)[BK / 16],
                                           const uint4 (&vb)[BK / 16], uint64_t pos, uint64_t C, LaneRun& ra,
                                           LaneRun& rb, const Emitter<E, DIRECT>& ea, const Emitter<E, DIRECT>& eb) {
  Blk ba, bb;
  blk_init<sentinel<Step>()>(ba, pos, C, ra);
  blk_init<sentinel<Step>()>(bb, pos, C, rb);
  uint32_t sa = ra.s, sb = rb.s;
  constexpr int NW = BK / 4;
  uint32_t wa[NW], wb[NW];
#pragma unroll
  for (int i = 0; i < BK / 16; ++i) {
    wa[4 * i + 0] = va[i].x;
    wa[4 * i + 1] = va[i].y;
    wa[4 * i + 2] = va[i].z;
    wa[4 * i + 3] = va[i].w;
    wb[4 * i + 0] = vb[i].x;
    wb[4 * i + 1] = vb[i].y;
    wb[4 * i + 2] = vb[i].z;
    wb[4 * i + 3] = vb[i].w;
  }
  typename Step::Pre pa = st.prep(wa[0]), pb = st.prep(wb[0]);
#define DG_W2(J)                                                                              \
  if ((J) < NW) {                                                                             \
    const typename Step::Pre ca = pa, cb = pb;                                                \
    if ((J) + 1 < NW) {                                                                       \
      pa = st.prep(wa[(J) + 1 < NW ? (J) + 1 : 0]);                                           \
      pb = st.prep(wb[(J) + 1 < NW ? (J) + 1 : 0]);                                           \
    }                                                                                         \
    word_step2<J>(st, M, wa[(J) < NW ? (J) : 0], wb[(J) < NW ? (J) : 0], ca, cb, sa, sb, ba, bb, ra, rb, ea, eb); \
  }
  DG_W2(0) DG_W2(1) DG_W2(2) DG_W2(3) DG_W2(4) DG_W2(5) DG_W2(6) DG_W2(7)
  DG_W2(8) DG_W2(9) DG_W2(10) DG_W2(11) DG_W2(12) DG_W2(13) DG_W2(14) DG_W2(15)
  DG_W2(16) DG_W2(17) DG_W2(18) DG_W2(19) DG_W2(20) DG_W2(21) DG_W2(22) DG_W2(23)
  DG_W2(24) DG_W2(25) DG_W2(26) DG_W2(27) DG_W2(28) DG_W2(29) DG_W2(30) DG_W2(31)
#undef DG_W2
  blk_finish(ba, sa, ra);
  blk_finish(bb, sb, rb);
}

// Steppers whose dependent chain is LDS reads (pair: two per word, filter:
// four): the NEXT word's first chain read is issued as soon as this word's
// last state is known -- before this word's event test, event path and
// newline bookkeeping, which then run under that read's latency instead of
// in front of it (run_block_pipe). Bit k = stepper kind k.
#ifndef DGREP_PIPE_KINDS
#define DGREP_PIPE_KINDS ((1 << kStepPair) | (1 << kStepFilter))
#endif
template <class Step>
constexpr bool pipe_chain() {
  return ((DGREP_PIPE_KINDS) >> Step::kKind) & 1;
}

template <int BK, bool DEFER, class Step, int E, bool DIRECT>
__device__ __forceinline__ void run_block_pipe(const Step& st, uint32_t M, const uint4 (&v)[BK / 16], uint64_t pos,
                                               uint64_t C, LaneRun& r, const Emitter<E, DIRECT>& emit) {
  Blk b;
  blk_init<sentinel<Step>()>(b, pos, C, r);
  EvCap cap{0ull, 0u, 0u, 0u, 0u};  // DEFER: this block's captured event per lane
  constexpr int NW = BK / 4;
  uint32_t w[NW];
#pragma unroll
  for (int i = 0; i < BK / 16; ++i) {
    w[4 * i + 0] = v[i].x;
    w[4 * i + 1] = v[i].y;
    w[4 * i + 2] = v[i].z;
    w[4 * i + 3] = v[i].w;
  }
  // pa: word J's state-independent lookups, pb: word J + 1's; f: word J's
  // first chain read, in flight
  typename Step::Pre pa = st.prep(w[0]);
  uint32_t f = st.first(pa, r.s);
  typename Step::Pre pb = st.prep(w[1]);
  uint32_t s = r.s;
#define DG_WP(J)                                                                          \
  if ((J) < NW) {                                                                         \
    /* filter: keep each word's work in place (as word_step does) */                     \
    if (Step::kKind != kStepPair) __builtin_amdgcn_sched_barrier(0);                      \
    uint32_t s0, s1, s2, s3;                                                              \
    st.rest(pa, f, s0, s1, s2, s3);                                                       \
    if ((J) + 1 < NW) {                                                                   \
      f = st.first(pb, s3); /* issued before this word's events */                       \
      pa = pb;                                                                            \
      if ((J) + 2 < NW) pb = st.prep(w[(J) + 2 < NW ? (J) + 2 : 0]);                     \
    }                                                                                     \
    const uint32_t m = nl_mask(w[(J) < NW ? (J) : 0]);                                    \
    if constexpr (DEFER)                                                                  \
      word_events_defer<J>(st, M, m, s1, s3, b, r, emit, cap);                            \
    else                                                                                  \
      word_events<J>(st, M, m, s0, s1, s2, s3, b, r, emit);                               \
    s = s3;                                                                               \
  }
  DG_WP(0) DG_WP(1) DG_WP(2) DG_WP(3) DG_WP(4) DG_WP(5) DG_WP(6) DG_WP(7)
  DG_WP(8) DG_WP(9) DG_WP(10) DG_WP(11) DG_WP(12) DG_WP(13) DG_WP(14) DG_WP(15)
  DG_WP(16) DG_WP(17) DG_WP(18) DG_WP(19) DG_WP(20) DG_WP(21) DG_WP(22) DG_WP(23)
  DG_WP(24) DG_WP(25) DG_WP(26) DG_WP(27) DG_WP(28) DG_WP(29) DG_WP(30) DG_WP(31)
#undef DG_WP
  if constexpr (DEFER) flush_caps(st, M, cap, b, r, emit);
  blk_finish(b, s, r);
}

// DEFER: in-chunk blocks of the uniform loop (run_lane_from), see defer_events
template <int BK, bool MAP, class Step, int E, bool DIRECT, bool DEFER = false>
__device__ __forceinline__ void run_block(const Step& st, uint32_t M, const uint4 (&v)[BK / 16], uint64_t pos,
                                          uint64_t C, LaneRun& r, const Emitter<E, DIRECT>& emit) {
  if constexpr (!MAP && pipe_chain<Step>() && (Step::kKind == kStepPair || Step::kKind == kStepFilter)) {
    run_block_pipe<BK, DEFER>(st, M, v, pos, C, r, emit);
    return;
  }
  Blk b;
  blk_init<sentinel<Step>()>(b, pos, C, r);
  uint32_t s = r.s;
  // word j's state-independent work (Step::prep) is issued one word ahead
  constexpr int NW = BK / 4;
  uint32_t w[NW];
#pragma unroll
  for (int i = 0; i < BK / 16; ++i) {
    w[4 * i + 0] = v[i].x;
    w[4 * i + 1] = v[i].y;
    w[4 * i + 2] = v[i].z;
    w[4 * i + 3] = v[i].w;
  }
  uint32_t mlo = 0, mhi = 0;
  if constexpr (MAP) {
    const uint2 v = *emit.mapsl;
    mlo = v.x;
    mhi = v.y;
  }
  typename Step::Pre pre = st.prep(w[0]);
#define DG_W(J)                                                                         \
  if ((J) < NW) {                                                                       \
    const typename Step::Pre cur = pre;                                                 \
    word_step<J, MAP>(st, M, w[(J) < NW ? (J) : 0], cur, s, b, r, emit, mlo, mhi, [&] { \
      if ((J) + 1 < NW) pre = st.prep(w[(J) + 1 < NW ? (J) + 1 : 0]);                   \
    });                                                                                 \
  }
  DG_W(0) DG_W(1) DG_W(2) DG_W(3) DG_W(4) DG_W(5) DG_W(6) DG_W(7)
  DG_W(8) DG_W(9) DG_W(10) DG_W(11) DG_W(12) DG_W(13) DG_W(14) DG_W(15)
  DG_W(16) DG_W(17) DG_W(18) DG_W(19) DG_W(20) DG_W(21) DG_W(22) DG_W(23)
  DG_W(24) DG_W(25) DG_W(26) DG_W(27) DG_W(28) DG_W(29) DG_W(30) DG_W(31)
#undef DG_W
  if constexpr (MAP) {
    if (b.nlrun == 0u) *emit.mapsl = make_uint2(mlo, mhi);
  }
  blk_finish(b, s, r);
}

// Split loads: BK bytes of one lane, 16 B per load (through L2: non-temporal
// loads measured ~2x slower, the per-lane 16-B pieces of a 128-B line rely on it)
template <int BK>
__device__ __forceinline__ void load_block(uint4 (&v)[BK / 16], const uint8_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < BK / 16; ++i) v[i] = q[i];
}

// The last < BLOCK bytes of the split, one byte at a time, then the end of the
// split closes the last owned line (strings.Split's final piece).
template <class Step, int E, bool DIRECT>
__device__ __forceinline__ void run_tail(const Step& st, uint32_t M, const uint8_t* p, uint64_t pos, uint64_t avail, uint64_t C,
                         LaneRun& r, uint32_t& nl_chunk, bool& snap, const Emitter<E, DIRECT>& emit) {
  // Sheng chunk map: continued byte by byte while the chunk shows no '\n'
  const bool tm = Step::kKind == kStepSheng8 && emit.cmap && r.nl == 0u && pos < C;
  uint32_t mlo = 0, mhi = 0;
  if (tm) {
    const uint2 v = *emit.mapsl;
    mlo = v.x;
    mhi = v.y;
  }
  if constexpr (Step::kKind == kStepSheng8 && kLazyMapBytes != 0) {
    // the split ends before the lazy point (run_lane_from never reached it):
    // a '\n' already seen makes a LAZY record; else the map starts at byte 0
    if (emit.cmap && pos < kLazyMapBytes) {
      if (r.nl != 0u) {
        *emit.cmap = make_uint4(0u, 0u, kLazyNewline, 0u);
      } else {
        mlo = 0x03020100u;
        mhi = 0x07060504u;
        for (uint64_t q = 0; q < pos; ++q) st.compose_byte(p[q], mlo, mhi);
      }
    }
  }
  for (; pos < avail; ++pos) {
    if (pos == C) {
      nl_chunk = r.nl;
      snap = true;
      if (tm && r.nl == 0u) *emit.cmap = make_uint4(mlo, mhi, kNoNewline, 0u);
    }
    if (pos >= C && (r.term || !r.seen)) return;
    const uint32_t b = p[pos];
    const uint32_t s1 = st.byte(r.s, b);
    if constexpr (Step::kKind == kStepSheng8) {
      if (tm && r.nl == 0u && pos < C) {
        st.compose_byte(b, mlo, mhi);
        if (b == '\n') *emit.cmap = make_uint4(mlo, mhi, uint32_t(pos), 0u);
      }
    }

    if (b == '\n') {
      if (Step::is(s1, M) && r.seen && !(pos >= C && r.term)) emit(r, pos, r.prev_nl + 1, r.nl, cand_of(st, s1));
      r.seen = true;
      ++r.nl;
      r.prev_nl = int64_t(pos);
      if (pos >= C) r.term = true;
    }
    r.s = s1;
  }
  // the split ends inside the chunk (or at its end) before any '\n'
  if (tm && r.nl == 0u && avail <= C) *emit.cmap = make_uint4(mlo, mhi, kNoNewline, 0u);
  const uint32_t se = st.byte(r.s, uint32_t('\n'));
  if (!r.term && r.seen && Step::is(se, M)) emit(r, avail, r.prev_nl + 1, r.nl, cand_of(st, se));
}

__device__ __forceinline__ void lane_init(const ScanArgs& a, uint64_t cs, LaneRun& r) {
  r.s = a.start;
  r.nl = 0;
  r.prev_nl = -1;
  r.seen = (cs == 0);
  r.term = false;
  r.parked = false;
  r.nev = 0;
}

// The <= 256-state steppers and the filter park long lines in the main scan
// (slot mode; the overflow pass stops at the same point). The filter's state
// at the park point is not used (CAND has no exact DFA state): its parked
// lines are decided from their start on the whole DFA (long_dfa_* kernels).
// The wide stepper is a forced test path: its lanes read a long line to its end.
#ifndef DGREP_FILTER_PARK
#define DGREP_FILTER_PARK 1
#endif
template <class Step, bool DIRECT>
constexpr bool track_long() {
  return (Step::kKind == kStepSheng8 || Step::kKind == kStepPair || Step::kKind == kStepTable ||
          (Step::kKind == kStepFilter && DGREP_FILTER_PARK)) &&
         !DIRECT;
}
// the parked state as an index of ScanArgs::pend_states (stepper encoding ->
// DFA state of the blob)
template <class Step>
__device__ __forceinline__ uint32_t park_index(const ScanArgs& a, uint32_t s) {
  if constexpr (Step::kKind == kStepSheng8) return s & 0xffu;
  else if constexpr (Step::kKind == kStepPair) return (s - Step::kT2) / a.pair_div;
  else if constexpr (Step::kKind == kStepFilter) return 0;  // re-run from the line start
  else return s;
}

// Past the chunk end the lane stops once its last owned line is finished
// (term) -- or at once if it owns no line at all (no '\n' in its chunk: the
// chunk lies inside a line an earlier lane owns).
__device__ __forceinline__ bool lane_done(uint64_t pos, uint64_t C, const LaneRun& r) {
  return pos >= C && (r.term || !r.seen);
}

// Sheng with chunk maps: a line still open kParkAfter bytes past the chunk end
// is parked at the chunk end (its state there was kept in the lane's map slot);
// the resolution composes the maps of the chunks from C on, so the owner's
// extra work is bounded by kParkAfter instead of a whole chunk.
constexpr uint64_t kParkAfter = 4096;
static_assert(kParkAfter % Tune<StepSheng8>::B == 0, "park point must be a block boundary");

// The lane's last line is still open kParkLate bytes past its chunk end (it
// started in the lane's chunk): park it as PENDING -- state and position go to
// the pending list, the lane's record for it is resolved by the long-line
// kernels -- instead of reading on alone. Round 5: 4 KiB past C (was 2 C): the
// resolution goes on from the parked state (the filter's re-runs the line from
// its start), and a lane reading on to 2 C held its wave (63 lanes done at C)
// for a whole second chunk in every tile holding a long line's start (long_c4
// scan 7.3 ms per 16 GiB against C4's 4.3). DGREP_PARK_AFTER=0: 2 C.
#ifndef DGREP_PARK_AFTER
#define DGREP_PARK_AFTER 4096
#endif
template <class Step>
__device__ __forceinline__ uint64_t park_point(uint64_t C) {
  if constexpr (DGREP_PARK_AFTER != 0) return C + DGREP_PARK_AFTER;
  return 2 * C;
}
static_assert(DGREP_PARK_AFTER % 128 == 0, "park point must be a block boundary");
template <class Step, int E>
__device__ __forceinline__ void park_pending(const ScanArgs& a, uint64_t cs, uint64_t pos, LaneRun& r,
                                             const Emitter<E, false>& emit, uint32_t s) {
  const unsigned long long idx = atomicAdd(a.pend_count, 1ull);
  if (idx < a.pend_cap) {
    PendingLine P;
    P.line_start = cs + uint64_t(r.prev_nl + 1);
    P.resume = cs + pos;
    P.state = park_index<Step>(a, s);
    P.matched = 0;
    P.len = 0;
    a.pend[idx] = P;
  }
  emit.pending(r, r.prev_nl + 1, r.nl, idx);
  r.term = true;
  r.parked = true;
}

// Sheng chunk maps, lazily: a lane that reaches kLazyMapBytes without a '\n'
// composes the map of those bytes now (read again, from L2) and goes on in
// map mode; in text nearly every lane has met a '\n' by then, so the wave
// skips map mode entirely (same-box A/B, C2: map-mode blocks from byte 0 cost
// 0.8 %, profiles/r04/ablation).
template <class Step>
__device__ __forceinline__ void lazy_map(const Step& st, const uint8_t* p, uint2* mapsl) {
  uint32_t lo = 0x03020100u, hi = 0x07060504u;
#pragma unroll 1
  for (uint32_t q = 0; q < kLazyMapBytes; q += 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(p + q);
    st.compose(st.prep(v.x), 3, lo, hi);
    st.compose(st.prep(v.y), 3, lo, hi);
    st.compose(st.prep(v.z), 3, lo, hi);
    st.compose(st.prep(v.w), 3, lo, hi);
  }
  *mapsl = make_uint2(lo, hi);
}

// Steppers whose in-chunk blocks run in a separate wave-uniform loop (see
// run_lane_from). Bit k = stepper kind k. Same-box A/B (profiles/r05/ablation/
// uniform_main.txt): C3 kernel 0.577-0.579 -> 0.581-0.584 (the latch's ~100
// SALU of exit-mask merges per two blocks gone); C2 (Sheng) unchanged, C4
// (filter) 0.479-0.485 -> 0.475-0.476, so pair only.
#ifndef DGREP_UNIFORM_MAIN
#define DGREP_UNIFORM_MAIN (1 << kStepPair)
#endif
template <class Step, bool DIRECT>
constexpr bool uniform_main() {
  return !DIRECT && (((DGREP_UNIFORM_MAIN) >> Step::kKind) & 1);
}

// Runs a lane (see file comment) from chunk-relative position pos0 over
// BK-byte blocks with direct per-lane loads, prefetching the next block while
// the current one is stepped (two register buffers, ping-pong). Returns the
// number of '\n' inside the lane's own chunk [cs, cs + C).
template <int BK, class Step, int E, bool DIRECT>
__device__ __forceinline__ uint32_t run_lane_from(const ScanArgs& a, const Step& st, uint64_t cs, uint64_t pos0,
                                                  LaneRun& r, const Emitter<E, DIRECT>& emit, const uint32_t C) {
  const uint32_t M = a.start_m;
  const uint64_t avail = cs < a.n ? a.n - cs : 0;
  if (avail <= pos0) {
    // the split ends exactly here: strings.Split's final piece
    const uint32_t se = st.byte(r.s, uint32_t('\n'));
    if (!r.term && r.seen && Step::is(se, M)) emit(r, avail, r.prev_nl + 1, r.nl, cand_of(st, se));
    return r.nl;
  }

  const uint8_t* __restrict__ p = a.data + cs;
  uint32_t nl_chunk = 0;
  bool snap = false;
  uint64_t pos = pos0;
  uint4 A[BK / 16], B[BK / 16];
  constexpr bool kTrack = track_long<Step, DIRECT>();
  const bool park = kTrack && a.pend != nullptr;
  // Sheng chunk maps (a.chunk_map): a block goes through the map-tracking copy
  // while any lane of the wave has not met its chunk's first '\n' yet
  // (wave-uniform branch; in text, the first few blocks of a chunk)
  constexpr bool kMap = kTrack && Step::kKind == kStepSheng8;
  const bool maps = kMap && emit.cmap != nullptr;
  if (maps && pos0 == 0) *emit.mapsl = make_uint2(0x03020100u, 0x07060504u);  // identity
  if (pos0 + BK <= avail) load_block<BK>(A, p + pos0);
#define DG_STEP(V, NX)                                                                     \
  if (kMap && __ballot(maps && r.nl == 0u && pos >= kLazyMapBytes && pos < uint64_t(C)) != 0) \
    run_block<BK, kMap>(st, M, V, pos, uint64_t(C), r, emit);                              \
  else                                                                                     \
    run_block<BK, false>(st, M, V, pos, uint64_t(C), r, emit);
// in-chunk blocks of the wave-uniform loop: no map mode (pair only), events deferred
#define DG_STEP_U(V) run_block<BK, false, Step, E, DIRECT, defer_events<Step, DIRECT>()>(st, M, V, pos, uint64_t(C), r, emit);
#define DG_CHECK                                                                           \
  if constexpr (kMap && kLazyMapBytes != 0) {                                              \
    if (maps && pos == kLazyMapBytes) {                                                    \
      if (r.nl != 0u)                                                                      \
        *emit.cmap = make_uint4(0u, 0u, kLazyNewline, 0u); /* resolved from the bytes */  \
      else                                                                                 \
        lazy_map(st, p, emit.mapsl);                                                       \
    }                                                                                      \
  }                                                                                        \
  if (pos == uint64_t(C)) {                                                                \
    nl_chunk = r.nl;                                                                       \
    snap = true;                                                                           \
    if (kMap && maps) {                                                                    \
      if (r.nl == 0u) {                                                                    \
        const uint2 mv = *emit.mapsl; /* the whole chunk: no '\n' in it */                \
        *emit.cmap = make_uint4(mv.x, mv.y, kNoNewline, 0u);                               \
      }                                                                                    \
      emit.mapsl->x = r.s; /* the state at C: a line still open at C + kParkAfter */       \
    }                                                                                      \
  }                                                                                        \
  if (lane_done(pos, uint64_t(C), r)) break;                                               \
  if constexpr (DIRECT) {                                                                  \
    if (emit.park_at && pos == emit.park_at) {                                             \
      /* the main scan parked this line here: the same pending entry decides it */         \
      emit.pending_direct(r, r.prev_nl + 1, r.nl);                                         \
      r.term = true;                                                                       \
      break;                                                                               \
    }                                                                                      \
  }                                                                                        \
  if constexpr (kTrack) {                                                                  \
    if (maps && pos == uint64_t(C) + kParkAfter) {                                         \
      /* parked at C: the chunk maps from C on finish it */                                \
      park_pending<Step, E>(a, cs, uint64_t(C), r, emit, emit.mapsl->x);                   \
      break;                                                                               \
    }                                                                                      \
    if (park && !maps && pos == park_point<Step>(uint64_t(C))) {                           \
      park_pending<Step, E>(a, cs, pos, r, emit, r.s);                                     \
      break;                                                                               \
    }                                                                                      \
  }                                                                                        \
  if (pos + BK > avail) {                                                                  \
    run_tail(st, M, p, pos, avail, uint64_t(C), r, nl_chunk, snap, emit);                  \
    break;                                                                                 \
  }
  static_assert(!(uniform_main<Step, DIRECT>() && kMap), "the uniform in-chunk loop has no chunk-map mode");
  if constexpr (uniform_main<Step, DIRECT>()) {
    // The blocks inside the chunk of a wave whose lanes all hold C + BK bytes:
    // no lane leaves before C, so this loop's trip count is wave-uniform --
    // scalar loop control, none of the per-lane exit masks (and their SALU
    // merges at every latch) of the loop below, which then runs only from the
    // last whole pair of blocks before C on. It steps two blocks per trip and
    // never past C: a forced chunk of an odd number of blocks (4224 B) leaves
    // its last block to the loop below, which takes the pos == C snapshot.
    if (pos < uint64_t(C) && __all(avail >= uint64_t(C) + BK)) {
      while (pos + 2 * BK <= uint64_t(C)) {
        if constexpr (kMap && kLazyMapBytes != 0) {
          if (maps && pos == kLazyMapBytes) {
            if (r.nl != 0u)
              *emit.cmap = make_uint4(0u, 0u, kLazyNewline, 0u);
            else
              lazy_map(st, p, emit.mapsl);
          }
        }
        load_block<BK>(B, p + pos + BK);
        DG_STEP_U(A)
        pos += BK;
        if constexpr (kMap && kLazyMapBytes != 0) {
          if (maps && pos == kLazyMapBytes) {
            if (r.nl != 0u)
              *emit.cmap = make_uint4(0u, 0u, kLazyNewline, 0u);
            else
              lazy_map(st, p, emit.mapsl);
          }
        }
        load_block<BK>(A, p + pos + BK);
        DG_STEP_U(B)
        pos += BK;
      }
    }
  }
  for (;;) {
    DG_CHECK
    load_block<BK>(B, p + (pos + 2 * BK <= avail ? pos + BK : pos));  // prefetch (or a harmless re-read)
    DG_STEP(A, B)
    pos += BK;
    DG_CHECK
    load_block<BK>(A, p + (pos + 2 * BK <= avail ? pos + BK : pos));
    DG_STEP(B, A)
    pos += BK;
  }
#undef DG_STEP
#undef DG_STEP_U
#undef DG_CHECK
  if (!snap) nl_chunk = r.nl;
  return nl_chunk;
}

template <int BK, class Step, int E, bool DIRECT>
__device__ __forceinline__ uint32_t run_lane(const ScanArgs& a, const Step& st, uint64_t cs, LaneRun& r,
                                             const Emitter<E, DIRECT>& emit, const uint32_t C) {
  lane_init(a, cs, r);
  if (cs >= a.n) return 0;
  return run_lane_from<BK>(a, st, cs, 0, r, emit, C);
}

// Two chunks per lane (csa, csb), both wholly inside the split, stepped in
// lockstep over [0, C) with direct loads (two independent dependency chains
// per lane); then each finishes its last owned line on its own.
template <int C, int BK, class Step, int E>
__device__ __forceinline__ void run_lane2(const ScanArgs& a, const Step& st, uint64_t csa, uint64_t csb, LaneRun& ra,
                                          LaneRun& rb, const Emitter<E, false>& ea, const Emitter<E, false>& eb,
                                          uint32_t& nla, uint32_t& nlb) {
  static_assert(C % (2 * BK) == 0, "chunk must hold an even number of blocks");
  const uint32_t M = a.start_m;
  lane_init(a, csa, ra);
  lane_init(a, csb, rb);
  const uint8_t* pa = a.data + csa;
  const uint8_t* pb = a.data + csb;
  uint4 A0[BK / 16], A1[BK / 16], B0[BK / 16], B1[BK / 16];
  load_block<BK>(A0, pa);
  load_block<BK>(B0, pb);
  for (uint32_t pos = 0; pos < uint32_t(C); pos += 2 * BK) {
    load_block<BK>(A1, pa + pos + BK);
    load_block<BK>(B1, pb + pos + BK);
    run_block2<BK>(st, M, A0, B0, pos, uint64_t(C), ra, rb, ea, eb);
    if (pos + 2 * BK < uint32_t(C)) {
      load_block<BK>(A0, pa + pos + 2 * BK);
      load_block<BK>(B0, pb + pos + 2 * BK);
    }
    run_block2<BK>(st, M, A1, B1, pos + BK, uint64_t(C), ra, rb, ea, eb);
  }
  nla = ra.nl;
  nlb = rb.nl;
  run_lane_from<BK>(a, st, csa, uint64_t(C), ra, ea, uint32_t(C));
  run_lane_from<BK>(a, st, csb, uint64_t(C), rb, eb, uint32_t(C));
}

// The Sheng stepper's lane chunk is chosen per split on the host
// (adaptive_chunk_bytes): the fixed chunks of the other steppers leave the
// last round of tiles over the resident waves part-empty, which at 16-KiB
// chunks costs up to a sixth of a 16-GiB split's time.
// Only one-chunk-per-lane steppers take the runtime chunk: the two-chunk path
// (run_lane2) is compiled for Tune::C.
template <class Step, int TBL>
constexpr bool adaptive_chunk() {
  return (Step::kKind == kStepSheng8 || Step::kKind == kStepPair || Step::kKind == kStepFilter) &&
         streams_of<Step, TBL>() == 1;
}
template <class Step, int TBL>
__device__ __forceinline__ uint32_t lane_chunk(const ScanArgs& a) {
  if constexpr (adaptive_chunk<Step, TBL>()) return a.chunk;
  return uint32_t(Tune<Step>::C);
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

// Calls f(byte) for every byte of [a, e), read in aligned 16-byte pieces (the
// next piece is loaded while this one is stepped; the scan read the line long
// ago, so its bytes come from HBM). f returns false to stop early. (Windows of
// two or four pieces in flight measured slower on C4: 0.498-0.502 -> 0.487-0.493.)
template <class F>
__device__ __forceinline__ void for_line_bytes(const uint8_t* data, uint64_t a, uint64_t e, F&& f) {
  if (a >= e) return;
  uint4 nxt = *reinterpret_cast<const uint4*>(data + (a & ~uint64_t(15)));
  for (uint64_t q = a & ~uint64_t(15); q < e; q += 16) {
    const uint4 w = nxt;
    if (q + 16 < e) nxt = *reinterpret_cast<const uint4*>(data + q + 16);
    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
    bool go = true;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint64_t pos = q + uint64_t(j);
      if (go && pos >= a && pos < e) go = f((ws[j >> 2] >> (8 * (j & 3))) & 0xffu);
    }
    if (!go) return;
  }
}

// waves per SIMD the register allocation must leave room for
template <class Step>
constexpr int waves_per_simd() {
  return Step::kKind == kStepSheng8  ? DGREP_SHENG_WAVES
         : Step::kKind == kStepTable ? DGREP_TABLE_WAVES
         : Step::kKind == kStepPair  ? DGREP_PAIR_WAVES
                                     : kFilterThreads / 256;  // one workgroup per CU
}

// the next tile for this wave: waves + (claims so far), wave-uniform
// (DGREP_DYNAMIC_TILES 0: the static stride t + waves, for A/B)
#ifndef DGREP_DYNAMIC_TILES
#define DGREP_DYNAMIC_TILES 1
#endif
__device__ __forceinline__ uint64_t claim_tile(const ScanArgs& a) {
  uint64_t c = 0;
  if ((threadIdx.x & 63u) == 0) c = atomicAdd(a.tile_next, 1ull);
  const uint32_t lo = uint32_t(__shfl(uint32_t(c), 0, 64)), hi = uint32_t(__shfl(uint32_t(c >> 32), 0, 64));
  return (uint64_t(hi) << 32) | lo;
}
__device__ __forceinline__ uint64_t next_tile(const ScanArgs& a, uint64_t t, uint64_t waves) {
  if (!DGREP_DYNAMIC_TILES) return t + waves;
  return waves + claim_tile(a);
}
__device__ __forceinline__ uint64_t first_tile(int tid, int NT) {
  return uint64_t(blockIdx.x) * uint64_t(NT / 64) + uint64_t(tid >> 6);
}

// One wave = one tile of 64 chunks. Waves never synchronise with each other:
// the tile's exclusive scans run on the wave's lanes (DPP/bpermute) and one
// lane reserves the tile's staging range with a single atomic.

template <class Step, int TBL, int NT>
__global__ __launch_bounds__(NT, waves_per_simd<Step>()) void scan_dfa8_kernel(ScanArgs a) {
  constexpr int E = Tune<Step>::E, BK = Tune<Step>::B;
  const uint32_t C = lane_chunk<Step, TBL>(a);
  // per-lane slot stride: E slots per stream, plus the dummy of flat_emit
  constexpr int ES = E * streams_of<Step, TBL>() + (flat_emit<Step, false>() ? 1 : 0);
  static_assert(!flat_emit<Step, false>() || streams_of<Step, TBL>() == 1, "dummy slot: one stream per lane");
  __shared__ ScanSmem<TBL, ES, NT, Step::kKind == kStepSheng8> sm;
  const int tid = int(threadIdx.x);
  for (uint32_t i = uint32_t(tid) * 16u; i < a.table_bytes; i += NT * 16u)
    *reinterpret_cast<uint4*>(sm.tbl + i) = *reinterpret_cast<const uint4*>(a.table + i);
  __syncthreads();

  const Step st = make_step<Step>(sm.tbl, a);
  constexpr int S = streams_of<Step, TBL>();  // chunks per lane: chunk k of a tile is k * 64 + lane
  uint32_t* slots = sm.slots + tid * ES * 2;
  const int lane = tid & 63;
  const uint64_t waves = uint64_t(gridDim.x) * (NT / 64);
  const uint64_t kTile = uint64_t(kTileLanes) * uint64_t(S) * uint64_t(C);
  // Tiles: the first one per wave by its index, every further one CLAIMED from
  // a counter (one atomic per tile), so a wave that runs faster takes more
  // tiles. Resident waves do not progress at one rate (the sequencer favours
  // older waves): with a static stride the youngest waves set the kernel's
  // end. Same box, C2 pattern: 12 / 18 / 32 GiB splits ran 9 % below 16 GiB,
  // whose 2.67 rounds happened to give the young waves one tile less.
  for (uint64_t t = first_tile(tid, NT); t < a.ntiles; t = next_tile(a, t, waves)) {
    uint64_t cs[S];
    LaneRun r[S];
    uint32_t nlc[S];
#pragma unroll
    for (int k = 0; k < S; ++k) cs[k] = t * kTile + (uint64_t(k) * kTileLanes + uint64_t(lane)) * uint64_t(C);
    const bool full = (t + 1) * kTile <= a.n;  // wave-uniform: the whole tile lies inside the split
    uint64_t* const tails = a.tails + (uint64_t(blockIdx.x) * NT + uint64_t(tid)) * S;
    if constexpr (S == 2) {
      Emitter<E, false> e0{&a, slots, cs[0], 0, 0}, e1{&a, slots + E * 2, cs[1], 0, 0};
      e0.tail = tails;
      e1.tail = tails + 1;
      if (a.spill) {
        // one spill area per stream
        uint2* sp0 = a.spill + ((uint64_t(blockIdx.x) * NT + uint64_t(tid)) * S) * a.spill_per_lane;
        e0.spill = sp0;
        e1.spill = sp0 + a.spill_per_lane;
        e0.spill_cap = e1.spill_cap = a.spill_per_lane;
      }
      if (full) {
        run_lane2<Tune<Step>::C, BK>(a, st, cs[0], cs[1], r[0], r[1], e0, e1, nlc[0], nlc[1]);
      } else {
        nlc[0] = run_lane<BK>(a, st, cs[0], r[0], e0, C);
        nlc[1] = run_lane<BK>(a, st, cs[1], r[1], e1, C);
      }
    } else {
      Emitter<E, false> em{&a, slots, cs[0], 0, 0};
      em.tail = tails;
      if constexpr (Step::kKind == kStepSheng8) {
        if (a.chunk_map && cs[0] < a.n) {
          em.cmap = reinterpret_cast<uint4*>(a.chunk_map + t * kTileLanes + uint64_t(lane));
          em.mapsl = &sm.maps[tid];
        }
      }
      if (a.spill) {
        em.spill = a.spill + (uint64_t(blockIdx.x) * NT + uint64_t(tid)) * S * a.spill_per_lane;
        em.spill_cap = a.spill_per_lane;
      }
      nlc[0] = run_lane<BK>(a, st, cs[0], r[0], em, C);
    }
    if constexpr (track_long<Step, false>()) {
      // '\n' per chunk (chunk index = t * 64 S + 64 k + lane): where the long-line
      // kernels look for a parked line's end
      if (a.chunk_nl) {
#pragma unroll
        for (int k = 0; k < S; ++k)
          if (cs[k] < a.n) a.chunk_nl[t * kTileLanes * S + uint64_t(k) * kTileLanes + uint64_t(lane)] = nlc[k];
      }

    }

    // tile-wide exclusive scans of (newlines, matching lines) over the tile's
    // chunks in split order (stream 0's 64 chunks, then stream 1's)
    uint32_t nl_off[S], ev_off[S], nl_tot = 0, ev_tot = 0;
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const uint32_t nl_inc = wave_incl_scan(nlc[k]);
      const uint32_t ev_inc = wave_incl_scan(r[k].nev);
      nl_off[k] = nl_tot + nl_inc - nlc[k];
      ev_off[k] = ev_tot + ev_inc - r[k].nev;
      nl_tot += __shfl(nl_inc, 63, 64);
      ev_tot += __shfl(ev_inc, 63, 64);
    }
    unsigned long long base = 0;
    if (lane == 0) {
      if (ev_tot) base = atomicAdd(a.counter, (unsigned long long)ev_tot);
      TileInfo ti;
      ti.base = base;
      ti.count = ev_tot;
      ti.nl = nl_tot;
      a.tiles[t] = ti;
    }
    base = (uint64_t(uint32_t(__shfl(uint32_t(base >> 32), 0, 64))) << 32) | uint32_t(__shfl(uint32_t(base), 0, 64));
#pragma unroll
    for (int k = 0; k < S && ev_tot != 0; ++k) {  // ev_tot: wave-uniform
      const uint32_t nev = r[k].nev;
      const uint32_t* sl = slots + k * E * 2;
      const bool spill = a.spill != nullptr;
      const uint2* sp = spill ? a.spill + ((uint64_t(blockIdx.x) * NT + uint64_t(tid)) * S + k) * a.spill_per_lane
                              : nullptr;
      const uint64_t o0 = base + ev_off[k];
      if (nev <= uint32_t(E) + (spill ? a.spill_per_lane : 0u)) {
        for (uint32_t j = 0; j < nev; ++j) {
          const uint64_t o = o0 + j;
          if (o < a.capacity) {
            uint32_t w0, w1;
            if (j < uint32_t(E)) {
              w0 = sl[j * 2 + 0];
              w1 = sl[j * 2 + 1];
            } else {
              const uint2 w = sp[j - uint32_t(E)];
              w0 = w.x;
              w1 = w.y;
            }
            // kSlotLong: the lane's last line, whose length (or pending
            // index) the lane kept in its tails entry
            uint64_t len = w1 & kSlotLong;
            uint32_t flags = (w1 & kCandidateBit) ? kMetaCand : 0u;
            uint32_t off = w0 & 0xffffu, rel = w0 >> 16;
            if (len == kSlotLong) {
              len = tails[k];
              if (len & kTailAtEnd) {
                // the line starts at the chunk end (C = 64 KiB does not fit
                // the slot's 16 bits): every '\n' of the chunk lies before it
                off = C;
                rel = nlc[k];
              }
              if (len & kTailPending) flags |= kMetaPend;
              len &= ~(kTailPending | kTailAtEnd);
            }
            StagedLine L;
            L.start = cs[k] + off;
            L.len_lo = uint32_t(len);
            L.meta = (nl_off[k] + rel) | flags | (flags & kMetaPend ? 0u : uint32_t(len >> 32) << kLenHiShift);
            a.staging[o] = L;
          }
        }
      } else {
        // more matching lines than LDS slots: scan_overflow_kernel re-runs
        // this chunk and writes straight to its final staging positions
        const unsigned long long q = atomicAdd(a.overflow_count, 1ull);
        if (q < a.overflow_cap) {
          OverflowLane ol;
          ol.cs = cs[k];
          ol.out_base = o0;
          ol.nl_prefix = nl_off[k];
          // a parked last line: its pending index + 1 (the pass stops there too)
          ol.pend = r[k].parked ? uint32_t(tails[k] & ~(kTailPending | kTailAtEnd)) + 1u : 0u;
          a.overflow[q] = ol;
        }
      }
    }
  }
}

// Lanes that owned more matching lines than their LDS slots are re-run here,
// one WAVE per such lane chunk: the chunk is cut into up to 64 sub-chunks of
// SC bytes (a multiple of the block) and sub-lane j applies the same
// line-ownership rule to sub-chunk j (it owns the lines that start in it after
// its first '\n'; sub-chunk 0 is the lane's own chunk start, so the lane's
// lines are exactly the union). Pass 1 counts each sub-lane's matching lines
// and '\n' (no writes), a wave scan turns the counts into offsets, pass 2
// re-runs every sub-chunk writing its lines straight to their final staging
// positions. Each chunk is read twice, but by 64 lanes at once, so dense
// matches no longer serialise on one thread per chunk.
constexpr int kOverflowThreads = 256;
template <class Step, int TBL>
__global__ __launch_bounds__(kOverflowThreads) void scan_overflow_kernel(ScanArgs a, uint64_t nover) {
  constexpr int E = Tune<Step>::E, BK = Tune<Step>::B;
  const uint32_t C = lane_chunk<Step, TBL>(a);
  __shared__ ScanSmem<TBL, 1, 1> sm;
  for (uint32_t i = threadIdx.x * 16u; i < a.table_bytes; i += kOverflowThreads * 16u)
    *reinterpret_cast<uint4*>(sm.tbl + i) = *reinterpret_cast<const uint4*>(a.table + i);
  __syncthreads();
  const Step st = make_step<Step>(sm.tbl, a);
  const uint32_t lane = threadIdx.x & 63u;
  // sub-chunk: C / 64 rounded UP to a whole block, so at most 64 of them
  const uint32_t sc = ((C + 63u) / 64u + uint32_t(BK) - 1u) / uint32_t(BK) * uint32_t(BK);
  const uint32_t nsub = (C + sc - 1) / sc;  // <= 64 (C and sc are multiples of BK)
  const uint64_t waves = uint64_t(gridDim.x) * (kOverflowThreads / 64);
  for (uint64_t k = uint64_t(blockIdx.x) * (kOverflowThreads / 64) + (threadIdx.x >> 6); k < nover; k += waves) {
    const OverflowLane ol = a.overflow[k];  // wave-uniform
    const bool live = lane < nsub;
    const uint64_t cs = ol.cs + uint64_t(lane) * sc;
    const uint32_t len = live ? min(sc, C - lane * sc) : 0u;
    // where the main scan parked the lane's last line (park_pending): C +
    // kParkAfter with Sheng chunk maps, else park_point -- relative to this sub-lane
    const uint64_t park = Step::kKind == kStepSheng8 && a.chunk_map ? uint64_t(C) + kParkAfter : park_point<Step>(uint64_t(C));
    const uint64_t park_at = ol.pend ? park - uint64_t(lane) * sc : 0;
    LaneRun r;
    uint32_t nl = 0, nev = 0;
    if (live) {
      // out_base = capacity: every write of the counting pass is skipped
      Emitter<E, true> cnt{&a, nullptr, cs, a.capacity, 0};
      cnt.park_at = park_at;
      nl = run_lane<BK>(a, st, cs, r, cnt, len);
      nev = r.nev;
    }
    const uint32_t nl_off = wave_incl_scan(nl) - nl;
    const uint32_t ev_off = wave_incl_scan(nev) - nev;
    if (live && nev) {
      Emitter<E, true> ed{&a, nullptr, cs, ol.out_base + ev_off, ol.nl_prefix + nl_off};
      ed.park_at = park_at;
      ed.park_idx = ol.pend - 1u;
      run_lane<BK>(a, st, cs, r, ed, len);
    }
  }
}

#if DG_PART(0)
// ---- filter verification (kStepFilter) -------------------------------------
// One wave per tile: every candidate line (kCandidateBit) of the tile's staged
// lines is re-run from its start on the WHOLE DFA and kept iff the '\n' after
// it enters start_m (grep.go:21 on that line); the tile's kept lines are
// compacted in place, in order, and its count updated; `removed` receives the
// dropped candidates. The whole DFA is numbered breadth-first from start (the
// runtime's order), so the rows a candidate line spends most of its bytes in
// are the first ones: kVerifyHotBytes of them are copied to LDS, the rest are
// read from HBM (L2-resident: [state][class], u16 entries, or u32 above 65535
// states). A line is read in aligned 16-byte pieces.
// The whole DFA (breadth-first ids, [state][class]) as the verification and
// long-line kernels read it: rows [0, hot_n / K) in LDS, optionally DfaXRec
// records for the next xn states (LDS), the rest from HBM (L2-resident).
template <typename E, bool XI = false>
struct FullDfa {
  const E* hot;  // LDS
  const __attribute__((address_space(1))) E* full;
  const uint32_t* cls;  // LDS
  uint32_t K, hot_n;    // hot_n = (resident rows) * K >= K
  // XI (the whole-DFA LDS image, runtime build_ximg): the DfaXRec of state
  // s >= xh at xr[s - xh]; its default row (a resident or an extra row) in hot
  const uint2* xr = nullptr;
  uint32_t xh = 0;
  // 32-bit index math: s * K + c < 2^21 * 256 (the compiler's state budget)
  __device__ __forceinline__ uint32_t next(uint32_t s, uint32_t b) const { return next_cls(s, cls[b]); }
  __device__ __forceinline__ uint32_t next_cls(uint32_t s, uint32_t c) const {
    const uint32_t i = __umul24(s, K) + c;
    if (i < hot_n) return uint32_t(hot[i]);
    return cold(s, c, i);
  }
  // a state past the resident rows: XI, its record (straight-line: the default
  // row's entry read unconditionally, then the exceptions selected) -- no HBM
  // read, so no vmcnt wait on the chain (a possible HBM result here made every
  // step wait for the segment's data prefetch); else the HBM table
  __device__ __forceinline__ uint32_t cold(uint32_t s, uint32_t c, uint32_t i) const {
    if constexpr (XI) {
      const uint2 r = xr[s - xh];
      uint32_t t = uint32_t(hot[__umul24(r.x & 0xffffu, K) + c]);
      t = c == (r.x >> 24) ? (r.y >> 16) : t;
      t = c == ((r.x >> 16) & 0xffu) ? (r.y & 0xffffu) : t;
      return t;
    } else {
      return uint32_t(full[i]);
    }
  }
  // state after bytes [a, e) from s, stopping at the absorbing `matched`
  __device__ __forceinline__ uint32_t run(const uint8_t* data, uint64_t a, uint64_t e, uint32_t s,
                                          uint32_t matched) const {
    if (s == matched) return s;
    for_line_bytes(data, a, e, [&](uint32_t b) {
      s = next(s, b);
      return s != matched;
    });
    return s;
  }
};

constexpr uint32_t kVerifyHotBytes = 48 * 1024;
constexpr uint32_t kVerifyLookback = 256;  // bytes a wave-verified segment's entry state is guessed from

// The tile loop shared by both verification kernels: line_matches(a, e)
// decides the candidate [a, e) (grep.go:21 on that line).
// Candidate lines longer than kVerifyWaveBytes are decided by the whole wave
// (WavePred): one lane walking a 60 KiB line on the DFA held the kernel for
// milliseconds (long-line workloads); see verify_kernel.
constexpr uint64_t kVerifyWaveBytes = 16384;
struct NoWavePred {
  __device__ bool operator()(uint64_t, uint64_t) const { return false; }
};
template <class Pred, class WavePred = NoWavePred>
__device__ __forceinline__ void verify_tiles(const VerifyArgs& v, Pred&& line_matches, WavePred&& wave_matches = {}) {
  constexpr bool kWave = !std::is_same<std::decay_t<WavePred>, NoWavePred>::value;
  const uint32_t lane = threadIdx.x & 63u, wpb = blockDim.x / 64u;
  const uint64_t waves = uint64_t(gridDim.x) * wpb;
  for (uint64_t t = uint64_t(blockIdx.x) * wpb + (threadIdx.x >> 6); t < v.ntiles; t += waves) {
    const TileInfo ti = v.tiles[t];
    if (ti.count == 0) continue;
    uint32_t kept = 0;
    for (uint32_t k0 = 0; k0 < ti.count; k0 += 64) {
      const uint32_t k = k0 + lane;
      const uint64_t src = ti.base + k;
      bool keep = false, wave = false;
      StagedLine L;
      if (k < ti.count && src < v.staging_cap) {
        L = v.staging[src];
        keep = true;
        if (L.meta & kMetaPend) {
          // a long line parked by the scan, resolved from the chunk maps
          const PendingLine P = v.pend[L.len_lo];
          keep = P.matched != 0u;
          L.len_lo = uint32_t(P.len);
          L.meta = staged_rel(L) | (uint32_t(P.len >> 32) << kLenHiShift);
        } else if (L.meta & kMetaCand) {
          L.meta &= ~kMetaCand;
          if (kWave && staged_len(L) > kVerifyWaveBytes)
            wave = true;
          else
            keep = line_matches(L.start, L.start + staged_len(L));
        }
      }
      if constexpr (kWave) {
        // the batch's long candidates, one at a time by all 64 lanes
        const uint64_t len = wave ? staged_len(L) : 0u;
        for (uint64_t wm = __ballot(wave); wm; wm &= wm - 1) {
          const int j = __ffsll((unsigned long long)wm) - 1;
          const uint64_t a = (uint64_t(uint32_t(__shfl(uint32_t(L.start >> 32), j, 64))) << 32) |
                             uint32_t(__shfl(uint32_t(L.start), j, 64));
          const uint64_t n = (uint64_t(uint32_t(__shfl(uint32_t(len >> 32), j, 64))) << 32) |
                             uint32_t(__shfl(uint32_t(len), j, 64));
          const bool r = wave_matches(a, a + n);
          if (int(lane) == j) keep = r;
        }
      }
      const uint64_t m = __ballot(keep);
      const uint32_t pos = uint32_t(__popcll(m & ((1ull << lane) - 1ull)));
      if (keep) v.staging[ti.base + kept + pos] = L;  // in place: never beyond this batch's reads
      kept += uint32_t(__popcll(m));
    }
    if (lane == 0 && kept != ti.count) {
      v.tiles[t].count = kept;
      atomicAdd(v.removed, (unsigned long long)(ti.count - kept));
    }
  }
}

// XR: the whole-DFA LDS image (runtime build_ximg) in one 1024-thread
// workgroup's LDS, one resident workgroup per CU; else the first
// kVerifyHotBytes of rows in each 256-thread workgroup's LDS, the rest in HBM
template <typename E, bool XR>
__global__ __launch_bounds__(XR ? 1024 : 256) void verify_kernel(VerifyArgs v) {
  constexpr uint32_t NT = XR ? 1024 : 256;
  constexpr uint32_t kLds = XR ? 158u * 1024u : kVerifyHotBytes;
  __shared__ uint32_t cls[256];
  __shared__ __attribute__((aligned(16))) uint8_t lbuf[kLds];
  if (threadIdx.x < 256) cls[threadIdx.x] = v.cls[threadIdx.x];
  E* const hot = reinterpret_cast<E*>(lbuf);
  const uint32_t hot_n = XR ? v.x_hot * v.nclasses : v.hot_entries;
  if constexpr (XR) {
    for (uint32_t i = threadIdx.x * 16u; i < v.ximg_bytes; i += NT * 16u)
      *reinterpret_cast<uint4*>(lbuf + i) = *reinterpret_cast<const uint4*>(v.ximg + i);
  } else {
    const E* full = static_cast<const E*>(v.full);
    for (uint32_t i = threadIdx.x; i < hot_n; i += NT) hot[i] = full[i];
  }
  __syncthreads();
  const __attribute__((address_space(1))) E* gfull = (const __attribute__((address_space(1))) E*)v.full;
  const uint32_t K = v.nclasses, cn = cls['\n'];
  FullDfa<E, XR> d{hot, gfull, cls, K, hot_n};
  if constexpr (XR) {
    d.xr = reinterpret_cast<const uint2*>(lbuf + v.xr_off);
    d.xh = v.x_hot;
  }
  auto next = [&](uint32_t s, uint32_t c) __attribute__((always_inline)) -> uint32_t { return d.next_cls(s, c); };
  // state after [a, e) from s, stopping at the absorbing MATCHED state
  auto run = [&](uint64_t a, uint64_t e, uint32_t s) __attribute__((always_inline)) -> uint32_t {
    if (s == v.matched) return s;
    for_line_bytes(v.data, a, e, [&](uint32_t b) {
      s = next(s, cls[b]);
      return s != v.matched;
    });
    return s;
  };
  verify_tiles(
      v, [&](uint64_t a, uint64_t e) { return next(run(a, e, v.start), cn) == v.start_m; },
      [&](uint64_t a, uint64_t e) {
        // a long candidate by the whole wave: lane j runs segment j from a
        // GUESSED entry state (the state after the kVerifyLookback bytes
        // before it, from start: exact for keyword automata such as config
        // 4's); the lanes then compose in order from the true state, re-running
        // (all lanes alike) a segment whose guess was wrong -- exact for any DFA
        const uint64_t n = e - a, seg = (n + 63) / 64, lane = threadIdx.x & 63u;
        const uint64_t sb = a + min(n, lane * seg), se = a + min(n, (lane + 1) * seg);
        const uint64_t from = sb - min(sb - a, uint64_t(kVerifyLookback));
        const uint32_t g = run(from, sb, v.start);
        const uint32_t x = run(sb, se, g);
        uint32_t s = v.start;
        for (int j = 0; j < 64 && s != v.matched; ++j) {
          const uint32_t gj = uint32_t(__shfl(g, j, 64)), xj = uint32_t(__shfl(x, j, 64));
          if (gj == s)
            s = xj;
          else
            s = run(a + min(n, uint64_t(j) * seg), a + min(n, uint64_t(j + 1) * seg), s);
        }
        return next(s, cn) == v.start_m || s == v.matched;
      });
}

// ---- NFA verification (DGREP_DFA_PARTIAL) -----------------------------------
// A pattern whose DFA exceeds the compiler's budget ships its first DFA states
// (the filter) and an NFA program (include/dgrep_blob.h): per rune class, a
// bit-parallel step over at most 1024 positions (the NFA's rune-set states),
// with the UTF-8 decoder trie and the context flags (line start, previous rune
// a word character) the DFA construction uses. One lane per candidate line;
// the program is small and stays in L2. The position sets live in registers:
// the kernel is instantiated for up to 256 positions (8 words, the common
// case) and up to DGREP_NFA_MAX_POS (32 words).
constexpr uint32_t kNfaMaxWords = DGREP_NFA_MAX_POS / 32;
constexpr uint32_t kNfaSmallWords = 8;

struct NfaView {
  const int32_t* child;
  const uint32_t *depth, *word, *has, *init, *init_m, *cl, *mx, *end_init, *end_x;
  uint32_t nw, nctx, fffd, has_word;
};

__device__ __forceinline__ NfaView nfa_view(const uint32_t* g) {
  NfaView n;
  const uint32_t nw = g[2], nrc = g[3], nnodes = g[4], nctx = g[5], npos = g[1];
  n.nw = nw;
  n.nctx = nctx;
  n.fffd = g[6];
  n.has_word = g[7];
  const uint32_t* p = g + 8;
  n.child = reinterpret_cast<const int32_t*>(p);
  p += size_t(nnodes) * 256;
  n.depth = p;
  p += nnodes;
  n.word = p;
  p += nrc;
  n.has = p;
  p += size_t(nrc) * nw;
  n.init = p;
  p += 2 * nctx * nw;
  n.init_m = p;
  p += 2 * nctx;
  n.cl = p;
  p += size_t(npos) * nctx * nw;
  n.mx = p;
  p += nctx * nw;
  n.end_init = p;
  p += 4;
  n.end_x = p;
  return n;
}

template <uint32_t NW>
struct NfaRun {
  uint32_t P[NW];  // positions consumed by the last rune
  uint32_t begin, pw, node;  // no rune yet on the line; previous rune is a word char; decoder node
  bool matched;
};

// one rune of class c (DfaBuilder::step, per position)
template <uint32_t NW>
__device__ __forceinline__ void nfa_rune(const NfaView& g, NfaRun<NW>& r, uint32_t c) {
  const uint32_t nwf = g.word[c];
  const uint32_t ctx = g.has_word ? r.pw * 2u + nwf : 0u;
  const uint32_t nw = g.nw;
  const uint32_t* ini = g.init + (size_t(r.begin) * g.nctx + ctx) * nw;
  const uint32_t* mx = g.mx + size_t(ctx) * nw;
  bool m = g.init_m[r.begin * g.nctx + ctx] != 0u;
  uint32_t S[NW];
#pragma unroll
  for (uint32_t j = 0; j < NW; ++j) S[j] = j < nw ? ini[j] : 0u;
#pragma unroll
  for (uint32_t w = 0; w < NW; ++w) {
    uint32_t bits = r.P[w];
    if (bits & (w < nw ? mx[w] : 0u)) m = true;
    while (bits) {
      const uint32_t x = w * 32u + uint32_t(__builtin_ctz(bits));
      bits &= bits - 1u;
      const uint32_t* row = g.cl + (size_t(x) * g.nctx + ctx) * nw;
#pragma unroll
      for (uint32_t j = 0; j < NW; ++j)
        if (j < nw) S[j] |= row[j];
    }
  }
  if (m) {
    r.matched = true;
    return;
  }
  const uint32_t* hc = g.has + size_t(c) * nw;
#pragma unroll
  for (uint32_t j = 0; j < NW; ++j) r.P[j] = j < nw ? (S[j] & hc[j]) : 0u;
  r.begin = 0;
  r.pw = g.has_word ? nwf : 0u;
}

// one byte through the UTF-8 decoder trie (Go's utf8.DecodeRune: a byte that
// breaks a sequence flushes its pending bytes as U+FFFD and is decoded afresh)
template <uint32_t NW>
__device__ __forceinline__ void nfa_byte(const NfaView& g, NfaRun<NW>& r, uint32_t b) {
  int32_t v = g.child[size_t(r.node) * 256 + b];
  if (r.node != 0 && v == -1) {
    for (uint32_t i = 0, d = g.depth[r.node]; i < d && !r.matched; ++i) nfa_rune(g, r, g.fffd);
    r.node = 0;
    if (r.matched) return;
    v = g.child[b];
  }
  if (v <= -2) {
    r.node = 0;
    nfa_rune(g, r, uint32_t(-2 - v));
  } else if (v == -1) {
    nfa_rune(g, r, g.fffd);
  } else {
    r.node = uint32_t(v);
  }
}

template <uint32_t NW>
__device__ __forceinline__ bool nfa_line_matches(const NfaView& g, const uint8_t* data, uint64_t a, uint64_t e) {
  NfaRun<NW> r;
#pragma unroll
  for (uint32_t j = 0; j < NW; ++j) r.P[j] = 0;
  r.begin = 1;
  r.pw = 0;
  r.node = 0;
  r.matched = false;
  for_line_bytes(data, a, e, [&](uint32_t b) {
    nfa_byte(g, r, b);
    return !r.matched;
  });
  for (uint32_t i = 0, d = g.depth[r.node]; i < d && !r.matched; ++i) nfa_rune(g, r, g.fffd);
  if (r.matched) return true;
  bool m = g.end_init[r.begin * 2u + r.pw] != 0u;
  const uint32_t* ex = g.end_x + size_t(r.pw) * g.nw;
#pragma unroll
  for (uint32_t w = 0; w < NW; ++w)
    if (w < g.nw && (r.P[w] & ex[w])) m = true;
  return m;
}

// The staged lines of a scan with PENDING lines and no filter candidates: only
// the pending ones change (kept iff they match; length filled in).
__global__ __launch_bounds__(256) void resolve_tiles_kernel(VerifyArgs v) {
  verify_tiles(v, [](uint64_t, uint64_t) { return true; });
}

// ---- long lines -------------------------------------------------------------
// A line the scan parked (park_pending) is finished here, in parallel over its
// bytes instead of by one lane: long_end_kernel finds its end ('\n' or the
// split's end) from the per-chunk '\n' counts; the host cuts [resume, end) into
// segments; long_map_kernel computes each segment's transition map (every
// state at once: each lane the map of its 1/64 of the segment, then the wave
// composes the 64 maps in order); long_fin_kernel applies a line's segment maps
// in order to its parked state, and the line matches iff '\n' then enters
// start_m (the DFA's own rule, also for the split's unterminated last line).
// States are the blob's (u8 table [S][256], S <= 256).

// one wave per parked line
__global__ __launch_bounds__(256) void long_end_kernel(LongArgs la) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t waves = uint64_t(gridDim.x) * 4;
  for (uint64_t i = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); i < la.npend; i += waves) {
    PendingLine P = la.pend[i];
    uint64_t c = P.resume / la.chunk, end = la.n;
    for (;; c += 64) {
      const uint64_t cc = c + lane;
      const bool past = cc >= la.nchunks;
      const uint64_t hit = __ballot(past || la.chunk_nl[cc < la.nchunks ? cc : 0] != 0u);
      if (!hit) continue;
      const uint64_t ch = c + uint64_t(__builtin_ctzll(hit));
      if (ch < la.nchunks) {
        // the first '\n' of chunk ch: 64 lanes x 16 B per round
        const uint64_t cb = ch * la.chunk, ce = cb + la.chunk < la.n ? cb + la.chunk : la.n;
        for (uint64_t q0 = cb; q0 < ce; q0 += 1024) {
          const uint64_t q = q0 + 16u * lane;
          uint32_t first = 0xffffffffu;
          if (q < ce) {
            uint4 v;
            if (q + 16 <= la.n) {
              v = *reinterpret_cast<const uint4*>(la.data + q);
            } else {
              uint32_t w[4] = {0, 0, 0, 0};
              for (uint64_t b = q; b < la.n; ++b) w[(b - q) >> 2] |= uint32_t(la.data[b]) << (8 * ((b - q) & 3));
              v = make_uint4(w[0], w[1], w[2], w[3]);
            }
            const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
            for (int k = 3; k >= 0; --k) {
              const uint32_t m = nl_mask(ws[k]);
              if (m && q + 4u * uint32_t(k) + (uint32_t(__builtin_ctz(m)) >> 3) < ce)
                first = 4u * uint32_t(k) + (uint32_t(__builtin_ctz(m)) >> 3);
            }
          }
          const uint64_t h2 = __ballot(first != 0xffffffffu);
          if (h2) {
            const int l = __builtin_ctzll(h2);
            end = q0 + 16u * uint32_t(l) + uint32_t(__shfl(int(first), l, 64));
            break;
          }
        }
      }
      break;
    }
    if (lane == 0) {
      P.end = end;
      la.pend[i] = P;
    }
  }
}

// one wave per segment; the map of a piece is computed with every DFA state at
// once: S <= 8 as Sheng byte vectors (8 next states per input byte, two v_perm
// per byte), else one map of S bytes per lane in LDS
constexpr int kLongWaves = 1;  // waves per workgroup of long_map_kernel (its LDS holds one [S][256] table)
__global__ __launch_bounds__(64 * kLongWaves) void long_map_kernel(LongArgs la) {
  __shared__ __attribute__((aligned(16))) uint8_t tbl[256 * 256];
  __shared__ __attribute__((aligned(16))) uint8_t maps[64 * kLongWaves * 256];
  __shared__ uint2 v8[256];  // S <= 8: V[b] = the 8 next states of byte b
  const uint32_t S = la.nstates, lane = threadIdx.x & 63u;
  for (uint32_t i = threadIdx.x * 16u; i < S * 256u; i += 64u * kLongWaves * 16u)
    *reinterpret_cast<uint4*>(tbl + i) = *reinterpret_cast<const uint4*>(la.tbl + i);
  __syncthreads();
  if (S <= 8) {
    for (uint32_t b = threadIdx.x; b < 256; b += 64u * kLongWaves) {
      uint32_t vx = 0, vy = 0;
      for (uint32_t s = 0; s < 4; ++s) {
        vx |= uint32_t(tbl[(s < S ? s : 0) * 256u + b]) << (8 * s);
        vy |= uint32_t(tbl[(s + 4 < S ? s + 4 : 0) * 256u + b]) << (8 * s);
      }
      v8[b] = make_uint2(vx, vy);
    }
    __syncthreads();
  }
  uint8_t* my = maps + threadIdx.x * 256u;
  const uint64_t waves = uint64_t(gridDim.x) * kLongWaves;
  for (uint64_t g = uint64_t(blockIdx.x) * kLongWaves + (threadIdx.x >> 6); g < la.nseg; g += waves) {
    const LongSeg sg = la.seg[g];
    // this lane's piece: [a, e), 16-aligned cuts
    const uint64_t span = sg.end - sg.begin;
    const uint64_t per = ((span + 63) / 64 + 15) & ~uint64_t(15);
    const uint64_t a = sg.begin + per * lane < sg.end ? sg.begin + per * lane : sg.end;
    const uint64_t e = a + per < sg.end ? a + per : sg.end;
    uint8_t* out = la.segmap + g * 256u;
    if (S <= 8) {
      uint32_t lo = 0x03020100u, hi = 0x07060504u;
      for_line_bytes(la.data, a, e, [&](uint32_t b) {
        const uint2 v = v8[b];
        lo = __builtin_amdgcn_perm(v.y, v.x, lo);
        hi = __builtin_amdgcn_perm(v.y, v.x, hi);
        return true;
      });
      // compose the 64 lane maps in lane (= byte) order
      uint32_t alo = 0x03020100u, ahi = 0x07060504u;
      for (int l = 0; l < 64; ++l) {
        const uint32_t ml = __shfl(lo, l, 64), mh = __shfl(hi, l, 64);
        alo = __builtin_amdgcn_perm(mh, ml, alo);
        ahi = __builtin_amdgcn_perm(mh, ml, ahi);
      }
      if (lane < 8u) out[lane] = uint8_t((lane < 4 ? alo >> (8 * lane) : ahi >> (8 * (lane - 4))) & 0xffu);
    } else {
      for (uint32_t s = 0; s < S; ++s) my[s] = uint8_t(s);
      for_line_bytes(la.data, a, e, [&](uint32_t b) {
        for (uint32_t s = 0; s < S; ++s) my[s] = tbl[uint32_t(my[s]) * 256u + b];
        return true;
      });
      __builtin_amdgcn_wave_barrier();
      // lane j follows states j, j + 64, ... through the 64 lane maps in order
      uint8_t* wm = maps + (threadIdx.x & ~63u) * 256u;
      for (uint32_t s = lane; s < S; s += 64) {
        uint32_t x = s;
        for (int l = 0; l < 64; ++l) x = wm[uint32_t(l) * 256u + x];
        out[s] = uint8_t(x);
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// one lane per parked line
__global__ __launch_bounds__(256) void long_fin_kernel(LongArgs la) {
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < la.npend; i += uint64_t(gridDim.x) * 256) {
    PendingLine P = la.pend[i];
    uint32_t s = la.st2id[P.state];
    for (uint64_t g = la.seg_off[i]; g < la.seg_off[i + 1]; ++g) s = la.segmap[g * 256u + s];
    P.matched = la.tbl[s * 256u + uint32_t('\n')] == la.start_m ? 1u : 0u;
    P.len = P.end - P.line_start;
    la.pend[i] = P;
  }
}

// Sheng stepper (<= 8 states): the scan left every lane chunk's map
// (ChunkMap), so a parked line is finished without reading its bytes again:
// from its parked state, apply the whole-chunk maps of the chunks after the
// park position, in order, up to the first chunk holding a '\n', whose map
// ends with that '\n' (the line matches iff the state is then start_m); or,
// no '\n' to the split's end, the last chunk's map and then V['\n'] (the
// split's unterminated last line, grep.go:17). One workgroup per parked line:
// each thread composes kLsPer consecutive chunk maps, the wave and then the
// workgroup compose theirs in order (v_perm on 8-state byte maps).
constexpr int kLsThreads = 256;
constexpr int kLsPer = 4;

// the map "a, then b" (byte s = b[a[s]])
__device__ __forceinline__ uint2 map_then(uint2 a, uint2 b) {
  return make_uint2(__builtin_amdgcn_perm(b.y, b.x, a.x), __builtin_amdgcn_perm(b.y, b.x, a.y));
}

__global__ __launch_bounds__(kLsThreads) void long_sheng_kernel(LongArgs la) {
  __shared__ uint2 wmap[kLsThreads / 64];
  __shared__ uint32_t whit[kLsThreads / 64];
  __shared__ uint64_t wend[kLsThreads / 64];
  __shared__ uint32_t wlazy[kLsThreads / 64];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint2 ident = make_uint2(0x03020100u, 0x07060504u);
  for (uint64_t i = blockIdx.x; i < la.npend; i += gridDim.x) {
    const PendingLine P = la.pend[i];
    uint32_t s = P.state;
    uint64_t end = la.n;
    bool lazy = false;  // the stopping chunk is a LAZY record: `end` is its start
    for (uint64_t c0 = P.resume / la.chunk;; c0 += uint64_t(kLsThreads) * kLsPer) {
      // this thread's chunks, in order, up to the first that holds a '\n' (or
      // lies past the split)
      const uint64_t cb = c0 + uint64_t(threadIdx.x) * kLsPer;
      ChunkMap cm[kLsPer];
#pragma unroll
      for (int j = 0; j < kLsPer; ++j) {
        const uint4 v = cb + j < la.nchunks ? *reinterpret_cast<const uint4*>(la.chunk_map + cb + j)
                                            : make_uint4(0u, 0u, kNoNewline, 1u);  // pad 1: past the split
        cm[j] = ChunkMap{v.x, v.y, v.z, v.w};
      }
      uint2 m = ident;
      bool stop = false, lz = false;
      uint64_t e = 0;
#pragma unroll
      for (int j = 0; j < kLsPer; ++j) {
        if (stop) continue;
        if (cm[j].pad) {  // past the split's end
          stop = true;
          e = la.n;
        } else if (cm[j].first == kLazyNewline) {  // no map: stop before this chunk
          stop = lz = true;
          e = (cb + j) * la.chunk;
        } else {
          m = map_then(m, make_uint2(cm[j].lo, cm[j].hi));
          if (cm[j].first != kNoNewline) {
            stop = true;
            e = (cb + j) * la.chunk + cm[j].first;
          }
        }
      }
      // the wave: threads up to its first stopping one, composed in order
      const uint64_t hb = __ballot(stop);
      const uint32_t hl = hb ? uint32_t(__builtin_ctzll(hb)) : 64u;
      if (lane > hl) m = ident;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint2 o = make_uint2(__shfl_down(m.x, d, 64), __shfl_down(m.y, d, 64));
        if ((lane & uint32_t(2 * d - 1)) == 0u && lane + uint32_t(d) < 64u) m = map_then(m, o);
      }
      if (lane == 0) {
        wmap[w] = m;
        whit[w] = hl;
      }
      if (lane == hl) {
        wend[w] = e;
        wlazy[w] = lz ? 1u : 0u;
      }
      __syncthreads();
      uint32_t wf = kLsThreads / 64;
      for (uint32_t k = 0; k < kLsThreads / 64; ++k) {
        if (wf == kLsThreads / 64) {
          const uint2 t = wmap[k];
          s = __builtin_amdgcn_perm(t.y, t.x, s) & 0xffu;
          if (whit[k] < 64u) wf = k;
        }
      }
      if (wf < kLsThreads / 64) {
        end = wend[wf];
        lazy = wlazy[wf] != 0u;
      }
      __syncthreads();  // wmap / whit / wend are rewritten by the next round
      if (wf < kLsThreads / 64) break;
    }
    // a LAZY chunk: its first '\n' lies in its first kLazyMapBytes; s is the
    // state at the chunk's start, so step its bytes through that '\n'
    if (lazy && threadIdx.x == 0) {
      for (uint64_t q = end;; ++q) {
        const uint32_t b = la.data[q];
        const uint2 v = la.sheng_v[b];
        s = __builtin_amdgcn_perm(v.y, v.x, s) & 0xffu;
        if (b == uint32_t('\n')) {
          end = q;
          break;
        }
      }
    }
    // end < n: the last map ended with the line's '\n'; end == n: the split
    // ended first, and its end closes the line (V['\n'] applied)
    if (!lazy && end == la.n) s = __builtin_amdgcn_perm(la.nl_hi, la.nl_lo, s) & 0xffu;
    if (threadIdx.x == 0) {
      PendingLine Q = P;
      Q.end = end;
      Q.len = end - P.line_start;
      Q.matched = s == la.sheng_m ? 1u : 0u;
      la.pend[i] = Q;
    }
    __syncthreads();
  }
}

// ---- long lines of the filter stepper (> 256 states) ---------------------------
// A parked line is decided on the WHOLE DFA (breadth-first ids, u16/u32 table in
// HBM with its leading rows in LDS, as verify_kernel) in parallel over its
// bytes: the host cuts [line_start, end) into segments; long_dfa_seg1_kernel
// runs each segment on one lane from up to kLongGuesses GUESSED entry states --
// the states the DFA reaches over the kLongLookback bytes before the segment
// from kLongSeeds start states (for keyword automata such as config 4's, the
// state after any 12+ bytes no longer depends on what came before, so one
// guess is exact) -- and records each guess with its exit state;
// long_dfa_fix_kernel then walks each line's segments in order from the true
// state, takes a segment's exit when its guess was right and re-runs the
// segment from the true state when it was not (exact for any DFA).
constexpr uint32_t kLongLookback = 256;
constexpr uint64_t kLongSeedBytes = 64;  // lookback bytes every seed steps (long_dfa_seg1_kernel)
#ifndef DGREP_LONG_SEEDS_RUN
#define DGREP_LONG_SEEDS_RUN kLongSeeds  // seeds stepped (<= kLongSeeds; 1: start only, the round-5 single guess)
#endif
constexpr int kLongSeedsRun = DGREP_LONG_SEEDS_RUN;
static_assert(kLongSeedsRun >= 1 && kLongSeedsRun <= kLongSeeds, "DGREP_LONG_SEEDS_RUN");


// one 1024-thread workgroup per CU holds the DFA's first kLongDfaHotBytes of
// rows (breadth-first: the states keyword text spends its bytes in; C4's
// depth <= 3 rows need ~110 KiB) -- the segment lanes' table reads stay in LDS
constexpr int kLongDfaThreads = 1024;
constexpr uint32_t kLongDfaHotBytes = 120 * 1024;  // rows alone (u32 DFAs)
constexpr uint32_t kLongDfaLdsBytes = 158 * 1024;  // rows + DfaXRec (u16 DFAs)

// One segment per lane, read in 64-byte blocks (four 16-B loads, the next
// block in flight while this one is stepped). Two segments per lane in
// 16-B pieces kept 2,048 read streams per CU live, more 128-B lines than L2
// holds: each line came from HBM several times (long_c4 seg kernel 21 ms per
// 16 GiB, 0.67 TB/s of segment bytes).
// 16-B pieces per block (4: 64 B, half a line: eight pieces spill at 1024 threads)
#ifndef DGREP_SEG_PIECES
#define DGREP_SEG_PIECES 4
#endif
constexpr int kSegPieces = DGREP_SEG_PIECES;
template <typename E, bool XI>
__global__ __launch_bounds__(kLongDfaThreads) void long_dfa_seg1_kernel(LongDfaArgs la) {
  __shared__ uint32_t cls[256];
  __shared__ uint8_t cls8[256];
  __shared__ __attribute__((aligned(16))) uint8_t lbuf[kLongDfaLdsBytes];
  // classes pre-scaled to the entry size: a step's table address is one v_mad
  if (threadIdx.x < 256) {
    cls[threadIdx.x] = uint32_t(la.cls[threadIdx.x]) * uint32_t(sizeof(E));
    cls8[threadIdx.x] = uint8_t(la.cls[threadIdx.x]);
  }
  // a byte's scaled class, from the u8 copy: bytes b and b + 128 share a bank,
  // so ASCII text reads it conflict-free (the u32 table's bank is b % 32: 'a',
  // 'A' and '!' collide), for one more VALU op per byte (long_c4p +3.7 %,
  // long_c4 unchanged, profiles/r06/long_ab/cls8_*)
  auto cl = [&](uint32_t b) __attribute__((always_inline)) -> uint32_t {
    return uint32_t(cls8[b]) * uint32_t(sizeof(E));
  };
  E* const hot = reinterpret_cast<E*>(lbuf);
  const uint32_t hot_n = XI ? la.x_hot * la.nclasses : min(la.seg_hot_entries, uint32_t(kLongDfaHotBytes / sizeof(E)));
  if constexpr (XI) {
    for (uint32_t i = threadIdx.x * 16u; i < la.ximg_bytes; i += kLongDfaThreads * 16u)
      *reinterpret_cast<uint4*>(lbuf + i) = *reinterpret_cast<const uint4*>(la.ximg + i);
  } else {
    const E* full = static_cast<const E*>(la.full);
    for (uint32_t i = threadIdx.x; i < hot_n; i += kLongDfaThreads) hot[i] = full[i];
  }
  __syncthreads();
  FullDfa<E, XI> d{hot, (const __attribute__((address_space(1))) E*)la.full, cls, la.nclasses, hot_n};
  if constexpr (XI) {
    d.xr = reinterpret_cast<const uint2*>(lbuf + la.xr_off);
    d.xh = la.x_hot;
  }
  // one DFA step on scaled class ce: the entry's LDS address in one v_mad,
  // clamped to the resident rows (one v_min) and read unconditionally; a state
  // past them takes the cold path behind a ballot, which replaces the value
  const uint32_t KE = la.nclasses * uint32_t(sizeof(E)), hot_end = hot_n * uint32_t(sizeof(E));
  auto step_c = [&](uint32_t s, uint32_t ce) __attribute__((always_inline)) -> uint32_t {
    const uint32_t ad = __umul24(s, KE) + ce;
    uint32_t t = uint32_t(*reinterpret_cast<const E*>(lbuf + min(ad, hot_end - uint32_t(sizeof(E)))));
    const bool k = ad >= hot_end;
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(k) != 0, 0)) {
      if (k) t = d.cold(s, ce / uint32_t(sizeof(E)), ad / uint32_t(sizeof(E)));
    }
    return t;
  };
  auto step = [&](uint32_t s, uint32_t byte) __attribute__((always_inline)) -> uint32_t {
    return step_c(s, cl(byte));
  };
  auto word_cls = [&](uint32_t w, uint32_t (&c)[4]) __attribute__((always_inline)) {
    c[0] = cl(w & 0xffu);
    c[1] = cl((w >> 8) & 0xffu);
    c[2] = cl((w >> 16) & 0xffu);
    c[3] = cl(w >> 24);
  };
  // state after bytes [a, e) from s: the bytes up to the first 64-B boundary
  // and after the last one singly, the blocks between unrolled with no
  // position test, the next block in flight
  auto run = [&](uint64_t a, uint64_t e, uint32_t s) __attribute__((always_inline)) -> uint32_t {
    constexpr uint64_t kB = 16u * kSegPieces;
    const uint64_t A = min(e, (a + kB - 1) & ~(kB - 1)), Eb = max(A, e & ~(kB - 1));
    for (uint64_t p = a; p < A; ++p) s = step(s, la.data[p]);
    if (A < Eb) {
      const uint4* src = reinterpret_cast<const uint4*>(la.data + A);
      const uint64_t nb = (Eb - A) / kB;
      uint4 cur[kSegPieces], nxt[kSegPieces];
#pragma unroll
      for (int k = 0; k < kSegPieces; ++k) cur[k] = src[k];
      // the classes of the next word are read while this word is stepped
      uint32_t cn[4];
      word_cls(cur[0].x, cn);
      for (uint64_t blk = 0; blk < nb; ++blk) {
        const uint64_t nx = blk + 1 < nb ? blk + 1 : blk;  // the last block re-reads itself
#pragma unroll
        for (int k = 0; k < kSegPieces; ++k) nxt[k] = src[nx * kSegPieces + k];
#pragma unroll
        for (int wi = 0; wi < 4 * kSegPieces; ++wi) {
          const uint32_t c[4] = {cn[0], cn[1], cn[2], cn[3]};
          const int wn = wi + 1;
          const uint4 v = wn < 4 * kSegPieces ? cur[wn >> 2] : nxt[0];
          word_cls((wn & 3) == 0 ? v.x : (wn & 3) == 1 ? v.y : (wn & 3) == 2 ? v.z : v.w, cn);
          s = step_c(s, c[0]);
          s = step_c(s, c[1]);
          s = step_c(s, c[2]);
          s = step_c(s, c[3]);
        }
#pragma unroll
        for (int k = 0; k < kSegPieces; ++k) cur[k] = nxt[k];
      }
    }
    for (uint64_t p = Eb; p < e; ++p) s = step(s, la.data[p]);
    return s;
  };
  for (uint64_t g = uint64_t(blockIdx.x) * kLongDfaThreads + threadIdx.x; g < la.nseg;
       g += uint64_t(gridDim.x) * kLongDfaThreads) {
    const LongSeg A = la.seg[g];
    const uint64_t fa = la.seg_from[g];
    // The guesses: the states the lookback [fa, begin) leads to from start and
    // from the seeds (kLongSeeds chains in lockstep), distinct, absorbing ones
    // left out (the fix kernel stops there); a line's first segment has exactly
    // one entry state, start. A DFA that forgets its past within the lookback
    // (config 4's keywords) gives one guess; one that keeps a finite memory of
    // the whole line (the parity of some byte, "a k since the last z") gives
    // one guess per memory class, and the entry state is nearly always among them.
    // The seeds run together over the lookback's first kLongSeedBytes only:
    // chains that meet there stay together, so the rest of the lookback steps
    // just the distinct ones (config 4's keyword automaton: one chain after ~12
    // bytes; a parity: two).
    uint32_t gs[kLongGuesses];
    uint32_t ng = 1;
    gs[0] = la.start;
    if (A.begin != fa) {
      uint32_t sd[kLongSeedsRun];
#pragma unroll
      for (int i = 0; i < kLongSeedsRun; ++i) sd[i] = la.seed[i];
      const uint64_t mid = min(A.begin, fa + kLongSeedBytes);
      for_line_bytes(la.data, fa, mid, [&](uint32_t b) {
        const uint32_t ce = cl(b);
#pragma unroll
        for (int i = 0; i < kLongSeedsRun; ++i) sd[i] = step_c(sd[i], ce);
        return true;
      });
      ng = 0;
#pragma unroll
      for (int i = 0; i < kLongSeedsRun; ++i) {
        bool fresh = sd[i] != la.matched && sd[i] != la.dead && ng < uint32_t(kLongGuesses);
#pragma unroll
        for (int k = 0; k < kLongGuesses; ++k) fresh = fresh && !(uint32_t(k) < ng && gs[k] == sd[i]);
        if (fresh) gs[ng++] = sd[i];
      }
      if (ng == 0) gs[ng++] = sd[0];  // every seed absorbed: the fix kernel stops before this segment anyway
      for (uint32_t k = 0; k < ng; ++k) gs[k] = run(mid, A.begin, gs[k]);
    }
    for (uint32_t k = 0; k < uint32_t(kLongGuesses); ++k) {
      la.seg_guess[k * la.nseg + g] = k < ng ? gs[k] : kNoGuess;
      la.seg_exit[k * la.nseg + g] = k < ng ? run(A.begin, A.end, gs[k]) : kNoGuess;
    }
  }
}

template <typename E>
__global__ __launch_bounds__(256) void long_dfa_fix_kernel(LongDfaArgs la) {
  __shared__ uint32_t cls[256];
  __shared__ __attribute__((aligned(16))) E hot[kVerifyHotBytes / sizeof(E)];
  cls[threadIdx.x] = la.cls[threadIdx.x];
  const E* full = static_cast<const E*>(la.full);
  for (uint32_t i = threadIdx.x; i < la.hot_entries; i += 256) hot[i] = full[i];
  __syncthreads();
  const FullDfa<E> d{hot, (const __attribute__((address_space(1))) E*)la.full, cls, la.nclasses, la.hot_entries};
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < la.npend; i += uint64_t(gridDim.x) * 256) {
    PendingLine P = la.pend[i];
    uint32_t s = la.start;
    // in order from the true state: a segment whose guesses hold one is taken
    // whole; else it is re-run from the true state (exact for any DFA); an
    // absorbing state ends the walk. A segment's guesses and exits do not
    // depend on s: the next segment's are loaded while this one is decided, so
    // the walk pays one memory latency per segment, not one per guess read.
    const uint64_t g0 = la.seg_off[i], ge = la.seg_off[i + 1];
    uint32_t gv[kLongGuesses], xv[kLongGuesses];
    auto load = [&](uint64_t g, uint32_t(&gq)[kLongGuesses], uint32_t(&xq)[kLongGuesses]) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < kLongGuesses; ++k) {
        gq[k] = la.seg_guess[uint64_t(k) * la.nseg + g];
        xq[k] = la.seg_exit[uint64_t(k) * la.nseg + g];
      }
    };
    if (g0 < ge) load(g0, gv, xv);
    for (uint64_t g = g0; g < ge && s != la.matched && s != la.dead; ++g) {
      uint32_t gn[kLongGuesses], xn[kLongGuesses];
      load(min(g + 1, ge - 1), gn, xn);
      uint32_t x = kNoGuess;
#pragma unroll
      for (int k = 0; k < kLongGuesses; ++k) x = (x == kNoGuess && gv[k] == s) ? xv[k] : x;
#pragma unroll
      for (int k = 0; k < kLongGuesses; ++k) {
        gv[k] = gn[k];
        xv[k] = xn[k];
      }
      if (x != kNoGuess) {
        s = x;
      } else {
        const LongSeg sg = la.seg[g];
        s = d.run(la.data, sg.begin, sg.end, s, la.matched);
      }
    }
    P.matched = (s == la.matched || d.next(s, uint32_t('\n')) == la.start_m) ? 1u : 0u;
    P.len = P.end - P.line_start;
    la.pend[i] = P;
  }
}

template <uint32_t NW>
__global__ __launch_bounds__(256) void verify_nfa_kernel(VerifyArgs v) {
  const NfaView g = nfa_view(v.nfa);
  verify_tiles(v, [&](uint64_t a, uint64_t e) { return nfa_line_matches<NW>(g, v.data, a, e); });
}

// ---- ordering passes ------------------------------------------------------
// Tiles append their lines to the staging buffer in atomic order; these passes
// place every tile's lines at its final output index (exclusive prefix of the
// per-tile counts) with the 1-based number of its first line (1 + exclusive
// prefix of the per-tile '\n' counts), in split order. tile_block_sum_kernel
// reduces each block of 64 tiles (one wave per block: 128 blocks for a 16 GiB
// split at 32 KiB chunks); order_lines_kernel (one wave per tile) adds the block
// sums before its block and the tiles of its block before it, then copies. Two
// launches either way: a single-workgroup scan of all tile counts took 16-100 us
// per split (it is latency-bound on one CU), the block sums ~2 us.
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

__global__ __launch_bounds__(256) void tile_block_sum_kernel(const TileInfo* tiles, uint64_t ntiles, uint64_t* bsum_c,
                                                             uint64_t* bsum_l) {
  const uint64_t nb = (ntiles + 63) / 64;
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t b = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); b < nb; b += uint64_t(gridDim.x) * 4) {
    const uint64_t t = b * 64 + lane;
    uint64_t c = 0, l = 0;
    if (t < ntiles) {
      const TileInfo ti = tiles[t];
      c = ti.count;
      l = ti.nl;
    }
    c = wave_sum_u64(c);
    l = wave_sum_u64(l);
    if (lane == 0) {
      bsum_c[b] = c;
      bsum_l[b] = l;
    }
  }
}

// one wave per tile: its prefix, then its staged lines copied to their final slots (SoA)
#ifndef DGREP_ORDER_UNROLL
#define DGREP_ORDER_UNROLL 4
#endif
constexpr uint32_t kOrderUnroll = DGREP_ORDER_UNROLL;
// streaming (nontemporal) stores for the three output arrays, for A/B
__global__ __launch_bounds__(256) void order_lines_kernel(const TileInfo* tiles, const StagedLine* staging,
                                                          uint64_t ntiles, const uint64_t* bsum_c,
                                                          const uint64_t* bsum_l, uint64_t staging_cap,
                                                          uint64_t capacity, uint64_t* line_no, uint64_t* start,
                                                          uint64_t* len) {
  const uint64_t waves = uint64_t(gridDim.x) * 4;
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t t = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); t < ntiles; t += waves) {
    const TileInfo ti = tiles[t];
    if (ti.count == 0) continue;
    const uint64_t b = t / 64;
    uint64_t pc = 0, pl = 0;
    for (uint64_t j = lane; j < b; j += 64) {
      pc += bsum_c[j];
      pl += bsum_l[j];
    }
    const uint64_t tt = b * 64 + lane;
    if (tt < t) {
      const TileInfo x = tiles[tt];
      pc += x.count;
      pl += x.nl;
    }
    const uint64_t o = wave_sum_u64(pc), lb = wave_sum_u64(pl) + 1;
    // kOrderUnroll records per lane in flight: every load of a round is issued
    // before its stores (the stores may alias the staging buffer for all the
    // compiler knows, so a plain loop waited out one HBM latency per 64 records)
    for (uint32_t k0 = 0; k0 < ti.count; k0 += 64u * kOrderUnroll) {
      StagedLine L[kOrderUnroll];
      bool ok[kOrderUnroll];
#pragma unroll
      for (uint32_t u = 0; u < kOrderUnroll; ++u) {
        const uint32_t k = k0 + u * 64u + lane;
        const uint64_t src = ti.base + k, dst = o + k;
        ok[u] = k < ti.count && src < staging_cap && dst < capacity;
        if (ok[u]) L[u] = staging[src];
      }
#pragma unroll
      for (uint32_t u = 0; u < kOrderUnroll; ++u) {
        const uint64_t dst = o + k0 + u * 64u + lane;
        if (ok[u]) {
          line_no[dst] = lb + staged_rel(L[u]);
          start[dst] = L[u].start;
          len[dst] = staged_len(L[u]);
        }
      }
    }
  }
}

#endif  // DG_PART(0)

// ---- host-side launchers (called from dgrep_runtime.cpp) ----------------

#if DG_PART(0)
uint32_t scan_table_row() { return kRow; }
uint32_t scan_max_lane_chunk() { return uint32_t(kMaxLaneChunk); }
#endif

namespace {
template <class Step>
constexpr int threads_of() {
  return Step::kKind == kStepFilter ? kFilterThreads : kScanThreads;
}
template <class Step, int TBL>
hipError_t launch_t(const ScanArgs& a, int grid, hipStream_t stream) {
  constexpr int NT = threads_of<Step>();
  hipLaunchKernelGGL((scan_dfa8_kernel<Step, TBL, NT>), dim3(grid), dim3(NT), 0, stream, a);
  return hipGetLastError();
}
template <class Step, int TBL>
hipError_t overflow_t(const ScanArgs& a, uint64_t nover, hipStream_t stream) {
  constexpr uint64_t wpb = kOverflowThreads / 64;
  int grid = int((nover + wpb - 1) / wpb);
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL((scan_overflow_kernel<Step, TBL>), dim3(grid), dim3(kOverflowThreads), 0, stream, a, nover);
  return hipGetLastError();
}
template <class Step, int TBL>
hipError_t occ_t(int* b) {
  constexpr int NT = threads_of<Step>();
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(b, scan_dfa8_kernel<Step, TBL, NT>, NT, 0);
}

// Adaptive chunk: a power of two from the compiled chunk (its floor) up to
// kShengMaxChunk, the largest that still gives every resident wave at least
// one tile. Measured on C2 (profiles/r01/ablation/chunk_sweep.txt): 32 KiB
// runs 5.1 TB/s, 16 KiB 4.74-4.88, 8 KiB 4.54, 4 KiB 4.29, but 14,592 B (a
// chunk sized to fill whole rounds exactly) 4.13: keep powers of two. The LDS
// slots pack a line's chunk-relative start (<= C) and '\n' index (<= C) in 16
// bits each, with a start of exactly C = 65,536 flagged in the lane's tail:
// 64 KiB is the hard limit (the adaptive choice stops at kShengMaxChunk).
// `dens_cap` (0 = none) is the largest chunk whose expected matching lines,
// at the match density of the previous scan of this pattern, fill at most a
// quarter of a lane's LDS slots: a denser pattern keeps smaller chunks instead
// of sending many lanes through the overflow pass (C4 at 16 KiB: 0.8 % of the
// lanes overflow and the pass costs 8 % of the scan; at 8 KiB 0.07 %).
// The adaptive Sheng chunk stops at 32 KiB: 64 KiB chunks (what a >= 30 GiB
// split would take) are parity-correct since r05 but measured no faster, C5 32
// GiB same box: 0.670-0.671 at 64 KiB vs 0.672-0.674 at 32 KiB (the access
// pattern's ceiling had predicted +2-3 %); dgrep_set_lane_chunk forces 64 KiB.
#ifndef DGREP_SHENG_MAX_CHUNK
#define DGREP_SHENG_MAX_CHUNK 32768
#endif
constexpr uint64_t kShengMaxChunk = DGREP_SHENG_MAX_CHUNK;
static_assert(kShengMaxChunk <= uint64_t(kMaxLaneChunk), "adaptive chunk above the slot limit");
// Per-stepper ceiling: the pair stepper stops at 9 KiB (4.5 KiB doubled once).
// Round 2 (static tiles) measured 8 KiB 4.43 ms, 16 KiB 4.39, 32 KiB 4.71 per
// 16 GiB (at 32 KiB most of its ~40 records per lane and tile go through the
// HBM spill area); with tiles claimed dynamically, 8 KiB was at least as fast
// as 16 KiB on each of three boxes (profiles/r04/ablation/c3_chunk*.txt).
// Round 6, same box: 7 KiB (and 9 KiB) beat the power of two between them by
// 2.5-3.5 % on two boxes (C3 kernel 0.567-0.575 -> 0.586-0.588), where the bare
// access pattern (tools/pattern_ceiling) reads all three at one rate: a
// 2^13-byte stride between a wave's lane streams costs the latency-bound pair
// kernel, not the memory (profiles/r06/ablation/pair_chunk_*). 9 KiB runs at
// least as fast as 7 KiB on every box tried (0-1 %; a fast box 0.633 -> 0.638,
// pair_chunk_7k_vs_9k_c3_boxM.txt), and 4.5 KiB, the small-split floor, is the
// best chunk of the bare access pattern (pattern_ceiling_sweep_pair_lds.txt).
#ifndef DGREP_PAIR_MAX_CHUNK
#define DGREP_PAIR_MAX_CHUNK 9216
#endif
// Doubling also stops below DGREP_MIN_TILES_X2 / 2 tiles per resident wave
// (Sheng, pair; the filter keeps 1):
// with tiles claimed dynamically, a split of exactly 2 tiles per wave ran 7 %
// slower than 4 tiles of half the chunk (12 GiB: 32 KiB 4,462-4,580 GB/s,
// 16 KiB 5,152), while 2.67 (16 GiB) and 5.33 (32 GiB) tiles per wave at
// 32 KiB beat 16 KiB (profiles/r04/ablation/chunk_dyn.txt).
// The filter stops at 64 KiB (one tile per resident wave on a 16 GiB split):
// same box, C4 0.499-0.500 at 32 KiB -> 0.505-0.506 at 64 KiB, verification
// 0.18 -> 0.16 ms (profiles/r06/ablation/filter_chunk_64k_c4_boxJ.txt), where
// the Sheng stepper loses 6 % at 64 KiB (sheng_chunk_64k_c2_boxJ.txt).
#ifndef DGREP_FILTER_MAX_CHUNK
#define DGREP_FILTER_MAX_CHUNK 65536
#endif
#ifndef DGREP_MIN_TILES_X2
#define DGREP_MIN_TILES_X2 5
#endif
uint32_t adaptive_chunk_bytes(uint64_t n, uint64_t waves, uint64_t floor_c, uint64_t dens_cap,
                              uint64_t max_c = kShengMaxChunk, uint64_t min_tiles_x2 = DGREP_MIN_TILES_X2) {
  uint64_t c = floor_c;
  while (c * 2 <= max_c && 2 * n >= min_tiles_x2 * waves * uint64_t(kTileLanes) * c * 2 &&
         (!dens_cap || c * 2 <= dens_cap))
    c *= 2;
  return uint32_t(c);
}
}  // namespace

// The stepper entry points (one per op), instantiated by their build part.
namespace scan_ops {
struct TileOp {
  uint64_t* bytes;
  uint32_t* chunk;
  uint32_t* waves_per_block;
  uint64_t n, resident_blocks;
  uint32_t force;
  double density;  // matching lines per byte seen by the previous scan (0: unknown)
  uint32_t* slots;
  uint32_t spill_per_lane;
  template <class S, int T>
  hipError_t run() const {
    uint64_t c = uint64_t(Tune<S>::C);
    // a lane's record capacity: its LDS slots, plus the HBM spill area of the
    // one-chunk-per-lane steppers
    constexpr uint32_t E = uint32_t(Tune<S>::E);
    const uint32_t cap = E + (adaptive_chunk<S, T>() ? spill_per_lane : 0u);
    *slots = cap;
    // at most a quarter of the capacity expected in use: an overflowing lane
    // costs two latency-bound passes of the overflow kernel over its chunk
    const uint64_t dens_cap = density > 0 ? uint64_t(double(cap) / (4.0 * density)) : 0;
    if constexpr (adaptive_chunk<S, T>())
      c = force ? uint64_t(force)
                : adaptive_chunk_bytes(n, resident_blocks * uint64_t(threads_of<S>() / 64), c, dens_cap,
                                       S::kKind == kStepPair     ? DGREP_PAIR_MAX_CHUNK
                                       : S::kKind == kStepFilter ? DGREP_FILTER_MAX_CHUNK
                                                                 : kShengMaxChunk,
                                       // the filter keeps 32 KiB at 2 tiles per wave (C4: 16 KiB -1.5 %)
                                       S::kKind == kStepFilter ? 2 : DGREP_MIN_TILES_X2);
    *chunk = uint32_t(c);
    *waves_per_block = uint32_t(threads_of<S>() / 64);
    *bytes = uint64_t(kTileLanes) * uint64_t(streams_of<S, T>()) * c;
    return hipSuccess;
  }
};
struct OccOp {
  int* b;
  template <class S, int T>
  hipError_t run() const { return occ_t<S, T>(b); }
};
struct LaunchOp {
  const ScanArgs* a;
  int grid;
  hipStream_t s;
  template <class S, int T>
  hipError_t run() const { return launch_t<S, T>(*a, grid, s); }
};
struct OverflowOp {
  const ScanArgs* a;
  uint64_t n;
  hipStream_t s;
  template <class S, int T>
  hipError_t run() const { return overflow_t<S, T>(*a, n, s); }
};

// stepper by kind, LDS image by size; one function per build part
template <class Op>
hipError_t part_sheng(int, uint32_t, const Op& op) {
  return op.template run<StepSheng8, 2048>();
}
template <class Op>
hipError_t part_pair(int kind, uint32_t table_bytes, const Op& op) {
  if (kind & kKindW32) {
    if (table_bytes <= 8192) return op.template run<StepPair, 8192>();
    return op.template run<StepPair, int(kPairW32MaxImage)>();  // C3 (15.6 KiB)
  }
  if (table_bytes <= 16384) return op.template run<StepPair16, 16384>();
  return op.template run<StepPair16, int(kPairMaxImage)>();
}
template <class Op>
hipError_t part_table(int, uint32_t table_bytes, const Op& op) {
  if (table_bytes <= 16 * kRow) return op.template run<StepTable, 16 * kRow>();
  if (table_bytes <= 32 * kRow) return op.template run<StepTable, 32 * kRow>();
  if (table_bytes <= 64 * kRow) return op.template run<StepTable, 64 * kRow>();
  if (table_bytes <= 128 * kRow) return op.template run<StepTable, 128 * kRow>();
  return op.template run<StepTable, 256 * kRow>();
}
template <class Op>
hipError_t part_big(int kind, uint32_t, const Op& op) {
  return op.template run<StepFilter, int(kFilterImageBytes)>();
}
// explicit instantiations in their part, extern elsewhere
#define DG_OPS(PFX, FN)                                                   \
  PFX hipError_t FN<TileOp>(int, uint32_t, const TileOp&);                \
  PFX hipError_t FN<OccOp>(int, uint32_t, const OccOp&);                  \
  PFX hipError_t FN<LaunchOp>(int, uint32_t, const LaunchOp&);            \
  PFX hipError_t FN<OverflowOp>(int, uint32_t, const OverflowOp&);
#if DG_PART(1)
DG_OPS(template, part_sheng)
#else
DG_OPS(extern template, part_sheng)
#endif
#if DG_PART(2)
DG_OPS(template, part_pair)
#else
DG_OPS(extern template, part_pair)
#endif
#if DG_PART(3)
DG_OPS(template, part_table)
#else
DG_OPS(extern template, part_table)
#endif
#if DG_PART(4)
DG_OPS(template, part_big)
#else
DG_OPS(extern template, part_big)
#endif
#undef DG_OPS

// One switch for every entry point: stepper by kind.
template <class Op>
hipError_t dispatch(int kind, uint32_t table_bytes, const Op& op) {
  const int k = kind & ~kKindW32;
  if (k == kStepSheng8) return part_sheng(k, table_bytes, op);
  if (k == kStepPair) return part_pair(kind, table_bytes, op);
  if (k == kStepFilter) return part_big(k, table_bytes, op);
  return part_table(k, table_bytes, op);
}
}  // namespace scan_ops

#if DG_PART(0)
using namespace scan_ops;

uint64_t scan_tile_bytes(int kind, uint32_t table_bytes, uint64_t n, uint64_t resident_blocks, uint32_t force,
                         double density, uint32_t spill_per_lane, uint32_t* chunk, uint32_t* waves_per_block,
                         uint32_t* slots, uint32_t* threads, bool* spills) {
  uint64_t b = 0;
  (void)dispatch(kind, table_bytes,
                 TileOp{&b, chunk, waves_per_block, n, resident_blocks, force, density, slots, spill_per_lane});
  *threads = *waves_per_block * 64;
  const int k = kind & ~kKindW32;
  *spills = k == kStepSheng8 || k == kStepPair || k == kStepFilter;
  return b;
}
hipError_t scan_dfa_occupancy(int kind, uint32_t table_bytes, int* blocks_per_cu) {
  return dispatch(kind, table_bytes, OccOp{blocks_per_cu});
}
hipError_t scan_dfa(int kind, const ScanArgs& a, int grid, hipStream_t stream) {
  return dispatch(kind, a.table_bytes, LaunchOp{&a, grid, stream});
}
hipError_t scan_dfa_overflow(int kind, const ScanArgs& a, uint64_t nover, hipStream_t stream) {
  return dispatch(kind, a.table_bytes, OverflowOp{&a, nover, stream});
}

// out_off / line_base: scratch of ceil(ntiles / 64) entries each (block sums)
hipError_t order_lines(const TileInfo* tiles, const StagedLine* staging, uint64_t ntiles, uint64_t* out_off,
                       uint64_t* line_base, uint64_t staging_cap, uint64_t capacity, uint64_t* line_no,
                       uint64_t* start, uint64_t* len, hipStream_t stream) {
  // out_off / line_base hold the 64-tile block sums (ceil(ntiles / 64) each)
  const uint64_t nb = (ntiles + 63) / 64;
  const uint64_t bgrid = std::min<uint64_t>((nb + 3) / 4, 4096);
  if (bgrid) hipLaunchKernelGGL(tile_block_sum_kernel, dim3(bgrid), dim3(256), 0, stream, tiles, ntiles, out_off, line_base);
  uint64_t grid = (ntiles + 3) / 4;
  if (grid > 16384) grid = 16384;
  hipLaunchKernelGGL(order_lines_kernel, dim3(grid), dim3(256), 0, stream, tiles, staging, ntiles, out_off,
                     line_base, staging_cap, capacity, line_no, start, len);
  return hipGetLastError();
}

uint32_t verify_hot_bytes() { return kVerifyHotBytes; }

hipError_t long_lines_end(const LongArgs& la, hipStream_t stream) {
  uint64_t grid = (la.npend + 3) / 4;
  if (grid > 16384) grid = 16384;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(long_end_kernel, dim3(grid), dim3(256), 0, stream, la);
  return hipGetLastError();
}
hipError_t long_lines_resolve(const LongArgs& la, hipStream_t stream) {
  if (la.nseg) {
    uint64_t grid = (la.nseg + kLongWaves - 1) / kLongWaves;
    if (grid > 65536) grid = 65536;
    hipLaunchKernelGGL(long_map_kernel, dim3(grid), dim3(64 * kLongWaves), 0, stream, la);
  }
  uint64_t grid = (la.npend + 255) / 256;
  if (grid > 4096) grid = 4096;
  if (grid) hipLaunchKernelGGL(long_fin_kernel, dim3(grid), dim3(256), 0, stream, la);
  return hipGetLastError();
}

hipError_t long_lines_sheng(const LongArgs& la, hipStream_t stream) {
  const uint64_t grid = la.npend < 4096 ? la.npend : 4096;
  if (grid) hipLaunchKernelGGL(long_sheng_kernel, dim3(grid), dim3(kLsThreads), 0, stream, la);
  return hipGetLastError();
}

uint32_t long_lookback() { return kLongLookback; }
uint32_t long_guesses() { return uint32_t(kLongGuesses); }
uint32_t long_seeds() { return uint32_t(kLongSeeds); }
uint32_t long_dfa_hot_bytes() { return kLongDfaHotBytes; }
uint32_t long_dfa_lds_bytes() { return kLongDfaLdsBytes; }

hipError_t long_lines_dfa(const LongDfaArgs& la, bool u32, hipStream_t stream) {
  if (la.nseg) {
    uint64_t grid = (la.nseg + kLongDfaThreads - 1) / kLongDfaThreads;
    if (grid > 65536) grid = 65536;
    if (u32)
      hipLaunchKernelGGL((long_dfa_seg1_kernel<uint32_t, false>), dim3(grid), dim3(kLongDfaThreads), 0, stream, la);
    else if (la.ximg)
      hipLaunchKernelGGL((long_dfa_seg1_kernel<uint16_t, true>), dim3(grid), dim3(kLongDfaThreads), 0, stream, la);
    else
      hipLaunchKernelGGL((long_dfa_seg1_kernel<uint16_t, false>), dim3(grid), dim3(kLongDfaThreads), 0, stream, la);
  }
  uint64_t grid = (la.npend + 255) / 256;
  if (grid > 4096) grid = 4096;
  if (grid) {
    if (u32)
      hipLaunchKernelGGL(long_dfa_fix_kernel<uint32_t>, dim3(grid), dim3(256), 0, stream, la);
    else
      hipLaunchKernelGGL(long_dfa_fix_kernel<uint16_t>, dim3(grid), dim3(256), 0, stream, la);
  }
  return hipGetLastError();
}

hipError_t verify_candidates(const VerifyArgs& v, bool candidates, hipStream_t stream) {
  uint64_t grid = (v.ntiles + 3) / 4;
  if (grid > 16384) grid = 16384;
  if (grid == 0) return hipSuccess;
  if (!candidates)
    hipLaunchKernelGGL(resolve_tiles_kernel, dim3(grid), dim3(256), 0, stream, v);
  else if (v.nfa && v.nfa_words <= kNfaSmallWords)
    hipLaunchKernelGGL(verify_nfa_kernel<kNfaSmallWords>, dim3(grid), dim3(256), 0, stream, v);
  else if (v.nfa)
    hipLaunchKernelGGL(verify_nfa_kernel<kNfaMaxWords>, dim3(grid), dim3(256), 0, stream, v);
  else if (v.full_u32)
    hipLaunchKernelGGL((verify_kernel<uint32_t, false>), dim3(grid), dim3(256), 0, stream, v);
  else if (v.ximg)
    // one persistent 1024-thread workgroup per CU: the LDS copy once per CU
    hipLaunchKernelGGL((verify_kernel<uint16_t, true>), dim3(std::min<uint64_t>(v.num_cus, (v.ntiles + 15) / 16)),
                       dim3(1024), 0, stream, v);
  else
    hipLaunchKernelGGL((verify_kernel<uint16_t, false>), dim3(grid), dim3(256), 0, stream, v);
  return hipGetLastError();
}

#endif  // DG_PART(0)

}  // namespace dgrep
