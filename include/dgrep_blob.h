/*
 * dgrep_blob.h — layout of a compiled pattern ("DFA blob").
 *
 * Produced by dgrep_compile (the pattern compiler), consumed by
 * dgrep_load_dfa. A Go front end (regexp/syntax) may emit the
 * same layout. All integers little-endian.
 *
 * The automaton runs over the raw bytes of a split and restarts at every
 * '\n', so one pass over the split evaluates regexp.Match on every line of
 * strings.Split(contents, "\n") (application/grep.go:17-21):
 *   - state `start` is the state at the beginning of every line;
 *   - trans[s][class('\n')] is `start_m` if the line ending there matches,
 *     else `start`; `start_m` behaves exactly like `start` otherwise, so a
 *     matching line is recognised by "the state after a '\n' is start_m";
 *   - the last line of a split (no trailing '\n') matches iff
 *     trans[s_end][class('\n')] == start_m.
 */
#ifndef DGREP_BLOB_H
#define DGREP_BLOB_H
#include <stdint.h>

#define DGREP_BLOB_MAGIC 0x50524744u /* "DGRP" */
#define DGREP_BLOB_VERSION 1u

typedef struct {
  uint32_t magic;
  uint32_t version;
  uint32_t flags;    /* DGREP_DFA_* */
  uint32_t nstates;
  uint32_t nclasses;
  uint32_t start;
  uint32_t start_m;
  uint32_t nfa_bytes; /* size of the NFA program after trans (0 unless DGREP_DFA_PARTIAL) */
  uint8_t byte_class[256];
  /* followed by uint32_t trans[nstates * nclasses] (row-major by state), then
   * nfa_bytes of NFA program (DGREP_DFA_PARTIAL only, see below) */
} dgrep_blob_header;

/*
 * DGREP_DFA_PARTIAL: the minimal DFA would exceed the compiler's state budget
 * (e.g. [ab]*a[ab]{24}, a.{20}$). `trans` then holds the first nstates - 1
 * states of the subset construction in breadth-first order (unminimized, every
 * row exact) and state nstates - 1 is CAND: every transition into a state that
 * was not kept. A line that never enters CAND is decided by the DFA exactly; a
 * line that does is decided by the NFA program, a bit-parallel simulation of
 * the same automaton over rune classes (positions = the NFA's rune-set states):
 *
 *   u32 magic DGREP_NFA_MAGIC, npos (<= DGREP_NFA_MAX_POS), nw = ceil(npos/32),
 *       nrc (rune classes), nnodes (UTF-8 decoder trie nodes), nctx (1, or 4 if
 *       the pattern has \b or \B: ctx = 2 * prev_word + next_word), fffd (rune
 *       class of U+FFFD), has_word
 *   i32 child[nnodes][256]  decoder: >= 1 interior node, -1 invalid sequence,
 *                           <= -2 complete rune of class -2 - v (node 0 = root)
 *   u32 depth[nnodes]       pending bytes at a node (flushed as U+FFFD)
 *   u32 word[nrc]           class is an ASCII word character
 *   u32 has[nrc][nw]        positions whose rune set holds the class
 *   u32 init[2][nctx][nw]   [begin][ctx]: positions in the closure of the start
 *   u32 init_m[2][nctx]     ... and whether that closure reaches Match
 *   u32 cl[npos][nctx][nw]  positions in the closure after consuming position x
 *   u32 mx[nctx][nw]        positions whose closure reaches Match
 *   u32 end_init[2][2]      [begin][prev_word]: start's closure at end of line matches
 *   u32 end_x[2][nw]        [prev_word]: positions whose closure at end of line matches
 *
 * Per rune of class c with consumed-position set P (empty at a line start,
 * begin = 1): S = init[begin][ctx] | OR_{x in P} cl[x][ctx]; the line matches
 * if init_m[begin][ctx] or P & mx[ctx] != 0; else P = S & has[c], begin = 0,
 * prev_word = word[c]. At the end of the line (pending decoder bytes flushed as
 * U+FFFD runes) it matches if end_init[begin][prev_word] or P & end_x[prev_word].
 */
#define DGREP_NFA_MAGIC 0x3141464eu /* "NFA1" */
#define DGREP_NFA_MAX_POS 1024u

#endif
