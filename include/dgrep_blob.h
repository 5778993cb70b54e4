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
  uint32_t reserved;
  uint8_t byte_class[256];
  /* followed by uint32_t trans[nstates * nclasses] (row-major by state) */
} dgrep_blob_header;

#endif
