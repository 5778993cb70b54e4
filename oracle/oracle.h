/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's Map hot path (application/grep.go:13-36)
 * and of the Go standard-library algorithms it calls: strings.Split,
 * regexp.Match (= regexp/syntax Parse with Perl flags + Simplify + Compile +
 * an unanchored NFA search over utf8-decoded runes) and, for the after-Map
 * parity sink, hash/fnv ihash (map_reduce/worker.go:13-17) and the
 * encoding/json KeyValue line (map_reduce/worker.go:92-93).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker. The product (libdgrep.so) never
 * links or calls it.
 *
 * PARITY UNPINNED: the reference ships no tests, fixtures or golden vectors
 *  and its algorithm lives in the Go standard library,
 * which is absent from /root/reference and from this image (no Go toolchain,
 * here or on the GPU box). This restatement follows Go 1.18 (go.mod:3) from
 * the published regexp/syntax behaviour; it is cross-checked against Python
 * `re` (bytes mode) and GNU grep on the subset where their semantics agree
 * with Go's (tests/test_oracle.py), which pins the subset but not Go itself.
 */
#ifndef DGREP_ORACLE_H
#define DGREP_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  ORC_OK = 0,
  ORC_ESYNTAX = 1,      /* Go's regexp.Compile would fail: every line is "no match" */
  ORC_EUNSUPPORTED = 2, /* valid Go, but outside what this restatement models */
};

typedef struct orc_re orc_re;

/* Parse + compile `pat` (n bytes) with Go's Perl flags (regexp.Compile). */
int orc_compile(const char* pat, size_t n, orc_re** out, char* err, size_t errlen);
/* regexp.Match semantics on one line: unanchored, boolean. */
int orc_match(const orc_re* re, const unsigned char* s, size_t n);
void orc_free(orc_re* re);
/* The same verdicts as orc_match, memoized: a lazy DFA whose states are
 * orc_match's own (pc set, previous-rune class) pairs, built on demand (one
 * matcher per thread). Used by orc_map_mt for whole-split checks. */
typedef struct orc_matcher orc_matcher;
orc_matcher* orc_matcher_new(const orc_re* re);
int orc_matcher_match(orc_matcher* m, const unsigned char* s, size_t n);
void orc_matcher_free(orc_matcher* m);

/*
 * grep.go Map restatement: split `contents` on '\n' (strings.Split: k newlines
 * give k+1 lines), test each line with regexp.Match, emit matching lines in
 * ascending order as (1-based line number, byte start, byte length).
 * recompile_per_line != 0 re-parses the pattern for every line exactly as
 * grep.go:21 does (regexp.Match compiles on each call). Returns the number of
 * matching lines (records beyond `cap` are counted but not stored), or -1 if
 * the pattern is unsupported by the restatement. A Go syntax error yields 0.
 */
int64_t orc_map(const char* pat, size_t patn, const unsigned char* contents, size_t n,
                int recompile_per_line, uint64_t* line_no, uint64_t* start, uint64_t* len,
                uint64_t cap);
/* Same as orc_map with one thread per slice of lines (pattern compiled once). */
int64_t orc_map_mt(const char* pat, size_t patn, const unsigned char* contents, size_t n,
                   int nthreads, uint64_t* line_no, uint64_t* start, uint64_t* len, uint64_t cap);

/* map_reduce/worker.go:13-17: FNV-1a 32 & 0x7fffffff. */
uint32_t orc_ihash(const unsigned char* key, size_t n);
/* fmt.Sprintf("%s (line number #%v)", filename, line) (grep.go:25). Returns length. */
size_t orc_format_key(const char* filename, size_t fn, uint64_t line, char* out, size_t cap);
/* json.NewEncoder(f).Encode(&KeyValue{k,v}) line incl. trailing '\n' (worker.go:92-93). */
size_t orc_json_kv(const unsigned char* k, size_t kn, const unsigned char* v, size_t vn, char* out,
                   size_t cap);

#ifdef __cplusplus
}
#endif
#endif
