/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h). PARITY UNPINNED.
 *
 * Restatement of the reference's Map hot path and its parity sink:
 *   orc_map         application/grep.go:13-36  (strings.Split + regexp.Match per line)
 *   orc_ihash       map_reduce/worker.go:13-17 (hash/fnv New32a, & 0x7fffffff)
 *   orc_format_key  application/grep.go:25     (fmt.Sprintf "%s (line number #%v)")
 *   orc_json_kv     map_reduce/worker.go:92-93 (json.Encoder.Encode(&kv), HTML-escaping on)
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* grep.go:17-29. strings.Split(contents, "\n") yields k+1 pieces for k
 * newlines (a trailing '\n' gives a final empty line; an empty file gives
 * one empty line). Each piece is matched on its own; the error returned by
 * regexp.Match is discarded (grep.go:21), so a bad pattern matches nothing. */
int64_t orc_map(const char* pat, size_t patn, const unsigned char* contents, size_t n,
                int recompile_per_line, uint64_t* line_no, uint64_t* start, uint64_t* len,
                uint64_t cap) {
  orc_re* re = NULL;
  int st = orc_compile(pat, patn, &re, NULL, 0);
  if (st == ORC_EUNSUPPORTED) { orc_free(re); return -1; }
  int64_t cnt = 0;
  size_t ls = 0;
  uint64_t ln = 0;
  for (;;) {
    const unsigned char* nl = ls < n ? memchr(contents + ls, '\n', n - ls) : NULL;
    size_t le = nl ? (size_t)(nl - contents) : n;
    ln++;
    int m;
    if (recompile_per_line) {
      /* regexp.Match(pattern, b) = Compile(pattern) then Match(b) */
      orc_re* r2 = NULL;
      orc_compile(pat, patn, &r2, NULL, 0);
      m = orc_match(r2, contents + ls, le - ls);
      orc_free(r2);
    } else {
      m = orc_match(re, contents + ls, le - ls);
    }
    if (m) {
      if ((uint64_t)cnt < cap) {
        if (line_no) line_no[cnt] = ln;
        if (start) start[cnt] = ls;
        if (len) len[cnt] = (uint64_t)(le - ls);
      }
      cnt++;
    }
    if (!nl) break;
    ls = le + 1;
  }
  orc_free(re);
  return cnt;
}

typedef struct {
  const orc_re* re;
  const unsigned char* c;
  size_t lo, hi;        /* byte range of whole lines [lo, hi) */
  uint64_t first_line;  /* 1-based number of the line starting at lo */
  int last;             /* this slice owns the final (possibly empty) line */
  uint64_t* ln; uint64_t* st; uint64_t* lens; uint64_t cnt, cap;
} Slice;

static void* slice_run(void* arg) {
  Slice* s = (Slice*)arg;
  orc_matcher* mt = orc_matcher_new(s->re);
  size_t ls = s->lo;
  uint64_t ln = s->first_line;
  s->cnt = 0;
  while (ls < s->hi || (s->last && ls == s->hi)) {
    const unsigned char* nl = ls < s->hi ? memchr(s->c + ls, '\n', s->hi - ls) : NULL;
    size_t le = nl ? (size_t)(nl - s->c) : s->hi;
    if (orc_matcher_match(mt, s->c + ls, le - ls)) {
      if (s->cnt >= s->cap) {
        s->cap = s->cap ? s->cap * 2 : 1024;
        s->ln = realloc(s->ln, s->cap * sizeof(uint64_t));
        s->st = realloc(s->st, s->cap * sizeof(uint64_t));
        s->lens = realloc(s->lens, s->cap * sizeof(uint64_t));
      }
      s->ln[s->cnt] = ln; s->st[s->cnt] = ls; s->lens[s->cnt] = (uint64_t)(le - ls);
      s->cnt++;
    }
    ln++;
    if (!nl) break;
    ls = le + 1;
  }
  orc_matcher_free(mt);
  return NULL;
}

int64_t orc_map_mt(const char* pat, size_t patn, const unsigned char* contents, size_t n,
                   int nthreads, uint64_t* line_no, uint64_t* start, uint64_t* len, uint64_t cap) {
  orc_re* re = NULL;
  int st = orc_compile(pat, patn, &re, NULL, 0);
  if (st == ORC_EUNSUPPORTED) { orc_free(re); return -1; }
  if (nthreads < 1) nthreads = 1;
  Slice* sl = calloc((size_t)nthreads, sizeof(Slice));
  pthread_t* th = calloc((size_t)nthreads, sizeof(pthread_t));
  /* cut at line starts; count lines before each cut to number them */
  size_t prev = 0;
  uint64_t line = 1;
  for (int t = 0; t < nthreads; t++) {
    size_t cut = (t == nthreads - 1) ? n : (n / (size_t)nthreads) * (size_t)(t + 1);
    if (cut < prev) cut = prev;
    if (t != nthreads - 1) {
      const unsigned char* nl = cut < n ? memchr(contents + cut, '\n', n - cut) : NULL;
      cut = nl ? (size_t)(nl - contents) + 1 : n;
    }
    sl[t].re = re; sl[t].c = contents; sl[t].lo = prev; sl[t].hi = cut;
    /* the first slice that reaches n owns the final (possibly empty) line */
    sl[t].first_line = line; sl[t].last = (cut == n && (t == 0 || sl[t - 1].hi < n));
    for (size_t i = prev; i < cut; i++) line += contents[i] == '\n';
    prev = cut;
  }
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, slice_run, &sl[t]);
  int64_t cnt = 0;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    for (uint64_t i = 0; i < sl[t].cnt; i++, cnt++) {
      if ((uint64_t)cnt < cap) {
        if (line_no) line_no[cnt] = sl[t].ln[i];
        if (start) start[cnt] = sl[t].st[i];
        if (len) len[cnt] = sl[t].lens[i];
      }
    }
    free(sl[t].ln); free(sl[t].st); free(sl[t].lens);
  }
  free(sl); free(th);
  orc_free(re);
  return cnt;
}

uint32_t orc_ihash(const unsigned char* key, size_t n) {
  uint32_t h = 2166136261u;
  for (size_t i = 0; i < n; i++) { h ^= key[i]; h *= 16777619u; }
  return h & 0x7fffffffu;
}

size_t orc_format_key(const char* filename, size_t fn, uint64_t line, char* out, size_t cap) {
  char num[32];
  int k = snprintf(num, sizeof num, "%llu", (unsigned long long)line);
  size_t need = fn + strlen(" (line number #") + (size_t)k + 1;
  if (out && cap >= need) {
    memcpy(out, filename, fn);
    size_t o = fn;
    memcpy(out + o, " (line number #", 15); o += 15;
    memcpy(out + o, num, (size_t)k); o += (size_t)k;
    out[o++] = ')';
  }
  return need;
}

static size_t json_str(const unsigned char* s, size_t n, char* out, size_t o, size_t cap) {
  static const char hex[] = "0123456789abcdef";
#define PUT(ch) do { if (o < cap) out[o] = (char)(ch); o++; } while (0)
  PUT('"');
  size_t i = 0;
  while (i < n) {
    unsigned char b = s[i];
    if (b < 0x80) {
      int safe = b >= 0x20 && b != '"' && b != '\\' && b != '<' && b != '>' && b != '&';
      if (safe) { PUT(b); i++; continue; }
      PUT('\\');
      if (b == '\\' || b == '"') PUT(b);
      else if (b == '\n') PUT('n');
      else if (b == '\r') PUT('r');
      else if (b == '\t') PUT('t');
      else { PUT('u'); PUT('0'); PUT('0'); PUT(hex[b >> 4]); PUT(hex[b & 15]); }
      i++;
      continue;
    }
    /* utf8.DecodeRune: invalid -> �; U+2028/2029 escaped */
    int need = 0; unsigned lo = 0x80, hi = 0xBF; unsigned r = 0; int ok = 1;
    if (b >= 0xC2 && b <= 0xDF) { need = 2; r = b & 0x1F; }
    else if (b >= 0xE0 && b <= 0xEF) { need = 3; r = b & 0x0F; if (b == 0xE0) lo = 0xA0; if (b == 0xED) hi = 0x9F; }
    else if (b >= 0xF0 && b <= 0xF4) { need = 4; r = b & 7; if (b == 0xF0) lo = 0x90; if (b == 0xF4) hi = 0x8F; }
    else ok = 0;
    if (ok && i + (size_t)need > n) ok = 0;
    if (ok && (s[i + 1] < lo || s[i + 1] > hi)) ok = 0;
    for (int k = 1; ok && k < need; k++) {
      if (k > 1 && (s[i + k] < 0x80 || s[i + k] > 0xBF)) ok = 0;
      r = (r << 6) | (s[i + k] & 0x3F);
    }
    if (!ok) {
      const char* e = "\\ufffd";
      for (int k = 0; k < 6; k++) PUT(e[k]);
      i++;
      continue;
    }
    if (r == 0x2028 || r == 0x2029) {
      const char* e = "\\u202";
      for (int k = 0; k < 5; k++) PUT(e[k]);
      PUT(hex[r & 15]);
    } else {
      for (int k = 0; k < need; k++) PUT(s[i + k]);
    }
    i += (size_t)need;
  }
  PUT('"');
#undef PUT
  return o;
}

size_t orc_json_kv(const unsigned char* k, size_t kn, const unsigned char* v, size_t vn, char* out,
                   size_t cap) {
  size_t o = 0;
  const char* a = "{\"Key\":";
  for (const char* x = a; *x; x++) { if (o < cap) out[o] = *x; o++; }
  o = json_str(k, kn, out, o, cap);
  const char* b = ",\"Value\":";
  for (const char* x = b; *x; x++) { if (o < cap) out[o] = *x; o++; }
  o = json_str(v, vn, out, o, cap);
  if (o < cap) out[o] = '}';
  o++;
  if (o < cap) out[o] = '\n';
  o++;
  return o;
}
