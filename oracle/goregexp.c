/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h). PARITY UNPINNED.
 *
 * Restatement of Go 1.18 regexp as called by application/grep.go:21
 * (`regexp.Match(pattern, []byte(line))`):
 *   [Go stdlib] regexp/syntax/parse.go  Parse(pattern, syntax.Perl)   -> parse_*()
 *   [Go stdlib] regexp/syntax/simplify.go (Repeat expansion)          -> compile_node()
 *   [Go stdlib] regexp/syntax/compile.go  (Thompson program)          -> compile_node()
 *   [Go stdlib] regexp/exec.go + pike VM, unanchored boolean search   -> orc_match()
 *   [Go stdlib] unicode/utf8.DecodeRune (bad byte = U+FFFD, width 1)  -> dec_rune()
 * The parser keeps Go's operator-stack shape (push / concat / alternate /
 * swapVerticalBar / parseRightParen) so that its accept/reject decisions
 * follow parse.go statement by statement.
 */
#include "oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "unicode_tables.inc"

#define MAXRUNE 0x10FFFF
#define RUNEERR 0xFFFD
#define MIN_FOLD 0x41
#define MAX_FOLD 0x1E943

/* ---- utf8 (Go unicode/utf8 DecodeRune) ---------------------------------- */
static int dec_rune(const unsigned char* s, size_t n, int* size) {
  if (n == 0) { *size = 0; return RUNEERR; }
  unsigned c0 = s[0];
  if (c0 < 0x80) { *size = 1; return (int)c0; }
  int need; unsigned lo = 0x80, hi = 0xBF; unsigned r;
  if (c0 >= 0xC2 && c0 <= 0xDF) { need = 2; r = c0 & 0x1F; }
  else if (c0 >= 0xE0 && c0 <= 0xEF) {
    need = 3; r = c0 & 0x0F;
    if (c0 == 0xE0) lo = 0xA0; else if (c0 == 0xED) hi = 0x9F;
  } else if (c0 >= 0xF0 && c0 <= 0xF4) {
    need = 4; r = c0 & 0x07;
    if (c0 == 0xF0) lo = 0x90; else if (c0 == 0xF4) hi = 0x8F;
  } else { *size = 1; return RUNEERR; }
  if (n < (size_t)need) { *size = 1; return RUNEERR; }
  if (s[1] < lo || s[1] > hi) { *size = 1; return RUNEERR; }
  r = (r << 6) | (s[1] & 0x3F);
  for (int i = 2; i < need; i++) {
    if (s[i] < 0x80 || s[i] > 0xBF) { *size = 1; return RUNEERR; }
    r = (r << 6) | (s[i] & 0x3F);
  }
  *size = need;
  return (int)r;
}

/* ---- rune-range class helpers (sorted, merged pairs) --------------------- */
typedef struct { int* r; int n, cap; } Class; /* n = number of ints (2 per range) */

static void cls_push(Class* c, int lo, int hi) {
  if (c->n + 2 > c->cap) {
    c->cap = c->cap ? c->cap * 2 : 16;
    c->r = (int*)realloc(c->r, sizeof(int) * c->cap);
  }
  c->r[c->n++] = lo; c->r[c->n++] = hi;
}
static int cmp_pair(const void* a, const void* b) {
  const int* x = (const int*)a; const int* y = (const int*)b;
  if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
  return x[1] < y[1] ? 1 : (x[1] > y[1] ? -1 : 0);
}
/* cleanClass: sort + merge (parse.go cleanClass) */
static void cls_clean(Class* c) {
  if (c->n <= 2) return;
  qsort(c->r, c->n / 2, sizeof(int) * 2, cmp_pair);
  int w = 2;
  for (int i = 2; i < c->n; i += 2) {
    int lo = c->r[i], hi = c->r[i + 1];
    if (lo <= c->r[w - 1] + 1) {
      if (hi > c->r[w - 1]) c->r[w - 1] = hi;
      continue;
    }
    c->r[w] = lo; c->r[w + 1] = hi; w += 2;
  }
  c->n = w;
}
/* negateClass (parse.go negateClass), input must be clean */
static void cls_negate(Class* c) {
  Class o = {0};
  int next = 0;
  for (int i = 0; i < c->n; i += 2) {
    if (c->r[i] > next) cls_push(&o, next, c->r[i] - 1);
    next = c->r[i + 1] + 1;
  }
  if (next <= MAXRUNE) cls_push(&o, next, MAXRUNE);
  free(c->r);
  *c = o;
}
static int cls_has(const int* r, int n, int x) {
  int lo = 0, hi = n / 2;
  while (lo < hi) {
    int m = (lo + hi) / 2;
    if (x < r[2 * m]) hi = m;
    else if (x > r[2 * m + 1]) lo = m + 1;
    else return 1;
  }
  return 0;
}

/* ---- case folding --------------------------------------------------------
 * [Go stdlib] unicode.SimpleFold: orc_fold lists, sorted by rune, the next
 * member of every simple-case-folding orbit of two or more runes (generated
 * from Unicode 13.0, the version of Go 1.18's tables; at most 4 members). */
static int fold_next(int r) {
  int lo = 0, hi = orc_nfold;
  while (lo < hi) {
    int m = (lo + hi) / 2, x = (int)orc_fold[2 * m];
    if (x == r) return (int)orc_fold[2 * m + 1];
    if (x < r) lo = m + 1;
    else hi = m;
  }
  return -1;
}
/* the orbit of r, r first; returns its size (1..4) */
static int fold_orbit(int r, int out[4]) {
  int k = 0;
  out[k++] = r;
  for (int x = fold_next(r); x >= 0 && x != r && k < 4; x = fold_next(x)) out[k++] = x;
  return k;
}

/* ---- AST (regexp/syntax.Regexp) ------------------------------------------- */
enum {
  OP_NOMATCH = 1, OP_EMPTY, OP_LITERAL, OP_CLASS, OP_ANYNOTNL, OP_ANY,
  OP_BEGINLINE, OP_ENDLINE, OP_BEGINTEXT, OP_ENDTEXT, OP_WORDB, OP_NOWORDB,
  OP_CAPTURE, OP_STAR, OP_PLUS, OP_QUEST, OP_REPEAT, OP_CONCAT, OP_ALT,
  OP_PSEUDO = 128, OP_LPAREN, OP_VBAR
};
enum { F_FOLD = 1, F_DOTNL = 2, F_ONELINE = 4, F_NONGREEDY = 8 };

typedef struct Node {
  int op, flags;
  Class cls;          /* OP_LITERAL: single rune in cls.r[0]; OP_CLASS: ranges */
  struct Node** sub;
  int nsub, subcap;
  int min, max, cap;
} Node;

static Node* node_new(int op, int flags) {
  Node* n = (Node*)calloc(1, sizeof(Node));
  n->op = op; n->flags = flags;
  return n;
}
static void node_add(Node* n, Node* s) {
  if (n->nsub == n->subcap) {
    n->subcap = n->subcap ? n->subcap * 2 : 4;
    n->sub = (Node**)realloc(n->sub, sizeof(Node*) * n->subcap);
  }
  n->sub[n->nsub++] = s;
}
static void node_free(Node* n) {
  if (!n) return;
  for (int i = 0; i < n->nsub; i++) node_free(n->sub[i]);
  free(n->sub); free(n->cls.r); free(n);
}

/* ---- parser state (regexp/syntax.parser) ---------------------------------- */
typedef struct {
  Node** st; int nst, cst;
  int flags;
  int numcap;
  int err;          /* Go would return an error */
  int unsupported;  /* valid Go we do not model */
  const char* msg;
} Parser;

static void push_raw(Parser* p, Node* n) {
  if (p->nst == p->cst) {
    p->cst = p->cst ? p->cst * 2 : 16;
    p->st = (Node**)realloc(p->st, sizeof(Node*) * p->cst);
  }
  p->st[p->nst++] = n;
}
static void p_push(Parser* p, Node* n) { push_raw(p, n); }
static Node* p_op(Parser* p, int op) {
  Node* n = node_new(op, p->flags);
  p_push(p, n);
  return n;
}
static void fail(Parser* p, const char* m) { if (!p->err) { p->err = 1; p->msg = m; } }

/* nextRune (parse.go): invalid UTF-8 is an error; empty input gives RuneError */
static int next_rune(Parser* p, const unsigned char** t, const unsigned char* end) {
  int sz;
  int c = dec_rune(*t, (size_t)(end - *t), &sz);
  if (c == RUNEERR && sz == 1) { fail(p, "invalid UTF-8"); return -1; }
  *t += sz;
  return c;
}

/* p.literal(r) */
static void p_literal(Parser* p, int r) {
  Node* n = node_new(OP_LITERAL, p->flags);
  cls_push(&n->cls, r, r);
  p_push(p, n);
}

/* appendFoldedRange (parse.go) */
static void append_folded_range(Parser* p, Class* c, int lo, int hi) {
  if ((lo <= MIN_FOLD && hi >= MAX_FOLD) || hi < MIN_FOLD || lo > MAX_FOLD) {
    cls_push(c, lo, hi);
    return;
  }
  if (lo < MIN_FOLD) { cls_push(c, lo, MIN_FOLD - 1); lo = MIN_FOLD; }
  if (hi > MAX_FOLD) { cls_push(c, MAX_FOLD + 1, hi); hi = MAX_FOLD; }
  for (int x = lo; x <= hi; x++) {
    int o[4];
    int k = fold_orbit(x, o);
    for (int i = 0; i < k; i++) cls_push(c, o[i], o[i]);
  }
}

/* charGroup tables (perl_groups.go) */
typedef struct { const char* name; int sign; const int* r; int n; } Group;
static const int g_digit[] = {'0', '9'};
static const int g_space[] = {'\t', '\n', '\f', '\f', '\r', '\r', ' ', ' '};
static const int g_word[] = {'0', '9', 'A', 'Z', '_', '_', 'a', 'z'};
static const int g_alnum[] = {'0', '9', 'A', 'Z', 'a', 'z'};
static const int g_alpha[] = {'A', 'Z', 'a', 'z'};
static const int g_ascii[] = {0, 0x7F};
static const int g_blank[] = {'\t', '\t', ' ', ' '};
static const int g_cntrl[] = {0, 0x1F, 0x7F, 0x7F};
static const int g_graph[] = {'!', '~'};
static const int g_lower[] = {'a', 'z'};
static const int g_print[] = {' ', '~'};
static const int g_punct[] = {'!', '/', ':', '@', '[', '`', '{', '~'};
static const int g_pspace[] = {'\t', '\r', ' ', ' '};
static const int g_upper[] = {'A', 'Z'};
static const int g_xdigit[] = {'0', '9', 'A', 'F', 'a', 'f'};
#define GN(a) ((int)(sizeof(a) / sizeof(int)))
static const Group perl_groups[] = {
  {"\\d", +1, g_digit, GN(g_digit)}, {"\\D", -1, g_digit, GN(g_digit)},
  {"\\s", +1, g_space, GN(g_space)}, {"\\S", -1, g_space, GN(g_space)},
  {"\\w", +1, g_word, GN(g_word)},   {"\\W", -1, g_word, GN(g_word)},
};
#define PX(nm, arr) {"[:" nm ":]", +1, arr, GN(arr)}, {"[:^" nm ":]", -1, arr, GN(arr)}
static const Group posix_groups[] = {
  PX("alnum", g_alnum), PX("alpha", g_alpha), PX("ascii", g_ascii), PX("blank", g_blank),
  PX("cntrl", g_cntrl), PX("digit", g_digit), PX("graph", g_graph), PX("lower", g_lower),
  PX("print", g_print), PX("punct", g_punct), PX("space", g_pspace), PX("upper", g_upper),
  PX("word", g_word),   PX("xdigit", g_xdigit),
};

/* appendGroup (parse.go): folds the group under (?i), then adds or negates */
static void append_group(Parser* p, Class* c, const Group* g) {
  Class tmp = {0};
  for (int i = 0; i < g->n; i += 2) {
    if (p->flags & F_FOLD) append_folded_range(p, &tmp, g->r[i], g->r[i + 1]);
    else cls_push(&tmp, g->r[i], g->r[i + 1]);
  }
  cls_clean(&tmp);
  if (g->sign < 0) cls_negate(&tmp);
  for (int i = 0; i < tmp.n; i += 2) cls_push(c, tmp.r[i], tmp.r[i + 1]);
  free(tmp.r);
}

/* parsePerlClassEscape: returns 1 and advances if t starts with \d \D \s \S \w \W */
static int parse_perl_class_escape(Parser* p, const unsigned char** t, const unsigned char* end, Class* c) {
  if (end - *t < 2 || (*t)[0] != '\\') return 0;
  for (size_t i = 0; i < sizeof(perl_groups) / sizeof(perl_groups[0]); i++) {
    if ((*t)[1] == (unsigned char)perl_groups[i].name[1]) {
      append_group(p, c, &perl_groups[i]);
      *t += 2;
      return 1;
    }
  }
  return 0;
}

/* parseNamedClass: 1 = consumed, 0 = not a named class, sets err on bad name */
static int parse_named_class(Parser* p, const unsigned char** t, const unsigned char* end, Class* c) {
  const unsigned char* s = *t;
  if (end - s < 2 || s[0] != '[' || s[1] != ':') return 0;
  const unsigned char* q = NULL;
  for (const unsigned char* x = s + 2; x + 1 < end; x++)
    if (x[0] == ':' && x[1] == ']') { q = x; break; }
  if (!q) return 0;
  size_t nl = (size_t)(q + 2 - s);
  for (size_t i = 0; i < sizeof(posix_groups) / sizeof(posix_groups[0]); i++) {
    if (strlen(posix_groups[i].name) == nl && memcmp(posix_groups[i].name, s, nl) == 0) {
      append_group(p, c, &posix_groups[i]);
      *t = q + 2;
      return 1;
    }
  }
  fail(p, "invalid character class range (posix name)");
  return -1;
}

/* parseUnicodeClass: \pN, \p{Name}, \PN, \P{^Name}. 1 consumed, 0 not, -1 error */
static int parse_unicode_class(Parser* p, const unsigned char** t, const unsigned char* end, Class* c) {
  const unsigned char* s = *t;
  if (end - s < 2 || s[0] != '\\' || (s[1] != 'p' && s[1] != 'P')) return 0;
  int sign = s[1] == 'P' ? -1 : +1;
  const unsigned char* x = s + 2;
  int sz;
  int ch = dec_rune(x, (size_t)(end - x), &sz);
  if (ch == RUNEERR && sz == 1) return 0; /* Go: nextRune err -> return (no class) */
  const unsigned char *name, *name_end, *rest;
  if (ch != '{') {
    name = x; name_end = x + sz; rest = x + sz;
  } else {
    const unsigned char* close = memchr(s, '}', (size_t)(end - s));
    if (!close) { fail(p, "invalid character class range (no })"); return -1; }
    name = s + 3; name_end = close; rest = close + 1;
    /* checkUTF8(name) */
    for (const unsigned char* y = name; y < name_end;) {
      int k; int r = dec_rune(y, (size_t)(name_end - y), &k);
      if (r == RUNEERR && k == 1) { fail(p, "invalid UTF-8"); return -1; }
      y += k;
    }
  }
  if (name < name_end && name[0] == '^') { sign = -sign; name++; }
  size_t nl = (size_t)(name_end - name);
  Class tmp = {0};
  int fold_tab = 0, found = 0;
  if (nl == 3 && memcmp(name, "Any", 3) == 0) {
    cls_push(&tmp, 0, MAXRUNE); found = 1;
  } else {
    for (int i = 0; i < orc_ncategories; i++) {
      if (strlen(orc_categories[i].name) == nl && memcmp(orc_categories[i].name, name, nl) == 0) {
        for (int j = 0; j < orc_categories[i].n; j++)
          cls_push(&tmp, (int)orc_categories[i].r[2 * j], (int)orc_categories[i].r[2 * j + 1]);
        fold_tab = orc_categories[i].fold;
        found = 1;
        break;
      }
    }
    /* unicodeTable (parse.go): unicode.Categories, then unicode.Scripts */
    for (int i = 0; !found && i < orc_nscripts; i++) {
      if (strlen(orc_scripts[i].name) == nl && memcmp(orc_scripts[i].name, name, nl) == 0) {
        for (int j = 0; j < orc_scripts[i].n; j++)
          cls_push(&tmp, (int)orc_scripts[i].r[2 * j], (int)orc_scripts[i].r[2 * j + 1]);
        fold_tab = orc_scripts[i].fold;
        found = 1;
      }
    }
  }
  if (!found) { free(tmp.r); fail(p, "invalid character class range (unicode name)"); return -1; }
  if ((p->flags & F_FOLD) && fold_tab) {
    /* FoldCategory / FoldScript (parseUnicodeClass): add the runes that simple-fold into the table */
    Class closed = {0};
    cls_clean(&tmp);
    for (int i = 0; i < tmp.n; i += 2) {
      int lo = tmp.r[i] < MIN_FOLD ? MIN_FOLD : tmp.r[i], hi = tmp.r[i + 1] > MAX_FOLD ? MAX_FOLD : tmp.r[i + 1];
      for (int x = lo; x <= hi; x++) {
        int o[4];
        int k = fold_orbit(x, o);
        for (int j = 1; j < k; j++) cls_push(&closed, o[j], o[j]);
      }
    }
    for (int i = 0; i < closed.n; i += 2) cls_push(&tmp, closed.r[i], closed.r[i + 1]);
    free(closed.r);
  }
  cls_clean(&tmp);
  if (sign < 0) cls_negate(&tmp);
  for (int i = 0; i < tmp.n; i += 2) cls_push(c, tmp.r[i], tmp.r[i + 1]);
  free(tmp.r);
  *t = rest;
  return 1;
}

static int unhex(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
static int isalnum_ascii(int c) {
  return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z');
}

/* parseEscape: t points at '\\'. returns rune or -1 on error */
static int parse_escape(Parser* p, const unsigned char** tp, const unsigned char* end) {
  const unsigned char* t = *tp + 1;
  if (t >= end) { fail(p, "trailing backslash"); return -1; }
  int c = next_rune(p, &t, end);
  if (c < 0) return -1;
  int r;
  switch (c) {
    case '1': case '2': case '3': case '4': case '5': case '6': case '7':
      if (t >= end || *t < '0' || *t > '7') break; /* backreference: unsupported by Go */
      /* fallthrough */
    case '0':
      r = c - '0';
      for (int i = 1; i < 3; i++) {
        if (t >= end || *t < '0' || *t > '7') break;
        r = r * 8 + (*t - '0');
        t++;
      }
      *tp = t;
      return r;
    case 'x': {
      if (t >= end) break;
      c = next_rune(p, &t, end);
      if (c < 0) return -1;
      if (c == '{') {
        int nhex = 0; r = 0;
        for (;;) {
          if (t >= end) goto bad;
          c = next_rune(p, &t, end);
          if (c < 0) return -1;
          if (c == '}') break;
          int v = unhex(c);
          if (v < 0) goto bad;
          r = r * 16 + v;
          if (r > MAXRUNE) goto bad;
          nhex++;
        }
        if (nhex == 0) goto bad;
        *tp = t;
        return r;
      }
      int x = unhex(c);
      int sz;
      c = dec_rune(t, (size_t)(end - t), &sz);
      if (c == RUNEERR && sz == 1) { fail(p, "invalid UTF-8"); return -1; }
      t += sz;
      int y = unhex(c);
      if (x < 0 || y < 0) break;
      *tp = t;
      return x * 16 + y;
    }
    case 'a': *tp = t; return 7;
    case 'f': *tp = t; return 12;
    case 'n': *tp = t; return 10;
    case 'r': *tp = t; return 13;
    case 't': *tp = t; return 9;
    case 'v': *tp = t; return 11;
    default:
      if (c < 0x80 && !isalnum_ascii(c)) { *tp = t; return c; }
      break;
  }
bad:
  fail(p, "invalid escape sequence");
  return -1;
}

/* parseClassChar */
static int parse_class_char(Parser* p, const unsigned char** t, const unsigned char* end) {
  if (*t >= end) { fail(p, "missing closing ]"); return -1; }
  if (**t == '\\') return parse_escape(p, t, end);
  return next_rune(p, t, end);
}

/* parseClass: t points at '[' */
static void parse_class(Parser* p, const unsigned char** tp, const unsigned char* end) {
  const unsigned char* t = *tp + 1;
  Node* re = node_new(OP_CLASS, p->flags);
  Class* c = &re->cls;
  int sign = +1;
  if (t < end && *t == '^') { sign = -1; t++; } /* ClassNL set: no '\n' pre-insert */
  int first = 1;
  while (t >= end || *t != ']' || first) {
    /* PerlX set: '-' anywhere is fine */
    first = 0;
    if (end - t > 2 && t[0] == '[' && t[1] == ':') {
      int k = parse_named_class(p, &t, end, c);
      if (k < 0) { node_free(re); return; }
      if (k > 0) continue;
    }
    {
      int k = parse_unicode_class(p, &t, end, c);
      if (k < 0) { node_free(re); return; }
      if (k > 0) continue;
    }
    if (parse_perl_class_escape(p, &t, end, c)) continue;
    int lo = parse_class_char(p, &t, end);
    if (lo < 0) { node_free(re); return; }
    int hi = lo;
    if (end - t >= 2 && t[0] == '-' && t[1] != ']') {
      t++;
      hi = parse_class_char(p, &t, end);
      if (hi < 0) { node_free(re); return; }
      if (hi < lo) { fail(p, "invalid character class range"); node_free(re); return; }
    }
    if (p->flags & F_FOLD) append_folded_range(p, c, lo, hi);
    else cls_push(c, lo, hi);
  }
  t++; /* ] */
  cls_clean(c);
  if (sign < 0) cls_negate(c);
  p_push(p, re);
  *tp = t;
}

/* repeatIsValid (parse.go) */
static int repeat_is_valid(const Node* re, int n) {
  if (re->op == OP_REPEAT) {
    int m = re->max;
    if (m == 0) return 1;
    if (m < 0) m = re->min;
    if (m > n) return 0;
    if (m > 0) n /= m;
  }
  for (int i = 0; i < re->nsub; i++)
    if (!repeat_is_valid(re->sub[i], n)) return 0;
  return 1;
}

/* p.repeat: `after` may be advanced past a non-greedy '?' */
static void p_repeat(Parser* p, int op, int min, int max, const unsigned char** after,
                     const unsigned char* end, int last_repeat) {
  int flags = p->flags;
  if (*after < end && **after == '?') { (*after)++; flags ^= F_NONGREEDY; }
  if (last_repeat) { fail(p, "invalid nested repetition operator"); return; }
  if (p->nst == 0) { fail(p, "missing argument to repetition operator"); return; }
  Node* sub = p->st[p->nst - 1];
  if (sub->op >= OP_PSEUDO) { fail(p, "missing argument to repetition operator"); return; }
  Node* re = node_new(op, flags);
  re->min = min; re->max = max;
  node_add(re, sub);
  p->st[p->nst - 1] = re;
  if (op == OP_REPEAT && (min >= 2 || max >= 2) && !repeat_is_valid(re, 1000))
    fail(p, "invalid repeat count");
}

/* parseInt / parseRepeat (parse.go). returns 1 if a repeat was parsed */
static int parse_int(const unsigned char** s, const unsigned char* end, int* n) {
  const unsigned char* t = *s;
  if (t >= end || *t < '0' || *t > '9') return 0;
  if (end - t >= 2 && t[0] == '0' && t[1] >= '0' && t[1] <= '9') return 0;
  const unsigned char* d = t;
  while (t < end && *t >= '0' && *t <= '9') t++;
  *n = 0;
  for (const unsigned char* x = d; x < t; x++) {
    if (*n >= 100000000) { *n = -1; break; }
    *n = *n * 10 + (*x - '0');
  }
  *s = t;
  return 1;
}
static int parse_repeat(const unsigned char* s, const unsigned char* end, int* min, int* max,
                        const unsigned char** rest) {
  if (s >= end || *s != '{') return 0;
  s++;
  if (!parse_int(&s, end, min)) return 0;
  if (s >= end) return 0;
  if (*s != ',') {
    *max = *min;
  } else {
    s++;
    if (s >= end) return 0;
    if (*s == '}') *max = -1;
    else if (!parse_int(&s, end, max)) return 0;
    else if (*max < 0) *min = -1;
  }
  if (s >= end || *s != '}') return 0;
  *rest = s + 1;
  return 1;
}

/* concat / alternate collapse the stack above the nearest pseudo-op */
static void p_concat(Parser* p) {
  int i = p->nst;
  while (i > 0 && p->st[i - 1]->op < OP_PSEUDO) i--;
  int k = p->nst - i;
  Node* n;
  if (k == 0) n = node_new(OP_EMPTY, p->flags);
  else if (k == 1) n = p->st[i];
  else { n = node_new(OP_CONCAT, p->flags); for (int j = i; j < p->nst; j++) node_add(n, p->st[j]); }
  p->nst = i;
  push_raw(p, n);
}
static void p_alternate(Parser* p) {
  int i = p->nst;
  while (i > 0 && p->st[i - 1]->op < OP_PSEUDO) i--;
  int k = p->nst - i;
  Node* n;
  if (k == 0) n = node_new(OP_NOMATCH, p->flags);
  else if (k == 1) n = p->st[i];
  else { n = node_new(OP_ALT, p->flags); for (int j = i; j < p->nst; j++) node_add(n, p->st[j]); }
  p->nst = i;
  push_raw(p, n);
}
/* swapVerticalBar: if the stack is [... VBAR x], make it [... x VBAR] so
 * the branches below a bar accumulate; returns 1 if a bar was found. */
static int p_swap_vbar(Parser* p) {
  int n = p->nst;
  if (n >= 2 && p->st[n - 2]->op == OP_VBAR) {
    Node* t = p->st[n - 1];
    p->st[n - 1] = p->st[n - 2];
    p->st[n - 2] = t;
    return 1;
  }
  return 0;
}
/* branches are collected as plain stack entries below the bar; bars carry
 * no payload here (Go folds them into the bar node, same semantics). */
static void p_vertical_bar(Parser* p) {
  p_concat(p);
  if (!p_swap_vbar(p)) p_op(p, OP_VBAR);
}
static void p_right_paren(Parser* p) {
  p_concat(p);
  if (p_swap_vbar(p)) p->nst--, node_free(p->st[p->nst]);
  p_alternate(p);
  int n = p->nst;
  if (n < 2) { fail(p, "unexpected )"); return; }
  Node* re1 = p->st[n - 1];
  Node* re2 = p->st[n - 2];
  if (re2->op != OP_LPAREN) { fail(p, "unexpected )"); return; }
  p->nst -= 2;
  p->flags = re2->flags;
  if (re2->cap == 0) { free(re2); p_push(p, re1); }
  else { re2->op = OP_CAPTURE; node_add(re2, re1); p_push(p, re2); }
}

/* Note on swapVerticalBar: after a bar, each finished branch is swapped
 * below the bar, so the stack reads [LPAREN b1 b2 ... VBAR cur]. p_alternate
 * then sees [b1 b2 ... cur] once the bar is popped. */

static int is_valid_capture_name(const unsigned char* s, size_t n) {
  if (n == 0) return 0;
  for (size_t i = 0; i < n; i++)
    if (s[i] != '_' && !isalnum_ascii(s[i])) return 0;
  return 1;
}

/* parsePerlFlags: t points at "(?" */
static void parse_perl_flags(Parser* p, const unsigned char** tp, const unsigned char* end) {
  const unsigned char* t = *tp;
  if (end - t > 4 && t[2] == 'P' && t[3] == '<') {
    const unsigned char* close = memchr(t, '>', (size_t)(end - t));
    if (!close) { fail(p, "invalid named capture"); return; }
    const unsigned char* name = t + 4;
    for (const unsigned char* y = name; y < close;) {
      int k; int r = dec_rune(y, (size_t)(close - y), &k);
      if (r == RUNEERR && k == 1) { fail(p, "invalid UTF-8"); return; }
      y += k;
    }
    if (!is_valid_capture_name(name, (size_t)(close - name))) { fail(p, "invalid named capture"); return; }
    p->numcap++;
    Node* re = p_op(p, OP_LPAREN);
    re->cap = p->numcap;
    *tp = close + 1;
    return;
  }
  t += 2;
  int flags = p->flags, sign = +1, saw = 0;
  while (t < end) {
    int c = next_rune(p, &t, end);
    if (c < 0) return;
    switch (c) {
      case 'i': flags |= F_FOLD; saw = 1; break;
      case 'm': flags &= ~F_ONELINE; saw = 1; break;
      case 's': flags |= F_DOTNL; saw = 1; break;
      case 'U': flags |= F_NONGREEDY; saw = 1; break;
      case '-':
        if (sign < 0) goto bad;
        sign = -1; flags = ~flags; saw = 0;
        break;
      case ':': case ')':
        if (sign < 0) {
          if (!saw) goto bad;
          flags = ~flags;
        }
        if (c == ':') { Node* re = p_op(p, OP_LPAREN); re->cap = 0; }
        p->flags = flags;
        *tp = t;
        return;
      default:
        goto bad;
    }
  }
bad:
  fail(p, "invalid or unsupported Perl syntax");
}

static Node* parse(const unsigned char* s, size_t n, Parser* p) {
  const unsigned char* t = s;
  const unsigned char* end = s + n;
  p->flags = F_ONELINE; /* syntax.Perl = ClassNL|OneLine|PerlX|UnicodeGroups */
  int last_repeat = 0;
  while (t < end && !p->err) {
    int repeat = 0;
    switch (*t) {
      default: {
        int c = next_rune(p, &t, end);
        if (c < 0) break;
        p_literal(p, c);
        break;
      }
      case '(':
        if (end - t >= 2 && t[1] == '?') { parse_perl_flags(p, &t, end); break; }
        p->numcap++;
        p_op(p, OP_LPAREN)->cap = p->numcap;
        t++;
        break;
      case '|': p_vertical_bar(p); t++; break;
      case ')': p_right_paren(p); t++; break;
      case '^': p_op(p, (p->flags & F_ONELINE) ? OP_BEGINTEXT : OP_BEGINLINE); t++; break;
      case '$': p_op(p, (p->flags & F_ONELINE) ? OP_ENDTEXT : OP_ENDLINE); t++; break;
      case '.': p_op(p, (p->flags & F_DOTNL) ? OP_ANY : OP_ANYNOTNL); t++; break;
      case '[': parse_class(p, &t, end); break;
      case '*': case '+': case '?': {
        int op = *t == '*' ? OP_STAR : (*t == '+' ? OP_PLUS : OP_QUEST);
        const unsigned char* after = t + 1;
        p_repeat(p, op, 0, 0, &after, end, last_repeat);
        repeat = 1;
        t = after;
        break;
      }
      case '{': {
        int min = 0, max = 0;
        const unsigned char* after;
        if (!parse_repeat(t, end, &min, &max, &after)) { p_literal(p, '{'); t++; break; }
        if (min < 0 || min > 1000 || max > 1000 || (max >= 0 && min > max)) {
          fail(p, "invalid repeat count");
          break;
        }
        p_repeat(p, OP_REPEAT, min, max, &after, end, last_repeat);
        repeat = 1;
        t = after;
        break;
      }
      case '\\': {
        if (end - t >= 2) {
          int done = 1;
          switch (t[1]) {
            case 'A': p_op(p, OP_BEGINTEXT); t += 2; break;
            case 'b': p_op(p, OP_WORDB); t += 2; break;
            case 'B': p_op(p, OP_NOWORDB); t += 2; break;
            case 'C': fail(p, "invalid escape \\C"); break;
            case 'Q': {
              const unsigned char* lit = t + 2;
              const unsigned char* lend = end;
              const unsigned char* nt = end;
              for (const unsigned char* x = t; x + 1 < end; x++)
                if (x[0] == '\\' && x[1] == 'E') { lend = x; nt = x + 2; break; }
              if (lend < lit) lend = lit; /* \Q\E handled: x starts at t, never inside "\Q" */
              while (lit < lend && !p->err) {
                int c = next_rune(p, &lit, lend);
                if (c < 0) break;
                p_literal(p, c);
              }
              t = nt;
              break;
            }
            case 'z': p_op(p, OP_ENDTEXT); t += 2; break;
            default: done = 0;
          }
          if (done) break;
        }
        Node* re = node_new(OP_CLASS, p->flags);
        int k = parse_unicode_class(p, &t, end, &re->cls);
        if (k < 0) { node_free(re); break; }
        if (k > 0) { p_push(p, re); break; }
        if (parse_perl_class_escape(p, &t, end, &re->cls)) { p_push(p, re); break; }
        node_free(re);
        int c = parse_escape(p, &t, end);
        if (c < 0) break;
        p_literal(p, c);
        break;
      }
    }
    last_repeat = repeat;
  }
  if (p->err) return NULL;
  p_concat(p);
  if (p_swap_vbar(p)) p->nst--, node_free(p->st[p->nst]);
  p_alternate(p);
  if (p->nst != 1) { fail(p, "missing closing )"); return NULL; }
  return p->st[0];
}

/* ---- program (regexp/syntax.Prog) ---------------------------------------- */
enum { I_FAIL, I_MATCH, I_NOP, I_ALT, I_EMPTY, I_RUNE, I_RUNEFOLD, I_ANY, I_ANYNOTNL };
enum { E_BEGINLINE = 1, E_ENDLINE = 2, E_BEGINTEXT = 4, E_ENDTEXT = 8, E_WORDB = 16, E_NOWORDB = 32 };

typedef struct { int op, out, out1, arg; int* r; int nr; } Inst;
struct orc_re {
  Inst* in; int n, cap;
  int start;
  int status;
};

static int emit(orc_re* pg, int op) {
  if (pg->n == pg->cap) {
    pg->cap = pg->cap ? pg->cap * 2 : 64;
    pg->in = (Inst*)realloc(pg->in, sizeof(Inst) * pg->cap);
  }
  Inst* i = &pg->in[pg->n];
  memset(i, 0, sizeof(*i));
  i->op = op; i->out = -1; i->out1 = -1;
  return pg->n++;
}

/* A fragment: entry pc + list of dangling out slots (encoded pc*2+which). */
typedef struct { int start; int* holes; int nh, ch; int nullable; } Frag;
static void hole_add(Frag* f, int h) {
  if (f->nh == f->ch) { f->ch = f->ch ? f->ch * 2 : 4; f->holes = (int*)realloc(f->holes, sizeof(int) * f->ch); }
  f->holes[f->nh++] = h;
}
static void patch(orc_re* pg, Frag* f, int target) {
  for (int i = 0; i < f->nh; i++) {
    int pc = f->holes[i] >> 1;
    if (f->holes[i] & 1) pg->in[pc].out1 = target; else pg->in[pc].out = target;
  }
  f->nh = 0;
}
static void frag_cat_holes(Frag* a, Frag* b) { for (int i = 0; i < b->nh; i++) hole_add(a, b->holes[i]); free(b->holes); b->holes = NULL; b->nh = b->ch = 0; }

static Frag f_single(orc_re* pg, int pc) { Frag f = {0}; f.start = pc; hole_add(&f, pc * 2); return f; }
static Frag f_nop(orc_re* pg) { return f_single(pg, emit(pg, I_NOP)); }

static Frag compile_node(orc_re* pg, const Node* n);

static Frag c_cat(orc_re* pg, Frag a, Frag b) { patch(pg, &a, b.start); free(a.holes); b.start = a.start; return b; }
static Frag c_alt(orc_re* pg, Frag a, Frag b) {
  int pc = emit(pg, I_ALT);
  pg->in[pc].out = a.start; pg->in[pc].out1 = b.start;
  Frag f = {0}; f.start = pc;
  frag_cat_holes(&f, &a); frag_cat_holes(&f, &b);
  return f;
}
static Frag c_quest(orc_re* pg, Frag a) {
  int pc = emit(pg, I_ALT);
  pg->in[pc].out = a.start;
  Frag f = {0}; f.start = pc;
  hole_add(&f, pc * 2 + 1);
  frag_cat_holes(&f, &a);
  return f;
}
static Frag c_star(orc_re* pg, Frag a) {
  int pc = emit(pg, I_ALT);
  pg->in[pc].out = a.start;
  patch(pg, &a, pc); free(a.holes);
  Frag f = {0}; f.start = pc; hole_add(&f, pc * 2 + 1);
  return f;
}
static Frag c_plus(orc_re* pg, Frag a) {
  int start = a.start;
  Frag s = c_star(pg, a);
  s.start = start;
  return s;
}

static Frag c_rune(orc_re* pg, const int* r, int nr, int fold) {
  int pc = emit(pg, fold ? I_RUNEFOLD : I_RUNE);
  pg->in[pc].r = (int*)malloc(sizeof(int) * (nr ? nr : 1));
  memcpy(pg->in[pc].r, r, sizeof(int) * nr);
  pg->in[pc].nr = nr;
  return f_single(pg, pc);
}
static Frag c_empty(orc_re* pg, int cond) {
  int pc = emit(pg, I_EMPTY);
  pg->in[pc].arg = cond;
  return f_single(pg, pc);
}

/* Simplify (simplify.go) for OpRepeat, then compile (compile.go). */
static Frag compile_node(orc_re* pg, const Node* n) {
  switch (n->op) {
    case OP_NOMATCH: { int pc = emit(pg, I_FAIL); Frag f = {0}; f.start = pc; return f; }
    case OP_EMPTY: return f_nop(pg);
    case OP_LITERAL: return c_rune(pg, n->cls.r, 2, (n->flags & F_FOLD) != 0);
    case OP_CLASS: return c_rune(pg, n->cls.r, n->cls.n, 0);
    case OP_ANYNOTNL: return f_single(pg, emit(pg, I_ANYNOTNL));
    case OP_ANY: return f_single(pg, emit(pg, I_ANY));
    case OP_BEGINLINE: return c_empty(pg, E_BEGINLINE);
    case OP_ENDLINE: return c_empty(pg, E_ENDLINE);
    case OP_BEGINTEXT: return c_empty(pg, E_BEGINTEXT);
    case OP_ENDTEXT: return c_empty(pg, E_ENDTEXT);
    case OP_WORDB: return c_empty(pg, E_WORDB);
    case OP_NOWORDB: return c_empty(pg, E_NOWORDB);
    case OP_CAPTURE: return compile_node(pg, n->sub[0]);
    case OP_STAR: return c_star(pg, compile_node(pg, n->sub[0]));
    case OP_PLUS: return c_plus(pg, compile_node(pg, n->sub[0]));
    case OP_QUEST: return c_quest(pg, compile_node(pg, n->sub[0]));
    case OP_CONCAT: {
      Frag f = compile_node(pg, n->sub[0]);
      for (int i = 1; i < n->nsub; i++) f = c_cat(pg, f, compile_node(pg, n->sub[i]));
      return f;
    }
    case OP_ALT: {
      Frag f = compile_node(pg, n->sub[n->nsub - 1]);
      for (int i = n->nsub - 2; i >= 0; i--) f = c_alt(pg, compile_node(pg, n->sub[i]), f);
      return f;
    }
    case OP_REPEAT: {
      /* x{n,m} -> x^n (x(x(...)?)?)?  ; x{n,} -> x^(n-1) x+ (n>=1) or x* */
      const Node* x = n->sub[0];
      int mn = n->min, mx = n->max;
      if (mx == -1) {
        if (mn == 0) return c_star(pg, compile_node(pg, x));
        Frag f = {0}; int have = 0;
        for (int i = 0; i < mn - 1; i++) {
          Frag g = compile_node(pg, x);
          f = have ? c_cat(pg, f, g) : g; have = 1;
        }
        Frag pl = c_plus(pg, compile_node(pg, x));
        return have ? c_cat(pg, f, pl) : pl;
      }
      if (mx == 0) return f_nop(pg);
      Frag f = {0}; int have = 0;
      for (int i = 0; i < mn; i++) {
        Frag g = compile_node(pg, x);
        f = have ? c_cat(pg, f, g) : g; have = 1;
      }
      if (mx > mn) {
        /* build nested optional suffix from the inside out */
        Frag suf = c_quest(pg, compile_node(pg, x));
        for (int i = mn + 1; i < mx; i++) {
          Frag g = compile_node(pg, x);
          suf = c_quest(pg, c_cat(pg, g, suf));
        }
        f = have ? c_cat(pg, f, suf) : suf; have = 1;
      }
      return f;
    }
  }
  return f_nop(pg);
}

int orc_compile(const char* pat, size_t n, orc_re** out, char* err, size_t errlen) {
  Parser p;
  memset(&p, 0, sizeof(p));
  Node* ast = parse((const unsigned char*)pat, n, &p);
  int status = ORC_OK;
  if (p.err) status = ORC_ESYNTAX;
  else if (p.unsupported) status = ORC_EUNSUPPORTED;
  if (err && errlen) snprintf(err, errlen, "%s", p.msg ? p.msg : "");
  orc_re* pg = (orc_re*)calloc(1, sizeof(orc_re));
  pg->status = status;
  if (status == ORC_OK) {
    Frag f = compile_node(pg, ast);
    int m = emit(pg, I_MATCH);
    patch(pg, &f, m);
    free(f.holes);
    pg->start = f.start;
  }
  if (ast) node_free(ast);
  for (int i = 0; i < p.nst; i++) if (p.st[i] != ast) node_free(p.st[i]);
  free(p.st);
  *out = pg;
  return status;
}

void orc_free(orc_re* re) {
  if (!re) return;
  for (int i = 0; i < re->n; i++) free(re->in[i].r);
  free(re->in);
  free(re);
}

/* ---- Pike-style NFA simulation (boolean, unanchored) ---------------------- */
static int is_word(int r) {
  return r >= 0 && r < 0x80 && (isalnum_ascii(r) || r == '_');
}
/* EmptyOpContext(r1, r2) (syntax/prog.go); -1 = text boundary */
static int empty_ctx(int r1, int r2) {
  int op = E_NOWORDB, b = 0;
  if (is_word(r1)) b = 1;
  else if (r1 == '\n') op |= E_BEGINLINE;
  else if (r1 < 0) op |= E_BEGINTEXT | E_BEGINLINE;
  if (is_word(r2)) b ^= 1;
  else if (r2 == '\n') op |= E_ENDLINE;
  else if (r2 < 0) op |= E_ENDTEXT | E_ENDLINE;
  if (b) op ^= (E_WORDB | E_NOWORDB);
  return op;
}

typedef struct { int* dense; int* sparse; int n; } SSet;
static int ss_has(SSet* s, int x) { unsigned i = (unsigned)s->sparse[x]; return i < (unsigned)s->n && s->dense[i] == x; }
static void ss_add(SSet* s, int x) { s->sparse[x] = s->n; s->dense[s->n++] = x; }

static int rune_match(const Inst* in, int r) {
  switch (in->op) {
    case I_ANY: return 1;
    case I_ANYNOTNL: return r != '\n';
    case I_RUNE: return cls_has(in->r, in->nr, r);
    case I_RUNEFOLD: {
      int o[4];
      int k = fold_orbit(in->r[0], o);
      for (int i = 0; i < k; i++) if (o[i] == r) return 1;
      return 0;
    }
  }
  return 0;
}

/* add pc and its epsilon closure (under ctx) to q; returns 1 if Match reached */
static int closure(const orc_re* pg, SSet* q, int pc, int ctx, int* stack) {
  int sp = 0;
  stack[sp++] = pc;
  while (sp) {
    int x = stack[--sp];
    if (x < 0 || ss_has(q, x)) continue;
    ss_add(q, x);
    const Inst* in = &pg->in[x];
    switch (in->op) {
      case I_MATCH: return 1;
      case I_NOP: stack[sp++] = in->out; break;
      case I_ALT: stack[sp++] = in->out1; stack[sp++] = in->out; break;
      case I_EMPTY: if ((in->arg & ~ctx) == 0) stack[sp++] = in->out; break;
      default: break;
    }
  }
  return 0;
}

int orc_match(const orc_re* pg, const unsigned char* s, size_t n) {
  if (pg->status != ORC_OK) return 0;
  int N = pg->n;
  int* mem = (int*)malloc(sizeof(int) * ((size_t)N * 6 + 16));
  SSet cur = {mem, mem + N, 0}, nxt = {mem + 2 * N, mem + 3 * N, 0};
  int* stack = mem + 4 * N; /* closure pushes <= 2 per added state + 1 */
  /* raw = states reached by the previous rune step, before closure */
  int* raw = (int*)malloc(sizeof(int) * (size_t)N + 4);
  int nraw = 0;
  int prev = -1;
  size_t pos = 0;
  int matched = 0;
  for (;;) {
    int sz = 0;
    int r = pos < n ? dec_rune(s + pos, n - pos, &sz) : -1;
    int ctx = empty_ctx(prev, r);
    cur.n = 0;
    for (int i = 0; i < nraw && !matched; i++) matched = closure(pg, &cur, raw[i], ctx, stack);
    if (!matched) matched = closure(pg, &cur, pg->start, ctx, stack);
    if (matched || r < 0) break;
    nraw = 0;
    nxt.n = 0;
    for (int i = 0; i < cur.n; i++) {
      const Inst* in = &pg->in[cur.dense[i]];
      if (in->op >= I_RUNE && rune_match(in, r) && in->out >= 0 && !ss_has(&nxt, in->out)) {
        ss_add(&nxt, in->out);
        raw[nraw++] = in->out;
      }
    }
    prev = r;
    pos += (size_t)sz;
  }
  free(raw);
  free(mem);
  return matched;
}

/* ---- memoized Pike VM: a lazy DFA over the same program -------------------
 * For whole-split checks (orc_map_mt). A state is what orc_match carries from
 * one rune to the next: the set of pcs reached by the last rune step (`raw`,
 * kept sorted) and the class of the previous rune -- the only part of it that
 * empty_ctx() reads: none yet (-1), an ASCII word character, '\n', or other.
 * The transition of a state on a rune, and its verdict at the end of the line,
 * are computed by exactly the closure/step code of orc_match and cached for
 * ASCII runes; other runes are computed every time. The cache is flushed when
 * it grows past its bounds. */
enum { PC_BOT = 0, PC_WORD = 1, PC_NL = 2, PC_OTHER = 3 };
static const int pc_rep[4] = {-1, 'a', '\n', ' '};
static int prev_class(int r) { return r < 0 ? PC_BOT : is_word(r) ? PC_WORD : r == '\n' ? PC_NL : PC_OTHER; }

#define LZ_MATCHED (-2)
#define LZ_UNKNOWN (-1)
#define LZ_MAX_STATES 8192
#define LZ_MAX_ARENA (1 << 22)

typedef struct {
  int set_off, nset, prev;
  int endm; /* -1 unknown, else the end-of-line verdict */
  int next[128];
} LzState;

struct orc_matcher {
  const orc_re* pg;
  LzState* st; int nst;
  int* arena; int narena;
  int* hash; int hcap; /* open addressing: state index + 1, 0 = empty */
  SSet cur, nxt;
  int* mem; int* stack; int* raw;
  int start_state;
};

static uint64_t lz_hash(const int* s, int n, int prev) {
  uint64_t h = 1469598103934665603ull ^ (uint64_t)prev;
  for (int i = 0; i < n; i++) { h ^= (uint64_t)(unsigned)s[i]; h *= 1099511628211ull; }
  return h ^ (h >> 29);
}

static int cmp_int(const void* a, const void* b) { int x = *(const int*)a, y = *(const int*)b; return (x > y) - (x < y); }

static void lz_reset(orc_matcher* m) {
  m->nst = 0;
  m->narena = 0;
  memset(m->hash, 0, sizeof(int) * (size_t)m->hcap);
}

/* intern (sorted set, prev); returns the state index */
static int lz_intern(orc_matcher* m, const int* s, int n, int prev) {
  uint64_t h = lz_hash(s, n, prev);
  for (uint64_t i = h & (uint64_t)(m->hcap - 1);; i = (i + 1) & (uint64_t)(m->hcap - 1)) {
    int e = m->hash[i];
    if (!e) {
      LzState* x = &m->st[m->nst];
      x->set_off = m->narena; x->nset = n; x->prev = prev; x->endm = LZ_UNKNOWN;
      for (int k = 0; k < 128; k++) x->next[k] = LZ_UNKNOWN;
      memcpy(m->arena + m->narena, s, sizeof(int) * (size_t)n);
      m->narena += n;
      m->hash[i] = ++m->nst;
      return m->nst - 1;
    }
    const LzState* x = &m->st[e - 1];
    if (x->prev == prev && x->nset == n && !memcmp(m->arena + x->set_off, s, sizeof(int) * (size_t)n)) return e - 1;
  }
}

/* closure of the state's set and of the start under ctx(prev, r): 1 = Match */
static int lz_closure(orc_matcher* m, const int* set, int n, int prev, int r) {
  const int ctx = empty_ctx(pc_rep[prev], r);
  m->cur.n = 0;
  int matched = 0;
  for (int i = 0; i < n && !matched; i++) matched = closure(m->pg, &m->cur, set[i], ctx, m->stack);
  if (!matched) matched = closure(m->pg, &m->cur, m->pg->start, ctx, m->stack);
  return matched;
}

/* the transition of state `si` on rune r >= 0 (LZ_MATCHED or a state index);
 * *sip is updated if the cache had to be flushed */
static int lz_step(orc_matcher* m, int* sip, int r) {
  LzState* x = &m->st[*sip];
  int n = x->nset, prev = x->prev;
  /* the set may move if the cache is flushed below: work on a copy */
  memcpy(m->raw, m->arena + x->set_off, sizeof(int) * (size_t)n);
  if (lz_closure(m, m->raw, n, prev, r)) return LZ_MATCHED;
  int nraw = 0;
  m->nxt.n = 0;
  for (int i = 0; i < m->cur.n; i++) {
    const Inst* in = &m->pg->in[m->cur.dense[i]];
    if (in->op >= I_RUNE && rune_match(in, r) && in->out >= 0 && !ss_has(&m->nxt, in->out)) {
      ss_add(&m->nxt, in->out);
      m->raw[nraw++] = in->out;
    }
  }
  qsort(m->raw, (size_t)nraw, sizeof(int), cmp_int);
  if (m->nst + 2 > LZ_MAX_STATES || m->narena + nraw + m->pg->n > LZ_MAX_ARENA) {
    /* flush: re-intern the current state first so the caller's index stays valid */
    int* keep = (int*)malloc(sizeof(int) * ((size_t)n + 1));
    memcpy(keep, m->arena + m->st[*sip].set_off, sizeof(int) * (size_t)n);
    lz_reset(m);
    m->start_state = lz_intern(m, NULL, 0, PC_BOT);
    *sip = lz_intern(m, keep, n, prev);
    free(keep);
  }
  return lz_intern(m, m->raw, nraw, prev_class(r));
}

orc_matcher* orc_matcher_new(const orc_re* pg) {
  orc_matcher* m = (orc_matcher*)calloc(1, sizeof(orc_matcher));
  m->pg = pg;
  if (pg->status != ORC_OK) return m;
  int N = pg->n;
  m->st = (LzState*)malloc(sizeof(LzState) * LZ_MAX_STATES);
  m->arena = (int*)malloc(sizeof(int) * (size_t)LZ_MAX_ARENA);
  m->hcap = 4 * LZ_MAX_STATES;
  m->hash = (int*)calloc((size_t)m->hcap, sizeof(int));
  m->mem = (int*)malloc(sizeof(int) * ((size_t)N * 6 + 16));
  m->cur = (SSet){m->mem, m->mem + N, 0};
  m->nxt = (SSet){m->mem + 2 * N, m->mem + 3 * N, 0};
  m->stack = m->mem + 4 * N;
  m->raw = (int*)malloc(sizeof(int) * ((size_t)N + 4));
  m->start_state = lz_intern(m, NULL, 0, PC_BOT);
  return m;
}

int orc_matcher_match(orc_matcher* m, const unsigned char* s, size_t n) {
  if (m->pg->status != ORC_OK) return 0;
  int si = m->start_state;
  size_t pos = 0;
  while (pos < n) {
    int r, sz;
    if (s[pos] < 0x80) { r = s[pos]; sz = 1; } else r = dec_rune(s + pos, n - pos, &sz);
    int nx = r < 128 ? m->st[si].next[r] : LZ_UNKNOWN;
    if (nx == LZ_UNKNOWN) {
      int cur = si;
      nx = lz_step(m, &cur, r);
      if (nx != LZ_MATCHED && r < 128) m->st[cur].next[r] = nx;
      else if (nx == LZ_MATCHED && r < 128) m->st[cur].next[r] = LZ_MATCHED;
    }
    if (nx == LZ_MATCHED) return 1;
    si = nx;
    pos += (size_t)sz;
  }
  LzState* x = &m->st[si];
  if (x->endm == LZ_UNKNOWN) {
    memcpy(m->raw, m->arena + x->set_off, sizeof(int) * (size_t)x->nset);
    x->endm = lz_closure(m, m->raw, x->nset, x->prev, -1);
  }
  return x->endm;
}

void orc_matcher_free(orc_matcher* m) {
  if (!m) return;
  free(m->st); free(m->arena); free(m->hash); free(m->mem); free(m->raw);
  free(m);
}
