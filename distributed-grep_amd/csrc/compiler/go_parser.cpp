// go_parser.cpp — Go regexp/syntax front end of the dgrep pattern compiler.
//
// application/grep.go:21 calls regexp.Match(pattern, line), i.e.
// regexp.Compile(pattern) = syntax.Parse(pattern, syntax.Perl) on every line.
// This is a recursive-descent parser for that dialect [Go stdlib: RE2 syntax,
// Perl flags ClassNL|OneLine|PerlX|UnicodeGroups, Go 1.18 per go.mod:3]. It
// accepts and rejects exactly the patterns Go does (a rejected pattern makes
// every line a non-match, because grep.go:21 discards the error), including
// the dialect's corner cases:
//   * `{` that does not start a well-formed {n}, {n,}, {n,m} is a literal;
//     counts above 1000 and nested counts whose product exceeds 1000 are errors;
//   * stacked repetition operators (`a**`, `a{2}*`) are errors, but a
//     repetition may follow a flag group: `a(?i)*` repeats `a`;
//   * `(?i)` etc. last until the end of the enclosing group, across `|`;
//   * escapes: \a\f\t\n\r\v, octal \0.. / \1-\7 followed by an octal digit,
//     \xHH, \x{H..}, \Q..\E, \A \z \b \B, \pN \p{Name} \PN \p{^Name},
//     \d\D\s\S\w\W; any other escaped ASCII letter/digit (and \C) is an error;
//     escaped ASCII punctuation is literal;
//   * classes: `]` first is literal, `-` anywhere (PerlX), [:name:] and
//     [:^name:], ranges with hi < lo are errors; `[]` and `[\b]` are errors;
//   * invalid UTF-8 anywhere in the pattern is an error.
// Captures and greediness do not change a boolean match and are not kept.
#include <algorithm>
#include <cstring>
#include <string>

#include "regex_ast.hpp"

namespace dgrep {

namespace {
#include "unicode_tables.inc"

constexpr int32_t kMinFold = 0x41;    // [Go stdlib] regexp/syntax minFold
constexpr int32_t kMaxFold = 0x1E943; // [Go stdlib] regexp/syntax maxFold (Unicode 13)

enum : int { kFoldCase = 1, kDotNL = 2 };

// Go utf8.DecodeRune: (RuneError, 1) for any invalid or truncated sequence,
// (RuneError, 0) for empty input.
int32_t decode_rune(const uint8_t* s, size_t n, int* size) {
  if (n == 0) { *size = 0; return kRuneError; }
  uint32_t c = s[0];
  if (c < 0x80) { *size = 1; return int32_t(c); }
  int need;
  uint32_t lo = 0x80, hi = 0xBF, r;
  if (c >= 0xC2 && c <= 0xDF) { need = 2; r = c & 0x1F; }
  else if (c >= 0xE0 && c <= 0xEF) { need = 3; r = c & 0x0F; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
  else if (c >= 0xF0 && c <= 0xF4) { need = 4; r = c & 0x07; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
  else { *size = 1; return kRuneError; }
  if (n < size_t(need) || s[1] < lo || s[1] > hi) { *size = 1; return kRuneError; }
  r = (r << 6) | (s[1] & 0x3F);
  for (int i = 2; i < need; ++i) {
    if (s[i] < 0x80 || s[i] > 0xBF) { *size = 1; return kRuneError; }
    r = (r << 6) | (s[i] & 0x3F);
  }
  *size = need;
  return int32_t(r);
}

bool in_table(const unsigned int* r, int nranges, int32_t x) {
  int lo = 0, hi = nranges;
  while (lo < hi) {
    int m = (lo + hi) / 2;
    if (x < int32_t(r[2 * m])) hi = m;
    else if (x > int32_t(r[2 * m + 1])) lo = m + 1;
    else return true;
  }
  return false;
}

bool ascii_alnum(int32_t c) { return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }

// [Go stdlib] unicode.SimpleFold orbit of r (every rune equivalent to r under
// simple case folding, r included): dg_fold lists, sorted by rune, the next
// member of each orbit of two or more (tools/gen_unicode_tables.py, Unicode
// 13.0 as in Go 1.18); a rune not listed folds only to itself.
int fold_next(int32_t r) {
  int lo = 0, hi = dg_nfold;
  while (lo < hi) {
    const int m = (lo + hi) / 2;
    const int32_t x = int32_t(dg_fold[2 * m]);
    if (x == r) return int32_t(dg_fold[2 * m + 1]);
    if (x < r) lo = m + 1;
    else hi = m;
  }
  return -1;
}
void fold_orbit(int32_t r, RuneSet* out) {
  out->add(r, r);
  for (int32_t x = fold_next(r); x >= 0 && x != r; x = fold_next(x)) out->add(x, x);
}

struct Group {
  const char* name;
  int sign;
  std::initializer_list<int32_t> r;  // pairs
};

const Group kPerlGroups[] = {
    {"d", +1, {'0', '9'}}, {"D", -1, {'0', '9'}},
    {"s", +1, {'\t', '\n', '\f', '\r', ' ', ' '}}, {"S", -1, {'\t', '\n', '\f', '\r', ' ', ' '}},
    {"w", +1, {'0', '9', 'A', 'Z', '_', '_', 'a', 'z'}}, {"W", -1, {'0', '9', 'A', 'Z', '_', '_', 'a', 'z'}},
};

struct Posix {
  const char* name;
  std::initializer_list<int32_t> r;
};
const Posix kPosix[] = {
    {"alnum", {'0', '9', 'A', 'Z', 'a', 'z'}}, {"alpha", {'A', 'Z', 'a', 'z'}}, {"ascii", {0, 0x7F}},
    {"blank", {'\t', '\t', ' ', ' '}},          {"cntrl", {0, 0x1F, 0x7F, 0x7F}}, {"digit", {'0', '9'}},
    {"graph", {'!', '~'}},                     {"lower", {'a', 'z'}},           {"print", {' ', '~'}},
    {"punct", {'!', '/', ':', '@', '[', '`', '{', '~'}}, {"space", {'\t', '\r', ' ', ' '}},
    {"upper", {'A', 'Z'}},                     {"word", {'0', '9', 'A', 'Z', '_', '_', 'a', 'z'}},
    {"xdigit", {'0', '9', 'A', 'F', 'a', 'f'}},
};

class GoParser {
 public:
  GoParser(const uint8_t* s, size_t n) : p_(s), end_(s + n) {}

  ParseResult run() {
    ParseResult out;
    ReP re = alternation();
    if (!syntax_error_ && p_ < end_) syntax("unexpected )");  // alternation stops only at ')' or end
    if (syntax_error_) {
      out.status = ParseResult::GoSyntaxError;
      out.message = msg_;
    } else if (unsupported_) {
      out.status = ParseResult::Unsupported;
      out.message = msg_;
    } else {
      out.re = std::move(re);
    }
    return out;
  }

 private:
  const uint8_t* p_;
  const uint8_t* end_;
  int flags_ = 0;
  int depth_ = 0;
  bool syntax_error_ = false, unsupported_ = false;
  std::string msg_;

  void syntax(const char* m) {
    if (!syntax_error_) { syntax_error_ = true; msg_ = m; }
  }
  void unsupported(const char* m) {
    if (!unsupported_) { unsupported_ = true; if (!syntax_error_) msg_ = m; }
  }
  bool failed() const { return syntax_error_; }
  size_t left() const { return size_t(end_ - p_); }

  bool read_rune(int32_t* r) {  // Go nextRune
    int sz;
    *r = decode_rune(p_, left(), &sz);
    if (*r == kRuneError && sz == 1) { syntax("invalid UTF-8"); return false; }
    p_ += sz;
    return true;
  }

  static ReP make(Re::Kind k) { return ReP(new Re(k)); }
  static ReP make_set(RuneSet s) {
    ReP r = make(Re::Set);
    s.normalize();
    r->set = std::move(s);
    return r;
  }
  static ReP make_assert(AssertKind k) {
    ReP r = make(Re::Assert);
    r->assert_kind = k;
    return r;
  }

  ReP literal(int32_t c) {
    RuneSet s;
    if (flags_ & kFoldCase) {
      fold_orbit(c, &s);
    } else {
      s.add(c, c);
    }
    return make_set(std::move(s));
  }

  // [Go stdlib] appendFoldedRange, with its [minFold, maxFold] shortcuts.
  void add_folded_range(RuneSet* s, int32_t lo, int32_t hi) {
    if ((lo <= kMinFold && hi >= kMaxFold) || hi < kMinFold || lo > kMaxFold) { s->add(lo, hi); return; }
    if (lo < kMinFold) { s->add(lo, kMinFold - 1); lo = kMinFold; }
    if (hi > kMaxFold) { s->add(kMaxFold + 1, hi); hi = kMaxFold; }
    for (int32_t x = lo; x <= hi; ++x) fold_orbit(x, s);
  }

  void add_range(RuneSet* s, int32_t lo, int32_t hi) {
    if (flags_ & kFoldCase) add_folded_range(s, lo, hi);
    else s->add(lo, hi);
  }

  // [Go stdlib] appendGroup: fold the (ASCII) group under (?i), then add or negate it.
  void add_group(RuneSet* s, int sign, std::initializer_list<int32_t> r) {
    RuneSet g;
    for (auto it = r.begin(); it != r.end(); it += 2) add_range(&g, it[0], it[1]);
    g.normalize();
    if (sign < 0) g.negate();
    s->add(g);
  }

  // \d \D \s \S \w \W at p_; returns true and consumes on success.
  bool perl_class(RuneSet* s) {
    if (left() < 2 || p_[0] != '\\') return false;
    for (const Group& g : kPerlGroups) {
      if (p_[1] == uint8_t(g.name[0])) {
        add_group(s, g.sign, g.r);
        p_ += 2;
        return true;
      }
    }
    return false;
  }

  // [:name:] / [:^name:] at p_ (inside a class). 1 consumed, 0 not a named class, -1 error.
  int posix_class(RuneSet* s) {
    if (left() < 2 || p_[0] != '[' || p_[1] != ':') return 0;
    const uint8_t* close = nullptr;
    for (const uint8_t* x = p_ + 2; x + 1 < end_; ++x)
      if (x[0] == ':' && x[1] == ']') { close = x; break; }
    if (!close) return 0;
    std::string name(reinterpret_cast<const char*>(p_ + 2), size_t(close - (p_ + 2)));
    int sign = +1;
    if (!name.empty() && name[0] == '^') { sign = -1; name.erase(0, 1); }
    for (const Posix& g : kPosix) {
      if (name == g.name) {
        add_group(s, sign, g.r);
        p_ = close + 2;
        return 1;
      }
    }
    syntax("invalid character class range");
    return -1;
  }

  // \pN, \p{Name}, \PN, \p{^Name} at p_. 1 consumed, 0 not a unicode class, -1 error.
  int unicode_class(RuneSet* s) {
    if (left() < 2 || p_[0] != '\\' || (p_[1] != 'p' && p_[1] != 'P')) return 0;
    int sign = p_[1] == 'P' ? -1 : +1;
    const uint8_t* t = p_ + 2;
    int sz;
    int32_t c = decode_rune(t, size_t(end_ - t), &sz);
    if (c == kRuneError && sz == 1) { syntax("invalid UTF-8"); return -1; }
    std::string name;
    const uint8_t* rest;
    if (c != '{') {
      name.assign(reinterpret_cast<const char*>(t), size_t(sz));
      rest = t + sz;
    } else {
      const uint8_t* close = static_cast<const uint8_t*>(memchr(p_, '}', left()));
      if (!close) { syntax("invalid character class range"); return -1; }
      for (const uint8_t* y = p_ + 3; y < close;) {
        int k;
        int32_t r = decode_rune(y, size_t(close - y), &k);
        if (r == kRuneError && k == 1) { syntax("invalid UTF-8"); return -1; }
        y += k;
      }
      name.assign(reinterpret_cast<const char*>(p_ + 3), size_t(close - (p_ + 3)));
      rest = close + 1;
    }
    if (!name.empty() && name[0] == '^') { sign = -sign; name.erase(0, 1); }
    RuneSet tab;
    bool found = false, folds = false;
    if (name == "Any") {
      tab.add(0, kMaxRune);
      found = true;
    } else {
      for (int i = 0; i < dg_ncategories; ++i) {
        if (name == dg_categories[i].name) {
          for (int j = 0; j < dg_categories[i].n; ++j)
            tab.add(int32_t(dg_categories[i].r[2 * j]), int32_t(dg_categories[i].r[2 * j + 1]));
          folds = dg_categories[i].fold != 0;
          found = true;
          break;
        }
      }
    }
    if (!found) {
      // [Go stdlib] regexp/syntax unicodeTable: unicode.Categories first, then
      // unicode.Scripts (with unicode.FoldScript as the fold table)
      for (int i = 0; i < dg_nscripts; ++i) {
        if (name == dg_scripts[i].name) {
          for (int j = 0; j < dg_scripts[i].n; ++j)
            tab.add(int32_t(dg_scripts[i].r[2 * j]), int32_t(dg_scripts[i].r[2 * j + 1]));
          folds = dg_scripts[i].fold != 0;
          found = true;
          break;
        }
      }
    }
    if (!found) { syntax("invalid character class range"); return -1; }
    if ((flags_ & kFoldCase) && folds) {
      // [Go stdlib] unicode.FoldCategory / FoldScript: the runes outside the
      // table that simple-fold to runes inside it -- the table's orbit closure
      RuneSet closed;
      tab.normalize();
      for (const auto& rg : tab.ranges())
        for (int32_t x = std::max(rg.first, kMinFold); x <= std::min(rg.second, kMaxFold); ++x) fold_orbit(x, &closed);
      tab.add(closed);
    }
    tab.normalize();
    if (sign < 0) tab.negate();
    s->add(tab);
    p_ = rest;
    return 1;
  }

  static int unhex(int32_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }

  // Single-character escape at p_ ('\\'). [Go stdlib] parseEscape.
  bool escape(int32_t* out) {
    ++p_;
    if (p_ >= end_) { syntax("trailing backslash at end of expression"); return false; }
    int32_t c;
    if (!read_rune(&c)) return false;
    if (c >= '1' && c <= '7' && !(p_ < end_ && *p_ >= '0' && *p_ <= '7')) {
      syntax("invalid escape sequence (backreference)");
      return false;
    }
    if (c >= '0' && c <= '7') {
      int32_t r = c - '0';
      for (int i = 1; i < 3 && p_ < end_ && *p_ >= '0' && *p_ <= '7'; ++i) r = r * 8 + (*p_++ - '0');
      *out = r;
      return true;
    }
    switch (c) {
      case 'x': {
        if (p_ >= end_) break;
        int32_t d;
        if (!read_rune(&d)) return false;
        if (d == '{') {
          int32_t r = 0;
          int nhex = 0;
          for (;;) {
            if (p_ >= end_) { syntax("invalid escape sequence"); return false; }
            if (!read_rune(&d)) return false;
            if (d == '}') break;
            int v = unhex(d);
            if (v < 0) { syntax("invalid escape sequence"); return false; }
            r = r * 16 + v;
            if (r > kMaxRune) { syntax("invalid escape sequence"); return false; }
            ++nhex;
          }
          if (nhex == 0) { syntax("invalid escape sequence"); return false; }
          *out = r;
          return true;
        }
        int x = unhex(d);
        int sz;
        int32_t e = decode_rune(p_, left(), &sz);
        if (e == kRuneError && sz == 1) { syntax("invalid UTF-8"); return false; }
        p_ += sz;
        int y = unhex(e);
        if (x < 0 || y < 0) break;
        *out = x * 16 + y;
        return true;
      }
      case 'a': *out = 7; return true;
      case 'f': *out = 12; return true;
      case 'n': *out = 10; return true;
      case 'r': *out = 13; return true;
      case 't': *out = 9; return true;
      case 'v': *out = 11; return true;
      default:
        if (c < 0x80 && !ascii_alnum(c)) { *out = c; return true; }
        break;
    }
    syntax("invalid escape sequence");
    return false;
  }

  bool class_char(int32_t* out) {
    if (p_ >= end_) { syntax("missing closing ]"); return false; }
    if (*p_ == '\\') return escape(out);
    return read_rune(out);
  }

  // [...] at p_. [Go stdlib] parseClass with ClassNL|PerlX.
  ReP char_class() {
    ++p_;
    RuneSet s;
    int sign = +1;
    if (p_ < end_ && *p_ == '^') { sign = -1; ++p_; }
    bool first = true;
    while (p_ >= end_ || *p_ != ']' || first) {
      first = false;
      if (left() > 2 && p_[0] == '[' && p_[1] == ':') {
        int k = posix_class(&s);
        if (k < 0) return nullptr;
        if (k > 0) continue;
      }
      int k = unicode_class(&s);
      if (k < 0) return nullptr;
      if (k > 0) continue;
      if (perl_class(&s)) continue;
      int32_t lo, hi;
      if (!class_char(&lo)) return nullptr;
      hi = lo;
      if (left() >= 2 && p_[0] == '-' && p_[1] != ']') {
        ++p_;
        if (!class_char(&hi)) return nullptr;
        if (hi < lo) { syntax("invalid character class range"); return nullptr; }
      }
      add_range(&s, lo, hi);
    }
    ++p_;  // ]
    s.normalize();
    if (sign < 0) s.negate();
    return make_set(std::move(s));
  }

  // {n}, {n,}, {n,m} at p_; false if not well formed (then `{` is a literal).
  static bool parse_int(const uint8_t*& t, const uint8_t* end, int* n) {
    if (t >= end || *t < '0' || *t > '9') return false;
    if (end - t >= 2 && t[0] == '0' && t[1] >= '0' && t[1] <= '9') return false;  // no leading zeros
    const uint8_t* d = t;
    while (t < end && *t >= '0' && *t <= '9') ++t;
    long v = 0;
    for (const uint8_t* x = d; x < t; ++x) {
      if (v >= 100000000) { v = -1; break; }
      v = v * 10 + (*x - '0');
    }
    *n = int(v);
    return true;
  }
  bool braces(int* lo, int* hi, const uint8_t** after) const {
    const uint8_t* t = p_ + 1;
    if (!parse_int(t, end_, lo)) return false;
    if (t >= end_) return false;
    if (*t != ',') {
      *hi = *lo;
    } else {
      ++t;
      if (t >= end_) return false;
      if (*t == '}') *hi = -1;
      else if (!parse_int(t, end_, hi)) return false;
      else if (*hi < 0) *lo = -1;
    }
    if (t >= end_ || *t != '}') return false;
    *after = t + 1;
    return true;
  }

  // [Go stdlib] repeatIsValid: nested counted repetitions may not multiply
  // beyond 1000 copies of the innermost expression.
  static bool repeat_valid(const Re& re, int n) {
    if (re.kind == Re::Repeat) {
      int m = re.max;
      if (m == 0) return true;
      if (m < 0) m = re.min;
      if (m > n) return false;
      if (m > 0) n /= m;
    }
    for (const ReP& s : re.sub)
      if (!repeat_valid(*s, n)) return false;
    return true;
  }

  // Body of a group after its opening token; restores the flags in force
  // before the group (Go: parseRightParen restores the '(' flags).
  ReP group_body(int saved_flags) {
    if (++depth_ > 1000) unsupported("nesting deeper than 1000 groups");
    ReP r = alternation();
    --depth_;
    if (failed()) return nullptr;
    if (p_ >= end_) { syntax("missing closing )"); return nullptr; }
    ++p_;  // )
    flags_ = saved_flags;
    return r;
  }

  // "(?" at p_: named capture, flag group, or flag directive. Returns true
  // on success; *item is null for a bare directive like (?i).
  bool perl_group(ReP* item) {
    if (left() > 4 && p_[2] == 'P' && p_[3] == '<') {
      const uint8_t* close = static_cast<const uint8_t*>(memchr(p_, '>', left()));
      if (!close) { syntax("invalid named capture"); return false; }
      const uint8_t* name = p_ + 4;
      for (const uint8_t* y = name; y < close;) {
        int k;
        int32_t r = decode_rune(y, size_t(close - y), &k);
        if (r == kRuneError && k == 1) { syntax("invalid UTF-8"); return false; }
        y += k;
      }
      if (close == name) { syntax("invalid named capture"); return false; }
      for (const uint8_t* y = name; y < close; ++y)
        if (*y != '_' && !ascii_alnum(*y)) { syntax("invalid named capture"); return false; }
      p_ = close + 1;
      *item = group_body(flags_);
      return !failed();
    }
    p_ += 2;
    int flags = flags_;
    bool negated = false, saw = false;
    while (p_ < end_) {
      int32_t c;
      if (!read_rune(&c)) return false;
      switch (c) {
        case 'i': negated ? flags &= ~kFoldCase : flags |= kFoldCase; saw = true; break;
        case 'm': saw = true; break;  // ^/$ at line ends == text ends: lines hold no '\n'
        case 's': negated ? flags &= ~kDotNL : flags |= kDotNL; saw = true; break;
        case 'U': saw = true; break;  // greediness does not change a boolean match
        case '-':
          if (negated) { syntax("invalid or unsupported Perl syntax"); return false; }
          negated = true;
          saw = false;
          break;
        case ':':
        case ')': {
          if (negated && !saw) { syntax("invalid or unsupported Perl syntax"); return false; }
          if (c == ')') {
            flags_ = flags;
            *item = nullptr;
            return true;
          }
          int saved = flags_;
          flags_ = flags;
          *item = group_body(saved);
          return !failed();
        }
        default:
          syntax("invalid or unsupported Perl syntax");
          return false;
      }
    }
    syntax("invalid or unsupported Perl syntax");
    return false;
  }

  ReP alternation() {
    std::vector<ReP> branches;
    branches.push_back(concatenation());
    while (!failed() && p_ < end_ && *p_ == '|') {
      ++p_;
      branches.push_back(concatenation());
    }
    if (failed()) return nullptr;
    if (branches.size() == 1) return std::move(branches[0]);
    ReP a = make(Re::Alt);
    a->sub = std::move(branches);
    return a;
  }

  void apply_repeat(std::vector<ReP>& items, Re::Kind k, int lo, int hi, bool last_repeat) {
    if (p_ < end_ && *p_ == '?') ++p_;  // non-greedy: same boolean language
    if (last_repeat) { syntax("invalid nested repetition operator"); return; }
    if (items.empty()) { syntax("missing argument to repetition operator"); return; }
    ReP r = make(k);
    r->min = lo;
    r->max = hi;
    r->sub.push_back(std::move(items.back()));
    if (k == Re::Repeat && (lo >= 2 || hi >= 2) && !repeat_valid(*r, 1000)) {
      syntax("invalid repeat count");
      return;
    }
    items.back() = std::move(r);
  }

  ReP concatenation() {
    std::vector<ReP> items;
    bool last_repeat = false;
    while (!failed() && p_ < end_ && *p_ != '|' && *p_ != ')') {
      bool repeat = false;
      switch (*p_) {
        case '(':
          if (left() >= 2 && p_[1] == '?') {
            ReP g;
            if (perl_group(&g) && g) items.push_back(std::move(g));
          } else {
            ++p_;
            ReP g = group_body(flags_);
            if (g) items.push_back(std::move(g));
          }
          break;
        case '^': ++p_; items.push_back(make_assert(AssertKind::BeginText)); break;
        case '$': ++p_; items.push_back(make_assert(AssertKind::EndText)); break;
        case '.': {
          ++p_;
          RuneSet s;
          if (flags_ & kDotNL) s.add(0, kMaxRune);
          else { s.add(0, '\n' - 1); s.add('\n' + 1, kMaxRune); }
          items.push_back(make_set(std::move(s)));
          break;
        }
        case '[': {
          ReP c = char_class();
          if (c) items.push_back(std::move(c));
          break;
        }
        case '*': case '+': case '?': {
          Re::Kind k = *p_ == '*' ? Re::Star : (*p_ == '+' ? Re::Plus : Re::Quest);
          ++p_;
          apply_repeat(items, k, 0, 0, last_repeat);
          repeat = true;
          break;
        }
        case '{': {
          int lo = 0, hi = 0;
          const uint8_t* after;
          if (!braces(&lo, &hi, &after)) {
            ++p_;
            items.push_back(literal('{'));
            break;
          }
          if (lo < 0 || lo > 1000 || hi > 1000 || (hi >= 0 && lo > hi)) { syntax("invalid repeat count"); break; }
          p_ = after;
          apply_repeat(items, Re::Repeat, lo, hi, last_repeat);
          repeat = true;
          break;
        }
        case '\\': {
          if (left() >= 2) {
            bool done = true;
            switch (p_[1]) {
              case 'A': p_ += 2; items.push_back(make_assert(AssertKind::BeginText)); break;
              case 'z': p_ += 2; items.push_back(make_assert(AssertKind::EndText)); break;
              case 'b': p_ += 2; items.push_back(make_assert(AssertKind::WordBoundary)); break;
              case 'B': p_ += 2; items.push_back(make_assert(AssertKind::NotWordBoundary)); break;
              case 'C': syntax("invalid escape sequence \\C"); break;
              case 'Q': {
                const uint8_t* lit = p_ + 2;
                const uint8_t* lend = end_;
                const uint8_t* next = end_;
                for (const uint8_t* x = lit; x + 1 < end_; ++x)
                  if (x[0] == '\\' && x[1] == 'E') { lend = x; next = x + 2; break; }
                p_ = lit;
                while (!failed() && p_ < lend) {
                  int sz;
                  int32_t c = decode_rune(p_, size_t(lend - p_), &sz);
                  if (c == kRuneError && sz == 1) { syntax("invalid UTF-8"); break; }
                  p_ += sz;
                  items.push_back(literal(c));
                }
                if (!failed()) p_ = next;
                break;
              }
              default: done = false;
            }
            if (done) break;
          }
          RuneSet s;
          int k = unicode_class(&s);
          if (k < 0) break;
          if (k > 0 || perl_class(&s)) {
            s.normalize();
            items.push_back(make_set(std::move(s)));
            break;
          }
          int32_t c;
          if (escape(&c)) items.push_back(literal(c));
          break;
        }
        default: {
          int32_t c;
          if (read_rune(&c)) items.push_back(literal(c));
          break;
        }
      }
      last_repeat = repeat;
    }
    if (failed()) return nullptr;
    if (items.empty()) return make(Re::Empty);
    if (items.size() == 1) return std::move(items[0]);
    ReP c = make(Re::Concat);
    c->sub = std::move(items);
    return c;
  }
};

}  // namespace

void RuneSet::normalize() {
  if (r_.size() < 2) return;
  std::sort(r_.begin(), r_.end());
  size_t w = 0;
  for (size_t i = 1; i < r_.size(); ++i) {
    if (r_[i].first <= r_[w].second + 1) {
      if (r_[i].second > r_[w].second) r_[w].second = r_[i].second;
    } else {
      r_[++w] = r_[i];
    }
  }
  r_.resize(w + 1);
}

void RuneSet::negate() {
  std::vector<std::pair<int32_t, int32_t>> o;
  int32_t next = 0;
  for (auto& p : r_) {
    if (p.first > next) o.emplace_back(next, p.first - 1);
    next = p.second + 1;
  }
  if (next <= kMaxRune) o.emplace_back(next, kMaxRune);
  r_ = std::move(o);
}

bool RuneSet::contains(int32_t c) const {
  size_t lo = 0, hi = r_.size();
  while (lo < hi) {
    size_t m = (lo + hi) / 2;
    if (c < r_[m].first) hi = m;
    else if (c > r_[m].second) lo = m + 1;
    else return true;
  }
  return false;
}

ReP Re::clone() const {
  ReP r(new Re(kind));
  r->set = set;
  r->assert_kind = assert_kind;
  r->min = min;
  r->max = max;
  for (const ReP& s : sub) r->sub.push_back(s->clone());
  return r;
}

ParseResult parse_go_regexp(const uint8_t* pattern, size_t n) { return GoParser(pattern, n).run(); }

}  // namespace dgrep
