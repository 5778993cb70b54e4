// dfa_builder.cpp — AST -> NFA -> byte DFA -> minimal DFA -> blob.
//
// The DFA evaluates, in one left-to-right pass over a split, what
// application/grep.go:17-21 computes line by line:
//     for each line of strings.Split(contents, "\n"): regexp.Match(pattern, line)
//
// * Unanchored search: the NFA start state is re-injected before every rune
//   (a match may begin at any rune boundary of the line).
// * Runes are decoded exactly as Go's utf8.DecodeRune does it: a byte that does
//   not begin a complete valid sequence is U+FFFD of width 1, and decoding
//   resumes at the next byte. The DFA carries a "pending bytes" component (a
//   node of a UTF-8 decoding trie); when a sequence breaks, every pending byte
//   is emitted as U+FFFD before the breaking byte is decoded afresh.
// * Empty-width assertions (^ $ \A \z \b \B) are resolved when the next rune (or
//   end of line) is known, from two flags kept in the state: "no rune consumed
//   yet on this line" and "previous rune is an ASCII word character".
// * Once a line matches, the DFA parks in MATCHED until the '\n'. On '\n' every
//   state moves to START_M if its line matched, else to START; START_M is a copy
//   of START, so "state after '\n' == START_M" marks a matching line.
//
// Code points are first partitioned into rune classes (all sets of the pattern
// agree on every member), so the subset construction works per rune class and
// the decoder trie collapses to a handful of nodes for typical patterns.
#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../../include/dgrep.h"
#include "../../../include/dgrep_blob.h"
#include "compiler.hpp"

namespace dgrep {

namespace {

constexpr size_t kMaxNfaStates = 4u << 20;
constexpr size_t kMaxDfaStates = 1u << 21;
// states a partial DFA keeps (the filter stepper holds at most 65535 rows)
constexpr size_t kPartialKeep = 65534;

// ---------------------------------------------------------------- NFA ----
struct NState {
  enum Kind : uint8_t { Eps, Split, Set, Assert, Match, Fail } kind;
  uint8_t amask = 0;
  int32_t out = -1, out1 = -1, set = -1;
};

struct Frag {
  int32_t start;
  std::vector<int32_t> holes;  // state*2 + which
};

class NfaBuilder {
 public:
  std::vector<NState> st;
  std::vector<RuneSet> sets;
  bool too_large = false;
  uint8_t used_asserts = 0;

  int32_t add(NState s) {
    if (st.size() >= kMaxNfaStates) { too_large = true; return 0; }
    st.push_back(s);
    return int32_t(st.size() - 1);
  }
  void patch(Frag& f, int32_t to) {
    for (int32_t h : f.holes) {
      if (h & 1) st[h >> 1].out1 = to;
      else st[h >> 1].out = to;
    }
    f.holes.clear();
  }
  Frag single(NState s) {
    int32_t i = add(s);
    return Frag{i, {i * 2}};
  }
  Frag eps() { return single(NState{NState::Eps}); }
  Frag cat(Frag a, Frag b) {
    patch(a, b.start);
    b.start = a.start;
    return b;
  }
  Frag alt(Frag a, Frag b) {
    NState s{NState::Split};
    s.out = a.start;
    s.out1 = b.start;
    int32_t i = add(s);
    Frag f{i, std::move(a.holes)};
    f.holes.insert(f.holes.end(), b.holes.begin(), b.holes.end());
    return f;
  }
  Frag quest(Frag a) {
    NState s{NState::Split};
    s.out = a.start;
    int32_t i = add(s);
    Frag f{i, std::move(a.holes)};
    f.holes.push_back(i * 2 + 1);
    return f;
  }
  Frag star(Frag a) {
    NState s{NState::Split};
    s.out = a.start;
    int32_t i = add(s);
    patch(a, i);
    return Frag{i, {i * 2 + 1}};
  }
  Frag plus(Frag a) {
    int32_t first = a.start;
    Frag f = star(std::move(a));
    f.start = first;
    return f;
  }

  Frag build(const Re& re) {
    if (too_large) return eps();
    switch (re.kind) {
      case Re::NoMatch: return Frag{add(NState{NState::Fail}), {}};
      case Re::Empty: return eps();
      case Re::Set: {
        NState s{NState::Set};
        s.set = int32_t(sets.size());
        sets.push_back(re.set);
        return single(s);
      }
      case Re::Assert: {
        NState s{NState::Assert};
        s.amask = uint8_t(re.assert_kind);
        used_asserts |= s.amask;
        return single(s);
      }
      case Re::Concat: {
        Frag f = build(*re.sub[0]);
        for (size_t i = 1; i < re.sub.size(); ++i) f = cat(std::move(f), build(*re.sub[i]));
        return f;
      }
      case Re::Alt: {
        Frag f = build(*re.sub.back());
        for (size_t i = re.sub.size() - 1; i-- > 0;) f = alt(build(*re.sub[i]), std::move(f));
        return f;
      }
      case Re::Star: return star(build(*re.sub[0]));
      case Re::Plus: return plus(build(*re.sub[0]));
      case Re::Quest: return quest(build(*re.sub[0]));
      case Re::Repeat: {
        // [Go stdlib] simplify.go: x{n,m} = x^n (x(x..)?)? ; x{n,} = x^(n-1) x+ ; x{0} = empty
        const Re& x = *re.sub[0];
        int mn = re.min, mx = re.max;
        if (mx == -1) {
          if (mn == 0) return star(build(x));
          Frag f = plus(build(x));
          for (int i = 0; i < mn - 1 && !too_large; ++i) f = cat(build(x), std::move(f));
          return f;
        }
        if (mx == 0) return eps();
        bool have = false;
        Frag f{0, {}};
        if (mx > mn) {
          Frag suf = quest(build(x));
          for (int i = mn + 1; i < mx && !too_large; ++i) suf = quest(cat(build(x), std::move(suf)));
          f = std::move(suf);
          have = true;
        }
        for (int i = 0; i < mn && !too_large; ++i) {
          f = have ? cat(build(x), std::move(f)) : build(x);
          have = true;
        }
        return f;
      }
    }
    return eps();
  }
};

// ------------------------------------------------------ rune classes ----
bool is_word_rune(int32_t c) {
  return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_';
}

struct RuneClasses {
  std::vector<int32_t> lo;    // interval starts (sorted); interval i = [lo[i], lo[i+1]-1]
  std::vector<int32_t> cls;   // rune class of interval i
  int n = 0;
  std::vector<uint8_t> word;  // per class
  std::vector<std::vector<uint64_t>> set_has;  // per set: bitset over classes

  int of(int32_t c) const {
    size_t i = size_t(std::upper_bound(lo.begin(), lo.end(), c) - lo.begin()) - 1;
    return cls[i];
  }
  bool has(int set, int c) const { return (set_has[set][size_t(c) >> 6] >> (c & 63)) & 1; }
};

RuneClasses make_rune_classes(const std::vector<RuneSet>& sets, bool split_word) {
  std::vector<int32_t> b{0};
  for (const RuneSet& s : sets)
    for (auto& r : s.ranges()) {
      b.push_back(r.first);
      if (r.second < kMaxRune) b.push_back(r.second + 1);
    }
  if (split_word) {
    for (int32_t x : {int32_t('0'), int32_t('9' + 1), int32_t('A'), int32_t('Z' + 1), int32_t('_'), int32_t('_' + 1),
                      int32_t('a'), int32_t('z' + 1)})
      b.push_back(x);
  }
  b.push_back(0x80);  // keep ASCII and non-ASCII apart (decoder leaves vs root)
  std::sort(b.begin(), b.end());
  b.erase(std::unique(b.begin(), b.end()), b.end());

  // signature of each interval: membership in every set (+ word-ness)
  size_t nsets = sets.size();
  size_t words = (nsets + 1 + 63) / 64;
  std::vector<size_t> cursor(nsets, 0);
  std::unordered_map<std::string, int> sig2cls;
  RuneClasses rc;
  rc.lo = b;
  rc.cls.resize(b.size());
  std::vector<uint64_t> sig(words);
  std::vector<std::vector<uint64_t>> cls_sig;
  for (size_t i = 0; i < b.size(); ++i) {
    int32_t x = b[i];
    std::fill(sig.begin(), sig.end(), 0);
    for (size_t s = 0; s < nsets; ++s) {
      const auto& rr = sets[s].ranges();
      size_t& k = cursor[s];
      while (k < rr.size() && rr[k].second < x) ++k;
      if (k < rr.size() && rr[k].first <= x) sig[s >> 6] |= 1ull << (s & 63);
    }
    if (split_word && is_word_rune(x)) sig[nsets >> 6] |= 1ull << (nsets & 63);
    std::string key(reinterpret_cast<const char*>(sig.data()), sig.size() * 8);
    auto it = sig2cls.find(key);
    int c;
    if (it == sig2cls.end()) {
      c = int(cls_sig.size());
      sig2cls.emplace(std::move(key), c);
      cls_sig.push_back(sig);
    } else {
      c = it->second;
    }
    rc.cls[i] = c;
  }
  rc.n = int(cls_sig.size());
  rc.word.resize(size_t(rc.n));
  for (int c = 0; c < rc.n; ++c) rc.word[size_t(c)] = split_word && ((cls_sig[size_t(c)][nsets >> 6] >> (nsets & 63)) & 1);
  size_t cw = (size_t(rc.n) + 63) / 64;
  rc.set_has.assign(nsets, std::vector<uint64_t>(cw, 0));
  for (int c = 0; c < rc.n; ++c)
    for (size_t s = 0; s < nsets; ++s)
      if ((cls_sig[size_t(c)][s >> 6] >> (s & 63)) & 1) rc.set_has[s][size_t(c) >> 6] |= 1ull << (c & 63);
  return rc;
}

// ---------------------------------------------------- UTF-8 decoder ----
// Node 0 is the root (nothing pending). child[node][b]:
//   >= 1           : interior node (more continuation bytes needed)
//   kInvalid (-1)  : sequence broken at this byte
//   <= -2          : complete rune of class (-2 - v)
constexpr int32_t kInvalid = -1;
inline int32_t leaf(int c) { return -2 - c; }
inline bool is_leaf(int32_t v) { return v <= -2; }
inline int leaf_class(int32_t v) { return -2 - v; }

struct Decoder {
  std::vector<std::array<int32_t, 256>> child;
  std::vector<int> depth;  // bytes pending at this node
  std::unordered_map<std::string, int> memo;

  int intern(int d, const std::array<int32_t, 256>& ch) {
    std::string key(reinterpret_cast<const char*>(ch.data()), sizeof(int32_t) * 256);
    key.push_back(char(d));
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
    int id = int(child.size());
    child.push_back(ch);
    depth.push_back(d);
    memo.emplace(std::move(key), id);
    return id;
  }

  // node after `d` bytes of a sequence with `rem` continuation bytes still to
  // come; `prefix` holds the code point bits so far; [clo, chi] = valid next byte
  int make(const RuneClasses& rc, int d, int rem, int32_t prefix, int clo, int chi) {
    std::array<int32_t, 256> ch;
    ch.fill(kInvalid);
    for (int c = clo; c <= chi; ++c) {
      int32_t v = (prefix << 6) | (c & 0x3F);
      ch[size_t(c)] = rem == 1 ? leaf(rc.of(v)) : make(rc, d + 1, rem - 1, v, 0x80, 0xBF);
    }
    return intern(d, ch);
  }

  void build(const RuneClasses& rc) {
    child.emplace_back();
    depth.push_back(0);
    std::array<int32_t, 256> root;
    root.fill(kInvalid);
    for (int b = 0; b < 0x80; ++b) root[size_t(b)] = leaf(rc.of(b));
    for (int b = 0xC2; b <= 0xDF; ++b) root[size_t(b)] = make(rc, 1, 1, b & 0x1F, 0x80, 0xBF);
    for (int b = 0xE0; b <= 0xEF; ++b) {
      int lo = b == 0xE0 ? 0xA0 : 0x80, hi = b == 0xED ? 0x9F : 0xBF;
      root[size_t(b)] = make(rc, 1, 2, b & 0x0F, lo, hi);
    }
    for (int b = 0xF0; b <= 0xF4; ++b) {
      int lo = b == 0xF0 ? 0x90 : 0x80, hi = b == 0xF4 ? 0x8F : 0xBF;
      root[size_t(b)] = make(rc, 1, 3, b & 0x07, lo, hi);
    }
    child[0] = root;
  }
};

// ------------------------------------------------ subset construction ----
struct VecHash {
  size_t operator()(const std::vector<int32_t>& v) const {
    uint64_t h = 1469598103934665603ull;
    for (int32_t x : v) { h ^= uint32_t(x); h *= 1099511628211ull; }
    return size_t(h);
  }
};

class DfaBuilder {
 public:
  DfaBuilder(const NfaBuilder& nfa, int32_t nfa_start, const RuneClasses& rc, const Decoder& dec)
      : nfa_(nfa), start_(nfa_start), rc_(rc), dec_(dec), mark_(nfa.st.size(), 0) {
    has_begin_ = (nfa.used_asserts & uint8_t(AssertKind::BeginText)) != 0;
    has_word_ = (nfa.used_asserts & (uint8_t(AssertKind::WordBoundary) | uint8_t(AssertKind::NotWordBoundary))) != 0;
    fffd_ = rc.of(kRuneError);
  }

  // returns false if the state budget is exceeded; then *partial holds the
  // first states of the construction with CAND (DGREP_DFA_PARTIAL)
  bool run(CompiledDfa* out, CompiledDfa* partial, size_t budget);
  // the NFA program of a partial blob (dgrep_blob.h); false above DGREP_NFA_MAX_POS positions
  bool nfa_program(std::vector<uint32_t>* prog);

 private:
  const NfaBuilder& nfa_;
  int32_t start_;
  const RuneClasses& rc_;
  const Decoder& dec_;
  bool has_begin_, has_word_;
  int fffd_;

  // core = (Q, begin, prev_word); Q = NFA states reached by the last rune step
  std::vector<std::vector<int32_t>> core_q_;
  std::vector<uint8_t> core_flags_;  // bit0 begin, bit1 prev word
  std::unordered_map<std::vector<int32_t>, int, VecHash> core_ids_;
  std::unordered_map<uint64_t, int> step_memo_;  // (core, rc) -> core or kMatched
  std::vector<int8_t> end_memo_;                 // core -> accepts at end (-1 unknown)

  std::vector<uint32_t> mark_;
  uint32_t gen_ = 0;
  std::vector<int32_t> stack_, clos_;

  static constexpr int kMatched = -1;

  int intern_core(std::vector<int32_t> q, uint8_t flags) {
    std::vector<int32_t> key = q;
    key.push_back(-1 - int32_t(flags));
    auto it = core_ids_.find(key);
    if (it != core_ids_.end()) return it->second;
    int id = int(core_q_.size());
    core_q_.push_back(std::move(q));
    core_flags_.push_back(flags);
    core_ids_.emplace(std::move(key), id);
    end_memo_.push_back(-1);
    return id;
  }

  // epsilon closure of Q ∪ {start} at a position whose context is
  // (begin, prev_word, next_word, at_end). Returns true if Match is reached.
  bool closure(const std::vector<int32_t>& q, bool begin, bool prev_word, bool next_word, bool at_end,
               bool with_start = true) {
    ++gen_;
    clos_.clear();
    stack_.clear();
    for (int32_t s : q) stack_.push_back(s);
    if (with_start) stack_.push_back(start_);
    bool wb = prev_word != next_word;
    while (!stack_.empty()) {
      int32_t x = stack_.back();
      stack_.pop_back();
      if (x < 0 || mark_[size_t(x)] == gen_) continue;
      mark_[size_t(x)] = gen_;
      const NState& s = nfa_.st[size_t(x)];
      switch (s.kind) {
        case NState::Match: return true;
        case NState::Eps: stack_.push_back(s.out); break;
        case NState::Split: stack_.push_back(s.out1); stack_.push_back(s.out); break;
        case NState::Set: clos_.push_back(x); break;
        case NState::Assert: {
          bool ok;
          switch (AssertKind(s.amask)) {
            case AssertKind::BeginText: ok = begin; break;
            case AssertKind::EndText: ok = at_end; break;
            case AssertKind::WordBoundary: ok = wb; break;
            default: ok = !wb; break;
          }
          if (ok) stack_.push_back(s.out);
          break;
        }
        case NState::Fail: break;
      }
    }
    return false;
  }

  int step(int core, int c) {
    uint64_t key = (uint64_t(uint32_t(core)) << 32) | uint32_t(c);
    auto it = step_memo_.find(key);
    if (it != step_memo_.end()) return it->second;
    uint8_t f = core_flags_[size_t(core)];
    bool word = rc_.word[size_t(c)];
    int result;
    if (closure(core_q_[size_t(core)], f & 1, f & 2, word, false)) {
      result = kMatched;
    } else {
      std::vector<int32_t> q;
      for (int32_t x : clos_) {
        const NState& s = nfa_.st[size_t(x)];
        if (rc_.has(s.set, c) && s.out >= 0) q.push_back(s.out);
      }
      std::sort(q.begin(), q.end());
      q.erase(std::unique(q.begin(), q.end()), q.end());
      uint8_t nf = uint8_t((has_word_ && word) ? 2 : 0);
      result = intern_core(std::move(q), nf);
    }
    step_memo_.emplace(key, result);
    return result;
  }

  bool accepts_at_end(int core) {
    int8_t& m = end_memo_[size_t(core)];
    if (m < 0) {
      uint8_t f = core_flags_[size_t(core)];
      m = closure(core_q_[size_t(core)], f & 1, f & 2, false, true) ? 1 : 0;
    }
    return m == 1;
  }
};

// NFA program (layout in dgrep_blob.h): the same step the subset construction
// memoizes per core (DfaBuilder::step), per position instead of per set.
bool DfaBuilder::nfa_program(std::vector<uint32_t>* prog) {
  std::vector<int32_t> pos_of(nfa_.st.size(), -1), pos_state;
  for (size_t i = 0; i < nfa_.st.size(); ++i)
    if (nfa_.st[i].kind == NState::Set) {
      pos_of[i] = int32_t(pos_state.size());
      pos_state.push_back(int32_t(i));
    }
  const uint32_t npos = uint32_t(pos_state.size());
  if (npos > DGREP_NFA_MAX_POS) return false;
  const uint32_t nw = std::max<uint32_t>(1, (npos + 31) / 32), nrc = uint32_t(rc_.n),
                 nnodes = uint32_t(dec_.child.size()), nctx = has_word_ ? 4 : 1;
  std::vector<uint32_t>& g = *prog;
  g = {DGREP_NFA_MAGIC, npos, nw, nrc, nnodes, nctx, uint32_t(fffd_), has_word_ ? 1u : 0u};
  for (const auto& ch : dec_.child)
    for (int b = 0; b < 256; ++b) g.push_back(uint32_t(ch[size_t(b)]));
  for (int d : dec_.depth) g.push_back(uint32_t(d));
  for (uint32_t c = 0; c < nrc; ++c) g.push_back(rc_.word[c] ? 1u : 0u);
  auto bits = [&](std::vector<uint32_t>& v, size_t at) {  // clos_ -> position bitset at v[at..]
    for (int32_t x : clos_) v[at + size_t(pos_of[size_t(x)]) / 32] |= 1u << (pos_of[size_t(x)] % 32);
  };
  const size_t has_at = g.size();
  g.resize(has_at + size_t(nrc) * nw, 0);
  for (uint32_t c = 0; c < nrc; ++c)
    for (uint32_t p = 0; p < npos; ++p)
      if (rc_.has(nfa_.st[size_t(pos_state[p])].set, int(c))) g[has_at + size_t(c) * nw + p / 32] |= 1u << (p % 32);
  auto ctx_pw = [&](uint32_t ctx) { return nctx == 4 && (ctx >> 1); };
  auto ctx_nw = [&](uint32_t ctx) { return nctx == 4 && (ctx & 1); };
  const size_t init_at = g.size();
  g.resize(init_at + 2 * size_t(nctx) * nw + 2 * size_t(nctx), 0);
  for (uint32_t b = 0; b < 2; ++b)
    for (uint32_t ctx = 0; ctx < nctx; ++ctx) {
      const bool m = closure({}, b != 0, ctx_pw(ctx), ctx_nw(ctx), false);
      if (m) g[init_at + 2 * size_t(nctx) * nw + b * nctx + ctx] = 1;
      else bits(g, init_at + (size_t(b) * nctx + ctx) * nw);
    }
  const size_t cl_at = g.size();
  g.resize(cl_at + size_t(npos) * nctx * nw + size_t(nctx) * nw, 0);
  const size_t mx_at = cl_at + size_t(npos) * nctx * nw;
  for (uint32_t p = 0; p < npos; ++p) {
    const int32_t to = nfa_.st[size_t(pos_state[p])].out;
    if (to < 0) continue;
    for (uint32_t ctx = 0; ctx < nctx; ++ctx) {
      if (closure({to}, false, ctx_pw(ctx), ctx_nw(ctx), false, false)) g[mx_at + size_t(ctx) * nw + p / 32] |= 1u << (p % 32);
      else bits(g, cl_at + (size_t(p) * nctx + ctx) * nw);
    }
  }
  const size_t end_at = g.size();
  g.resize(end_at + 4 + 2 * size_t(nw), 0);
  for (uint32_t b = 0; b < 2; ++b)
    for (uint32_t pw = 0; pw < 2; ++pw)
      g[end_at + b * 2 + pw] = closure({}, b != 0, pw != 0 && has_word_, false, true) ? 1u : 0u;
  for (uint32_t pw = 0; pw < 2; ++pw)
    for (uint32_t p = 0; p < npos; ++p) {
      const int32_t to = nfa_.st[size_t(pos_state[p])].out;
      if (to >= 0 && closure({to}, false, pw != 0 && has_word_, false, true, false))
        g[end_at + 4 + size_t(pw) * nw + p / 32] |= 1u << (p % 32);
    }
  return true;
}

bool DfaBuilder::run(CompiledDfa* out, CompiledDfa* partial, size_t budget) {
  // byte classes for construction: bytes that every decoder node treats alike
  std::unordered_map<std::string, int> bsig;
  uint8_t bclass[256];
  std::vector<int> rep;  // representative byte per class
  for (int b = 0; b < 256; ++b) {
    std::string key;
    if (b == '\n') key = "NL";
    else
      for (const auto& ch : dec_.child) key.append(reinterpret_cast<const char*>(&ch[size_t(b)]), 4);
    auto it = bsig.find(key);
    if (it == bsig.end()) {
      it = bsig.emplace(key, int(rep.size())).first;
      rep.push_back(b);
    }
    bclass[b] = uint8_t(it->second);
  }
  const int K = int(rep.size());
  const int nl_class = bclass[uint8_t('\n')];

  // DFA states: 0 = START, 1 = START_M, 2 = MATCHED, then (dnode, core) pairs
  const int start_core = intern_core({}, uint8_t(has_begin_ ? 1 : 0));
  std::unordered_map<uint64_t, int> ids;
  std::vector<std::pair<int, int>> states;  // (dnode, core); (-1,-1) for MATCHED
  states.push_back({0, start_core});
  states.push_back({0, start_core});
  states.push_back({-1, -1});
  ids.emplace((uint64_t(0) << 32) | uint32_t(start_core), 0);
  std::vector<int32_t> trans;
  trans.reserve(size_t(K) * 64);

  auto get_state = [&](int dnode, int core) -> int {
    if (core == kMatched) return 2;
    uint64_t key = (uint64_t(uint32_t(dnode)) << 32) | uint32_t(core);
    auto it = ids.find(key);
    if (it != ids.end()) return it->second;
    int id = int(states.size());
    states.push_back({dnode, core});
    ids.emplace(key, id);
    return id;
  };

  // feed one byte from the decoder root at `core`; returns (dnode, core')
  auto feed_root = [&](int core, int b, int* dnode) -> int {
    int32_t v = dec_.child[0][size_t(b)];
    if (is_leaf(v)) { *dnode = 0; return step(core, leaf_class(v)); }
    if (v == kInvalid) { *dnode = 0; return step(core, fffd_); }
    *dnode = v;
    return core;
  };

  for (size_t s = 0; s < states.size(); ++s) {
    if (states.size() > budget && s >= 3) {
      // Over budget: keep the first states (rows [0, L) are complete, in
      // breadth-first order) and send every other transition to CAND = L.
      const uint32_t L = uint32_t(std::min<size_t>(s, kPartialKeep));
      partial->nstates = L + 1;
      partial->nclasses = uint32_t(K);
      partial->start = 0;
      partial->start_m = 1;
      partial->flags = DGREP_DFA_PARTIAL;
      memcpy(partial->byte_class, bclass, 256);
      partial->trans.assign(size_t(L + 1) * size_t(K), L);
      for (size_t i = 0; i < L; ++i)
        for (int k = 0; k < K; ++k) {
          const uint32_t x = uint32_t(trans[i * size_t(K) + size_t(k)]);
          partial->trans[i * size_t(K) + size_t(k)] = x < L ? x : L;
        }
      partial->trans[size_t(L) * size_t(K) + size_t(nl_class)] = 0;
      return false;
    }
    const int dnode = states[s].first, core = states[s].second;
    for (int k = 0; k < K; ++k) {
      const int b = rep[size_t(k)];
      int next;
      if (s == 2) {
        next = k == nl_class ? 1 : 2;
      } else if (k == nl_class) {
        // end of line: flush pending bytes as U+FFFD, then test end-of-text
        int c = core;
        for (int i = 0; i < dec_.depth[size_t(dnode)] && c != kMatched; ++i) c = step(c, fffd_);
        bool acc = c == kMatched || accepts_at_end(c);
        next = acc ? 1 : 0;
      } else if (dnode == 0) {
        int nd;
        int c = feed_root(core, b, &nd);
        next = get_state(nd, c);
      } else {
        int32_t v = dec_.child[size_t(dnode)][size_t(b)];
        if (is_leaf(v)) {
          next = get_state(0, step(core, leaf_class(v)));
        } else if (v != kInvalid) {
          next = get_state(v, core);
        } else {
          int c = core;
          for (int i = 0; i < dec_.depth[size_t(dnode)] && c != kMatched; ++i) c = step(c, fffd_);
          if (c == kMatched) {
            next = 2;
          } else {
            int nd;
            int c2 = feed_root(c, b, &nd);
            next = get_state(nd, c2);
          }
        }
      }
      trans.push_back(next);
    }
  }
  const size_t S = states.size();

  // ---- Moore minimization; START_M starts in its own block ----
  std::vector<int32_t> color(S, 0), ncolor(S);
  color[1] = 1;
  int ncolors = 2;
  for (;;) {
    std::unordered_map<std::vector<int32_t>, int, VecHash> sig;
    std::vector<int32_t> key(size_t(K) + 1);
    for (size_t s = 0; s < S; ++s) {
      key[0] = color[s];
      for (int k = 0; k < K; ++k) key[size_t(k) + 1] = color[size_t(trans[s * size_t(K) + size_t(k)])];
      auto it = sig.find(key);
      if (it == sig.end()) it = sig.emplace(key, int(sig.size())).first;
      ncolor[s] = it->second;
    }
    int n = int(sig.size());
    color.swap(ncolor);
    if (n == ncolors) break;
    ncolors = n;
  }

  // renumber minimized states in BFS order from START
  std::vector<int32_t> rep_state(size_t(ncolors), -1);
  for (size_t s = 0; s < S; ++s)
    if (rep_state[size_t(color[s])] < 0) rep_state[size_t(color[s])] = int32_t(s);
  std::vector<int32_t> order_of(size_t(ncolors), -1), order;
  // START is state 0 and START_M state 1 (kept even when no line can reach it)
  order.push_back(color[0]);
  order_of[size_t(color[0])] = 0;
  if (color[1] != color[0]) {
    order.push_back(color[1]);
    order_of[size_t(color[1])] = 1;
  }
  for (size_t i = 0; i < order.size(); ++i) {
    int32_t r = rep_state[size_t(order[i])];
    for (int k = 0; k < K; ++k) {
      int32_t c = color[size_t(trans[size_t(r) * size_t(K) + size_t(k)])];
      if (order_of[size_t(c)] < 0) {
        order_of[size_t(c)] = int32_t(order.size());
        order.push_back(c);
      }
    }
  }
  const size_t M = order.size();
  std::vector<uint32_t> mtrans(M * size_t(K));
  for (size_t i = 0; i < M; ++i) {
    int32_t r = rep_state[size_t(order[i])];
    for (int k = 0; k < K; ++k)
      mtrans[i * size_t(K) + size_t(k)] = uint32_t(order_of[size_t(color[size_t(trans[size_t(r) * size_t(K) + size_t(k)])])]);
  }
  const uint32_t start = uint32_t(order_of[size_t(color[0])]);
  const uint32_t start_m = uint32_t(order_of[size_t(color[1])]);

  // final byte classes over the minimized table
  std::unordered_map<std::vector<int32_t>, int, VecHash> colsig;
  std::vector<int> kmap(static_cast<size_t>(K));
  std::vector<int> kept;
  for (int k = 0; k < K; ++k) {
    std::vector<int32_t> col(M);
    for (size_t i = 0; i < M; ++i) col[i] = int32_t(mtrans[i * size_t(K) + size_t(k)]);
    if (k == nl_class) col.push_back(-7);  // keep '\n' its own class
    auto it = colsig.find(col);
    if (it == colsig.end()) {
      it = colsig.emplace(col, int(kept.size())).first;
      kept.push_back(k);
    }
    kmap[size_t(k)] = it->second;
  }
  const size_t K2 = kept.size();
  out->nstates = uint32_t(M);
  out->nclasses = uint32_t(K2);
  out->start = start;
  out->start_m = start_m;
  for (int b = 0; b < 256; ++b) out->byte_class[b] = uint8_t(kmap[bclass[b]]);
  out->trans.resize(M * K2);
  for (size_t i = 0; i < M; ++i)
    for (size_t k = 0; k < K2; ++k) out->trans[i * K2 + k] = mtrans[i * size_t(K) + size_t(kept[k])];

  // whole-pattern flags
  const uint32_t nlk = out->byte_class[uint8_t('\n')];
  bool any = false, all = true;
  for (size_t i = 0; i < M; ++i) {
    bool acc = out->trans[i * K2 + nlk] == start_m;
    any |= acc;
    all &= acc;
  }
  out->flags = 0;
  if (!any) out->flags |= DGREP_DFA_MATCH_NONE;
  if (all) out->flags |= DGREP_DFA_MATCH_ALL;
  return true;
}

}  // namespace

// Builds the DFA for a parsed pattern. Returns DGREP_OK / DGREP_E_TOO_LARGE.
// state_budget (0 = kMaxDfaStates; tests pass a small one so that the partial
// DFA + NFA program path is checked on small patterns, dgrep_compile_budget).
int build_dfa(const Re& re, CompiledDfa* out, std::string* err, size_t state_budget) {
  NfaBuilder nfa;
  Frag f = nfa.build(re);
  int32_t m = nfa.add(NState{NState::Match});
  nfa.patch(f, m);
  if (nfa.too_large) { *err = "pattern expands beyond the NFA state budget"; return DGREP_E_TOO_LARGE; }
  bool word = (nfa.used_asserts & (uint8_t(AssertKind::WordBoundary) | uint8_t(AssertKind::NotWordBoundary))) != 0;
  RuneClasses rc = make_rune_classes(nfa.sets, word);
  Decoder dec;
  dec.build(rc);
  DfaBuilder b(nfa, f.start, rc, dec);
  const size_t budget = state_budget >= 3 && state_budget < kMaxDfaStates ? state_budget : kMaxDfaStates;
  CompiledDfa part;
  if (b.run(out, &part, budget)) return DGREP_OK;
  // over the DFA budget: the first states as a filter, the NFA program decides
  // the lines that leave them (DGREP_DFA_PARTIAL)
  if (part.nstates < 3 || !b.nfa_program(&part.nfa)) {
    *err = "DFA exceeds the state budget and the NFA has more than 1024 rune-set positions";
    return DGREP_E_TOO_LARGE;
  }
  *out = std::move(part);
  return DGREP_OK;
}

void dfa_match_none(CompiledDfa* out, uint32_t extra_flags) {
  // two states: START (0) and START_M (1, never reached); byte class 0 = all
  // bytes but '\n', class 1 = '\n'
  out->nstates = 2;
  out->nclasses = 2;
  out->start = 0;
  out->start_m = 1;
  for (int b = 0; b < 256; ++b) out->byte_class[b] = b == '\n' ? 1 : 0;
  out->trans = {0, 0, 0, 0};
  out->flags = DGREP_DFA_MATCH_NONE | extra_flags;
}

}  // namespace dgrep
