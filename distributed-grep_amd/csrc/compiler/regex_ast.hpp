// regex_ast.hpp — pattern AST for the dgrep pattern compiler.
//
// The compiler replaces the regexp.Compile that regexp.Match performs on every
// line at application/grep.go:21. Only what decides *whether* a line matches is
// kept: captures, greediness and leftmost-first preferences do not change a
// boolean unanchored match, so they are dropped; every character-consuming
// construct is reduced to a set of code points.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace dgrep {

constexpr int32_t kMaxRune = 0x10FFFF;
constexpr int32_t kRuneError = 0xFFFD;

// Sorted, non-overlapping, non-adjacent closed intervals of code points.
class RuneSet {
 public:
  void add(int32_t lo, int32_t hi) { r_.emplace_back(lo, hi); }
  void add(const RuneSet& o) { r_.insert(r_.end(), o.r_.begin(), o.r_.end()); }
  void normalize();  // sort + merge
  void negate();     // complement within [0, kMaxRune]; requires normalize()
  bool contains(int32_t c) const;
  bool empty() const { return r_.empty(); }
  const std::vector<std::pair<int32_t, int32_t>>& ranges() const { return r_; }

 private:
  std::vector<std::pair<int32_t, int32_t>> r_;
};

enum class AssertKind : uint8_t { BeginText = 1, EndText = 2, WordBoundary = 4, NotWordBoundary = 8 };

struct Re;
using ReP = std::unique_ptr<Re>;

struct Re {
  enum Kind : uint8_t { NoMatch, Empty, Set, Assert, Concat, Alt, Star, Plus, Quest, Repeat };
  Kind kind;
  RuneSet set;            // Set
  AssertKind assert_kind; // Assert
  int min = 0, max = 0;   // Repeat (max = -1: unbounded)
  std::vector<ReP> sub;

  explicit Re(Kind k) : kind(k), assert_kind(AssertKind::BeginText) {}
  ReP clone() const;
};

struct ParseResult {
  enum Status { Ok, GoSyntaxError, Unsupported } status = Ok;
  std::string message;
  ReP re;
};

// Parse `pattern` with the flags regexp.Compile uses (syntax.Perl:
// ClassNL|OneLine|PerlX|UnicodeGroups). A pattern that Go rejects gives
// GoSyntaxError; a valid pattern this compiler cannot model exactly gives
// Unsupported (never an approximation).
ParseResult parse_go_regexp(const uint8_t* pattern, size_t n);

}  // namespace dgrep
