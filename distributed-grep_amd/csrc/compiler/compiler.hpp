// compiler.hpp — internal interface between the Go-syntax front end, the DFA
// builder and the C ABI (dgrep_compile in compile_api.cpp).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "regex_ast.hpp"

namespace dgrep {

struct CompiledDfa {
  uint32_t flags = 0;
  uint32_t nstates = 0, nclasses = 0, start = 0, start_m = 0;
  uint8_t byte_class[256] = {0};
  std::vector<uint32_t> trans;  // nstates * nclasses, row-major
  std::vector<uint32_t> nfa;    // DGREP_DFA_PARTIAL: the NFA program (dgrep_blob.h)
};

// AST -> minimal line-matching DFA (see dfa_builder.cpp). DGREP_OK or DGREP_E_TOO_LARGE.
int build_dfa(const Re& re, CompiledDfa* out, std::string* err, size_t state_budget = 0);
// The automaton of a pattern that matches no line.
void dfa_match_none(CompiledDfa* out, uint32_t extra_flags);

}  // namespace dgrep
