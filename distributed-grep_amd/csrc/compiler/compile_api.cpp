// compile_api.cpp — dgrep_compile / dgrep_blob_* (C ABI, host only).
//
// Replaces the regexp.Compile that regexp.Match runs for every line at
// application/grep.go:21 with a single compilation per pattern. A pattern that
// Go rejects yields a valid "no line matches" blob, because grep.go:21 drops
// the error and treats every line as unmatched.
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../../include/dgrep.h"
#include "../../../include/dgrep_blob.h"
#include "compiler.hpp"

namespace {

void set_err(char* err, size_t errlen, const std::string& m) {
  if (err && errlen) {
    size_t n = m.size() < errlen - 1 ? m.size() : errlen - 1;
    memcpy(err, m.data(), n);
    err[n] = 0;
  }
}

int serialize(const dgrep::CompiledDfa& d, void** blob, size_t* blob_len) {
  size_t n = sizeof(dgrep_blob_header) + (d.trans.size() + d.nfa.size()) * sizeof(uint32_t);
  auto* p = static_cast<uint8_t*>(malloc(n));
  if (!p) return DGREP_E_NOMEM;
  dgrep_blob_header h;
  memset(&h, 0, sizeof h);
  h.magic = DGREP_BLOB_MAGIC;
  h.version = DGREP_BLOB_VERSION;
  h.flags = d.flags;
  h.nstates = d.nstates;
  h.nclasses = d.nclasses;
  h.start = d.start;
  h.start_m = d.start_m;
  h.nfa_bytes = uint32_t(d.nfa.size() * sizeof(uint32_t));
  memcpy(h.byte_class, d.byte_class, 256);
  memcpy(p, &h, sizeof h);
  memcpy(p + sizeof h, d.trans.data(), d.trans.size() * sizeof(uint32_t));
  if (!d.nfa.empty()) memcpy(p + sizeof h + d.trans.size() * sizeof(uint32_t), d.nfa.data(), h.nfa_bytes);
  *blob = p;
  *blob_len = n;
  return DGREP_OK;
}

}  // namespace

extern "C" int dgrep_compile(const char* pattern, size_t n, void** blob, size_t* blob_len, char* err,
                             size_t errlen) {
  if (!blob || !blob_len || (!pattern && n)) return DGREP_E_INVALID;
  *blob = nullptr;
  *blob_len = 0;
  dgrep::ParseResult pr = dgrep::parse_go_regexp(reinterpret_cast<const uint8_t*>(pattern ? pattern : ""), n);
  dgrep::CompiledDfa dfa;
  if (pr.status == dgrep::ParseResult::GoSyntaxError) {
    set_err(err, errlen, "go regexp syntax error: " + pr.message);
    dgrep::dfa_match_none(&dfa, DGREP_DFA_GO_SYNTAX_ERROR);
    return serialize(dfa, blob, blob_len);
  }
  if (pr.status == dgrep::ParseResult::Unsupported) {
    set_err(err, errlen, "unsupported: " + pr.message);
    return DGREP_E_UNSUPPORTED;
  }
  std::string msg;
  int rc;
  try {
    rc = dgrep::build_dfa(*pr.re, &dfa, &msg);
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "out of memory building the DFA");
    return DGREP_E_NOMEM;
  }
  if (rc != DGREP_OK) {
    set_err(err, errlen, msg);
    return rc;
  }
  return serialize(dfa, blob, blob_len);
}

extern "C" void dgrep_blob_free(void* blob) { free(blob); }

extern "C" int dgrep_blob_info_get(const void* blob, size_t n, dgrep_blob_info* info) {
  if (!blob || !info || n < sizeof(dgrep_blob_header)) return DGREP_E_INVALID;
  dgrep_blob_header h;
  memcpy(&h, blob, sizeof h);
  if (h.magic != DGREP_BLOB_MAGIC || h.version != DGREP_BLOB_VERSION) return DGREP_E_INVALID;
  if (h.nstates == 0 || h.nclasses == 0 || h.start >= h.nstates || h.start_m >= h.nstates) return DGREP_E_INVALID;
  if (n != sizeof h + size_t(h.nstates) * h.nclasses * sizeof(uint32_t) + h.nfa_bytes) return DGREP_E_INVALID;
  // a partial DFA carries its NFA program (header of 8 words at least), nothing else does
  if (bool(h.flags & DGREP_DFA_PARTIAL) != (h.nfa_bytes != 0) || h.nfa_bytes % 4 || (h.nfa_bytes && h.nfa_bytes < 32))
    return DGREP_E_INVALID;
  info->flags = h.flags;
  info->nstates = h.nstates;
  info->nclasses = h.nclasses;
  info->start = h.start;
  info->start_m = h.start_m;
  return DGREP_OK;
}
