// compile_api.cpp — dgrep_compile / dgrep_blob_* (C ABI, host only).
//
// Replaces the regexp.Compile that regexp.Match runs for every line at
// application/grep.go:21 with a single compilation per pattern. A pattern that
// Go rejects yields a valid "no line matches" blob, because grep.go:21 drops
// the error and treats every line as unmatched.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

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

// The NFA program of a partial blob (include/dgrep_blob.h), checked word by
// word before anything indexes with it: verify_nfa_kernel computes every table
// offset from the header, follows child[] as node indices and uses classes as
// indices, so a malformed program must never reach the device.
bool nfa_program_ok(const uint32_t* g, size_t words) {
  if (words < 8 || g[0] != DGREP_NFA_MAGIC) return false;
  const uint64_t npos = g[1], nw = g[2], nrc = g[3], nnodes = g[4], nctx = g[5], fffd = g[6], has_word = g[7];
  if (npos > DGREP_NFA_MAX_POS || nw != std::max<uint64_t>(1, (npos + 31) / 32)) return false;
  if (has_word > 1 || nctx != (has_word ? 4u : 1u) || nrc == 0 || fffd >= nrc || nnodes == 0 || nnodes > (1u << 20))
    return false;
  const uint64_t need = 8 + nnodes * 256 + nnodes + nrc + nrc * nw + 2 * nctx * nw + 2 * nctx + npos * nctx * nw +
                        nctx * nw + 4 + 2 * nw;
  if (need != words) return false;
  const int32_t* child = reinterpret_cast<const int32_t*>(g + 8);
  for (uint64_t i = 0; i < nnodes * 256; ++i) {
    const int64_t v = child[i];
    if (v == 0 || v >= int64_t(nnodes) || v < -1 - int64_t(nrc)) return false;  // interior >= 1, leaf class < nrc
  }
  const uint32_t* depth = g + 8 + nnodes * 256;
  if (depth[0] != 0) return false;
  for (uint64_t i = 0; i < nnodes; ++i)
    if (depth[i] > 3) return false;  // at most 3 pending bytes of a UTF-8 sequence
  const uint32_t* word = depth + nnodes;
  for (uint64_t i = 0; i < nrc; ++i)
    if (word[i] > 1) return false;
  // every position bitset: no bit at or beyond npos (the kernel indexes cl[] with them)
  const uint64_t top = npos - 32 * (nw - 1);  // valid bits of the last word (0..32)
  const uint32_t last = top >= 32 ? 0xffffffffu : (1u << top) - 1u;
  auto sets_ok = [&](const uint32_t* p, uint64_t nsets) {
    for (uint64_t s = 0; s < nsets; ++s)
      if (p[s * nw + nw - 1] & ~last) return false;
    return true;
  };
  const uint32_t* has = word + nrc;
  const uint32_t* init = has + nrc * nw;
  const uint32_t* init_m = init + 2 * nctx * nw;
  const uint32_t* cl = init_m + 2 * nctx;
  const uint32_t* mx = cl + npos * nctx * nw;
  const uint32_t* end_init = mx + nctx * nw;
  const uint32_t* end_x = end_init + 4;
  (void)end_init;
  return sets_ok(has, nrc) && sets_ok(init, 2 * nctx) && sets_ok(cl, npos * nctx) && sets_ok(mx, nctx) &&
         sets_ok(end_x, 2);
}

}  // namespace

extern "C" int dgrep_compile(const char* pattern, size_t n, void** blob, size_t* blob_len, char* err,
                             size_t errlen) {
  return dgrep_compile_budget(pattern, n, 0, blob, blob_len, err, errlen);
}

extern "C" int dgrep_compile_budget(const char* pattern, size_t n, uint32_t state_budget, void** blob,
                                    size_t* blob_len, char* err, size_t errlen) {
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
    rc = dgrep::build_dfa(*pr.re, &dfa, &msg, state_budget);
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
  for (int b = 0; b < 256; ++b)
    if (h.byte_class[b] >= h.nclasses) return DGREP_E_INVALID;
  const auto* p = static_cast<const uint8_t*>(blob) + sizeof h;
  const size_t ne = size_t(h.nstates) * h.nclasses;
  for (size_t i = 0; i < ne; ++i) {
    uint32_t t;
    memcpy(&t, p + 4 * i, 4);
    if (t >= h.nstates) return DGREP_E_INVALID;
  }
  if (h.nfa_bytes) {
    std::vector<uint32_t> prog(h.nfa_bytes / 4);
    memcpy(prog.data(), p + 4 * ne, h.nfa_bytes);
    if (!nfa_program_ok(prog.data(), prog.size())) return DGREP_E_INVALID;
  }
  info->flags = h.flags;
  info->nstates = h.nstates;
  info->nclasses = h.nclasses;
  info->start = h.start;
  info->start_m = h.start_m;
  return DGREP_OK;
}
