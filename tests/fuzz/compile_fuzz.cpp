// compile_fuzz.cpp -- host-only driver for the product's pattern compiler
// (csrc/compiler: go_parser.cpp, dfa_builder.cpp, compile_api.cpp), built with
// -fsanitize=address,undefined by tests/fuzz/Makefile. The worker process
// parses arbitrary user patterns with this code (dgrep_compile), so a memory
// bug there would kill the worker: tests/test_fuzz_compile.py feeds it random
// byte strings and regex-shaped patterns and requires a clean exit.
//
// Input (stdin): records of <u32 little-endian length><bytes>. For each pattern
// it calls dgrep_compile, checks the status is one of the documented codes and
// that an OK blob passes dgrep_blob_info_get with transitions in range, then
// frees it. Prints "<n> patterns: ok=<a> unsupported=<b> too_large=<c>".
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "dgrep.h"
#include "dgrep_blob.h"

int main() {
  std::vector<unsigned char> in;
  unsigned char buf[1 << 16];
  size_t r;
  while ((r = fread(buf, 1, sizeof buf, stdin)) > 0) in.insert(in.end(), buf, buf + r);
  size_t pos = 0, n = 0, ok = 0, unsup = 0, big = 0;
  while (pos + 4 <= in.size()) {
    uint32_t len;
    memcpy(&len, in.data() + pos, 4);
    pos += 4;
    if (pos + len > in.size()) break;
    // copy into an exact-size heap block so ASan sees any read past the pattern
    char* p = static_cast<char*>(malloc(len ? len : 1));
    memcpy(p, in.data() + pos, len);
    pos += len;
    void* blob = nullptr;
    size_t blen = 0;
    char err[128];
    const int rc = dgrep_compile(p, len, &blob, &blen, err, sizeof err);
    if (rc == DGREP_OK) {
      dgrep_blob_info info;
      if (dgrep_blob_info_get(blob, blen, &info) != DGREP_OK) {
        fprintf(stderr, "blob rejected for pattern #%zu\n", n);
        return 2;
      }
      dgrep_blob_header h;
      memcpy(&h, blob, sizeof h);
      const uint32_t* tr = reinterpret_cast<const uint32_t*>(static_cast<const unsigned char*>(blob) + sizeof h);
      for (size_t i = 0; i < size_t(h.nstates) * h.nclasses; ++i)
        if (tr[i] >= h.nstates) {
          fprintf(stderr, "transition out of range for pattern #%zu\n", n);
          return 3;
        }
      dgrep_blob_free(blob);
      ++ok;
    } else if (rc == DGREP_E_UNSUPPORTED) {
      ++unsup;
    } else if (rc == DGREP_E_TOO_LARGE) {
      ++big;
    } else {
      fprintf(stderr, "unexpected status %d for pattern #%zu: %s\n", rc, n, err);
      return 4;
    }
    free(p);
    ++n;
  }
  printf("%zu patterns: ok=%zu unsupported=%zu too_large=%zu\n", n, ok, unsup, big);
  return 0;
}
