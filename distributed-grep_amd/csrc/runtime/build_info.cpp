// build_info.cpp — provenance of this libdgrep.so (dgrep_build_info).
// The Makefile regenerates build/build_stamp.h whenever `git rev-parse HEAD`
// or the product sources' dirty state changes, so the string names the commit
// the binary was built from and the tuning knobs it was compiled with.
#include "../../../include/dgrep.h"
#include "build_stamp.h"

#ifndef DGREP_GIT_HEAD
#define DGREP_GIT_HEAD "unknown"
#endif
#ifndef DGREP_BUILD_FLAGS
#define DGREP_BUILD_FLAGS ""
#endif

extern "C" const char* dgrep_build_info(void) {
  return "head=" DGREP_GIT_HEAD " arch=gfx950 hipflags=" DGREP_BUILD_FLAGS;
}
