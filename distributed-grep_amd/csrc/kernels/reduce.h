// reduce.h — the grep reduce task (reduce.hip), shared with the runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dgrep {

// *d_count = number of '\n' in d_in[0:n) (the input's KeyValue lines).
hipError_t reduce_count_lines(const uint8_t* d_in, uint64_t n, uint64_t* d_count, hipStream_t s);

// Decodes the json.Encoder KeyValue lines of d_in[0:n) (nlines of them, each
// ending in '\n'), keeps one line per distinct key (the first in input
// order) and writes "key value\n" with the raw (decoded) strings into out
// (lines past out_cap are not written). d_info (device, 3 u64): [0] lines,
// [1] first malformed line (UINT64_MAX: none), [2] output bytes. With scratch ==
// nullptr or *scratch_bytes too small, only sets *scratch_bytes.
hipError_t reduce_lines(const uint8_t* d_in, uint64_t n, uint64_t nlines, void* scratch, size_t* scratch_bytes,
                        uint8_t* out, uint64_t out_cap, uint64_t* d_info, hipStream_t s);

}  // namespace dgrep
