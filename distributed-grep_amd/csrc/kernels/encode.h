// encode.h — partition + intermediate writer (encode.hip), shared with the runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dgrep {

struct EncodeArgs {
  const uint8_t* data;        // the HBM-resident split (16-byte aligned)
  uint64_t n;                 // its bytes (aligned 16-B reads never pass them)
  const uint64_t* line_no;    // scan records, ascending line order
  const uint64_t* start;
  const uint64_t* len;
  uint64_t count;
  const uint8_t* fname_json;  // the filename, JSON-escaped, without quotes (device)
  uint32_t fname_json_len;
  uint32_t key_hash0;         // FNV-1a state after "filename (line number #"
  uint32_t nreduce;
};

// Host helpers (same escaping / hashing code as the device path).
uint64_t json_escape_host(const uint8_t* s, uint64_t n, uint8_t* out);  // out = nullptr measures
uint32_t key_prefix_hash(const uint8_t* filename, uint64_t fn);

// Encodes every record's KeyValue line into `out`, partition-major, line order
// inside a partition. d_bounds (2 * nreduce + 1 u64, device): [p] = begin and
// [nreduce + p] = end byte of partition p, [2 * nreduce] = total bytes. Lines
// past out_cap are not written. With scratch == nullptr or *scratch_bytes too
// small, only sets *scratch_bytes to the size needed.
hipError_t encode_partitions(const EncodeArgs& a, void* scratch, size_t* scratch_bytes, uint8_t* out,
                             uint64_t out_cap, uint64_t* d_bounds, hipStream_t s);

}  // namespace dgrep
