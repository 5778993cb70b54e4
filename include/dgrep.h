/*
 * dgrep.h — C ABI of libdgrep.so, the MI355X-native Map hot path of
 * distributed-grep (bgilby59/distributed-grep).
 *
 * The reference path being replaced is the body of the grep plugin's Map:
 *
 *   application/grep.go:13-36
 *     lines := strings.Split(contents, "\n")                 // grep.go:17
 *     for line_number, line := range lines {                 // grep.go:20
 *         matched, _ := regexp.Match(pattern, []byte(line))  // grep.go:21
 *         if matched {                                       // grep.go:24-29
 *             k := fmt.Sprintf("%s (line number #%v)", filename, line_number+1)
 *             kva = append(kva, KeyValue{Key: k, Value: line})
 *
 * A cgo-built Map binds exactly these entry points: it
 * compiles `pattern` once (dgrep_compile -> dgrep_load_dfa, replacing the
 * per-line regexp.Compile inside regexp.Match at grep.go:21), scans the split
 * on the GPU (dgrep_scan, replacing grep.go:17-24), and rebuilds each
 * KeyValue on the host from (line_no, start, len): Key = Sprintf(filename,
 * line_no), Value = contents[start:start+len] (grep.go:25-28). Reduce
 * (grep.go:38-40) is unchanged.
 *
 * Conventions: every function returns an int status (DGREP_OK = 0). The
 * library borrows `data` only for the duration of a call; result arrays are
 * owned by the library until dgrep_result_free. Each entry point sets the
 * context's HIP device, so a Go goroutine may migrate between OS threads.
 * One context per device stream; contexts share no mutable state.
 */
#ifndef DGREP_H
#define DGREP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  DGREP_OK = 0,
  DGREP_E_INVALID = 1,     /* bad argument / malformed blob */
  DGREP_E_UNSUPPORTED = 2, /* valid Go regexp outside the compiler's subset: refuse, never guess */
  DGREP_E_TOO_LARGE = 3,   /* automaton exceeds the compiler's state budget */
  DGREP_E_HIP = 4,         /* HIP runtime error (message in dgrep_last_error) */
  DGREP_E_NOMEM = 5,
  DGREP_E_NO_DFA = 6,      /* scan before dgrep_load_dfa */
};

/* Flags carried in a compiled blob (dgrep_blob_info). */
enum {
  DGREP_DFA_GO_SYNTAX_ERROR = 1u << 0, /* Go's regexp.Compile rejects the pattern: no line matches (grep.go:21 drops err) */
  DGREP_DFA_MATCH_NONE = 1u << 1,      /* no line can match */
  DGREP_DFA_MATCH_ALL = 1u << 2,       /* every line matches (e.g. the shipped pattern "" at grep.go:11) */
  DGREP_DFA_PARTIAL = 1u << 3,         /* DFA beyond the state budget: first states + CAND + NFA program (dgrep_blob.h) */
};

typedef struct dgrep_ctx dgrep_ctx;

/* Matching lines of one split, ascending line order (grep.go:20 iteration
 * order). line_no is 1-based (grep.go:25 `line_number+1`); start/len index
 * the split's bytes; the line excludes its '\n' (strings.Split). len is 64-bit:
 * a Go string (and so a line of one) may be longer than 4 GiB. */
typedef struct {
  uint64_t count;
  uint64_t* line_no;
  uint64_t* start;
  uint64_t* len;
} dgrep_result;

typedef struct {
  uint32_t flags;
  uint32_t nstates;  /* minimized DFA states */
  uint32_t nclasses; /* byte equivalence classes */
  uint32_t start;
  uint32_t start_m;  /* the state entered by a '\n' that ends a matching line */
} dgrep_blob_info;

/* ---- pattern compiler (host only, no GPU needed) ------------------------ */
/* Replaces regexp.Compile(pattern) inside regexp.Match (grep.go:21) with Go
 * regexp/syntax Perl-flag semantics. A pattern Go rejects still returns
 * DGREP_OK with a blob flagged DGREP_DFA_GO_SYNTAX_ERROR|MATCH_NONE, because
 * the reference discards the error and matches nothing. `err` (optional)
 * receives a message for non-OK results. */
int dgrep_compile(const char* pattern, size_t n, void** blob, size_t* blob_len, char* err, size_t errlen);
/* Tests only: dgrep_compile with the DFA state budget lowered to state_budget
 * (0 = the default 2^21; values below 3 are ignored), so that the partial-blob
 * path (DGREP_DFA_PARTIAL) can be exercised with small patterns. */
int dgrep_compile_budget(const char* pattern, size_t n, uint32_t state_budget, void** blob, size_t* blob_len,
                         char* err, size_t errlen);
void dgrep_blob_free(void* blob);
/* Validates the whole blob (header, byte classes, every transition, and the
 * NFA program of a partial blob word by word) before reporting its header:
 * DGREP_E_INVALID if anything would index out of range. dgrep_load_dfa
 * calls it first. */
int dgrep_blob_info_get(const void* blob, size_t n, dgrep_blob_info* info);

/* ---- device context ------------------------------------------------------ */
/* The worker's device (map_reduce/worker.go:126-145 runs one map task at a
 * time per worker process, one file per task, coordinator.go:312,329-333): the
 * DGREP_DEVICE environment variable if set, else worker_id % device_count, where
 * a negative worker_id means the DGREP_WORKER_ID environment variable, else the
 * process id (the Go plugin has no worker id: WorkerID stays inside the RPC
 * reply, worker.go:144). A device that is not present -- DGREP_DEVICE=99 on an
 * 8-GPU node, or no GPU at all -- is DGREP_E_HIP; a DGREP_DEVICE that is not a
 * non-negative integer is DGREP_E_INVALID. */
int dgrep_pick_device(int worker_id, int* device);
int dgrep_open(int device, dgrep_ctx** ctx);
void dgrep_close(dgrep_ctx* ctx);
const char* dgrep_last_error(dgrep_ctx* ctx);
/* Use an existing hipStream_t (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL selects the context's own stream. */
int dgrep_set_stream(dgrep_ctx* ctx, void* hip_stream);
int dgrep_load_dfa(dgrep_ctx* ctx, const void* blob, size_t n);
/* Stepper selection for later dgrep_load_dfa calls (tests / tuning only; the
 * default picks by size: <= 8 states Sheng; else the pair stepper if its
 * two-byte table fits in LDS; else <= 256 states the u8 table; else the
 * filter: the DFA's shallowest states in LDS, lines that leave them verified
 * on the whole DFA).
 * force: 0 = that default, 2 = the u8 table (<= 256 states), 3 = pair
 * (dgrep_load_dfa fails with DGREP_E_UNSUPPORTED if it does not fit), 4 =
 * filter (the default above 256 states). 1 and 5 (the wide and word steppers
 * of earlier rounds, measured slower and removed) and anything outside 0-5 are
 * DGREP_E_INVALID. filter_rows != 0 caps the filter's LDS-resident rows (its
 * cut then sends nearly every line to verification). */
int dgrep_set_stepper(dgrep_ctx* ctx, int force, uint32_t filter_rows);
/* Tests / tuning: lane chunk of the Sheng (<= 8-state), pair and filter
 * steppers for later scans. 0 (default) = adaptive: the compiled chunk (4 KiB;
 * pair 4.5 KiB), doubled while every resident wave still gets a tile and the
 * matching lines the previous scan's density predicts fill at most a quarter
 * of a lane's record capacity, up to 32 KiB (Sheng), 64 KiB (filter) or 9 KiB (pair). Otherwise a
 * multiple of 128 in [4096, 65536] (the LDS slots hold 16-bit chunk offsets;
 * a line starting exactly at a 64 KiB chunk end is flagged separately);
 * anything else is DGREP_E_INVALID and leaves the setting unchanged. No effect
 * on the u8 table stepper (fixed 2 KiB chunks). */
int dgrep_set_lane_chunk(dgrep_ctx* ctx, uint32_t chunk_bytes);

/* Host bytes -> H2D -> scan -> D2H results. This is the call Map makes.
 * The H2D leg is the worker's split ingest (the bytes map_reduce/worker.go:72-76
 * reads with os.ReadFile and passes to Map at worker.go:141): pieces are
 * copied by CPU threads into pinned staging buffers while the copy engine
 * DMAs the previous piece (dgrep_set_ingest). */
int dgrep_scan(dgrep_ctx* ctx, const uint8_t* data, size_t n, dgrep_result* out);
/* Ingest pipeline of dgrep_scan: chunk_bytes per pinned staging buffer
 * (0 = one pageable hipMemcpyAsync, no staging), nbufs buffers in rotation,
 * threads CPU threads per piece copy (0 keeps the current value). Defaults:
 * 64 MiB x 4 buffers x 4 threads. */
int dgrep_set_ingest(dgrep_ctx* ctx, size_t chunk_bytes, int nbufs, int threads);
/* Wall time (ms) of the last dgrep_scan's ingest (host -> HBM), 0 for the
 * direct path. */
int dgrep_last_ingest_ms(dgrep_ctx* ctx, float* ms);
void dgrep_result_free(dgrep_result* r);

/* ---- partition + intermediate writer (map_reduce/worker.go:13-17,78-109) ---
 * The worker's writeMapOutput over one split's Map output, on the GPU: each
 * matching line's KeyValue{Key: Sprintf("%s (line number #%v)", filename,
 * line_no), Value: line} (application/grep.go:25-28) goes to partition
 * ihash(Key) % nreduce (FNV-1a 32 & 0x7fffffff, worker.go:13-17) as the line
 * json.NewEncoder(f).Encode(&kv) writes ({"Key":...,"Value":...}\n, HTML
 * escaping on, invalid UTF-8 as \ufffd, worker.go:92-93), in Map output
 * (line) order inside each partition. Partition p's bytes are
 * bytes[begin[p]:end[p]] -- exactly the content of mr-<task>-<p>. */
typedef struct {
  uint32_t nreduce;
  uint64_t total;   /* bytes over all partitions */
  uint64_t* begin;  /* nreduce byte offsets into bytes */
  uint64_t* end;
  uint8_t* bytes;
} dgrep_partitions;

/* Host split -> ingest -> scan -> encode -> host partitions (the Map +
 * writeMapOutput of one map task). */
int dgrep_map_partitions(dgrep_ctx* ctx, const uint8_t* data, size_t n, const char* filename, size_t fn,
                         uint32_t nreduce, dgrep_partitions* out);
void dgrep_partitions_free(dgrep_partitions* p);
/* Device form over dgrep_scan_device's records: writes into d_out (out_cap
 * bytes; *total receives the bytes needed -- if larger, call again with a
 * bigger buffer); part_begin/part_end are host arrays of nreduce entries. */
int dgrep_encode_device(dgrep_ctx* ctx, const void* d_data, size_t n, const uint64_t* d_line_no,
                        const uint64_t* d_start, const uint64_t* d_len, uint64_t count, const char* filename,
                        size_t fn, uint32_t nreduce, void* d_out, uint64_t out_cap, uint64_t* part_begin,
                        uint64_t* part_end, uint64_t* total);
/* Device time (ms) of the last encode (HIP events on the context stream). */
int dgrep_last_encode_ms(dgrep_ctx* ctx, float* ms);

/* ---- reduce task (map_reduce/worker.go:22-68,161-165; grep.go:38-40) ------
 * One reduce task of the grep job on the GPU: `data` = the concatenated
 * mr-<map>-<r> files of partition r (json.Encoder KeyValue lines, as
 * readReduceInput decodes them); the result is one "key value\n" line
 * (fmt "%v %v\n" of the raw strings) per distinct key with one of its values
 * (the grep Reduce returns values[0] after an unstable sort, so any value of
 * a duplicated key is a valid result), in input order of the kept lines (the
 * reference writes them in Go map order, i.e. unordered). A line that is not a
 * json.Encoder KeyValue line fails with DGREP_E_INVALID (never guessed). */
typedef struct {
  uint64_t lines_in; /* KeyValue lines read */
  uint64_t total;    /* output bytes */
  uint8_t* bytes;    /* the content of mr-out-<r> */
} dgrep_reduce_out;
int dgrep_reduce(dgrep_ctx* ctx, const uint8_t* data, size_t n, dgrep_reduce_out* out);
void dgrep_reduce_free(dgrep_reduce_out* r);

/* HBM-resident split (the data never leaves the device): results are written
 * to caller-provided device arrays of `capacity` entries; *count receives
 * the number of matching lines (if > capacity, nothing beyond capacity is
 * written: call again with a larger capacity). Asynchronous on the context
 * stream except for the 8-byte count readback. */
int dgrep_scan_device(dgrep_ctx* ctx, const void* d_data, size_t n, uint64_t* d_line_no, uint64_t* d_start,
                      uint64_t* d_len, uint64_t capacity, uint64_t* count);

/* ---- multi-GPU exchange -----------------------------------
 * Replaces the SFTP shipping of map output to the reducers
 * (map_reduce/coordinator.go:136-142) for workers on one node: each worker
 * process scans its split on its own GPU and the compacted match records --
 * never the line bytes -- are gathered to the reducing worker over RCCL
 * (xGMI). Callable from the Go worker through cgo like the rest of the ABI.
 * Setup: the root calls dgrep_comm_unique_id and hands the 128 bytes to the
 * other workers out of band (the worker's own channel, e.g. a file or its RPC);
 * every worker then calls dgrep_comm_open with its rank (collective: all
 * nranks must call it). The communicator uses the context's device and stream. */
#define DGREP_COMM_ID_BYTES 128
typedef struct dgrep_comm dgrep_comm;
int dgrep_comm_unique_id(void* id_out /* DGREP_COMM_ID_BYTES */);
int dgrep_comm_open(dgrep_ctx* ctx, const void* id, int nranks, int rank, dgrep_comm** comm);
void dgrep_comm_close(dgrep_comm* comm);
/* Gather every rank's records (a dgrep_scan_device result: `count` entries of
 * the three device arrays) to rank `root`, as 28-byte packed records
 * {u64 line_no, u64 start, u64 len, u32 split} (split = the caller's map task
 * id, so the root can rebuild each Key = Sprintf(filename[split], line_no),
 * application/grep.go:25), in rank order. Collective. The counts are
 * all-gathered first (8 B per rank), then one grouped send/recv moves exactly
 * sum(counts) x 28 bytes into a device buffer the communicator owns (grown as
 * needed): on the root *d_records points at it (valid until the next gather or
 * dgrep_comm_close), *total = sum(counts), and rank_counts (may be NULL)
 * receives the nranks counts. Other ranks: *d_records = NULL, *total = count. */
int dgrep_gather_records_device(dgrep_comm* comm, const uint64_t* d_line_no, const uint64_t* d_start,
                                const uint64_t* d_len, uint64_t count, uint32_t split, int root,
                                const void** d_records, uint64_t* total, uint64_t* rank_counts);
/* The same with host results on the root (SoA, malloc'd; free with
 * dgrep_gathered_free); other ranks get count 0. */
typedef struct {
  uint64_t count;
  uint64_t* line_no;
  uint64_t* start;
  uint64_t* len;
  uint32_t* split;
} dgrep_gathered;
int dgrep_gather_records(dgrep_comm* comm, const uint64_t* d_line_no, const uint64_t* d_start, const uint64_t* d_len,
                         uint64_t count, uint32_t split, int root, dgrep_gathered* out);
void dgrep_gathered_free(dgrep_gathered* g);
/* message for the communicator's last non-OK status (RCCL / HIP error text) */
const char* dgrep_comm_last_error(dgrep_comm* comm);

/* ---- bench / test tooling ------------------------------------------------ */
/* Fill d_out[0:n) with the seeded synthetic log corpus on
 * the device. kind: 0 = plain log lines, 1 = log lines with seeded
 * case-insensitive keywords planted (config 4), 2 = long lines (4 MiB mean)
 * between pages of log lines, 3 = kind 2 after one newline-free 1 GiB line,
 * 4 = kind 2 with config 4's keywords planted (csrc/kernels/synth.h). */
int dgrep_synth_corpus(dgrep_ctx* ctx, void* d_out, size_t n, uint64_t seed, int kind);
/* Host twin of dgrep_synth_corpus (same generator code): fills out[0:n). */
int dgrep_synth_corpus_host(void* out, size_t n, uint64_t seed, int kind);
/* Keyword i (0..999) of the seeded config-4 keyword set; returns its length. */
int dgrep_synth_keyword(uint64_t seed, int i, char* out16);
/* Device time (ms) of the last dgrep_scan* call's scan: the scan kernel
 * (every attempt, if the overflow list had to grow) plus the overflow pass,
 * measured with HIP events on the launch stream. */
int dgrep_last_kernel_ms(dgrep_ctx* ctx, float* ms);
/* dgrep_last_kernel_ms summed over the dgrep_scan_device calls since the
 * previous take (and their number), then reset: a benchmark reads its timed
 * steps' device time once, after them, with no host call between scans. */
int dgrep_take_kernel_ms(dgrep_ctx* ctx, double* sum_ms, uint64_t* scans);

/* What the last dgrep_scan* call did (tests, tuning, bench reports). */
typedef struct {
  uint32_t stepper;        /* 0 u8 table, 1 Sheng (<= 8 states), 3 pair (two bytes per lookup), 4 filter
                              (shallow DFA states in LDS + candidate verification) */
  uint32_t lane_chunk;     /* bytes per lane chunk */
  uint32_t lane_slots;     /* LDS slots per lane chunk for matching lines */
  uint32_t scan_attempts;  /* scan launches (2 if the overflow list had to grow) */
  uint64_t tiles;          /* wave tiles of the split */
  uint64_t overflow_lanes; /* lane chunks re-run by the overflow pass */
  uint64_t matches;        /* matching lines */
  float scan_ms;           /* scan kernel, all attempts */
  float overflow_ms;       /* overflow pass */
  float verify_ms;         /* filter stepper: re-run of the candidate lines on the whole DFA; Sheng: resolution
                              of the parked long lines */
  uint64_t candidates;     /* filter stepper: candidate lines dropped by that re-run */
  uint64_t pending;        /* Sheng: long lines parked by the scan and resolved from chunk maps */
  uint32_t reserved0;      /* round 5's order_in_scan (the in-scan ordering was removed in round 6): 0 */
  uint32_t reserved;
} dgrep_scan_stats;
/* Sized getter: out_size is the caller's sizeof(dgrep_scan_stats). The library
 * writes min(out_size, its own size) bytes, so a binding built against an
 * older (shorter) layout never has bytes written past its struct; a larger
 * caller struct gets its tail zeroed. out_size 0 is DGREP_E_INVALID. The
 * layout above is the round-5 one (80 bytes); fields are only ever appended. */
int dgrep_last_scan_stats(dgrep_ctx* ctx, dgrep_scan_stats* out, size_t out_size);

/* Provenance of this library: "head=<git commit>[-dirty] arch=gfx950
 * hipflags=<tuning -D knobs>" (static string). */
const char* dgrep_build_info(void);

#ifdef __cplusplus
}
#endif
#endif
