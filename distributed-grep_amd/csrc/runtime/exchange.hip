// exchange.hip — the multi-GPU exchange of the Map hot path (C ABI, RCCL).
//
// The reference ships each map task's output to the reducers by SFTP
// (map_reduce/coordinator.go:136-142, called per finished map task). On one
// node the workers' splits are scanned on their own GPUs, and only the
// compacted match records -- never line bytes -- travel to the reducing
// worker over RCCL (xGMI): SURVEY.md §8e. RCCL has no gatherv, so
//   1. the per-rank counts are all-gathered (one u64 per rank);
//   2. each rank packs its records into 28-B records {u64 line_no, u64 start,
//      u64 len, u32 split} on its device (one thread per record);
//   3. one ncclGroupStart/End holds a send per non-empty rank and the root's
//      matching receives, straight into one buffer in rank order: exactly
//      sum(counts) x 28 bytes cross xGMI, each sender on its own link.
// The root is the only rank that needs the counts on the host (to size and
// place its receives). Same record layout as dgrep/dist.py (the torch path).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/dgrep.h"

namespace dgrep {
int ctx_device(const dgrep_ctx* c);
hipStream_t ctx_stream(const dgrep_ctx* c);
}  // namespace dgrep

constexpr uint32_t kRecWords = 7;  // u32 words per packed record (28 B)

struct dgrep_comm {
  dgrep_ctx* ctx = nullptr;
  int device = 0, nranks = 1, rank = 0;
  ncclComm_t nccl = nullptr;
  uint64_t* d_counts = nullptr;  // [nranks] all-gathered counts; [nranks] = this rank's count
  uint32_t* d_pack = nullptr;    // this rank's packed records
  uint64_t pack_cap = 0;         // records
  uint32_t* d_recv = nullptr;    // root: every rank's packed records, rank order
  uint64_t recv_cap = 0;         // records
  std::vector<uint64_t> counts;
  std::string err;
};

namespace {

__global__ void pack_records_kernel(const uint64_t* __restrict__ line_no, const uint64_t* __restrict__ start,
                                    const uint64_t* __restrict__ len, uint64_t count, uint32_t split,
                                    uint32_t* __restrict__ out) {
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < count;
       i += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t a = line_no[i], b = start[i], c = len[i];
    uint32_t* o = out + i * kRecWords;
    o[0] = uint32_t(a);
    o[1] = uint32_t(a >> 32);
    o[2] = uint32_t(b);
    o[3] = uint32_t(b >> 32);
    o[4] = uint32_t(c);
    o[5] = uint32_t(c >> 32);
    o[6] = split;
  }
}

// the rank's count into device memory, in stream order (no pageable copy)
__global__ void put_count_kernel(uint64_t* dst, uint64_t v) { *dst = v; }

int fail(dgrep_comm* m, const std::string& what) {
  m->err = what;
  return DGREP_E_HIP;
}
#define HIPC(expr)                                                                    \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess) return fail(m, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)
#define NCCLC(expr)                                                                       \
  do {                                                                                    \
    ncclResult_t r_ = (expr);                                                             \
    if (r_ != ncclSuccess) return fail(m, std::string(#expr ": ") + ncclGetErrorString(r_)); \
  } while (0)

int grow(dgrep_comm* m, uint32_t** p, uint64_t* cap, uint64_t records) {
  if (*cap >= records && *p) return DGREP_OK;
  if (*p) HIPC(hipFree(*p));
  *p = nullptr;
  const uint64_t n = records + records / 8 + 1024;
  HIPC(hipMalloc(reinterpret_cast<void**>(p), n * kRecWords * 4));
  *cap = n;
  return DGREP_OK;
}

}  // namespace

extern "C" int dgrep_comm_unique_id(void* id_out) {
  if (!id_out) return DGREP_E_INVALID;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return DGREP_E_HIP;
  static_assert(sizeof(id) == DGREP_COMM_ID_BYTES, "RCCL unique id size");
  memcpy(id_out, &id, sizeof id);
  return DGREP_OK;
}

extern "C" int dgrep_comm_open(dgrep_ctx* ctx, const void* id, int nranks, int rank, dgrep_comm** out) {
  if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) return DGREP_E_INVALID;
  *out = nullptr;
  dgrep_comm* m = new dgrep_comm();
  m->ctx = ctx;
  m->device = dgrep::ctx_device(ctx);
  m->nranks = nranks;
  m->rank = rank;
  m->counts.assign(size_t(nranks), 0);
  *out = m;  // kept on failure too, so the caller can read the message
  HIPC(hipSetDevice(m->device));
  HIPC(hipMalloc(reinterpret_cast<void**>(&m->d_counts), (size_t(nranks) + 1) * sizeof(uint64_t)));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof uid);
  NCCLC(ncclCommInitRank(&m->nccl, nranks, uid, rank));
  return DGREP_OK;
}

extern "C" void dgrep_comm_close(dgrep_comm* m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  if (m->nccl) (void)ncclCommDestroy(m->nccl);
  if (m->d_counts) (void)hipFree(m->d_counts);
  if (m->d_pack) (void)hipFree(m->d_pack);
  if (m->d_recv) (void)hipFree(m->d_recv);
  delete m;
}

extern "C" int dgrep_gather_records_device(dgrep_comm* m, const uint64_t* d_line_no, const uint64_t* d_start,
                                           const uint64_t* d_len, uint64_t count, uint32_t split, int root,
                                           const void** d_records, uint64_t* total, uint64_t* rank_counts) {
  if (!m || !d_records || !total || root < 0 || root >= m->nranks || (count && (!d_line_no || !d_start || !d_len)))
    return DGREP_E_INVALID;
  *d_records = nullptr;
  *total = 0;
  HIPC(hipSetDevice(m->device));
  const hipStream_t s = dgrep::ctx_stream(m->ctx);
  int rc;
  // 1. counts: this rank's in slot [nranks], all-gathered into [0, nranks)
  hipLaunchKernelGGL(put_count_kernel, dim3(1), dim3(1), 0, s, m->d_counts + m->nranks, count);
  HIPC(hipGetLastError());
  NCCLC(ncclAllGather(m->d_counts + m->nranks, m->d_counts, 1, ncclUint64, m->nccl, s));
  // 2. pack
  if (count) {
    if ((rc = grow(m, &m->d_pack, &m->pack_cap, count)) != DGREP_OK) return rc;
    const uint64_t blocks = std::min<uint64_t>((count + 255) / 256, 4096);
    hipLaunchKernelGGL(pack_records_kernel, dim3(uint32_t(blocks)), dim3(256), 0, s, d_line_no, d_start, d_len,
                       count, split, m->d_pack);
    HIPC(hipGetLastError());
  }
  if (m->rank != root) {
    // 3. send, grouped like the root's receives (and like the torch path,
    // dgrep/dist.py: batch_isend_irecv on both sides)
    if (count) {
      NCCLC(ncclGroupStart());
      NCCLC(ncclSend(m->d_pack, count * kRecWords, ncclUint32, root, m->nccl, s));
      NCCLC(ncclGroupEnd());
    }
    HIPC(hipStreamSynchronize(s));
    *total = count;
    return DGREP_OK;
  }
  // root: the counts on the host place the receives
  HIPC(hipMemcpyAsync(m->counts.data(), m->d_counts, size_t(m->nranks) * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  uint64_t sum = 0;
  for (uint64_t c : m->counts) sum += c;
  if ((rc = grow(m, &m->d_recv, &m->recv_cap, sum)) != DGREP_OK) return rc;
  NCCLC(ncclGroupStart());
  uint64_t off = 0;
  for (int p = 0; p < m->nranks; ++p) {
    const uint64_t c = m->counts[size_t(p)];
    if (c && p == m->rank) {
      HIPC(hipMemcpyAsync(m->d_recv + off * kRecWords, m->d_pack, c * kRecWords * 4, hipMemcpyDeviceToDevice, s));
    } else if (c) {
      NCCLC(ncclRecv(m->d_recv + off * kRecWords, c * kRecWords, ncclUint32, p, m->nccl, s));
    }
    off += c;
  }
  NCCLC(ncclGroupEnd());
  HIPC(hipStreamSynchronize(s));
  *d_records = m->d_recv;
  *total = sum;
  if (rank_counts) memcpy(rank_counts, m->counts.data(), size_t(m->nranks) * sizeof(uint64_t));
  return DGREP_OK;
}

extern "C" int dgrep_gather_records(dgrep_comm* m, const uint64_t* d_line_no, const uint64_t* d_start,
                                    const uint64_t* d_len, uint64_t count, uint32_t split, int root,
                                    dgrep_gathered* out) {
  if (!out) return DGREP_E_INVALID;
  memset(out, 0, sizeof *out);
  const void* d = nullptr;
  uint64_t total = 0;
  int rc = dgrep_gather_records_device(m, d_line_no, d_start, d_len, count, split, root, &d, &total, nullptr);
  if (rc != DGREP_OK || m->rank != root || total == 0) return rc;
  std::vector<uint32_t> w(total * kRecWords);
  const hipStream_t s = dgrep::ctx_stream(m->ctx);
  HIPC(hipMemcpyAsync(w.data(), d, w.size() * 4, hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  out->line_no = static_cast<uint64_t*>(malloc(total * 8));
  out->start = static_cast<uint64_t*>(malloc(total * 8));
  out->len = static_cast<uint64_t*>(malloc(total * 8));
  out->split = static_cast<uint32_t*>(malloc(total * 4));
  if (!out->line_no || !out->start || !out->len || !out->split) {
    dgrep_gathered_free(out);
    return DGREP_E_NOMEM;
  }
  for (uint64_t i = 0; i < total; ++i) {
    const uint32_t* r = w.data() + i * kRecWords;
    out->line_no[i] = uint64_t(r[0]) | (uint64_t(r[1]) << 32);
    out->start[i] = uint64_t(r[2]) | (uint64_t(r[3]) << 32);
    out->len[i] = uint64_t(r[4]) | (uint64_t(r[5]) << 32);
    out->split[i] = r[6];
  }
  out->count = total;
  return DGREP_OK;
}

extern "C" void dgrep_gathered_free(dgrep_gathered* g) {
  if (!g) return;
  free(g->line_no);
  free(g->start);
  free(g->len);
  free(g->split);
  memset(g, 0, sizeof *g);
}

// message of the communicator's last failure
extern "C" const char* dgrep_comm_last_error(dgrep_comm* m) { return m ? m->err.c_str() : "null communicator"; }
