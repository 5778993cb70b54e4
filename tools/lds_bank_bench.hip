// lds_bank_bench.hip — LDS gather bank conflicts of the scan's per-byte table
// lookups on the synthetic log corpus (synth.h), one kernel per layout:
//   b32      u32 [256] at 4*b            (Pair UA/UB, Filter classes today)
//   u8       u8 [256] at b               (4 byte values share a dword)
//   u16      u16 [256] at 2*b
//   b64      u64 [256] at 8*b            (Sheng8 V[b] today)
//   b32lp    u32, lane-private banks: b*128 + 4*(lane%32)
//   b64lp    u64, lane-private banks: b*256 + 8*(lane%32)
// Every lane reads its own 4 KiB chunk of the corpus in 16-B pieces and looks
// up each byte R times (R copies of the table, same bank layout), so the LDS,
// not HBM, bounds the kernel. Run alone for times, under rocprofv3 --pmc
// SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE for the conflict cycles.
//   hipcc -O3 --offload-arch=gfx950 -I distributed-grep_amd/csrc/kernels tools/lds_bank_bench.hip -o tools/lds_bank_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "synth.h"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int kNT = 256, kChunk = 4096, kR = 4;

__global__ void synth_k(char* out, uint64_t n, uint64_t seed) {
  const uint64_t pages = (n + dgrep::synth::kPage - 1) / dgrep::synth::kPage;
  for (uint64_t p = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; p < pages; p += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t off = p * dgrep::synth::kPage;
    const uint32_t bytes = uint32_t(n - off < dgrep::synth::kPage ? n - off : dgrep::synth::kPage);
    dgrep::synth::page_fill(seed, p, 0, out + off, bytes);
  }
}

enum Mode { B32, U8, U16, B64, B32LP, B64LP };

template <int MODE>
__device__ __forceinline__ uint32_t look(const uint8_t* lds, uint32_t b, uint32_t lp, int k) {
  if constexpr (MODE == B32) return *reinterpret_cast<const uint32_t*>(lds + k * 1024 + 4 * b);
  if constexpr (MODE == U8) return lds[k * 256 + b];
  if constexpr (MODE == U16) return *reinterpret_cast<const uint16_t*>(lds + k * 512 + 2 * b);
  if constexpr (MODE == B64) {
    const uint2 v = *reinterpret_cast<const uint2*>(lds + k * 2048 + 8 * b);
    return v.x ^ v.y;
  }
  if constexpr (MODE == B32LP) return *reinterpret_cast<const uint32_t*>(lds + ((b ^ uint32_t(k)) << 7) + lp);
  if constexpr (MODE == B64LP) {
    const uint2 v = *reinterpret_cast<const uint2*>(lds + ((b ^ uint32_t(k)) << 8) + lp);
    return v.x ^ v.y;
  }
  return 0;
}

template <int MODE>
constexpr int table_bytes() {
  return MODE == B32 ? 1024 * kR : MODE == U8 ? 256 * kR : MODE == U16 ? 512 * kR : MODE == B64 ? 2048 * kR
         : MODE == B32LP ? 32768 : 65536;
}

template <int MODE>
__global__ __launch_bounds__(kNT) void gather_k(const uint8_t* data, uint64_t n, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[table_bytes<MODE>()];
  for (int i = threadIdx.x; i < table_bytes<MODE>() / 4; i += kNT) reinterpret_cast<uint32_t*>(lds)[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lp = MODE == B32LP ? 4u * (lane & 31u) : 8u * (lane & 31u);
  uint32_t acc = 0;
  const uint64_t lanes = uint64_t(gridDim.x) * kNT;
  for (uint64_t L = blockIdx.x * uint64_t(kNT) + threadIdx.x; L * kChunk < n; L += lanes) {
    const uint4* p = reinterpret_cast<const uint4*>(data + L * kChunk);
    for (int q = 0; q < kChunk / 16; ++q) {
      const uint4 v = p[q];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
#pragma unroll
          for (int k = 0; k < kR; ++k) acc += look<MODE>(lds, (w[j] >> (8 * bb)) & 0xffu, lp, k);
    }
  }
  out[blockIdx.x * kNT + threadIdx.x] = acc;
}

template <int MODE>
float run(const char* name, const uint8_t* d, uint64_t n, uint32_t* out, int grid) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(gather_k<MODE>, dim3(grid), dim3(kNT), 0, 0, d, n, out);
  CK(hipEventRecord(a));
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(gather_k<MODE>, dim3(grid), dim3(kNT), 0, 0, d, n, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= 5;
  const double lookups = double(n) * kR;
  printf("%-6s %8.3f ms  %7.1f G lookups/s  (%.2f lookups/clk/CU at 2.4 GHz)\n", name, ms, lookups / ms / 1e6,
         lookups / (ms * 1e-3) / 2.4e9 / 256);
  return ms;
}

int main(int argc, char** argv) {
  const uint64_t n = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 1ull << 30);
  const char* only = argc > 2 ? argv[2] : nullptr;
  uint8_t* d;
  uint32_t* out;
  CK(hipMalloc(&d, n));
  CK(hipMalloc(&out, 1 << 24));
  hipLaunchKernelGGL(synth_k, dim3(4096), dim3(256), 0, 0, reinterpret_cast<char*>(d), n, 2);
  CK(hipDeviceSynchronize());
  const int grid = 256 * 2;  // 2 workgroups (8 waves) per CU in every mode
  auto want = [&](const char* m) { return !only || !strcmp(only, m); };
  if (want("b32")) run<B32>("b32", d, n, out, grid);
  if (want("u8")) run<U8>("u8", d, n, out, grid);
  if (want("u16")) run<U16>("u16", d, n, out, grid);
  if (want("b64")) run<B64>("b64", d, n, out, grid);
  if (want("b32lp")) run<B32LP>("b32lp", d, n, out, grid);
  if (want("b64lp")) run<B64LP>("b64lp", d, n, out, grid);
  CK(hipDeviceSynchronize());
  return 0;
}
