// pattern_ceiling.hip -- the HBM read rate of the scan kernels' ACCESS PATTERN
// alone (no DFA), next to a coalesced streaming read, on the same split sizes:
// what fraction of its own pattern's ceiling the Sheng scan (C2) reaches.
//   coalesced  : each wave-instruction reads 1 KiB contiguous (16 B per lane)
//   lanechunk  : the scan's shape -- a tile is ONE wave's 64 lane chunks of C
//                bytes, 128-B blocks per lane (8 x 16 B), the next block loaded
//                while the current one is consumed, 256-thread workgroups with
//                53 KiB of LDS (3 per CU, as the Sheng kernel), the first tile
//                by index and later ones claimed from a counter
// Build: hipcc -O3 --offload-arch=gfx950 tools/pattern_ceiling.hip -o tools/pattern_ceiling
// Run:   tools/pattern_ceiling [GiB ...]     (prints one line per size and kernel)
//        env PC_LDS (LDS bytes per workgroup), PC_C (lane chunk), PC_DEPTH (128-B blocks in flight, 1-3)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int kThreads = 256;
constexpr int kLds = 53248;  // the Sheng scan kernel's LDS: 3 workgroups per CU

__global__ void fill_kernel(uint4* d, uint64_t n16) {
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x)
    d[i] = make_uint4(uint32_t(i), uint32_t(i >> 32), 0x0a0a0a0au, 0x61626364u);
}

__global__ __launch_bounds__(kThreads) void coalesced(const uint4* __restrict__ d, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * kThreads) {
    const uint4 v = d[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int DEPTH>
__global__ __launch_bounds__(kThreads, 3) void lanechunk(const uint8_t* __restrict__ d, uint64_t n, uint32_t C,
                                                        unsigned long long* next, uint32_t* out) {
  extern __shared__ uint32_t pad[];  // kLds bytes at launch: 3 workgroups per CU
  if (threadIdx.x == 0) pad[0] = 0;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t tile = 64ull * C, ntiles = n / tile;
  const uint64_t waves = uint64_t(gridDim.x) * (kThreads / 64);
  uint32_t acc = pad[0];
  for (uint64_t t = uint64_t(blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6); t < ntiles;) {
    const uint4* p = reinterpret_cast<const uint4*>(d + t * tile + uint64_t(lane) * C);
    // DEPTH blocks of 128 B in flight ahead of the one being consumed
    uint4 Q[DEPTH + 1][8];
#pragma unroll
    for (int k = 0; k < DEPTH; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) Q[k][i] = p[k * 8 + i];
    const uint32_t nb = C / 128;
    for (uint32_t b = 0; b < nb; ++b) {
      const uint32_t nx = b + DEPTH < nb ? b + DEPTH : nb - 1;
#pragma unroll
      for (int i = 0; i < 8; ++i) Q[DEPTH][i] = p[nx * 8 + i];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc ^= Q[0][i].x ^ Q[0][i].y ^ Q[0][i].z ^ Q[0][i].w;
#pragma unroll
      for (int k = 0; k < DEPTH; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i) Q[k][i] = Q[k + 1][i];
    }
    uint64_t c = 0;
    if (lane == 0) c = atomicAdd(next, 1ull);
    t = waves + ((uint64_t(uint32_t(__shfl(uint32_t(c >> 32), 0, 64))) << 32) | uint32_t(__shfl(uint32_t(c), 0, 64)));
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int occ = 0;
  const size_t lds = argc > 1 && getenv("PC_LDS") ? size_t(atoi(getenv("PC_LDS"))) : size_t(kLds);
  const int depth = getenv("PC_DEPTH") ? atoi(getenv("PC_DEPTH")) : 1;
  auto kern = depth == 2 ? lanechunk<2> : depth == 3 ? lanechunk<3> : lanechunk<1>;
  CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, kThreads, lds));
  const uint32_t C = getenv("PC_C") ? uint32_t(atoi(getenv("PC_C"))) : 32768u;
  double maxg = 0;
  for (int a = 1; a < argc; ++a) maxg = atof(argv[a]) > maxg ? atof(argv[a]) : maxg;
  if (argc < 2) maxg = 16;
  const uint64_t cap = uint64_t(maxg * (1ull << 30));
  uint8_t* d = nullptr;
  uint32_t* out = nullptr;
  unsigned long long* next = nullptr;
  CHK(hipMalloc(&d, cap));
  CHK(hipMalloc(&out, 4));
  CHK(hipMalloc(&next, 8));
  hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint4*>(d), cap / 16);
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int a = (argc < 2 ? 0 : 1); a < (argc < 2 ? 1 : argc); ++a) {
    const double g = argc < 2 ? 16.0 : atof(argv[a]);
    const uint64_t n = uint64_t(g * (1ull << 30)) / (64ull * C) * (64ull * C);
    for (int k = 0; k < 2; ++k) {
      float best = 1e30f, sum = 0.f;
      const int reps = 8;
      for (int r = 0; r < reps + 2; ++r) {
        CHK(hipMemset(next, 0, 8));
        CHK(hipEventRecord(e0, 0));
        if (k == 0)
          hipLaunchKernelGGL(coalesced, dim3(cus * 8), dim3(kThreads), 0, 0, reinterpret_cast<const uint4*>(d), n / 16,
                             out);
        else
          hipLaunchKernelGGL(kern, dim3(cus * occ), dim3(kThreads), lds, 0, d, n, C, next, out);
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) {
          sum += ms;
          best = ms < best ? ms : best;
        }
      }
      printf("%-10s C=%u depth=%d gib=%.1f occ=%d avg_ms=%.3f GB/s=%.0f frac=%.4f best_GB/s=%.0f\n", k ? "lanechunk" : "coalesced", C, depth, g,
             occ, sum / reps, n / (sum / reps * 1e-3) / 1e9, n / (sum / reps * 1e-3) / 8e12, n / (best * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
  return 0;
}
