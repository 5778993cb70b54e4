// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE for the scan's access
// patterns (MI355X_MICROARCH.md §HBM: FETCH_SIZE is exact only for wide
// coalesced streaming reads, where it counts half of the bytes; other widths
// are uncalibrated). Each kernel reads exactly n bytes once and is profiled
// on its own (distinct kernel names):
//   coalesced16   : lane i reads 16 B at i*16 of every 1 KiB step (coalesced)
//   lane64_T      : per-lane chunks of C bytes, 64-B blocks (4 x 16 B per lane
//                   per step, the filter/wide/table steppers' pattern), T threads
//   lane128_T     : the same with 128-B blocks (Sheng / pair)
// Build: hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
// Run:   rocprofv3 --pmc FETCH_SIZE --kernel-trace ... -- tools/fetch_calib [GiB] [C]
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

__global__ void fill_kernel(uint4* d, uint64_t n16) {
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x)
    d[i] = make_uint4(uint32_t(i), uint32_t(i >> 32), 0x0a0a0a0au, 0x61626364u);
}

__global__ __launch_bounds__(256) void coalesced16(const uint4* __restrict__ d, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * 256) {
    const uint4 v = d[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// per-lane chunks of C bytes, BK-byte blocks, next block prefetched (the scan
// kernels' run_lane_from shape); tiles of T lanes strided over the grid
template <int BK, int T>
__device__ __forceinline__ void lane_chunks(const uint8_t* __restrict__ d, uint64_t n, uint32_t C, uint32_t* out) {
  constexpr int NV = BK / 16;
  const uint64_t tile = uint64_t(T) * C, ntiles = n / tile;
  uint32_t acc = 0;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint4* p = reinterpret_cast<const uint4*>(d + t * tile + uint64_t(threadIdx.x) * C);
    uint4 A[NV], B[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) A[i] = p[i];
    const uint32_t nb = C / BK;
    for (uint32_t b = 0; b < nb; ++b) {
      const uint32_t nx = b + 1 < nb ? b + 1 : b;
#pragma unroll
      for (int i = 0; i < NV; ++i) B[i] = p[nx * NV + i];
#pragma unroll
      for (int i = 0; i < NV; ++i) acc ^= A[i].x ^ A[i].y ^ A[i].z ^ A[i].w;
#pragma unroll
      for (int i = 0; i < NV; ++i) A[i] = B[i];
    }
  }
  if (acc == 0x12345678u) out[1] = acc;
}
__global__ __launch_bounds__(256) void lane64_256(const uint8_t* d, uint64_t n, uint32_t C, uint32_t* out) {
  lane_chunks<64, 256>(d, n, C, out);
}
__global__ __launch_bounds__(256) void lane128_256(const uint8_t* d, uint64_t n, uint32_t C, uint32_t* out) {
  lane_chunks<128, 256>(d, n, C, out);
}
__global__ __launch_bounds__(1024) void lane64_1024(const uint8_t* d, uint64_t n, uint32_t C, uint32_t* out) {
  lane_chunks<64, 1024>(d, n, C, out);
}
__global__ __launch_bounds__(1024) void lane128_1024(const uint8_t* d, uint64_t n, uint32_t C, uint32_t* out) {
  lane_chunks<128, 1024>(d, n, C, out);
}

int main(int argc, char** argv) {
  const uint64_t n = uint64_t(argc > 1 ? atoi(argv[1]) : 4) << 30;
  const uint32_t C = argc > 2 ? uint32_t(atoi(argv[2])) : 32768;
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t* d;
  uint32_t* out;
  CHK(hipMalloc(&d, n));
  CHK(hipMalloc(&out, 64));
  fill_kernel<<<4096, 256>>>(reinterpret_cast<uint4*>(d), n / 16);
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  auto timed = [&](const char* name, auto launch) {
    launch();  // warm
    CHK(hipEventRecord(e0));
    launch();
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-14s %8.1f GB/s  (bytes read per launch: %llu)\n", name, n / (ms * 1e-3) / 1e9, (unsigned long long)n);
  };
  timed("coalesced16", [&] { coalesced16<<<cus * 8, 256>>>(reinterpret_cast<const uint4*>(d), n / 16, out); });
  timed("lane64_256", [&] { lane64_256<<<cus * 3, 256>>>(d, n, C, out); });
  timed("lane128_256", [&] { lane128_256<<<cus * 3, 256>>>(d, n, C, out); });
  timed("lane64_1024", [&] { lane64_1024<<<cus, 1024>>>(d, n, C, out); });
  timed("lane128_1024", [&] { lane128_1024<<<cus, 1024>>>(d, n, C, out); });
  CHK(hipDeviceSynchronize());
  return 0;
}
