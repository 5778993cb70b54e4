// microbench_scan.hip — ablation micro-benchmark for the scan kernel's lane
// loop (not part of the product). Each variant streams the same HBM-resident
// text with the product's chunk-per-lane access pattern and adds one cost at a
// time, so the profile of scan_dfa8_kernel can be attributed:
//   V0c  coalesced 16 B/lane streaming read (bandwidth reference)
//   V0   per-lane chunk streaming, 64-B blocks, prefetch 1 block
//   V0b  per-lane chunk streaming, prefetch 2 blocks
//   V1   V0 + DFA step per byte (LDS u8 table, 260-B rows)
//   V2   V1 + SWAR newline count per word
//   V3   V2 + per-word START_M check with a (never taken) branch
//   V4   V2 with NS independent chunk streams interleaved per lane (ILP)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench_scan.hip -o tools/microbench_scan
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                      \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
  } while (0)

constexpr int kT = 256;
constexpr uint32_t kRow = 260;

__device__ __forceinline__ uint32_t nl_mask(uint32_t w) {
  uint32_t x = w ^ 0x0a0a0a0au;
  uint32_t t = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;
  return ~t & 0x80808080u;
}
__device__ __forceinline__ uint32_t step(const uint8_t* tbl, uint32_t s, uint32_t w, uint32_t sel) {
  return tbl[__builtin_amdgcn_perm(s, w, sel) + (s << 2)];
}

struct Smem {
  uint8_t tbl[16 * kRow];
};

template <int MODE>
__device__ __forceinline__ void word(const uint8_t* tbl, uint32_t x, uint32_t& s, uint32_t& acc, uint32_t M,
                                     uint32_t* flag) {
  if (MODE == 0) {
    acc ^= x;
    return;
  }
  const uint32_t s0 = step(tbl, s, x, 0x0c0c0400u);
  const uint32_t s1 = step(tbl, s0, x, 0x0c0c0401u);
  const uint32_t s2 = step(tbl, s1, x, 0x0c0c0402u);
  const uint32_t s3 = step(tbl, s2, x, 0x0c0c0403u);
  if (MODE >= 2) acc += __popc(nl_mask(x));
  if (MODE >= 3) {
    if (__builtin_expect((s0 == M) | (s1 == M) | (s2 == M) | (s3 == M), 0)) atomicAdd(flag, 1u);
  }
  s = s3;
}

template <int MODE, int PF>
__global__ __launch_bounds__(kT) void lane_kernel(const uint8_t* __restrict__ data, uint64_t n, int C,
                                                  const uint8_t* table, uint32_t* out, uint32_t M) {
  __shared__ Smem sm;
  for (int i = threadIdx.x; i < int(sizeof(sm.tbl)); i += kT) sm.tbl[i] = table[i];
  __syncthreads();
  const uint64_t ntiles = n / (uint64_t(kT) * C);
  uint32_t acc = 0, s = 0;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint4* p = reinterpret_cast<const uint4*>(data + t * uint64_t(kT) * C + uint64_t(threadIdx.x) * C);
    const int nb = C / 64;
    uint4 A[4], B[4], D[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) A[i] = p[i];
    if (PF == 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) B[i] = p[4 + i];
    }
    for (int b = 0; b < nb; ++b) {
      if (PF == 1) {
        const int nx = b + 1 < nb ? b + 1 : b;
#pragma unroll
        for (int i = 0; i < 4; ++i) B[i] = p[nx * 4 + i];
      } else {
        const int nx = b + 2 < nb ? b + 2 : b;
#pragma unroll
        for (int i = 0; i < 4; ++i) D[i] = p[nx * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        word<MODE>(sm.tbl, A[i].x, s, acc, M, out + 1);
        word<MODE>(sm.tbl, A[i].y, s, acc, M, out + 1);
        word<MODE>(sm.tbl, A[i].z, s, acc, M, out + 1);
        word<MODE>(sm.tbl, A[i].w, s, acc, M, out + 1);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        A[i] = B[i];
        if (PF == 2) B[i] = D[i];
      }
    }
  }
  out[2 + blockIdx.x * kT + threadIdx.x] = acc ^ s;  // keep live
}

// NS independent streams per lane: lane handles chunks tid and tid + kT*k
template <int NS>
__global__ __launch_bounds__(kT) void multi_kernel(const uint8_t* __restrict__ data, uint64_t n, int C,
                                                   const uint8_t* table, uint32_t* out, uint32_t M) {
  __shared__ Smem sm;
  for (int i = threadIdx.x; i < int(sizeof(sm.tbl)); i += kT) sm.tbl[i] = table[i];
  __syncthreads();
  const uint64_t tile = uint64_t(kT) * C * NS;
  const uint64_t ntiles = n / tile;
  uint32_t acc = 0;
  uint32_t s[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) s[k] = 0;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint4* p[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k)
      p[k] = reinterpret_cast<const uint4*>(data + t * tile + (uint64_t(k) * kT + threadIdx.x) * C);
    const int nb = C / 64;
    uint4 A[NS][4], B[NS][4];
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
      for (int i = 0; i < 4; ++i) A[k][i] = p[k][i];
    for (int b = 0; b < nb; ++b) {
      const int nx = b + 1 < nb ? b + 1 : b;
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) B[k][i] = p[k][nx * 4 + i];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t* wa[NS];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
          for (int k = 0; k < NS; ++k) {
            const uint32_t x = q == 0 ? A[k][i].x : q == 1 ? A[k][i].y : q == 2 ? A[k][i].z : A[k][i].w;
            word<2>(sm.tbl, x, s[k], acc, M, out + 1);
          }
        }
        (void)wa;
      }
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) A[k][i] = B[k][i];
    }
  }
  uint32_t z = acc;
#pragma unroll
  for (int k = 0; k < NS; ++k) z ^= s[k];
  out[2 + blockIdx.x * kT + threadIdx.x] = z;
}

// Sheng-style DFA for <= 8 states: per input byte b an 8-byte vector
// V[b][s] = next state; one v_perm_b32 per byte is the whole dependent chain,
// and the LDS reads of V[b] do not depend on the state (ILP).
template <int MODE>
__global__ __launch_bounds__(kT) void sheng_kernel(const uint8_t* __restrict__ data, uint64_t n, int C,
                                                   const uint2* vtab, uint32_t* out, uint32_t M) {
  __shared__ uint2 V[256];
  for (int i = threadIdx.x; i < 256; i += kT) V[i] = vtab[i];
  __syncthreads();
  const uint64_t ntiles = n / (uint64_t(kT) * C);
  uint32_t acc = 0, s = 0;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint4* p = reinterpret_cast<const uint4*>(data + t * uint64_t(kT) * C + uint64_t(threadIdx.x) * C);
    const int nb = C / 64;
    uint4 A[4], B[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) A[i] = p[i];
    for (int b = 0; b < nb; ++b) {
      const int nx = b + 1 < nb ? b + 1 : b;
#pragma unroll
      for (int i = 0; i < 4; ++i) B[i] = p[nx * 4 + i];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t w4[4] = {A[i].x, A[i].y, A[i].z, A[i].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t x = w4[q];
          const uint2 m0 = V[x & 0xff], m1 = V[(x >> 8) & 0xff], m2 = V[(x >> 16) & 0xff], m3 = V[x >> 24];
          const uint32_t s0 = __builtin_amdgcn_perm(m0.y, m0.x, s);
          const uint32_t s1 = __builtin_amdgcn_perm(m1.y, m1.x, s0);
          const uint32_t s2 = __builtin_amdgcn_perm(m2.y, m2.x, s1);
          const uint32_t s3 = __builtin_amdgcn_perm(m3.y, m3.x, s2);
          if (MODE >= 2) acc += __popc(nl_mask(x));
          if (MODE >= 3) {
            if (__builtin_expect(((s0 & 0xff) == M) | ((s1 & 0xff) == M) | ((s2 & 0xff) == M) | ((s3 & 0xff) == M), 0))
              atomicAdd(out + 1, 1u);
          }
          s = s3;
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) A[i] = B[i];
    }
  }
  out[2 + blockIdx.x * kT + threadIdx.x] = acc ^ s;
}

template <int NS>
__global__ __launch_bounds__(kT) void sheng_multi(const uint8_t* __restrict__ data, uint64_t n, int C,
                                                  const uint2* vtab, uint32_t* out, uint32_t M) {
  __shared__ uint2 V[256];
  for (int i = threadIdx.x; i < 256; i += kT) V[i] = vtab[i];
  __syncthreads();
  const uint64_t tile = uint64_t(kT) * C * NS;
  const uint64_t ntiles = n / tile;
  uint32_t acc = 0;
  uint32_t s[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) s[k] = 0;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint4* p[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k)
      p[k] = reinterpret_cast<const uint4*>(data + t * tile + (uint64_t(k) * kT + threadIdx.x) * C);
    const int nb = C / 64;
    uint4 A[NS][4], B[NS][4];
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
      for (int i = 0; i < 4; ++i) A[k][i] = p[k][i];
    for (int b = 0; b < nb; ++b) {
      const int nx = b + 1 < nb ? b + 1 : b;
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) B[k][i] = p[k][nx * 4 + i];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
          for (int k = 0; k < NS; ++k) {
            const uint32_t x = q == 0 ? A[k][i].x : q == 1 ? A[k][i].y : q == 2 ? A[k][i].z : A[k][i].w;
            const uint2 m0 = V[x & 0xff], m1 = V[(x >> 8) & 0xff], m2 = V[(x >> 16) & 0xff], m3 = V[x >> 24];
            const uint32_t s0 = __builtin_amdgcn_perm(m0.y, m0.x, s[k]);
            const uint32_t s1 = __builtin_amdgcn_perm(m1.y, m1.x, s0);
            const uint32_t s2 = __builtin_amdgcn_perm(m2.y, m2.x, s1);
            const uint32_t s3 = __builtin_amdgcn_perm(m3.y, m3.x, s2);
            acc += __popc(nl_mask(x));
            if (__builtin_expect(((s0 & 0xff) == M) | ((s1 & 0xff) == M) | ((s2 & 0xff) == M) | ((s3 & 0xff) == M), 0))
              atomicAdd(out + 1, 1u);
            s[k] = s3;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) A[k][i] = B[k][i];
    }
  }
  uint32_t z = acc;
#pragma unroll
  for (int k = 0; k < NS; ++k) z ^= s[k];
  out[2 + blockIdx.x * kT + threadIdx.x] = z;
}

// V7/V8: coalesced loads through LDS. Per wave and per round, the 64 lanes'
// next R-byte segments (one per lane chunk, stride C) are fetched with
// global_load_lds_dwordx4: instruction k brings 64/P whole segments (P = R/16
// pieces each, so every instruction reads whole 64/128-B lines) into LDS row
// k; the piece order inside a segment is XOR-rotated by f(q) = (q / (16/P)) % P
// so the per-lane ds_read_b128 of piece j is bank-conflict-free. Single
// buffer: the next round is issued as soon as the lane has its pieces in
// registers.
template <int R, int MODE>
__global__ __launch_bounds__(kT) void glds_kernel(const uint8_t* __restrict__ data, uint64_t n, int C,
                                                  const uint2* vtab, uint32_t* out, uint32_t M) {
  constexpr int P = R / 16, SPI = 64 / P;
  __shared__ __attribute__((aligned(16))) uint8_t stage[kT / 64][64 * R];
  __shared__ uint2 V[256];
  for (int i = threadIdx.x; i < 256; i += kT) V[i] = vtab[i];
  __syncthreads();
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint8_t* st = stage[wv];
  const uint64_t ntiles = n / (64ull * C);
  const uint64_t waves = uint64_t(gridDim.x) * (kT / 64);
  uint32_t acc = 0, s = 0;
  const int lq = lane / P, lp = lane % P;
  const int fl = (lane / (16 / P)) % P;
  for (uint64_t t = uint64_t(blockIdx.x) * (kT / 64) + wv; t < ntiles; t += waves) {
    const uint8_t* tb = data + t * 64ull * C;
    auto issue = [&](int r) {
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int q = k * SPI + lq;
        const int pc = lp ^ ((q / (16 / P)) % P);
        __builtin_amdgcn_global_load_lds((const void*)(tb + uint64_t(q) * C + uint64_t(r) * R + 16 * pc),
                                         (void*)(st + k * 1024), 16, 0, 0);
      }
    };
    issue(0);
    const int nr = C / R;
    for (int r = 0; r < nr; ++r) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      uint4 v[P];
#pragma unroll
      for (int j = 0; j < P; ++j)
        v[j] = *reinterpret_cast<const uint4*>(st + (lane / SPI) * 1024 + 16 * ((lane % SPI) * P + (j ^ fl)));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (r + 1 < nr) issue(r + 1);
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const uint32_t w4[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t x = w4[q];
          if (MODE == 0) {
            acc ^= x;
            continue;
          }
          const uint2 m0 = V[x & 0xff], m1 = V[(x >> 8) & 0xff], m2 = V[(x >> 16) & 0xff], m3 = V[x >> 24];
          const uint32_t s0 = __builtin_amdgcn_perm(m0.y, m0.x, s);
          const uint32_t s1 = __builtin_amdgcn_perm(m1.y, m1.x, s0);
          const uint32_t s2 = __builtin_amdgcn_perm(m2.y, m2.x, s1);
          const uint32_t s3 = __builtin_amdgcn_perm(m3.y, m3.x, s2);
          acc += __popc(nl_mask(x));
          if (__builtin_expect(((s0 & 0xff) == M) | ((s1 & 0xff) == M) | ((s2 & 0xff) == M) | ((s3 & 0xff) == M), 0))
            atomicAdd(out + 1, 1u);
          s = s3;
        }
      }
    }
  }
  out[2 + blockIdx.x * kT + threadIdx.x] = acc ^ s;
}

__global__ void coalesced_kernel(const uint4* __restrict__ d, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x) {
    uint4 v = d[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[2 + blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void fill_kernel(uint8_t* d, uint64_t n) {
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    uint64_t h = i * 0x9e3779b97f4a7c15ull;
    h ^= h >> 29;
    uint8_t c = uint8_t('a' + (h % 26));
    if ((h >> 8) % 120 == 0) c = '\n';
    if ((h >> 16) % 9 == 0) c = ' ';
    d[i] = c;
  }
}

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  f();
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const uint64_t n = uint64_t(argc > 1 ? atoi(argv[1]) : 4) << 30;
  const int C = argc > 2 ? atoi(argv[2]) : 1024;
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t* d;
  uint32_t* out;
  uint8_t* tbl;
  CHK(hipMalloc(&d, n + 4096));
  CHK(hipMalloc(&out, (2 + 8192 * 256) * 4));
  CHK(hipMalloc(&tbl, 16 * kRow));
  fill_kernel<<<4096, 256>>>(d, n);
  // 'error' DFA-like table: 7 states, mostly back to 0
  std::vector<uint8_t> h(16 * kRow, 0);
  const char* pat = "error";
  for (int s = 0; s < 6; ++s)
    for (int b = 0; b < 256; ++b) {
      int nx = (b == pat[0]) ? 1 : 0;
      if (s < 5 && b == pat[s]) nx = s + 1;
      if (s == 5) nx = 5;
      if (b == '\n') nx = (s == 5) ? 6 : 0;
      h[s * kRow + b] = uint8_t(nx);
    }
  for (int b = 0; b < 256; ++b) h[6 * kRow + b] = h[0 * kRow + b];
  CHK(hipMemcpy(tbl, h.data(), h.size(), hipMemcpyHostToDevice));
  std::vector<uint8_t> vt(256 * 8, 0);
  for (int b = 0; b < 256; ++b)
    for (int st = 0; st < 8; ++st) vt[b * 8 + st] = st < 7 ? h[st * kRow + b] : 0;
  uint2* vtab;
  CHK(hipMalloc(&vtab, 256 * 8));
  CHK(hipMemcpy(vtab, vt.data(), vt.size(), hipMemcpyHostToDevice));
  CHK(hipDeviceSynchronize());
  const uint32_t M = 6;
  auto gbs = [&](float ms) { return double(n) / (ms * 1e-3) / 1e9; };
  const int reps = 5;
  if (argc > 3) {
    // glds variants: grid = resident blocks (grid-stride loops must not queue blocks)
    auto run = [&](const char* name, auto kern) {
      int occ = 0;
      CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, kT, 0));
      const int grid = cus * occ;
      float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(kT), 0, 0, d, n, C, vtab, out, M); }, reps);
      printf("%-22s %d WG/CU %8.1f GB/s\n", name, occ, gbs(ms));
    };
    float ms = timeit([&] { coalesced_kernel<<<cus * 8, kT>>>(reinterpret_cast<const uint4*>(d), n / 16, out); }, reps);
    printf("V0c coalesced          %8.1f GB/s\n", gbs(ms));
    run("V5b sheng8+nl+event", sheng_kernel<3>);
    run("V7  glds R=64 xor", glds_kernel<64, 0>);
    run("V7b glds R=128 xor", glds_kernel<128, 0>);
    run("V8  glds R=64 sheng", glds_kernel<64, 1>);
    run("V8b glds R=128 sheng", glds_kernel<128, 1>);
    return 0;
  }
  for (int occ : {4, 6, 8}) {
    const int grid = cus * occ;
    printf("--- grid %d WGs (%d per CU), C=%d, n=%.1f GiB\n", grid, occ, C, n / double(1 << 30));
    float ms;
    ms = timeit([&] { coalesced_kernel<<<grid, kT>>>(reinterpret_cast<const uint4*>(d), n / 16, out); }, reps);
    printf("V0c coalesced        %8.1f GB/s\n", gbs(ms));
    ms = timeit([&] { lane_kernel<0, 1><<<grid, kT>>>(d, n, C, tbl, out, M); }, reps);
    printf("V0  lane stream pf1  %8.1f GB/s\n", gbs(ms));
    ms = timeit([&] { lane_kernel<0, 2><<<grid, kT>>>(d, n, C, tbl, out, M); }, reps);
    printf("V0b lane stream pf2  %8.1f GB/s\n", gbs(ms));
    ms = timeit([&] { lane_kernel<1, 1><<<grid, kT>>>(d, n, C, tbl, out, M); }, reps);
    printf("V1  + DFA            %8.1f GB/s\n", gbs(ms));
    ms = timeit([&] { lane_kernel<1, 2><<<grid, kT>>>(d, n, C, tbl, out, M); }, reps);
    printf("V1b + DFA pf2        %8.1f GB/s\n", gbs(ms));
    ms = timeit([&] { lane_kernel<2, 1><<<grid, kT>>>(d, n, C, tbl, out, M); }, reps);
    printf("V2  + newline SWAR   %8.1f GB/s\n", gbs(ms));
    ms = timeit([&] { lane_kernel<3, 1><<<grid, kT>>>(d, n, C, tbl, out, M); }, reps);
    printf("V3  + event branch   %8.1f GB/s\n", gbs(ms));
    ms = timeit([&] { sheng_kernel<1><<<grid, kT>>>(d, n, C, vtab, out, M); }, reps);
    printf("V5  sheng8 DFA       %8.1f GB/s\n", gbs(ms));
    ms = timeit([&] { sheng_kernel<3><<<grid, kT>>>(d, n, C, vtab, out, M); }, reps);
    printf("V5b sheng8+nl+event  %8.1f GB/s\n", gbs(ms));
    ms = timeit([&] { sheng_multi<2><<<grid, kT>>>(d, n, C, vtab, out, M); }, reps);
    printf("V6  sheng8 x2 streams%8.1f GB/s\n", gbs(ms));
    ms = timeit([&] { multi_kernel<2><<<grid, kT>>>(d, n, C, tbl, out, M); }, reps);
    printf("V4  V2 x2 streams    %8.1f GB/s\n", gbs(ms));
    ms = timeit([&] { multi_kernel<4><<<grid, kT>>>(d, n, C, tbl, out, M); }, reps);
    printf("V4  V2 x4 streams    %8.1f GB/s\n", gbs(ms));
  }
  return 0;
}
