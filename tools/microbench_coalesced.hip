// microbench_coalesced.hip — ablation micro-benchmark for a COALESCED scan
// layout (not part of the product). Per step a wave reads 64 x W contiguous
// bytes, lane i the W bytes at i*W, and keeps D steps in flight in registers.
//   S<W,D>  streaming only (xor of every word): the access ceiling of the layout
//   M<W,D>  + per-lane 8-state transition map of its W bytes (2 v_perm per byte,
//           one ds_read_b64 per byte) and a DPP wave scan composing the maps
//           (Hillis-Steele, 6 steps), exclusive shift, carry to the next step
//   G<W,D>  the whole fast path (see piece_g); Gb with a sched_barrier per word
//   F<W,D>  M + SWAR newline mask / count and the per-byte START_M test with a
//           never-taken branch (everything the product's word step does)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench_coalesced.hip -o tools/microbench_coalesced
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                                  \
  do {                                                                                          \
    hipError_t e = (x);                                                                         \
    if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
  } while (0)

constexpr int kT = 256;
constexpr uint64_t kTile = 256 * 1024;
constexpr uint32_t kIdLo = 0x03020100u, kIdHi = 0x07060504u;

__device__ __forceinline__ uint32_t nl_mask(uint32_t w) {
  uint32_t x = w ^ 0x0a0a0a0au;
  uint32_t t = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;
  return ~t & 0x80808080u;
}
__device__ __forceinline__ uint32_t sel(uint2 v, uint32_t s) { return __builtin_amdgcn_perm(v.y, v.x, s); }

// x <- x o y (y applied first)
__device__ __forceinline__ void comp(uint32_t& lo, uint32_t& hi, uint32_t ylo, uint32_t yhi) {
  const uint32_t nlo = __builtin_amdgcn_perm(hi, lo, ylo);
  const uint32_t nhi = __builtin_amdgcn_perm(hi, lo, yhi);
  lo = nlo;
  hi = nhi;
}
#define SCAN_STEP(CTRL, RM)                                                                      \
  {                                                                                              \
    const uint32_t ylo = __builtin_amdgcn_update_dpp(kIdLo, lo, CTRL, RM, 0xf, false);          \
    const uint32_t yhi = __builtin_amdgcn_update_dpp(kIdHi, hi, CTRL, RM, 0xf, false);          \
    comp(lo, hi, ylo, yhi);                                                                      \
  }

template <int MODE, int L>
__device__ __forceinline__ void piece(const uint2* V, const uint4 (&v)[L], uint32_t M, uint32_t& acc, uint32_t& cin,
                                      uint32_t* flag) {
  if (MODE == 0) {
#pragma unroll
    for (int l = 0; l < L; ++l) acc ^= v[l].x ^ v[l].y ^ v[l].z ^ v[l].w;
    return;
  }
  uint32_t lo = kIdLo, hi = kIdHi, nlc = 0;
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const uint32_t w4[4] = {v[l].x, v[l].y, v[l].z, v[l].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t x = w4[j];
      const uint2 m0 = V[x & 0xffu], m1 = V[(x >> 8) & 0xffu], m2 = V[(x >> 16) & 0xffu], m3 = V[x >> 24];
      const uint32_t l0 = sel(m0, lo), h0 = sel(m0, hi);
      const uint32_t l1 = sel(m1, l0), h1 = sel(m1, h0);
      const uint32_t l2 = sel(m2, l1), h2 = sel(m2, h1);
      const uint32_t l3 = sel(m3, l2), h3 = sel(m3, h2);
      if (MODE >= 2) {
        const uint32_t m = nl_mask(x);
        nlc += __popc(m);
        if (__builtin_expect(((l0 & 0xffu) == M) | ((l1 & 0xffu) == M) | ((l2 & 0xffu) == M) | ((l3 & 0xffu) == M),
                             0))
          atomicAdd(flag, 1u);
      }
      lo = l3;
      hi = h3;
    }
  }
  // inclusive wave scan of the maps: row_shr 1,2,4,8 then row_bcast 15, 31
  SCAN_STEP(0x111, 0xf)
  SCAN_STEP(0x112, 0xf)
  SCAN_STEP(0x114, 0xf)
  SCAN_STEP(0x118, 0xf)
  SCAN_STEP(0x142, 0xa)
  SCAN_STEP(0x143, 0xc)
  const uint32_t elo = __builtin_amdgcn_update_dpp(kIdLo, lo, 0x138, 0xf, 0xf, false);  // wave_shr:1
  const uint32_t ehi = __builtin_amdgcn_update_dpp(kIdHi, hi, 0x138, 0xf, 0xf, false);
  const uint32_t e = __builtin_amdgcn_perm(ehi, elo, cin) & 0xffu;
  acc += e + nlc;
  cin = __builtin_amdgcn_perm(__builtin_amdgcn_readlane(hi, 63), __builtin_amdgcn_readlane(lo, 63), cin) & 0xffu;
}


// G: everything the product's coalesced fast path does per piece, branch-free
// in the word loop: map (2 perm/byte), newline mask/count, event-candidate flag,
// capture of the map at the word holding the first '\n', last '\n' position;
// then the three wave scans (map compose, '\n' count, last-'\n' max) and the
// exact replay of the first line's end. `SB` adds a sched_barrier per word.
template <int L, int FEAT>
__device__ __forceinline__ void piece_g(const uint2* V, const uint4 (&v)[L], const uint8_t* pp, uint32_t M,
                                        uint32_t& acc, uint32_t& cin, uint32_t& nlcar, int32_t& lastcar,
                                        uint32_t* flag) {
  uint32_t lo = kIdLo, hi = kIdHi, nlc = 0, cap_lo = kIdLo, cap_hi = kIdHi, cap_j = 0, cap_x = 0, lastm = 0, lastj = 0;
  uint32_t seenm = 0;
  uint32_t ev = 0;
  uint32_t w[4 * L];
#pragma unroll
  for (int l = 0; l < L; ++l) { w[4 * l] = v[l].x; w[4 * l + 1] = v[l].y; w[4 * l + 2] = v[l].z; w[4 * l + 3] = v[l].w; }
#pragma unroll
  for (int j = 0; j < 4 * L; ++j) {
    const uint32_t x = w[j];
    const uint2 m0 = V[x & 0xffu], m1 = V[(x >> 8) & 0xffu], m2 = V[(x >> 16) & 0xffu], m3 = V[x >> 24];
    const uint32_t m = nl_mask(x);
    if (FEAT & 4) {
      // seenm: all ones once a '\n' was seen; the capture keeps the map, the
      // word and its index from before that word (bit-select, no predicate)
      cap_lo = ((cap_lo & seenm) | (lo & ~seenm));
      cap_hi = (cap_hi & seenm) | (hi & ~seenm);
      cap_x = (cap_x & seenm) | (x & ~seenm);
      cap_j = (cap_j & seenm) | (uint32_t(j) & ~seenm);
      seenm |= uint32_t(int32_t(0u - m) >> 31);
    }
    const uint32_t l0 = sel(m0, lo), h0 = sel(m0, hi);
    const uint32_t l1 = sel(m1, l0), h1 = sel(m1, h0);
    const uint32_t l2 = sel(m2, l1), h2 = sel(m2, h1);
    const uint32_t l3 = sel(m3, l2), h3 = sel(m3, h2);
    if (FEAT & 2) {
      // byte 0 of l0..l3 gathered into one word, SWAR zero-byte test against M
      const uint32_t g = __builtin_amdgcn_perm(l1, l0, 0x0c0c0400u) | __builtin_amdgcn_perm(l3, l2, 0x04000c0cu);
      const uint32_t z = g ^ (M * 0x01010101u);
      ev |= ~(((z & 0x7f7f7f7fu) + 0x7f7f7f7fu) | z) & 0x80808080u;
    }
    if (FEAT & 1) nlc += __popc(m);
    if (FEAT & 8) if (m) { lastm = m; lastj = uint32_t(j); }
    lo = l3;
    hi = h3;
  }
  SCAN_STEP(0x111, 0xf)
  SCAN_STEP(0x112, 0xf)
  SCAN_STEP(0x114, 0xf)
  SCAN_STEP(0x118, 0xf)
  SCAN_STEP(0x142, 0xa)
  SCAN_STEP(0x143, 0xc)
  const uint32_t elo = __builtin_amdgcn_update_dpp(kIdLo, lo, 0x138, 0xf, 0xf, false);
  const uint32_t ehi = __builtin_amdgcn_update_dpp(kIdHi, hi, 0x138, 0xf, 0xf, false);
  const uint32_t e = __builtin_amdgcn_perm(ehi, elo, cin) & 0xffu;
  cin = __builtin_amdgcn_perm(__builtin_amdgcn_readlane(hi, 63), __builtin_amdgcn_readlane(lo, 63), cin) & 0xffu;
  // '\n' count: inclusive sum scan
  uint32_t c = nlc;
  c += __builtin_amdgcn_update_dpp(0u, c, 0x111, 0xf, 0xf, false);
  c += __builtin_amdgcn_update_dpp(0u, c, 0x112, 0xf, 0xf, false);
  c += __builtin_amdgcn_update_dpp(0u, c, 0x114, 0xf, 0xf, false);
  c += __builtin_amdgcn_update_dpp(0u, c, 0x118, 0xf, 0xf, false);
  c += __builtin_amdgcn_update_dpp(0u, c, 0x142, 0xa, 0xf, false);
  c += __builtin_amdgcn_update_dpp(0u, c, 0x143, 0xc, 0xf, false);
  const uint32_t nl_excl = nlcar + c - nlc;
  nlcar += __builtin_amdgcn_readlane(c, 63);
  // last '\n' position: inclusive max scan
  int32_t lp = lastm ? int32_t(4u * lastj + ((31u - __clz(lastm)) >> 3)) : -1;
  int32_t q = lp;
  q = max(q, __builtin_amdgcn_update_dpp(-1, q, 0x111, 0xf, 0xf, false));
  q = max(q, __builtin_amdgcn_update_dpp(-1, q, 0x112, 0xf, 0xf, false));
  q = max(q, __builtin_amdgcn_update_dpp(-1, q, 0x114, 0xf, 0xf, false));
  q = max(q, __builtin_amdgcn_update_dpp(-1, q, 0x118, 0xf, 0xf, false));
  q = max(q, __builtin_amdgcn_update_dpp(-1, q, 0x142, 0xa, 0xf, false));
  q = max(q, __builtin_amdgcn_update_dpp(-1, q, 0x143, 0xc, 0xf, false));
  const int32_t prev = max(lastcar, __builtin_amdgcn_update_dpp(-1, q, 0x138, 0xf, 0xf, false));
  lastcar = max(lastcar, __builtin_amdgcn_readlane(q, 63));
  uint32_t res = e + nl_excl + uint32_t(prev);
  if (FEAT & 4) {
    // replay the word holding the first '\n' from the captured map
    const uint32_t x = cap_x;
    res += cap_j;
    uint32_t s = __builtin_amdgcn_perm(cap_hi, cap_lo, e) & 0xffu;
    const uint32_t f = uint32_t(__builtin_ctz(nl_mask(x))) >> 3;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t t = sel(V[(x >> (8 * k)) & 0xffu], s) & 0xffu;
      s = uint32_t(k) <= f ? t : s;
    }
    res += s & seenm;
  }
  if (__builtin_expect(ev, 0)) atomicAdd(flag, res);
  acc += res;
}

template <int W, int D, int MODE>
__global__ __launch_bounds__(kT) void coal_kernel(const uint8_t* __restrict__ data, uint64_t ntiles, uint32_t M,
                                                  uint32_t* out) {
  constexpr int L = W / 16;
  constexpr uint32_t STEP = 64u * W;
  constexpr uint32_t NS = uint32_t(kTile / STEP);
  static_assert(NS % D == 0, "steps per tile must be a multiple of the depth");
  __shared__ uint2 V[256];
  const int tid = int(threadIdx.x);
  {
    uint32_t a = 0, b = 0;
    for (int s = 0; s < 4; ++s) a |= ((uint32_t(tid) * 37u + uint32_t(s) * 11u + 5u) & 7u) << (8 * s);
    for (int s = 0; s < 4; ++s) b |= ((uint32_t(tid) * 37u + uint32_t(s + 4) * 11u + 5u) & 7u) << (8 * s);
    V[tid] = make_uint2(a, b);
  }
  __syncthreads();
  const int lane = tid & 63;
  uint32_t acc = 0, cin = 0, nlcar = 0;
  int32_t lastcar = -1;
  const uint64_t waves = uint64_t(gridDim.x) * (kT / 64);
  for (uint64_t t = uint64_t(blockIdx.x) * (kT / 64) + uint64_t(tid >> 6); t < ntiles; t += waves) {
    const uint8_t* base = data + t * kTile + uint64_t(lane) * W;
    uint4 buf[D][L];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int l = 0; l < L; ++l) buf[d][l] = *reinterpret_cast<const uint4*>(base + d * STEP + l * 16);
    for (uint32_t s0 = 0; s0 < NS; s0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        uint4 cur[L];
#pragma unroll
        for (int l = 0; l < L; ++l) cur[l] = buf[d][l];
        if (s0 + d + D < NS) {
#pragma unroll
          for (int l = 0; l < L; ++l)
            buf[d][l] = *reinterpret_cast<const uint4*>(base + uint64_t(s0 + d + D) * STEP + l * 16);
        }
        if constexpr (MODE >= 16)
          piece_g<L, MODE - 16>(V, cur, base + uint64_t(s0 + d) * STEP, M, acc, cin, nlcar, lastcar, out + 1);
        else
          piece<MODE, L>(V, cur, M, acc, cin, out + 1);
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

static double run(const char* name, void (*k)(const uint8_t*, uint64_t, uint32_t, uint32_t*), const uint8_t* d,
                  uint64_t n, uint32_t* out, int cus) {
  int bpc = 0;
  CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k, kT, 0));
  hipFuncAttributes fa;
  CHK(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k)));
  const uint64_t ntiles = n / kTile;
  const int grid = int(uint64_t(cus) * bpc < ntiles ? uint64_t(cus) * bpc : ntiles);
  hipLaunchKernelGGL(k, dim3(grid), dim3(kT), 0, 0, d, ntiles, 8u, out);
  CHK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const int reps = 5;
  CHK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(kT), 0, 0, d, ntiles, 8u, out);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  const double gbs = double(ntiles * kTile) * reps / (ms * 1e-3) / 1e9;
  printf("%-10s vgpr=%3d wg/cu=%d  %7.1f GB/s\n", name, fa.numRegs, bpc, gbs);
  fflush(stdout);
  return gbs;
}

__global__ void fill(uint8_t* d, uint64_t n) {
  for (uint64_t i = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) * 8; i < n; i += uint64_t(gridDim.x) * blockDim.x * 8) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z ^= z >> 29;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 32;
    uint64_t w = 0;
    for (int k = 0; k < 8; ++k) {
      const uint32_t r = uint32_t(z >> (8 * k)) & 0xffu;
      const uint32_t c = r < 3 ? '\n' : 0x20u + (r % 95u);
      w |= uint64_t(c) << (8 * k);
    }
    *reinterpret_cast<uint64_t*>(d + i) = w;
  }
}

#define RUN(NAME, W, D, MODE) run(NAME, coal_kernel<W, D, MODE>, d, n, out, cus)

int main(int argc, char** argv) {
  const uint64_t n = uint64_t(argc > 1 ? atoi(argv[1]) : 8) << 30;
  uint8_t* d;
  uint32_t* out;
  CHK(hipMalloc(&d, n));
  CHK(hipMalloc(&out, 64));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, d, n);
  CHK(hipDeviceSynchronize());
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  printf("--- coalesced layouts, n=%.1f GiB, %d CUs\n", double(n) / (1 << 30), cus);
  RUN("S64x2", 64, 2, 0);
  RUN("M64x2", 64, 2, 1);
  RUN("M64x4", 64, 4, 1);
  RUN("G64x2f0", 64, 2, 16);
  RUN("G64x2f1", 64, 2, 17);
  RUN("G64x2f2", 64, 2, 18);
  RUN("G64x2f4", 64, 2, 20);
  RUN("G64x2f8", 64, 2, 24);
  RUN("G64x2f3", 64, 2, 19);
  RUN("G64x2f11", 64, 2, 27);
  RUN("G64x2f15", 64, 2, 31);
  RUN("G32x4f15", 32, 4, 31);
  RUN("G32x2f15", 32, 2, 31);
  return 0;
}
