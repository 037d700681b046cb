// Micro-benchmark (not part of the product): what bounds the many-round GF(2^8) scan (C5:
// 5 rounds, wave-uniform coefficients, 2 dwords per lane, 8 waves per CU like k_query's scan
// waves)?  Same loads and v_bitop3 count in every mode; only the mask source differs:
//   MODE 0: s_bfe_i32 per (round, bit) -- the product's form (1 SALU per 2 v_bitop3)
//   MODE 1: one mask for all 40 planes (1 SALU per row; wrong answers: isolates the SALU cost)
//   MODE 2: masks from a 256 x 8-dword table via s_load_dwordx8 (1 SMEM per round)
//   MODE 3: HBM only (one XOR per dword)
// Build: hipcc -O3 --offload-arch=gfx950 -o scan_salu scan_salu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint32_t mxor(uint32_t z, uint32_t x, uint32_t m) {
  return __builtin_amdgcn_bitop3_b32(z, x, m, 0x78);
}

constexpr int NQ = 5, VEC = 2, U = 8;

template <int MODE>
__global__ __launch_bounds__(512) void k(const uint8_t* __restrict__ shard, uint64_t nrec,
                                         const uint2* __restrict__ coef,
                                         const u32x8* __restrict__ mtab, uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  // 2 column groups of 512 B per 1 KiB record: wave w of the block takes group w & 1
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t grp = wv & 1;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (wv >> 1);
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  const uint64_t r0 = wave * nrec / nw, r1 = (wave + 1) * nrec / nw;
  const uint8_t* base = shard + grp * 512 + lane * 8;
  uint32_t Z[NQ][8][VEC];
#pragma unroll
  for (int a = 0; a < NQ; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int v = 0; v < VEC; ++v) Z[a][b][v] = 0;
  for (uint64_t r = r0; r + U <= r1; r += U) {
    u32x2 x[U];
    uint32_t c0[U], c1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(base + (r + u) * 1024));
      const uint2 q = coef[r + u];
      c0[u] = __builtin_amdgcn_readfirstlane(q.x);
      c1[u] = __builtin_amdgcn_readfirstlane(q.y);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (MODE == 3) {
        Z[0][0][0] ^= x[u].x;
        Z[0][0][1] ^= x[u].y;
        continue;
      }
      const uint32_t one = MODE == 1 ? (uint32_t)((int32_t)(c0[u] << 31) >> 31) : 0u;
#pragma unroll
      for (int a = 0; a < NQ; ++a) {
        const uint32_t ca = ((a < 4 ? c0[u] : c1[u]) >> (8 * (a & 3))) & 0xffu;
        uint32_t m[8];
        if constexpr (MODE == 2) {
          const u32x8 t = mtab[ca];
#pragma unroll
          for (int b = 0; b < 8; ++b) m[b] = t[b];
        } else {
#pragma unroll
          for (int b = 0; b < 8; ++b) m[b] = MODE == 1 ? one : 0u - ((ca >> b) & 1u);
        }
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          Z[a][b][0] = mxor(Z[a][b][0], x[u].x, m[b]);
          Z[a][b][1] = mxor(Z[a][b][1], x[u].y, m[b]);
        }
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int a = 0; a < NQ; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc ^= (Z[a][b][0] + 3 * Z[a][b][1]) * (2 * (8 * a + b) + 1);
  atomicXor(out + lane, acc);
}

__global__ void fill(uint8_t* d, size_t n, uint64_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n / 8; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    reinterpret_cast<uint64_t*>(d)[i] = z ^ (z >> 31);
  }
}

template <int MODE>
static int run(const uint8_t* shard, uint64_t nrec, const uint2* coef, const u32x8* mtab,
               uint32_t* out, int cus) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k<MODE>, dim3(cus), dim3(512), 0, 0, shard, nrec, coef, mtab, out);
  CK(hipEventRecord(e0));
  const int iters = 5;
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL(k<MODE>, dim3(cus), dim3(512), 0, 0, shard, nrec, coef, mtab, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  printf("MODE=%d  %.3f ms  %.1f GB/s\n", MODE, ms, nrec * 1024.0 / ms / 1e6);
  return 0;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t nrec = 1ull << 22;  // 4 GiB
  uint8_t* shard;
  uint2* coef;
  u32x8* mtab;
  uint32_t* out;
  CK(hipMalloc(&shard, nrec * 1024));
  CK(hipMalloc(&coef, nrec * 8));
  CK(hipMalloc(&mtab, 256 * 32));
  CK(hipMalloc(&out, 256));
  uint32_t h[256 * 8];
  for (int c = 0; c < 256; ++c)
    for (int b = 0; b < 8; ++b) h[c * 8 + b] = ((c >> b) & 1) ? 0xffffffffu : 0u;
  CK(hipMemcpy(mtab, h, sizeof(h), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, shard, nrec * 1024, 1);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint8_t*)coef, nrec * 8, 2);
  CK(hipDeviceSynchronize());
  run<3>(shard, nrec, coef, mtab, out, cus);
  run<0>(shard, nrec, coef, mtab, out, cus);
  run<1>(shard, nrec, coef, mtab, out, cus);
  run<2>(shard, nrec, coef, mtab, out, cus);
  run<0>(shard, nrec, coef, mtab, out, cus);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
