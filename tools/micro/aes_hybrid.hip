// Micro-benchmark (not part of the product): the hybrid question of north_star's "table-free /
// bitsliced AES" (DESIGN.md § AES): the depth-first leaf stage (k_subtree, pir_aes4.h) is bound
// by LDS lookups while its VALU issues well under its peak, and the bitsliced AES (aes_bs.h)
// uses the VALU alone.  Do waves running the bitsliced AES beside T-table waves on the SAME CU
// add AES blocks per second, or do the two forms just trade issue slots?
//
// One 1024-thread workgroup per CU (128 KiB of 4-table LDS, as k_subtree): the first 16 - B
// waves run the production 4-table T-box (aes_ctr_row4: 1 lane = 1 key), the last B waves the
// bitsliced AES (a quad = 32 keys), both for the same wall-clock budget (each wave loops until
// its shader clock passes the deadline) and count the AES blocks they finished.  Printed per
// B: blocks/s of each form and in all, for leaf blocks (1 block per key, as the leaf
// conversion) and internal nodes (3 CTR blocks under one key schedule; the bitsliced waves run
// them as 3 one-block calls, the three-block form needs 173 VGPRs and the workgroup has 128).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../erasurecodedpir_amd/csrc -o aes_hybrid aes_hybrid.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "pir_aes4.h"
#include "aes_bs.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

// counters[0] = T-table blocks, counters[1] = bitsliced blocks
template <int NB>
__global__ __launch_bounds__(1024) void k_hyb(int bs_waves, long long budget, uint32_t salt,
                                              unsigned long long* counters, uint32_t* out) {
  __shared__ uint32_t tab[pir::kTab4Bytes / 4];
  pir::load_tables4_n<1024>(tab);
  __syncthreads();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const long long t0 = clock64();
  unsigned long long n = 0;
  uint32_t acc = 0;
  if ((int)wave >= 16 - bs_waves) {
    const bs::Lane L(threadIdx.x & 3u);
    uint32_t key[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) key[i] = (g * 0x9E3779B9u) ^ (i * 0x85EBCA6Bu) ^ salt;
    while (clock64() - t0 < budget) {
#pragma unroll 1
      for (int b = 0; b < NB; ++b) {  // NB one-block calls (own key schedule each), chained
        uint32_t o[1][32];
        bs::aes_ctr<1>(L, key, o);
#pragma unroll
        for (int i = 0; i < 32; ++i) key[i] ^= o[0][i] ^ (uint32_t)b;
      }
      n += 32 / 4 * NB;  // per lane: a quad does 32 keys
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) acc ^= key[i];
    if ((threadIdx.x & 63) == 0) atomicAdd(&counters[1], n * 64);
  } else {
    const pir::Tab4 T(tab);
    uint4 seed = make_uint4(g * 0x9E3779B9u, g + salt, salt * 0x85EBCA6Bu, g ^ 0x5A5A5A5Au);
    while (clock64() - t0 < budget) {
      uint4 o[NB];
      pir::aes_ctr_row4<NB, 16>(T, seed, o);
      seed = pir::xor4(seed, o[0]);
#pragma unroll
      for (int b = 1; b < NB; ++b) acc ^= o[b].x ^ o[b].y;
      n += NB;
    }
    acc ^= seed.x ^ seed.w;
    if ((threadIdx.x & 63) == 0) atomicAdd(&counters[0], n * 64);
  }
  if (acc == 0x12345678u) out[g] = acc;
}

template <int NB>
static int run(int cus, unsigned long long* d_cnt, uint32_t* out) {
  const long long budget = 4000000;  // shader-clock ticks per wave (~2 ms)
  for (int B : {0, 1, 2, 4, 6, 8, 16}) {
    hipLaunchKernelGGL(k_hyb<NB>, dim3(cus), dim3(1024), 0, 0, B, budget / 8, 1u, d_cnt, out);
    CK(hipMemset(d_cnt, 0, 2 * sizeof(unsigned long long)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_hyb<NB>, dim3(cus), dim3(1024), 0, 0, B, budget, 2u, d_cnt, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long c[2];
    CK(hipMemcpy(c, d_cnt, sizeof c, hipMemcpyDeviceToHost));
    printf("%s  bitsliced waves %2d/16: T-table %7.2f  bitsliced %7.2f  total %7.2f G blocks/s"
           "  (%.3f ms)\n", NB == 1 ? "leaf block   " : "internal node", B, c[0] / ms / 1e6,
           c[1] / ms / 1e6, (c[0] + c[1]) / ms / 1e6, ms);
  }
  return 0;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  unsigned long long* d_cnt;
  uint32_t* out;
  CK(hipMalloc(&d_cnt, 2 * sizeof(unsigned long long)));
  CK(hipMalloc(&out, (size_t)cus * 1024 * 4));
  if (run<1>(cus, d_cnt, out)) return 1;
  if (run<3>(cus, d_cnt, out)) return 1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
