// Micro-benchmark (not part of the product): VALU issue rate of the scan's instruction forms
// on MI355X, no memory traffic.  Each wave runs ITERS x 32 independent accumulator updates.
//   MODE 0: v_bitop3_b32 z, z, x, s   (2 VGPR + 1 SGPR source: the scan's masked XOR)
//   MODE 1: v_bitop3_b32 z, z, x, m   (3 VGPR sources)
//   MODE 2: v_xor_b32 z, x, z         (2 VGPR sources)
//   MODE 3: v_xor_b32 z, s, z         (1 VGPR + 1 SGPR)
//   MODE 4: v_perm_b32 z, z, x, m     (3 VGPR sources: a byte-table lookup)
//   MODE 5: v_perm_b32 z, s, z, x     (SGPR table half + 2 VGPRs)
// Reports lane-ops/s chip-wide and the shader clock from s_memtime over the same interval.
// Build: hipcc -O3 --offload-arch=gfx950 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int MODE>
__global__ __launch_bounds__(1024) void k(uint32_t* out, uint32_t seed, int iters, uint64_t* clk) {
  uint32_t z[32];
  for (int i = 0; i < 32; ++i) z[i] = seed * (threadIdx.x + 7 * i);
  const uint32_t x = threadIdx.x * 0x9E3779B9u, m = threadIdx.x | 1u;
  const uint32_t s = __builtin_amdgcn_readfirstlane(seed ^ 0xFFFF0000u);
  const uint64_t t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      if constexpr (MODE == 0) z[i] = __builtin_amdgcn_bitop3_b32(z[i], x, s, 0x78);
      else if constexpr (MODE == 1) z[i] = __builtin_amdgcn_bitop3_b32(z[i], x, m, 0x78);
      else if constexpr (MODE == 2) z[i] ^= x;
      else if constexpr (MODE == 3) z[i] ^= s;
      else if constexpr (MODE == 4) z[i] = __builtin_amdgcn_perm(z[i], x, m);
      else z[i] = __builtin_amdgcn_perm(s, z[i], x);
    }
    asm volatile("" ::: "memory");
  }
  const uint64_t t1 = __builtin_readcyclecounter();
  uint32_t acc = 0;
  for (int i = 0; i < 32; ++i) acc += z[i] * (2 * i + 1);
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
  if (threadIdx.x == 0 && blockIdx.x == 0) *clk = t1 - t0;
}

template <int MODE>
static int run(uint32_t* out, uint64_t* dclk, int cus) {
  const int iters = 4000;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k<MODE>, dim3(cus), dim3(1024), 0, 0, out, 3u, 10, dclk);
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(k<MODE>, dim3(cus), dim3(1024), 0, 0, out, 3u, iters, dclk);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  uint64_t clk = 0;
  CK(hipMemcpy(&clk, dclk, 8, hipMemcpyDeviceToHost));
  const double ops = (double)cus * 1024 * iters * 32;
  printf("MODE=%d  %.3f ms  %.2f T lane-ops/s  %.1f lane-ops/clk/CU at %.2f GHz (s_memtime over %.3f ms)\n",
         MODE, ms, ops / ms / 1e9, ops / cus / (clk * 1.0), clk / (ms * 1e6), ms);
  return 0;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t* out;
  uint64_t* clk;
  CK(hipMalloc(&out, 4096));
  CK(hipMalloc(&clk, 8));
  run<0>(out, clk, cus);
  run<1>(out, clk, cus);
  run<2>(out, clk, cus);
  run<3>(out, clk, cus);
  run<4>(out, clk, cus);
  run<5>(out, clk, cus);
  run<0>(out, clk, cus);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
