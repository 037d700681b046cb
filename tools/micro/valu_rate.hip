// Micro-benchmark (not part of the product): VALU issue rate of the scan's instruction forms
// on MI355X, no memory traffic.  Each wave runs ITERS x 32 independent accumulator updates.
//   MODE 0: v_bitop3_b32 z, z, x, s   (2 VGPR + 1 SGPR source: the scan's masked XOR)
//   MODE 1: v_bitop3_b32 z, z, x, m   (3 VGPR sources)
//   MODE 2: v_xor_b32 z, x, z         (2 VGPR sources)
//   MODE 3: v_xor_b32 z, s, z         (1 VGPR + 1 SGPR)
//   MODE 4: v_perm_b32 z, z, x, m     (3 VGPR sources: a byte-table lookup)
//   MODE 5: v_perm_b32 z, s, z, x     (SGPR table half + 2 VGPRs)
//   MODE 6: v_and_or_b32 z, z, x, m   MODE 7: v_lshl_or_b32 z, z, 8, x   MODE 8: v_bfe_u32 z, z, 8, 8
//   MODE 9: v_alignbit_b32 z, z, x, 8 MODE 10: v_add_u32 z, z, x          MODE 11: v_bfi_b32 z, x, z, m
//   MODE 12: v_lshrrev_b32 z, 8, z    MODE 13: v_and_b32 z, z, x
//   MODE 14: v_mov_b32_sdwa z, x dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2
//   MODE 15: v_or_b32_sdwa z, z, x src1_sel:BYTE_3
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
      else if constexpr (MODE == 5) z[i] = __builtin_amdgcn_perm(s, z[i], x);
      else if constexpr (MODE == 6) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(z[i]) : "v"(x), "v"(m));
      else if constexpr (MODE == 7) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(z[i]) : "v"(x));
      else if constexpr (MODE == 8) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(z[i]));
      else if constexpr (MODE == 9) asm volatile("v_alignbit_b32 %0, %0, %1, 8" : "+v"(z[i]) : "v"(x));
      else if constexpr (MODE == 10) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(z[i]) : "v"(x));
      else if constexpr (MODE == 11) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(z[i]) : "v"(x), "v"(m));
      else if constexpr (MODE == 12) asm volatile("v_lshrrev_b32_e32 %0, 8, %0" : "+v"(z[i]));
      else if constexpr (MODE == 13) asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(z[i]) : "v"(x));
      else if constexpr (MODE == 14)
        asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(z[i]) : "v"(x));
      else asm volatile("v_or_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "+v"(z[i]) : "v"(x));
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
  run<6>(out, clk, cus);
  run<7>(out, clk, cus);
  run<8>(out, clk, cus);
  run<9>(out, clk, cus);
  run<10>(out, clk, cus);
  run<11>(out, clk, cus);
  run<12>(out, clk, cus);
  run<13>(out, clk, cus);
  run<14>(out, clk, cus);
  run<15>(out, clk, cus);
  run<0>(out, clk, cus);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
