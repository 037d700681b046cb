// Micro-benchmark (not part of the product): the production row-shape AES of a DPF tree node,
// G(seed) = AES_seed(0..2) with its on-the-fly key schedule (pir_aes.h aes_ctr_row<3,4>), and
// the leaf conversion block AES_seed(0) (aes_ctr_row<1,4>), in isolation: one 1024-thread
// workgroup per CU with the 64 KiB LDS tables, like k_query's tree waves.  Each lane expands
// ITERS independent seeds; outputs are XOR-folded.  Prints nodes/s; run under
// rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES for the instruction counts per node.
// Build: hipcc -O3 --offload-arch=gfx950 -I../../erasurecodedpir_amd/csrc -o aes_node aes_node.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "pir_aes.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int NB>
__global__ __launch_bounds__(1024) void k_node(int iters, uint32_t salt, uint32_t* out) {
  __shared__ uint32_t tab[pir::kTablesBytes / 4];
  pir::load_tables_n<1024>(tab);
  __syncthreads();
  const pir::Tab T(tab);
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int it = 0; it < iters; ++it) {
    const uint4 seed = make_uint4(g * 0x9E3779B9u ^ it, g + salt, it * 0x85EBCA6Bu, g ^ (it << 7));
    uint4 o[NB];
    pir::aes_ctr_row<NB, 1>(T, seed, o);
#pragma unroll
    for (int b = 0; b < NB; ++b) acc = pir::xor4(acc, o[b]);
  }
  const uint32_t v = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (v == 0x12345678u) out[g] = v;
}

template <int NB>
static int run(int cus, uint32_t* out, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_node<NB>, dim3(cus), dim3(1024), 0, 0, 4, 1u, out);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_node<NB>, dim3(cus), dim3(1024), 0, 0, iters, 2u, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double nodes = (double)cus * 1024 * iters;
  printf("NB=%d (%s)  %.3f ms  %.2f G keys/s  %.2f G blocks/s\n", NB,
         NB == 3 ? "internal node: 3 CTR blocks, 1 key schedule" : "leaf: 1 block, 1 key schedule",
         ms, nodes / ms / 1e6, nodes * NB / ms / 1e6);
  return 0;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t* out;
  CK(hipMalloc(&out, (size_t)cus * 1024 * 4));
  run<3>(cus, out, 2000);
  run<1>(cus, out, 4000);
  run<3>(cus, out, 2000);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
