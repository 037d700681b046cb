// Micro-benchmark (not part of the product): dependent-chain latency of one AES-128 PRG call
// (the tree's per-level critical path) in the execution shapes of pir_aes.h, one wave alone.
//   col : column shape, 16 lanes = 4 quads (quad r = CTR block r), aes_col()
//   row3: row shape, 1 lane = 1 node, 3 CTR blocks on one key schedule, aes_ctr_row<3,1>
//   row1: row shape, 1 block, aes_ctr_row<1,4>
// Each chain feeds block 0's output back as the next key (a tree descent).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../erasurecodedpir_amd/csrc -o aes_latency aes_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "pir_aes.h"

using namespace pir;

__global__ __launch_bounds__(1024) void k_col(int iters, uint32_t* out, long long* cyc) {
  __shared__ uint32_t tab[2 * 256 * 32];
  load_tables(tab);
  __syncthreads();
  if (threadIdx.x >= 64) {  // the other waves of a big workgroup park at a barrier
    __syncthreads();
    return;
  }
  const Tab T(tab);
  const uint32_t q = threadIdx.x & 3u, role = (threadIdx.x >> 2) & 3u;
  const uint32_t mq1 = q >= 1 ? ~0u : 0u, mq2 = q >= 2 ? ~0u : 0u;
  const uint32_t ptq = q == 3 ? (role << 24) : 0u;
  uint32_t s = 0x01020304u * (q + 1);
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    const uint32_t o = aes_col(T, s, ptq, mq1, mq2);
    s = (uint32_t)__shfl((int)o, (int)((threadIdx.x & ~15u) | q), 64);  // block 0 -> next key
  }
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
  if (blockDim.x > 64) __syncthreads();
}

template <int NB, int LASTW>
__global__ __launch_bounds__(1024) void k_row(int iters, uint32_t* out, long long* cyc) {
  __shared__ uint32_t tab[2 * 256 * 32];
  load_tables(tab);
  __syncthreads();
  const Tab T(tab);
  uint4 s = make_uint4(threadIdx.x, 1, 2, 3);
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    uint4 o[NB];
    aes_ctr_row<NB, LASTW>(T, s, o);
    s = o[0];
    if (NB > 1) s.x ^= o[NB - 1].x & 1u;
  }
  const long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s.x ^ s.y ^ s.z ^ s.w;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

static uint32_t* g_o;
static long long* g_c;
static const int kIters = 1000;

static void run(const char* name, void (*launch)()) {
  long long best = 1ll << 62;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float ms = 0;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(a);
    launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    long long c;
    (void)hipMemcpy(&c, g_c, 8, hipMemcpyDeviceToHost);
    if (c < best) best = c;
    (void)hipEventElapsedTime(&ms, a, b);
  }
  printf("%-6s %8.1f cycles per AES call; kernel %.3f ms for %d calls -> %.3f us per call\n", name,
         (double)best / kIters, ms, kIters, ms * 1e3 / kIters);
}

int main() {
  (void)hipMalloc(&g_o, 256 * 1024 * 4);
  (void)hipMalloc(&g_c, 8);
  run("col", [] { hipLaunchKernelGGL(k_col, dim3(1), dim3(64), 0, 0, kIters, g_o, g_c); });
  run("col256", [] { hipLaunchKernelGGL(k_col, dim3(256), dim3(64), 0, 0, kIters, g_o, g_c); });
  run("colWG", [] { hipLaunchKernelGGL(k_col, dim3(1), dim3(1024), 0, 0, kIters, g_o, g_c); });
  run("colWG256", [] { hipLaunchKernelGGL(k_col, dim3(256), dim3(1024), 0, 0, kIters, g_o, g_c); });
  run("row3", [] { hipLaunchKernelGGL((k_row<3, 1>), dim3(1), dim3(64), 0, 0, kIters, g_o, g_c); });
  run("row1", [] { hipLaunchKernelGGL((k_row<1, 4>), dim3(1), dim3(64), 0, 0, kIters, g_o, g_c); });
  // throughput: 256 CUs x W waves of row3 / row1 (blocks per second chip-wide)
  for (int w : {4, 8, 16}) {
    static int ws;
    ws = w;
    printf("row3 x %2d waves/CU: ", w);
    run("", [] { hipLaunchKernelGGL((k_row<3, 1>), dim3(256), dim3(64 * ws), 0, 0, kIters, g_o, g_c); });
    printf("row1 x %2d waves/CU: ", w);
    run("", [] { hipLaunchKernelGGL((k_row<1, 4>), dim3(256), dim3(64 * ws), 0, 0, kIters, g_o, g_c); });
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
