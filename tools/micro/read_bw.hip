// Micro-benchmark (not part of the product): the achievable HBM read rate on MI355X for the
// scan's access pattern -- every byte of a 16 GiB buffer read once with 16-byte non-temporal
// loads, XOR-folded per lane (so the loads cannot be dropped), one partial word per workgroup.
// Variants: rows in flight per lane (U) and workgroups per CU.  Prints TB/s per variant.
// Build: hipcc -O3 --offload-arch=gfx950 -o read_bw read_bw.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(512) void k_read(const u32x4* __restrict__ p, uint64_t n16, uint32_t* out) {
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // each wave reads contiguous 1 KiB rows (64 lanes x 16 B), waves interleaved across the grid
  u32x4 acc = {0, 0, 0, 0};
  uint64_t i = t;
  for (; i + (U - 1) * nthreads < n16; i += U * nthreads) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(p + i + u * nthreads);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= x[u];
  }
  for (; i < n16; i += nthreads) acc ^= __builtin_nontemporal_load(p + i);
  const uint32_t v = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (v == 0x9e3779b9u) out[blockIdx.x] = v;  // practically never: keeps the loads live
}

template <int U>
static int run(const u32x4* d, uint64_t n16, uint32_t* out, int cus, int bpc) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 grid(cus * bpc);
  hipLaunchKernelGGL(k_read<U>, grid, dim3(512), 0, 0, d, n16, out);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_read<U>, grid, dim3(512), 0, 0, d, n16, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  printf("U=%2d blocks/CU=%d  %.3f ms  %.3f TB/s\n", U, bpc, best, n16 * 16.0 / (best * 1e9));
  return 0;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t bytes = 16ull << 30;
  void* d;
  uint32_t* out;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&out, 4 * cus * 8));
  CK(hipMemset(d, 0x5a, bytes));
  const uint64_t n16 = bytes / 16;
  for (int bpc : {1, 2, 4}) {
    run<4>((const u32x4*)d, n16, out, cus, bpc);
    run<8>((const u32x4*)d, n16, out, cus, bpc);
    run<16>((const u32x4*)d, n16, out, cus, bpc);
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
