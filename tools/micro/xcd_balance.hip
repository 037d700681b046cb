// Micro-benchmark (not part of the product): do the 8 XCDs stream at the same rate?  k_query's
// traces (profiles/r04/r4z_xcd*.txt) show workgroups b with b odd finishing ~8 % after those with
// b even for the same work.  Here workgroup b (one 512-thread workgroup per CU, 8 waves, 8 rows
// of 1 KiB in flight per wave, 16-B non-temporal loads, XOR-folded) reads the contiguous region
// (b + shift) mod 256 of a 16 GiB buffer and records its end time (s_memrealtime, 100 MHz) and
// its XCC_ID; printed per XCC and per b mod 8: does the slow set follow the hardware XCD, the
// block number, or the region read?
// Build: hipcc -O3 --offload-arch=gfx950 -o xcd_balance xcd_balance.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int U = 8, NW = 8;
constexpr uint64_t ROW16 = 64;

__global__ __launch_bounds__(512) void k_read(const u32x4* __restrict__ p, uint64_t rows, int shift,
                                              uint64_t* stamp, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t nb = gridDim.x, b = blockIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t R = rows / nb, reg = (b + (uint64_t)shift) % nb;
  u32x4 acc = {0, 0, 0, 0};
  const uint64_t nk = R / NW;
  for (uint64_t k = 0; k + U <= nk; k += U) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(p + (reg * R + (k + u) * NW + w) * ROW16 + lane);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= x[u];
  }
  const uint32_t v = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (v == 0x9e3779b9u) out[blockIdx.x] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 0xf;  // HW_REG_XCC_ID[3:0]
    stamp[3 * b] = t0;
    stamp[3 * b + 1] = __builtin_amdgcn_s_memrealtime();
    stamp[3 * b + 2] = xcc;
  }
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t bytes = 16ull << 30, rows = bytes / 1024;
  u32x4* d;
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(d, 0x5a, bytes));
  uint32_t* out;
  uint64_t* st;
  CK(hipMalloc(&out, 4096 * 4));
  CK(hipMalloc(&st, cus * 3 * 8));
  std::vector<uint64_t> h(cus * 3);
  for (int shift : {0, 1, 0, 1, 8}) {
    hipLaunchKernelGGL(k_read, dim3(cus), dim3(512), 0, 0, d, rows, shift, st, out);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_read, dim3(cus), dim3(512), 0, 0, d, rows, shift, st, out);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull, tend = 0;
    for (int b = 0; b < cus; ++b) { t0 = std::min(t0, h[3 * b]); tend = std::max(tend, h[3 * b + 1]); }
    printf("shift %d: launch %.1f us (%.3f TB/s)\n", shift, (tend - t0) / 100.0, bytes / ((tend - t0) * 1e-8) / 1e12);
    for (int by = 0; by < 2; ++by) {
      for (int g = 0; g < 8; ++g) {
        std::vector<double> e;
        for (int b = 0; b < cus; ++b)
          if ((by == 0 ? (int)h[3 * b + 2] : b % 8) == g) e.push_back((h[3 * b + 1] - t0) / 100.0);
        if (e.empty()) continue;
        std::sort(e.begin(), e.end());
        printf("  %s %d: %3zu wgs  end med %8.1f  min %8.1f  max %8.1f us\n", by == 0 ? "xcc " : "b%8", g,
               e.size(), e[e.size() / 2], e.front(), e.back());
      }
    }
    fflush(stdout);
  }
  return 0;
}
