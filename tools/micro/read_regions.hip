// Micro-benchmark (not part of the product): does the HBM read rate depend on the shard size
// and on how rows are assigned to workgroups?  k_query gives workgroup b the contiguous region
// [b R, (b+1) R) of the shard (R = N / 256 rows) and streams it tile by tile; the read micro of
// round 2 (read_bw.hip) interleaves rows across the whole grid.  At 2^24 x 1 KiB both run at
// ~6.75 TB/s; the 2^27 x 1 KiB single engine (128 GiB) runs k_query at ~6.1 TB/s.
// For S = 16, 32, 64, 128 GiB this times a full read (16-B non-temporal loads, one 512-thread
// workgroup per CU, 8 waves, 8 rows of 1 KiB in flight per wave, XOR-folded) with rows assigned
//   region : workgroup b reads [b S/256, (b+1) S/256), its 8 waves interleaved by row (k_query)
//   tiles  : tile t (T rows) of the shard goes to workgroup t mod 256 (round-robin tiles)
//   grid   : row r goes to wave r mod (all waves) (read_bw.hip's order)
// Build: hipcc -O3 --offload-arch=gfx950 -o read_regions read_regions.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int U = 8;        // rows in flight per wave
constexpr int NW = 8;       // waves per workgroup
constexpr uint64_t ROW16 = 64;  // 16-B chunks per 1 KiB row

// mode 0 = region, 1 = tiles of `tile` rows, 2 = grid order
__global__ __launch_bounds__(512) void k_read(const u32x4* __restrict__ p, uint64_t rows, int mode,
                                              uint64_t tile, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t nb = gridDim.x, b = blockIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  auto row_of = [&](uint64_t k) -> uint64_t {  // k-th row of this wave
    if (mode == 0) {
      const uint64_t R = rows / nb;
      return b * R + k * NW + w;
    }
    if (mode == 1) {
      const uint64_t per_tile = tile / NW;  // rows of one tile for this wave
      const uint64_t t = k / per_tile, j = k % per_tile;
      return ((t * nb + b) * tile) + j * NW + w;
    }
    return (k * nb + b) * NW + w;
  };
  const uint64_t nk = rows / (nb * NW);
  for (uint64_t k = 0; k + U <= nk; k += U) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(p + row_of(k + u) * ROW16 + lane);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= x[u];
  }
  const uint32_t v = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (v == 0x9e3779b9u) out[blockIdx.x] = v;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t maxb = 128ull << 30;
  u32x4* d;
  CK(hipMalloc(&d, maxb));
  CK(hipMemset(d, 0x5a, maxb));
  uint32_t* out;
  CK(hipMalloc(&out, 4096 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[3] = {"region", "tiles", "grid"};
  for (uint64_t gib : {16ull, 32ull, 64ull, 128ull}) {
    const uint64_t rows = (gib << 30) / 1024;
    for (int mode = 0; mode < 3; ++mode) {
      const uint64_t tile = 4096;
      hipLaunchKernelGGL(k_read, dim3(cus), dim3(512), 0, 0, d, rows, mode, tile, out);
      CK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_read, dim3(cus), dim3(512), 0, 0, d, rows, mode, tile, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      printf("%4llu GiB  %-6s  %8.3f ms  %6.3f TB/s\n", (unsigned long long)gib, names[mode], best,
             (double)(gib << 30) / (best * 1e-3) / 1e12);
      fflush(stdout);
    }
  }
  return 0;
}
