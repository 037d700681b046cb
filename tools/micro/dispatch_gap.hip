// Micro-benchmark (not part of the product): what sets the ~6.3 us between a lone query's
// k_reduce and the next query's k_query (profiles/r05/r5af_lone_gaps_depth4_depth16.txt), when
// k_query -> k_reduce shows no gap at all?  Candidates: k_query's private segment (its VGPR
// spills use scratch; k_reduce has none), its 95 KiB of LDS, or its 1024-thread workgroups.
// Back-to-back pairs on one stream, timed under rocprofv3 --kernel-trace (the gap = next start
// minus previous end):  small (4 x 1024 threads, no scratch) -> big, with big one of
//   0: 256 x 1024 threads, 96 KiB LDS, no scratch
//   1: the same with a private segment (a dynamically indexed local array)
//   2: 256 x 256 threads, no LDS, no scratch
//   3: mode 1 followed by a small kernel WITH a private segment
//   4: mode 1 launches back to back (no small kernel)
//   5: mode 1 with a 16-B private segment
//   6: mode 2 with an 80-B private segment
//   7: mode 0 with a hipEventRecord after each small kernel (pir_engine's ws_release)
//   8: mode 0 with a hipStreamWaitEvent on an already-complete event before each big kernel
//   9: mode 1 with the private segment never touched at run time
// Build: hipcc -O3 --offload-arch=gfx950 -o dispatch_gap dispatch_gap.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(1024) void k_small(uint32_t* out) {
  if (threadIdx.x == 0 && out[blockIdx.x] == 0x9e3779b9u) out[blockIdx.x] = 1;
}

// k_small with a private segment of its own
__global__ __launch_bounds__(1024) void k_small_scratch(uint32_t* out, uint32_t k) {
  volatile uint32_t loc[16];
  for (int i = 0; i < 16; ++i) loc[i] = threadIdx.x + i;
  if (threadIdx.x == 0 && loc[k & 15] == 0x9e3779b9u) out[blockIdx.x] = 1;
}

// ~20 us of work per workgroup so every launch is a kernel of k_query's shape
__device__ inline void spin(uint32_t us) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((uint32_t)(__builtin_amdgcn_s_memrealtime() - t0) < us * 100u) __builtin_amdgcn_s_sleep(4);
}

__global__ __launch_bounds__(1024) void k_big_lds(uint32_t* out, uint32_t us) {
  __shared__ uint32_t lds[24 * 1024];  // 96 KiB
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  spin(us);
  if (lds[(threadIdx.x + 1) & 1023] == 0x9e3779b9u) out[blockIdx.x] = 1;
}

__global__ __launch_bounds__(1024) void k_big_lds_scratch(uint32_t* out, uint32_t us, uint32_t k) {
  __shared__ uint32_t lds[24 * 1024];
  volatile uint32_t loc[16];  // private segment
  for (int i = 0; i < 16; ++i) loc[i] = threadIdx.x + i;
  lds[threadIdx.x] = loc[(threadIdx.x + k) & 15];
  __syncthreads();
  spin(us);
  if (lds[(threadIdx.x + 1) & 1023] == 0x9e3779b9u) out[blockIdx.x] = 1;
}

// a 16-B private segment instead of 80 B
__global__ __launch_bounds__(1024) void k_big_lds_scratch16(uint32_t* out, uint32_t us, uint32_t k) {
  __shared__ uint32_t lds[24 * 1024];
  volatile uint32_t loc[4];
  for (int i = 0; i < 4; ++i) loc[i] = threadIdx.x + i;
  lds[threadIdx.x] = loc[(threadIdx.x + k) & 3];
  __syncthreads();
  spin(us);
  if (lds[(threadIdx.x + 1) & 1023] == 0x9e3779b9u) out[blockIdx.x] = 1;
}

// 256-thread workgroups (a quarter of the waves) with the 80-B private segment
__global__ __launch_bounds__(256) void k_big_plain_scratch(uint32_t* out, uint32_t us, uint32_t k) {
  volatile uint32_t loc[16];
  for (int i = 0; i < 16; ++i) loc[i] = threadIdx.x + i;
  spin(us);
  if (loc[k & 15] == 0x9e3779b9u) out[blockIdx.x] = 1;
}

// an 80-B private segment that no lane touches at run time (k != 12345 in every launch)
__global__ __launch_bounds__(1024) void k_big_lds_scratch_cold(uint32_t* out, uint32_t us, uint32_t k) {
  __shared__ uint32_t lds[24 * 1024];
  lds[threadIdx.x] = threadIdx.x;
  if (k == 12345u) {
    volatile uint32_t loc[16];
    for (int i = 0; i < 16; ++i) loc[i] = threadIdx.x + i;
    lds[threadIdx.x] = loc[(threadIdx.x + k) & 15];
  }
  __syncthreads();
  spin(us);
  if (lds[(threadIdx.x + 1) & 1023] == 0x9e3779b9u) out[blockIdx.x] = 1;
}

__global__ __launch_bounds__(256) void k_big_plain(uint32_t* out, uint32_t us) {
  spin(us);
  if (threadIdx.x == 0 && out[blockIdx.x] == 0x9e3779b9u) out[blockIdx.x] = 1;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t* out;
  CK(hipMalloc(&out, 4096 * 4));
  CK(hipMemset(out, 0, 4096 * 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (int mode = 0; mode < 10; ++mode) {
    for (int r = 0; r < 40; ++r) {
      if (mode == 8) CK(hipStreamWaitEvent(s, ev, 0));
      if (mode == 9) hipLaunchKernelGGL(k_big_lds_scratch_cold, dim3(cus), dim3(1024), 0, s, out, 20u, (uint32_t)r);
      if (mode == 0 || mode == 7 || mode == 8) hipLaunchKernelGGL(k_big_lds, dim3(cus), dim3(1024), 0, s, out, 20u);
      if (mode == 1) hipLaunchKernelGGL(k_big_lds_scratch, dim3(cus), dim3(1024), 0, s, out, 20u, (uint32_t)r);
      if (mode == 2) hipLaunchKernelGGL(k_big_plain, dim3(cus), dim3(256), 0, s, out, 20u);
      if (mode == 5) hipLaunchKernelGGL(k_big_lds_scratch16, dim3(cus), dim3(1024), 0, s, out, 20u, (uint32_t)r);
      if (mode == 6) hipLaunchKernelGGL(k_big_plain_scratch, dim3(cus), dim3(256), 0, s, out, 20u, (uint32_t)r);
      if (mode == 3 || mode == 4) hipLaunchKernelGGL(k_big_lds_scratch, dim3(cus), dim3(1024), 0, s, out, 20u, (uint32_t)r);
      if (mode == 3) hipLaunchKernelGGL(k_small_scratch, dim3(4), dim3(1024), 0, s, out, (uint32_t)r);
      if (mode <= 2 || mode >= 5) hipLaunchKernelGGL(k_small, dim3(4), dim3(1024), 0, s, out);
      if (mode == 7) CK(hipEventRecord(ev, s));
    }
    CK(hipStreamSynchronize(s));
    printf("mode %d done\n", mode);
  }
  return 0;
}
