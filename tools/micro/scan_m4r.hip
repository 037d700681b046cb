// Micro-benchmark (not part of the product): the many-round GF(2^8) scan of configs[4] (5 rounds,
// wave-uniform coefficients, 1 KiB records), four Russians over rows (pir_m4r.h) against the
// product's plane-table form, at several lane widths, wave counts and round splits.
//   REF  : 8 masks per (row, round) from a 256 x 8-dword table, one v_bitop3 per (plane, dword)
//   M4R  : pir::m4r_fold4 per group of 4 rows (VEC = 1 or 2 dwords per lane)
//   SPLIT = 2: the waves of a pair read the same rows; one folds rounds 0-2, the other 3-4
//   (fewer accumulators per wave, rows read twice from L2)
// Every variant XORs its planes into one 40 x 256-word array (partition-independent), compared
// with REF's on the host.
// Build: hipcc -O3 --offload-arch=gfx950 -I../../erasurecodedpir_amd/csrc -o scan_m4r scan_m4r.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "pir_m4r.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

constexpr int NQ = 5;

template <int VEC>
__device__ __forceinline__ void ldx(const uint8_t* p, uint32_t* v) {
  if constexpr (VEC == 2) {
    const u32x2 q = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
    v[0] = q.x; v[1] = q.y;
  } else {
    v[0] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p));
  }
}

// lane k = plane k of rounds [A0, A0 + NA): bit (k % 8) of the 4 rows' round (A0 + k / 8) bytes
template <int A0>
__device__ __forceinline__ uint32_t plane_index(const uint32_t* c0, const uint32_t* c1, uint32_t lane) {
  const uint32_t a = A0 + (lane >> 3), sh = 8u * (a & 3u) + (lane & 7u);
  uint32_t vi = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) vi |= (((a >= 4 ? c1[i] : c0[i]) >> sh) & 1u) << i;
  return vi;
}

template <int MODE, int WAVES, int VEC, int SPLIT, int U>
__global__ __launch_bounds__(WAVES * 64) void k(const uint8_t* __restrict__ shard, uint64_t nrec,
                                                const uint2* __restrict__ coef,
                                                const u32x8* __restrict__ mtab,
                                                uint32_t* __restrict__ out) {
  constexpr int GROUPS = 1024 / (64 * VEC * 4);
  constexpr int PER = WAVES / GROUPS / SPLIT;  // row-waves per block
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t grp = wv % GROUPS;
  const uint32_t half = (wv / GROUPS) % SPLIT;
  const uint64_t wave = (uint64_t)blockIdx.x * PER + wv / (GROUPS * SPLIT);
  const uint64_t nw = (uint64_t)gridDim.x * PER;
  const uint64_t r0 = wave * nrec / nw, r1 = (wave + 1) * nrec / nw;
  const uint8_t* base = shard + grp * (64 * VEC * 4) + lane * VEC * 4;
  constexpr int NA = SPLIT == 1 ? NQ : 3;
  uint32_t Z[NA][8][VEC];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int v = 0; v < VEC; ++v) Z[a][b][v] = 0;
  uint32_t xn[U][VEC];
  auto load_batch = [&](uint64_t r) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < U; ++u) ldx<VEC>(base + (r + u < r1 ? r + u : r0) * 1024, xn[u]);
  };
  load_batch(r0);
  for (uint64_t r = r0; r < r1; r += U) {
    uint32_t x[U][VEC], c0[U], c1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) x[u][v] = xn[u][v];
      const uint2 cc = coef[r + u];  // uniform: scalar loads
      c0[u] = cc.x;
      c1[u] = cc.y;
    }
    load_batch(r + U);
    if constexpr (MODE == 0) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int a = 0; a < NQ; ++a) {
          const uint32_t ca = ((a < 4 ? c0[u] : c1[u]) >> (8 * (a & 3))) & 0xffu;
          const u32x8 t = mtab[ca];
#pragma unroll
          for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int v = 0; v < VEC; ++v)
              Z[a][b][v] = __builtin_amdgcn_bitop3_b32(Z[a][b][v], x[u][v], t[b], 0x78);
        }
    } else {
#pragma unroll
      for (int g = 0; g < U; g += 4) {
        if constexpr (SPLIT == 1) {
          pir::m4r_fold4<VEC, NQ>(Z, x[g], x[g + 1], x[g + 2], x[g + 3],
                                  plane_index<0>(c0 + g, c1 + g, lane));
        } else if (half == 0) {
          pir::m4r_fold4<VEC, 3>(Z, x[g], x[g + 1], x[g + 2], x[g + 3],
                                 plane_index<0>(c0 + g, c1 + g, lane));
        } else {
          auto& Z2 = reinterpret_cast<uint32_t(&)[2][8][VEC]>(Z);
          pir::m4r_fold4<VEC, 2>(Z2, x[g], x[g + 1], x[g + 2], x[g + 3],
                                 plane_index<3>(c0 + g, c1 + g, lane));
        }
      }
    }
  }
  const uint32_t col = (grp * 64 + lane) * VEC;
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const int ag = SPLIT == 1 ? a : (half == 0 ? a : a + 3);
    if (ag >= NQ || (SPLIT == 2 && half == 1 && a >= 2)) continue;
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int v = 0; v < VEC; ++v) atomicXor(out + (ag * 8 + b) * 256 + col + v, Z[a][b][v]);
  }
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

static uint32_t ref_planes[40 * 256];
static bool have_ref = false;

template <int MODE, int WAVES, int VEC, int SPLIT, int U>
static int run(const char* name, const uint8_t* shard, uint64_t nrec, const uint2* coef,
               const u32x8* mtab, uint32_t* out, int cus) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipMemset(out, 0, 40 * 256 * 4));
  hipLaunchKernelGGL((k<MODE, WAVES, VEC, SPLIT, U>), dim3(cus), dim3(WAVES * 64), 0, 0, shard, nrec, coef, mtab, out);
  static uint32_t h[40 * 256];
  CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
  bool ok = true;
  if (!have_ref) { memcpy(ref_planes, h, sizeof(h)); have_ref = true; }
  else ok = memcmp(ref_planes, h, sizeof(h)) == 0;
  CK(hipEventRecord(e0));
  const int iters = 5;
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL((k<MODE, WAVES, VEC, SPLIT, U>), dim3(cus), dim3(WAVES * 64), 0, 0, shard, nrec, coef, mtab, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  printf("%-34s WAVES=%2d VEC=%d SPLIT=%d U=%d  %.3f ms  %.1f GB/s  planes %s\n", name, WAVES, VEC,
         SPLIT, U, ms, nrec * 1024.0 / ms / 1e6, ok ? "== REF" : "DIFFER");
  return 0;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t nrec = 3ull << 20;  // 3 GiB; rows per wave a multiple of 8 for every variant
  uint8_t* shard;
  uint2* coef;
  u32x8* mtab;
  uint32_t* out;
  CK(hipMalloc(&shard, nrec * 1024));
  CK(hipMalloc(&coef, (nrec + 64) * 8));
  CK(hipMalloc(&mtab, 256 * 32));
  CK(hipMalloc(&out, 40 * 256 * 4));
  uint32_t h[256 * 8];
  for (int c = 0; c < 256; ++c)
    for (int b = 0; b < 8; ++b) h[c * 8 + b] = ((c >> b) & 1) ? 0xffffffffu : 0u;
  CK(hipMemcpy(mtab, h, sizeof(h), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, shard, nrec * 1024, 1);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint8_t*)coef, (nrec + 64) * 8, 2);
  CK(hipDeviceSynchronize());
  run<0, 8, 2, 1, 8>("REF plane table", shard, nrec, coef, mtab, out, cus);
  run<0, 16, 2, 1, 8>("REF plane table", shard, nrec, coef, mtab, out, cus);
  run<1, 8, 2, 1, 8>("M4R", shard, nrec, coef, mtab, out, cus);
  run<1, 8, 2, 1, 4>("M4R", shard, nrec, coef, mtab, out, cus);
  run<1, 12, 2, 1, 4>("M4R", shard, nrec, coef, mtab, out, cus);
  run<1, 8, 1, 1, 8>("M4R", shard, nrec, coef, mtab, out, cus);
  run<1, 16, 1, 1, 8>("M4R", shard, nrec, coef, mtab, out, cus);
  run<1, 16, 1, 1, 4>("M4R", shard, nrec, coef, mtab, out, cus);
  run<1, 16, 2, 2, 4>("M4R split 3+2", shard, nrec, coef, mtab, out, cus);
  run<1, 16, 2, 2, 8>("M4R split 3+2", shard, nrec, coef, mtab, out, cus);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
