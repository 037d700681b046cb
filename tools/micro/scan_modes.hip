// Micro-benchmark (not part of the product): GF(2^8) multi-round accumulate strategies for the
// shard scan, on a device-resident shard of 1 KiB records with wave-uniform coefficients.
//   MODE 0: scalar branch per coefficient bit (XOR x into the bit plane when set)
//   MODE 1: branch-free, SGPR mask per bit (s_bfe_i32) + v_bitop3 (Z ^= x & m)
//   MODE 2: mixed, bits 0-3 branched, bits 4-7 masked
//   MODE 4: MODE 0 with an empty volatile asm in the taken block (keeps the scalar branch)
//   MODE 3: HBM only (one XOR per dword, no GF work)
// Build: hipcc -O3 --offload-arch=gfx950 -o scan_modes scan_modes.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int VEC>
__device__ __forceinline__ void ld(const uint8_t* p, uint32_t* v) {
  if constexpr (VEC == 4) {
    u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
    u32x2 q = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
    v[0] = q.x; v[1] = q.y;
  }
}

__device__ __forceinline__ uint32_t mxor(uint32_t z, uint32_t x, uint32_t m) {
  return __builtin_amdgcn_bitop3_b32(z, x, m, 0x78);  // z ^ (x & m)
}

template <int NQ, int VEC, int MODE, bool PF>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k(const uint8_t* __restrict__ shard, uint64_t nrec,
                                         uint32_t pitch, const uint8_t* __restrict__ coef,
                                         uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint32_t gy = gridDim.y;
  const uint64_t wave = (uint64_t)blockIdx.x * 8 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 8;
  const uint64_t r0 = wave * nrec / nw, r1 = (wave + 1) * nrec / nw;
  const uint32_t loff = (blockIdx.y * 64 + lane) * (VEC * 4);
  uint32_t Z[NQ][8][VEC];
#pragma unroll
  for (int a = 0; a < NQ; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int v = 0; v < VEC; ++v) Z[a][b][v] = 0;
  constexpr int U = 8;
  auto load = [&](uint64_t r, uint32_t (&x)[U][VEC], uint32_t (&c0)[U], uint32_t (&c1)[U]) {
    const uint8_t* gb = shard + r * pitch;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)gb, 0, U * pitch, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (VEC == 4) {
        u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, loff, u * pitch, 2);
        x[u][0] = q.x; x[u][1] = q.y; x[u][2] = q.z; x[u][3] = q.w;
      } else {
        u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(rs, loff, u * pitch, 2);
        x[u][0] = q.x; x[u][1] = q.y;
      }
      const uint64_t ru = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(r + u)) |
                          ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)((r + u) >> 32)) << 32);
      const uint2 q = reinterpret_cast<const uint2*>(coef)[ru];
      c0[u] = __builtin_amdgcn_readfirstlane(q.x);
      c1[u] = __builtin_amdgcn_readfirstlane(q.y);
    }
  };
  auto compute = [&](const uint32_t (&x)[U][VEC], const uint32_t (&c0)[U], const uint32_t (&c1)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int a = 0; a < NQ; ++a) {
        const uint32_t ca = ((a < 4 ? c0[u] : c1[u]) >> (8 * (a & 3))) & 0xffu;
        if constexpr (MODE == 3) {
#pragma unroll
          for (int v = 0; v < VEC; ++v) Z[a][0][v] ^= x[u][v];
        } else {
#pragma unroll
          for (int b = 0; b < 8; ++b) {
            const bool br = MODE == 0 || MODE == 4 || (MODE == 2 && b < 4);
            if (br) {
              if (ca & (1u << b)) {
                if constexpr (MODE == 4) __asm__ volatile("");
#pragma unroll
                for (int v = 0; v < VEC; ++v) Z[a][b][v] ^= x[u][v];
              }
            } else {
              const uint32_t m = (uint32_t)((int32_t)(ca << (31 - b)) >> 31);
#pragma unroll
              for (int v = 0; v < VEC; ++v) Z[a][b][v] = mxor(Z[a][b][v], x[u][v], m);
            }
          }
        }
      }
  };
  uint32_t xa[U][VEC], ca0[U], ca1[U];
  uint32_t xb[U][VEC], cb0[U], cb1[U];
  if constexpr (!PF) {
    for (uint64_t r = r0; r + U <= r1; r += U) {
      load(r, xa, ca0, ca1);
      compute(xa, ca0, ca1);
    }
  } else {
    uint64_t r = r0;
    if (r + U <= r1) load(r, xa, ca0, ca1);
    for (; r + U <= r1; r += 2 * U) {
      const bool nb = r + 2 * U <= r1;
      if (nb) load(r + U, xb, cb0, cb1);
      compute(xa, ca0, ca1);
      if (!nb) break;
      if (r + 3 * U <= r1) load(r + 2 * U, xa, ca0, ca1);
      compute(xb, cb0, cb1);
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int a = 0; a < NQ; ++a)
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      uint32_t t = Z[a][7][v];
#pragma unroll
      for (int b = 6; b >= 0; --b) t = (((t & 0x7f7f7f7fu) << 1) ^ (((t >> 7) & 0x01010101u) * 0x1du)) ^ Z[a][b][v];
      acc ^= t * (2 * a + 1) + v;
    }
  atomicXor(out + (blockIdx.y * 64 + lane) % 256, acc);
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

template <int NQ, int VEC, int MODE, bool PF>
static int run(const uint8_t* shard, uint64_t nrec, uint32_t pitch, const uint8_t* coef, uint32_t* out,
               int cus) {
  const uint32_t gy = pitch / (VEC * 4) / 64;
  dim3 grid(cus * 2 / gy, gy);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int it = 0; it < 2; ++it) hipLaunchKernelGGL((k<NQ, VEC, MODE, PF>), grid, dim3(512), 0, 0, shard, nrec, pitch, coef, out);
  CK(hipEventRecord(e0));
  const int iters = 5;
  for (int it = 0; it < iters; ++it) hipLaunchKernelGGL((k<NQ, VEC, MODE, PF>), grid, dim3(512), 0, 0, shard, nrec, pitch, coef, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  uint32_t h[256];
  CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
  uint32_t cs = 0;
  for (int i = 0; i < 256; ++i) cs ^= h[i] * (i + 1);
  printf("NQ=%d VEC=%d MODE=%d PF=%d  %.3f ms  %.1f GB/s  csum=%08x\n", NQ, VEC, MODE, (int)PF, ms,
         nrec * (double)pitch / ms / 1e6, cs);
  CK(hipMemset(out, 0, 1024));
  return 0;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t nrec = 1ull << 22;
  const uint32_t pitch = 1024;
  uint8_t *shard, *coef;
  uint32_t* out;
  CK(hipMalloc(&shard, nrec * pitch));
  CK(hipMalloc(&coef, nrec * 8));
  CK(hipMalloc(&out, 1024));
  CK(hipMemset(out, 0, 1024));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, shard, nrec * pitch, 1);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, coef, nrec * 8, 2);
  CK(hipDeviceSynchronize());
  run<1, 4, 3, false>(shard, nrec, pitch, coef, out, cus);
  run<1, 4, 3, true>(shard, nrec, pitch, coef, out, cus);
  run<1, 4, 0, false>(shard, nrec, pitch, coef, out, cus);
  run<1, 4, 0, true>(shard, nrec, pitch, coef, out, cus);
  run<1, 4, 1, false>(shard, nrec, pitch, coef, out, cus);
  run<1, 4, 1, true>(shard, nrec, pitch, coef, out, cus);
  run<1, 4, 2, false>(shard, nrec, pitch, coef, out, cus);
  run<1, 4, 2, true>(shard, nrec, pitch, coef, out, cus);
  run<1, 4, 4, false>(shard, nrec, pitch, coef, out, cus);
  run<1, 4, 4, true>(shard, nrec, pitch, coef, out, cus);
  run<2, 4, 0, false>(shard, nrec, pitch, coef, out, cus);
  run<2, 4, 0, true>(shard, nrec, pitch, coef, out, cus);
  run<2, 4, 1, false>(shard, nrec, pitch, coef, out, cus);
  run<2, 4, 1, true>(shard, nrec, pitch, coef, out, cus);
  run<2, 4, 2, false>(shard, nrec, pitch, coef, out, cus);
  run<2, 4, 2, true>(shard, nrec, pitch, coef, out, cus);
  run<2, 4, 4, false>(shard, nrec, pitch, coef, out, cus);
  run<2, 4, 4, true>(shard, nrec, pitch, coef, out, cus);
  run<5, 2, 3, false>(shard, nrec, pitch, coef, out, cus);
  run<5, 2, 3, true>(shard, nrec, pitch, coef, out, cus);
  run<5, 2, 0, false>(shard, nrec, pitch, coef, out, cus);
  run<5, 2, 0, true>(shard, nrec, pitch, coef, out, cus);
  run<5, 2, 1, false>(shard, nrec, pitch, coef, out, cus);
  run<5, 2, 1, true>(shard, nrec, pitch, coef, out, cus);
  run<5, 2, 2, false>(shard, nrec, pitch, coef, out, cus);
  run<5, 2, 2, true>(shard, nrec, pitch, coef, out, cus);
  run<5, 2, 4, false>(shard, nrec, pitch, coef, out, cus);
  run<5, 2, 4, true>(shard, nrec, pitch, coef, out, cus);
  run<8, 2, 0, false>(shard, nrec, pitch, coef, out, cus);
  run<8, 2, 0, true>(shard, nrec, pitch, coef, out, cus);
  run<8, 2, 1, false>(shard, nrec, pitch, coef, out, cus);
  run<8, 2, 1, true>(shard, nrec, pitch, coef, out, cus);
  run<8, 2, 2, false>(shard, nrec, pitch, coef, out, cus);
  run<8, 2, 2, true>(shard, nrec, pitch, coef, out, cus);
  run<8, 2, 4, false>(shard, nrec, pitch, coef, out, cus);
  run<8, 2, 4, true>(shard, nrec, pitch, coef, out, cus);
  return 0;
}
