// Micro-benchmark (not part of the product): GF(2^8) scan of one shard pass for G keys at once
// (256-B records = one wave row, wave-uniform coefficients), two accumulate strategies:
//   bitplane<G>: 8 bit-plane accumulators per key, SGPR mask per coefficient bit + v_bitop3
//   nibble<G>  : per record, tables T_lo[n] = n*x and T_hi[n] = (16n)*x in registers (n < 16),
//                then Y_q ^= T_lo[c_q & 15] ^ T_hi[c_q >> 4] (uniform index: VGPR indexing)
// Build: hipcc -O3 --offload-arch=gfx950 -o batch_scan batch_scan.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t xt(uint32_t x) {
  return ((x & 0x7f7f7f7fu) << 1) ^ (((x >> 7) & 0x01010101u) * 0x1du);
}
__device__ __forceinline__ uint32_t fold8(const uint32_t* z) {
  uint32_t t = z[7];
  for (int b = 6; b >= 0; --b) t = xt(t) ^ z[b];
  return t;
}

template <int G, int MODE>
__global__ __launch_bounds__(512) void k(const uint32_t* __restrict__ shard, uint64_t nrec,
                                         const uint8_t* __restrict__ coef, uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 8 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 8;
  const uint64_t r0 = wave * nrec / nw, r1 = (wave + 1) * nrec / nw;
  constexpr int NZ = MODE == 0 ? 8 * G : G;
  uint32_t Z[NZ];
#pragma unroll
  for (int i = 0; i < NZ; ++i) Z[i] = 0;
  constexpr int U = 4;
  for (uint64_t r = r0; r + U <= r1; r += U) {
    uint32_t x[U];
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(shard + r * 64), 0, U * 256, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, u * 256, 2);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t* cw = reinterpret_cast<const uint32_t*>(coef + (r + u) * G);
      if constexpr (MODE == 0) {
#pragma unroll
        for (int q4 = 0; q4 < G / 4; ++q4) {
          const uint32_t c4 = __builtin_amdgcn_readfirstlane(cw[q4]);
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int b = 0; b < 8; ++b) {
              const uint32_t m = (uint32_t)((int32_t)(c4 << (31 - (8 * j + b))) >> 31);
              Z[(4 * q4 + j) * 8 + b] = __builtin_amdgcn_bitop3_b32(Z[(4 * q4 + j) * 8 + b], x[u], m, 0x78);
            }
        }
      } else {
        uint32_t T[32];
        T[0] = 0;
        T[1] = x[u];
#pragma unroll
        for (int i = 2; i < 16; ++i) T[i] = (i & 1) ? (T[i - 1] ^ x[u]) : xt(T[i / 2]);
        T[16] = 0;
        T[17] = xt(T[8]);
#pragma unroll
        for (int i = 2; i < 16; ++i) T[16 + i] = (i & 1) ? (T[16 + i - 1] ^ T[17]) : xt(T[16 + i / 2]);
#pragma unroll
        for (int q4 = 0; q4 < G / 4; ++q4) {
          const uint32_t c4 = __builtin_amdgcn_readfirstlane(cw[q4]);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t c = (c4 >> (8 * j)) & 0xffu;
            Z[4 * q4 + j] = __builtin_amdgcn_bitop3_b32(Z[4 * q4 + j], T[c & 15], T[16 + (c >> 4)], 0x96);
          }
        }
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int q = 0; q < G; ++q) acc ^= (MODE == 0 ? fold8(&Z[8 * q]) : Z[q]) * (2 * q + 1);
  atomicXor(out + lane, acc);
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

template <int G, int MODE>
static int run(const uint32_t* shard, uint64_t nrec, const uint8_t* coef, uint32_t* out, int cus, int bpc) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  dim3 grid(cus * bpc);
  hipLaunchKernelGGL((k<G, MODE>), grid, dim3(512), 0, 0, shard, nrec, coef, out);
  CK(hipEventRecord(e0));
  const int iters = 3;
  for (int it = 0; it < iters; ++it) hipLaunchKernelGGL((k<G, MODE>), grid, dim3(512), 0, 0, shard, nrec, coef, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  uint32_t h[64];
  CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
  uint32_t cs = 0;
  for (int i = 0; i < 64; ++i) cs ^= h[i] * (i + 1);
  printf("G=%2d MODE=%d bpc=%d  %.3f ms/pass  %.4f ms/key  %.1f GB/s  csum=%08x\n", G, MODE, bpc, ms, ms / G,
         nrec * 256.0 / ms / 1e6, cs);
  CK(hipMemset(out, 0, 256));
  return 0;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t nrec = 1ull << 22;
  uint32_t* shard;
  uint8_t* coef;
  uint32_t* out;
  CK(hipMalloc(&shard, nrec * 256));
  CK(hipMalloc(&coef, nrec * 64));
  CK(hipMalloc(&out, 256));
  CK(hipMemset(out, 0, 256));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint8_t*)shard, nrec * 256, 1);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, coef, nrec * 64, 2);
  CK(hipDeviceSynchronize());
  run<8, 0>(shard, nrec, coef, out, cus, 2);
  run<8, 1>(shard, nrec, coef, out, cus, 2);
  run<16, 1>(shard, nrec, coef, out, cus, 2);
  run<32, 1>(shard, nrec, coef, out, cus, 2);
  run<64, 1>(shard, nrec, coef, out, cus, 2);
  run<64, 1>(shard, nrec, coef, out, cus, 1);
  return 0;
}
