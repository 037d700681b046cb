// Micro-benchmark (not part of the product): the many-round GF(2^8) scan (C5: 5 rounds,
// wave-uniform coefficients, 1 KiB records) with the per-round bit-plane accumulators
// Z[a][k] ^= x  (for every row whose round-a coefficient has bit k set).
//   MODE 2: the product's form -- 8 masks per (row, round) from a 256 x 8-dword table
//           (s_load_dwordx8), one v_bitop3 per (plane, dword); 2 dwords per lane
//   MODE 6: "four Russians" over rows -- per group of 4 rows the 16 XOR combinations of the
//           rows are built once (15 VALU) into 16 consecutive VGPRs; each plane then takes ONE
//           v_xor whose source register is selected by the plane's 4-bit index (the plane's
//           bit of the 4 coefficients) through GPR-index mode (s_set_gpr_idx_idx); 1 dword per
//           lane, the index nibbles from a spread table (nibble k of spread[c] = bit k of c)
//   MODE 3: HBM only (one XOR per dword)
// WAVES = waves per CU (8: 2 per SIMD like k_query's scan waves; 16: 4 per SIMD).
// Both computing modes produce the same planes; their checksums must agree.
// Build: hipcc -O3 --offload-arch=gfx950 -o scan_4r scan_4r.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

constexpr int NQ = 5;

__constant__ uint32_t c_spread[256];  // nibble k = bit k of c

__device__ __forceinline__ uint32_t mxor(uint32_t z, uint32_t x, uint32_t m) {
  return __builtin_amdgcn_bitop3_b32(z, x, m, 0x78);
}

#define Z8(a) "+v"(Z[a][0]), "+v"(Z[a][1]), "+v"(Z[a][2]), "+v"(Z[a][3]), "+v"(Z[a][4]), "+v"(Z[a][5]), "+v"(Z[a][6]), "+v"(Z[a][7])
#define PL(a, k, op)                                                 \
  "s_bfe_u32 %[t], %[w" #a "], " #op "\n\t"                          \
  "s_set_gpr_idx_idx %[t]\n\t"                                       \
  "v_xor_b32 %" #k ", v112, %" #k "\n\t"

// one group of 4 rows x 1 dword per lane into the 40 planes (operands 0-39 = Z[a][k])
__device__ __forceinline__ void fold4(uint32_t (&Z)[NQ][8], uint32_t x0, uint32_t x1, uint32_t x2,
                                      uint32_t x3, uint32_t w0, uint32_t w1, uint32_t w2,
                                      uint32_t w3, uint32_t w4) {
  uint32_t t;
  asm volatile(
      "v_mov_b32 v112, 0\n\t"
      "v_mov_b32 v113, %[x0]\n\t"
      "v_mov_b32 v114, %[x1]\n\t"
      "v_xor_b32 v115, %[x0], %[x1]\n\t"
      "v_mov_b32 v116, %[x2]\n\t"
      "v_xor_b32 v117, %[x0], %[x2]\n\t"
      "v_xor_b32 v118, %[x1], %[x2]\n\t"
      "v_xor_b32 v119, v115, %[x2]\n\t"
      "v_mov_b32 v120, %[x3]\n\t"
      "v_xor_b32 v121, %[x0], %[x3]\n\t"
      "v_xor_b32 v122, %[x1], %[x3]\n\t"
      "v_xor_b32 v123, v115, %[x3]\n\t"
      "v_xor_b32 v124, %[x2], %[x3]\n\t"
      "v_xor_b32 v125, v117, %[x3]\n\t"
      "v_xor_b32 v126, v118, %[x3]\n\t"
      "v_xor_b32 v127, v119, %[x3]\n\t"
      "s_set_gpr_idx_on 0, gpr_idx(SRC0)\n\t"
      PL(0, 0, 0x40000) PL(0, 1, 0x40004) PL(0, 2, 0x40008) PL(0, 3, 0x4000c)
      PL(0, 4, 0x40010) PL(0, 5, 0x40014) PL(0, 6, 0x40018) PL(0, 7, 0x4001c)
      PL(1, 8, 0x40000) PL(1, 9, 0x40004) PL(1, 10, 0x40008) PL(1, 11, 0x4000c)
      PL(1, 12, 0x40010) PL(1, 13, 0x40014) PL(1, 14, 0x40018) PL(1, 15, 0x4001c)
      PL(2, 16, 0x40000) PL(2, 17, 0x40004) PL(2, 18, 0x40008) PL(2, 19, 0x4000c)
      PL(2, 20, 0x40010) PL(2, 21, 0x40014) PL(2, 22, 0x40018) PL(2, 23, 0x4001c)
      PL(3, 24, 0x40000) PL(3, 25, 0x40004) PL(3, 26, 0x40008) PL(3, 27, 0x4000c)
      PL(3, 28, 0x40010) PL(3, 29, 0x40014) PL(3, 30, 0x40018) PL(3, 31, 0x4001c)
      PL(4, 32, 0x40000) PL(4, 33, 0x40004) PL(4, 34, 0x40008) PL(4, 35, 0x4000c)
      PL(4, 36, 0x40010) PL(4, 37, 0x40014) PL(4, 38, 0x40018) PL(4, 39, 0x4001c)
      "s_set_gpr_idx_off"
      : Z8(0), Z8(1), Z8(2), Z8(3), Z8(4), [t] "=&s"(t)
      : [x0] "v"(x0), [x1] "v"(x1), [x2] "v"(x2), [x3] "v"(x3), [w0] "s"(w0), [w1] "s"(w1),
        [w2] "s"(w2), [w3] "s"(w3), [w4] "s"(w4)
      : "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122",
        "v123", "v124", "v125", "v126", "v127", "m0");
}

template <int MODE, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k(const uint8_t* __restrict__ shard, uint64_t nrec,
                                                const uint2* __restrict__ coef,
                                                const u32x8* __restrict__ mtab,
                                                uint32_t* __restrict__ out) {
  constexpr int VEC = MODE == 6 ? 1 : 2;
  __shared__ uint32_t lmt[256 * 8];  // MODE 7: the mask table in LDS
  if constexpr (MODE == 7) {
    for (int i = threadIdx.x; i < 256 * 8; i += blockDim.x)
      lmt[i] = ((i >> 3) >> (i & 7)) & 1 ? 0xffffffffu : 0u;
    __syncthreads();
  }
  constexpr int GROUPS = 1024 / (64 * VEC * 4);  // column groups of a 1 KiB record
  constexpr int U = 8;
  const int lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t grp = wv % GROUPS;
  const uint64_t wave = (uint64_t)blockIdx.x * (WAVES / GROUPS) + wv / GROUPS;
  const uint64_t nw = (uint64_t)gridDim.x * (WAVES / GROUPS);
  const uint64_t r0 = wave * nrec / nw, r1 = (wave + 1) * nrec / nw;
  const uint8_t* base = shard + grp * (64 * VEC * 4) + lane * VEC * 4;
  uint32_t Z[NQ][8][VEC];
#pragma unroll
  for (int a = 0; a < NQ; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int v = 0; v < VEC; ++v) Z[a][b][v] = 0;
  // rolling pipeline (as k_query's scan waves): the next batch's rows and coefficients are in
  // flight while the current batch folds
  uint32_t xn[U][VEC];
  uint2 cn[U];
  auto load_batch = [&](uint64_t r) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t rr = r + u < r1 ? r + u : r0;
      if constexpr (VEC == 2) {
        const u32x2 q = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(base + rr * 1024));
        xn[u][0] = q.x;
        xn[u][VEC - 1] = q.y;
      } else {
        xn[u][0] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(base + rr * 1024));
      }
      cn[u] = coef[rr];
    }
  };
  if (r0 + U <= r1) load_batch(r0);
  for (uint64_t r = r0; r + U <= r1; r += U) {
    uint32_t x[U][VEC];
    uint32_t c0[U], c1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) x[u][v] = xn[u][v];
      c0[u] = __builtin_amdgcn_readfirstlane(cn[u].x);
      c1[u] = __builtin_amdgcn_readfirstlane(cn[u].y);
    }
    load_batch(r + U);
    if constexpr (MODE == 3) {
#pragma unroll
      for (int u = 0; u < U; ++u) Z[0][0][0] ^= x[u][0];
    } else if constexpr (MODE == 7) {
      // masks from an LDS copy of the table: two broadcast ds_read_b128 per (row, round) into
      // VGPRs -- no scalar instruction per plane or per round
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int a = 0; a < NQ; ++a) {
          const uint32_t ca = ((a < 4 ? c0[u] : c1[u]) >> (8 * (a & 3))) & 0xffu;
          const uint4* mp = reinterpret_cast<const uint4*>(lmt) + 2 * ca;
          const uint4 m0 = mp[0], m1 = mp[1];
          const uint32_t t[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
          for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int v = 0; v < VEC; ++v) Z[a][b][v] = mxor(Z[a][b][v], x[u][v], t[b]);
        }
    } else if constexpr (MODE == 2) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int a = 0; a < NQ; ++a) {
          const uint32_t ca = ((a < 4 ? c0[u] : c1[u]) >> (8 * (a & 3))) & 0xffu;
          const u32x8 t = mtab[ca];
#pragma unroll
          for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int v = 0; v < VEC; ++v) Z[a][b][v] = mxor(Z[a][b][v], x[u][v], t[b]);
        }
    } else {
#pragma unroll
      for (int g = 0; g < U; g += 4) {
        uint32_t w[NQ];
#pragma unroll
        for (int a = 0; a < NQ; ++a) {
          uint32_t acc = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t ca = ((a < 4 ? c0[g + i] : c1[g + i]) >> (8 * (a & 3))) & 0xffu;
            acc |= c_spread[ca] << i;
          }
          w[a] = acc;
        }
        uint32_t(&Zf)[NQ][8] = reinterpret_cast<uint32_t(&)[NQ][8]>(Z);
        fold4(Zf, x[g][0], x[g + 1][0], x[g + 2][0], x[g + 3][0], w[0], w[1], w[2], w[3], w[4]);
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int a = 0; a < NQ; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc ^= Z[a][b][v] * (2 * (8 * a + b) + 1);
  // checksum independent of the lane / dword split: XOR of every plane word times its plane
  atomicXor(out, acc);
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

template <int MODE, int WAVES>
static int run(const uint8_t* shard, uint64_t nrec, const uint2* coef, const u32x8* mtab,
               uint32_t* out, int cus) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipMemset(out, 0, 4));
  hipLaunchKernelGGL((k<MODE, WAVES>), dim3(cus), dim3(WAVES * 64), 0, 0, shard, nrec, coef, mtab, out);
  uint32_t sum = 0;
  CK(hipMemcpy(&sum, out, 4, hipMemcpyDeviceToHost));
  CK(hipEventRecord(e0));
  const int iters = 5;
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL((k<MODE, WAVES>), dim3(cus), dim3(WAVES * 64), 0, 0, shard, nrec, coef, mtab, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  printf("MODE=%d WAVES=%2d  %.3f ms  %.1f GB/s  checksum %08x\n", MODE, WAVES, ms,
         nrec * 1024.0 / ms / 1e6, sum);
  return 0;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t nrec = 1ull << 22;  // 4 GiB
  uint8_t* shard;
  uint2* coef;
  u32x8* mtab;
  uint32_t* out;
  CK(hipMalloc(&shard, nrec * 1024));
  CK(hipMalloc(&coef, nrec * 8));
  CK(hipMalloc(&mtab, 256 * 32));
  CK(hipMalloc(&out, 256));
  uint32_t h[256 * 8], sp[256];
  for (int c = 0; c < 256; ++c) {
    sp[c] = 0;
    for (int b = 0; b < 8; ++b) {
      h[c * 8 + b] = ((c >> b) & 1) ? 0xffffffffu : 0u;
      sp[c] |= (uint32_t)((c >> b) & 1) << (4 * b);
    }
  }
  CK(hipMemcpy(mtab, h, sizeof(h), hipMemcpyHostToDevice));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(c_spread), sp, sizeof(sp)));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, shard, nrec * 1024, 1);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint8_t*)coef, nrec * 8, 2);
  CK(hipDeviceSynchronize());
  run<3, 8>(shard, nrec, coef, mtab, out, cus);
  run<2, 8>(shard, nrec, coef, mtab, out, cus);
  run<6, 8>(shard, nrec, coef, mtab, out, cus);
  run<7, 8>(shard, nrec, coef, mtab, out, cus);
  run<2, 16>(shard, nrec, coef, mtab, out, cus);
  run<7, 16>(shard, nrec, coef, mtab, out, cus);
  run<6, 16>(shard, nrec, coef, mtab, out, cus);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
