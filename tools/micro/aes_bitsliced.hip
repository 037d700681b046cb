// Micro-benchmark (not part of the product): a table-free, bitsliced AES-128 for the DPF tree's
// PRG on gfx950, measured against the production T-table AES (pir_aes.h) on the same work.
//
// Layout ("DPP quad"): a quad of 4 lanes holds 32 nodes; lane q holds COLUMN q
// of each node's state and round key as 32 bit-planes (plane 8r + i = bit i of row r; bit j of a
// plane = node j).  Per round and lane:
//   SubBytes    4 Boyar-Peralta S-box circuits (34 AND + 94 XOR/XNOR as written; the compiler
//               fuses gates into v_bitop3) on the lane's own 4 bytes;
//   ShiftRows   row r of column q <- row r of column q+r: 8 DPP quad_perm moves per row 1..3;
//   MixColumns  + AddRoundKey on the lane's own column (xtime on planes is renaming + 3 XORs);
//   key         RotWord/SubWord: lane q takes byte (q+1)%4 of column 3 (broadcast from lane 3,
//               selected by v_bitop3), one S-box, the 4 bytes gathered back (DPP), and the
//               prefix XOR k'_q = T ^ k_0 ^ .. ^ k_q across the quad (2 DPP steps).
// An internal node is G(seed) = 3 CTR blocks under one key schedule, as aes_ctr_row<3,..>; a
// leaf block 1 block.  Seeds and outputs stay bitsliced (a bitsliced tree would keep them so:
// children are block-0/1 outputs of their parents), so no transposes are timed; a separate
// check transposes 32 seeds per quad and compares every output byte with the T-table AES.
//
// Prints, for both forms: nodes/s over all CUs.  Run under
//   rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE -- ./aes_bitsliced
// for instruction counts per node (VALU lane-ops per node = SQ_INSTS_VALU * 64 / nodes).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../erasurecodedpir_amd/csrc -o aes_bitsliced aes_bitsliced.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

#include "pir_aes.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

namespace bs {

template <int CTRL>
__device__ __forceinline__ uint32_t qp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t sel(uint32_t a, uint32_t b, uint32_t m) {  // m ? a : b
  return __builtin_amdgcn_bitop3_b32(a, b, m, 0xE4);  // table index = S0*4 + S1*2 + S2
}

// Boyar-Peralta S-box (verified exhaustively on the host, 256/256): x[i] = plane of bit i
// (U0 = bit 7 ... U7 = bit 0); y[i] = output bit i.
__device__ __forceinline__ void sbox(const uint32_t* x, uint32_t* y) {
  const uint32_t U0 = x[7], U1 = x[6], U2 = x[5], U3 = x[4], U4 = x[3], U5 = x[2], U6 = x[1],
                 U7 = x[0];
  const uint32_t T1 = U0 ^ U3, T2 = U0 ^ U5, T3 = U0 ^ U6, T4 = U3 ^ U5, T5 = U4 ^ U6;
  const uint32_t T6 = T1 ^ T5, T7 = U1 ^ U2, T8 = U7 ^ T6, T9 = U7 ^ T7, T10 = T6 ^ T7;
  const uint32_t T11 = U1 ^ U5, T12 = U2 ^ U5, T13 = T3 ^ T4, T14 = T6 ^ T11, T15 = T5 ^ T11;
  const uint32_t T16 = T5 ^ T12, T17 = T9 ^ T16, T18 = U3 ^ U7, T19 = T7 ^ T18, T20 = T1 ^ T19;
  const uint32_t T21 = U6 ^ U7, T22 = T7 ^ T21, T23 = T2 ^ T22, T24 = T2 ^ T10, T25 = T20 ^ T17;
  const uint32_t T26 = T3 ^ T16, T27 = T1 ^ T12;
  const uint32_t M1 = T13 & T6, M2 = T23 & T8, M3 = T14 ^ M1, M4 = T19 & U7, M5 = M4 ^ M1;
  const uint32_t M6 = T3 & T16, M7 = T22 & T9, M8 = T26 ^ M6, M9 = T20 & T17, M10 = M9 ^ M6;
  const uint32_t M11 = T1 & T15, M12 = T4 & T27, M13 = M12 ^ M11, M14 = T2 & T10, M15 = M14 ^ M11;
  const uint32_t M16 = M3 ^ M2, M17 = M5 ^ T24, M18 = M8 ^ M7, M19 = M10 ^ M15, M20 = M16 ^ M13;
  const uint32_t M21 = M17 ^ M15, M22 = M18 ^ M13, M23 = M19 ^ T25, M24 = M22 ^ M23;
  const uint32_t M25 = M22 & M20, M26 = M21 ^ M25, M27 = M20 ^ M21, M28 = M23 ^ M25;
  const uint32_t M29 = M28 & M27, M30 = M26 & M24, M31 = M20 & M23, M32 = M27 & M31;
  const uint32_t M33 = M27 ^ M25, M34 = M21 & M22, M35 = M24 & M34, M36 = M24 ^ M25;
  const uint32_t M37 = M21 ^ M29, M38 = M32 ^ M33, M39 = M23 ^ M30, M40 = M35 ^ M36;
  const uint32_t M41 = M38 ^ M40, M42 = M37 ^ M39, M43 = M37 ^ M38, M44 = M39 ^ M40;
  const uint32_t M45 = M42 ^ M41;
  const uint32_t M46 = M44 & T6, M47 = M40 & T8, M48 = M39 & U7, M49 = M43 & T16, M50 = M38 & T9;
  const uint32_t M51 = M37 & T17, M52 = M42 & T15, M53 = M45 & T27, M54 = M41 & T10;
  const uint32_t M55 = M44 & T13, M56 = M40 & T23, M57 = M39 & T19, M58 = M43 & T3;
  const uint32_t M59 = M38 & T22, M60 = M37 & T20, M61 = M42 & T1, M62 = M45 & T4, M63 = M41 & T2;
  const uint32_t L0 = M61 ^ M62, L1 = M50 ^ M56, L2 = M46 ^ M48, L3 = M47 ^ M55, L4 = M54 ^ M58;
  const uint32_t L5 = M49 ^ M61, L6 = M62 ^ L5, L7 = M46 ^ L3, L8 = M51 ^ M59, L9 = M52 ^ M53;
  const uint32_t L10 = M53 ^ L4, L11 = M60 ^ L2, L12 = M48 ^ M51, L13 = M50 ^ L0, L14 = M52 ^ M61;
  const uint32_t L15 = M55 ^ L1, L16 = M56 ^ L0, L17 = M57 ^ L1, L18 = M58 ^ L8, L19 = M63 ^ L4;
  const uint32_t L20 = L0 ^ L1, L21 = L1 ^ L7, L22 = L3 ^ L12, L23 = L18 ^ L2, L24 = L15 ^ L9;
  const uint32_t L25 = L6 ^ L10, L26 = L7 ^ L9, L27 = L8 ^ L10, L28 = L11 ^ L14, L29 = L11 ^ L17;
  y[7] = L6 ^ L24;
  y[6] = ~(L16 ^ L26);
  y[5] = ~(L19 ^ L28);
  y[4] = L6 ^ L21;
  y[3] = L20 ^ L22;
  y[2] = L25 ^ L29;
  y[1] = ~(L13 ^ L27);
  y[0] = ~(L6 ^ L23);
}

constexpr int kQ1230 = 0x39, kQ2301 = 0x4E, kQ3012 = 0x93, kQ3333 = 0xFF;
constexpr int kQ0000 = 0x00, kQ1111 = 0x55, kQ2222 = 0xAA;
constexpr int kQ0012 = 0x90, kQ0101 = 0x44;
constexpr uint32_t kRcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};

struct Lane {
  uint32_t mA, mB;    // byte (q+1)%4 select bits: bit 0 / bit 1 of that byte index
  uint32_t mq1, mq2;  // q >= 1, q >= 2
  uint32_t is0, is3;  // q == 0, q == 3
  __device__ explicit Lane(uint32_t q) {
    const uint32_t b = (q + 1) & 3u;
    mA = (b & 1u) ? ~0u : 0u;
    mB = (b & 2u) ? ~0u : 0u;
    mq1 = q >= 1 ? ~0u : 0u;
    mq2 = q >= 2 ? ~0u : 0u;
    is0 = q == 0 ? ~0u : 0u;
    is3 = q == 3 ? ~0u : 0u;
  }
};

// round key r+1 from round key r (k[32] = this lane's column, in place)
__device__ __forceinline__ void key_next(const Lane& L, uint32_t (&k)[32], int r) {
  uint32_t x[8], s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // byte (q+1)%4 of column 3
    const uint32_t b0 = qp<kQ3333>(k[i]), b1 = qp<kQ3333>(k[8 + i]);
    const uint32_t b2 = qp<kQ3333>(k[16 + i]), b3 = qp<kQ3333>(k[24 + i]);
    x[i] = sel(sel(b3, b2, L.mA), sel(b1, b0, L.mA), L.mB);
  }
  sbox(x, s);  // lane q: byte q of SubWord(RotWord(w3))
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t t0 = qp<kQ0000>(s[i]), t1 = qp<kQ1111>(s[i]), t2 = qp<kQ2222>(s[i]),
             t3 = qp<kQ3333>(s[i]);
    if ((kRcon[r] >> i) & 1u) t0 = ~t0;
    // prefix over the quad: P_q = k_0 ^ ... ^ k_q, then k'_q = T ^ P_q
    uint32_t y0 = k[i] ^ (qp<kQ0012>(k[i]) & L.mq1);
    uint32_t y1 = k[8 + i] ^ (qp<kQ0012>(k[8 + i]) & L.mq1);
    uint32_t y2 = k[16 + i] ^ (qp<kQ0012>(k[16 + i]) & L.mq1);
    uint32_t y3 = k[24 + i] ^ (qp<kQ0012>(k[24 + i]) & L.mq1);
    k[i] = __builtin_amdgcn_bitop3_b32(y0, qp<kQ0101>(y0) & L.mq2, t0, 0x96);
    k[8 + i] = __builtin_amdgcn_bitop3_b32(y1, qp<kQ0101>(y1) & L.mq2, t1, 0x96);
    k[16 + i] = __builtin_amdgcn_bitop3_b32(y2, qp<kQ0101>(y2) & L.mq2, t2, 0x96);
    k[24 + i] = __builtin_amdgcn_bitop3_b32(y3, qp<kQ0101>(y3) & L.mq2, t3, 0x96);
  }
}

// SubBytes + ShiftRows on this lane's column (out of place: w -> v)
__device__ __forceinline__ void sub_shift(const uint32_t (&w)[32], uint32_t (&v)[32]) {
  uint32_t s[32];
#pragma unroll
  for (int r = 0; r < 4; ++r) sbox(&w[8 * r], &s[8 * r]);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] = s[i];
    v[8 + i] = qp<kQ1230>(s[8 + i]);
    v[16 + i] = qp<kQ2301>(s[16 + i]);
    v[24 + i] = qp<kQ3012>(s[24 + i]);
  }
}

// MixColumns + AddRoundKey on this lane's column
__device__ __forceinline__ void mix_ark(const uint32_t (&a)[32], const uint32_t (&k)[32],
                                        uint32_t (&w)[32]) {
  uint32_t t[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = __builtin_amdgcn_bitop3_b32(a[i], a[8 + i], a[16 + i], 0x96) ^ a[24 + i];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int rn = (r + 1) & 3;
    uint32_t d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = a[8 * r + i] ^ a[8 * rn + i];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint32_t xt = i == 0 ? d[7] : d[i - 1];
      const uint32_t base = __builtin_amdgcn_bitop3_b32(a[8 * r + i], t[i], k[8 * r + i], 0x96);
      if (i == 1 || i == 3 || i == 4) xt = xt ^ d[7];
      w[8 * r + i] = base ^ xt;
    }
  }
}

// NB CTR blocks (counters 0..NB-1: BE128(c) = byte 15 = row 3 of column 3) under the key planes
// `key` (this lane's column), 10 rounds, outputs o[b] (this lane's column of block b)
template <int NB>
__device__ __forceinline__ void aes_ctr(const Lane& L, const uint32_t (&key)[32],
                                        uint32_t (&o)[NB][32]) {
  uint32_t k[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) k[i] = key[i];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      uint32_t v = k[i];
      if (i >= 24 && (((uint32_t)b >> (i - 24)) & 1u)) v ^= L.is3;  // counter byte
      o[b][i] = v;
    }
#pragma unroll 1
  for (int r = 0; r < 10; ++r) {
    key_next(L, k, r);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      uint32_t v[32];
      sub_shift(o[b], v);
      if (r < 9) {
        mix_ark(v, k, o[b]);
      } else {
#pragma unroll
        for (int i = 0; i < 32; ++i) o[b][i] = v[i] ^ k[i];
      }
    }
  }
}

}  // namespace bs

// throughput: every quad expands `iters` rounds of 32 nodes (seeds chained through block 0)
template <int NB>
__global__ __launch_bounds__(256) void k_bs(int iters, uint32_t salt, uint32_t* out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const bs::Lane L(threadIdx.x & 3u);
  uint32_t key[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) key[i] = (g * 0x9E3779B9u) ^ (i * 0x85EBCA6Bu) ^ salt;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t o[NB][32];
    bs::aes_ctr<NB>(L, key, o);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      uint32_t x = 0;
#pragma unroll
      for (int b = 0; b < NB; ++b) x ^= o[b][i];
      acc ^= x;
      key[i] = o[0][i] ^ (uint32_t)it;  // next 32 "children" (a tree descent of 32-node groups)
    }
  }
  if (acc == 0x12345678u) out[g] = acc;
}

// the production T-table node in the same harness (aes_node.hip's kernel)
template <int NB>
__global__ __launch_bounds__(1024) void k_tt(int iters, uint32_t salt, uint32_t* out) {
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

// correctness: 32 seeds per quad (seed[j] for node j), transposed in, 3 blocks, transposed out;
// out[(quad * 32 + j) * 12 + b * 4 + c] = word c of block b of node j
__global__ __launch_bounds__(64) void k_check(const uint4* __restrict__ seeds, uint32_t* __restrict__ out) {
  const uint32_t q = threadIdx.x & 3u, quad = (blockIdx.x * blockDim.x + threadIdx.x) >> 2;
  const bs::Lane L(q);
  const uint4* sd = seeds + quad * 32;
  uint32_t key[32];
  for (int p = 0; p < 32; ++p) {  // plane 8r + i of column q: bit (8r + i) of word q
    uint32_t v = 0;
    for (int j = 0; j < 32; ++j) {
      const uint4 s = sd[j];
      const uint32_t w = q == 0 ? s.x : (q == 1 ? s.y : (q == 2 ? s.z : s.w));
      v |= ((w >> p) & 1u) << j;
    }
    key[p] = v;
  }
  uint32_t o[3][32];
  bs::aes_ctr<3>(L, key, o);
  for (int b = 0; b < 3; ++b)
    for (int j = 0; j < 32; ++j) {
      uint32_t w = 0;
      for (int p = 0; p < 32; ++p) w |= ((o[b][p] >> j) & 1u) << p;
      out[(quad * 32 + j) * 12 + b * 4 + q] = w;
    }
}

__global__ void k_ref(const uint4* __restrict__ seeds, uint32_t* __restrict__ out, int n) {
  __shared__ uint32_t tab[pir::kTablesBytes / 4];
  pir::load_tables(tab);
  __syncthreads();
  const pir::Tab T(tab);
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    uint4 o[3];
    pir::aes_ctr_row<3, 4>(T, seeds[j], o);
    for (int b = 0; b < 3; ++b) {
      out[j * 12 + b * 4 + 0] = o[b].x; out[j * 12 + b * 4 + 1] = o[b].y;
      out[j * 12 + b * 4 + 2] = o[b].z; out[j * 12 + b * 4 + 3] = o[b].w;
    }
  }
}

template <typename F>
static int timed(const char* name, F launch, double nodes) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch(4);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  launch(0);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-62s %8.3f ms  %7.2f G nodes/s\n", name, ms, nodes / ms / 1e6);
  return 0;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  pir::upload_te0(0);
  uint32_t* out;
  CK(hipMalloc(&out, (size_t)cus * 4096 * 4 * 8));
  // correctness against the T-table AES: 64 quads x 32 nodes
  {
    const int nq = 64, n = nq * 32;
    std::vector<uint32_t> h(n * 4);
    uint64_t x = 0x243F6A8885A308D3ull;
    for (auto& v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint32_t)x; }
    uint4* d_seeds;
    uint32_t *d_a, *d_b;
    CK(hipMalloc(&d_seeds, n * 16));
    CK(hipMalloc(&d_a, n * 48));
    CK(hipMalloc(&d_b, n * 48));
    CK(hipMemcpy(d_seeds, h.data(), n * 16, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_check, dim3(nq * 4 / 64), dim3(64), 0, 0, d_seeds, d_a);
    hipLaunchKernelGGL(k_ref, dim3(1), dim3(256), 0, 0, d_seeds, d_b, n);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> a(n * 12), b(n * 12);
    CK(hipMemcpy(a.data(), d_a, n * 48, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), d_b, n * 48, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < n * 12; ++i) bad += a[i] != b[i];
    printf("bitsliced vs T-table AES-128-CTR (3 blocks, %d seeds): %s (%d words differ)\n", n,
           bad ? "DIFFER" : "equal", bad);
    if (bad) return 2;
  }
  const int itb = 40, itt = 2000;
  // bitsliced: 256-thread blocks, 4 per CU x 4 waves = 16 waves per CU (VGPR permitting)
  for (int bpc : {2, 4, 8}) {
    char name[128];
    snprintf(name, sizeof name, "bitsliced G(seed) 3 blocks, 32 nodes/quad, %d x 256 thr/CU", bpc);
    const int grid = cus * bpc;
    timed(name, [&](int warm) {
      hipLaunchKernelGGL(k_bs<3>, dim3(grid), dim3(256), 0, 0, warm ? warm : itb, 1u, out);
    }, (double)grid * 256 / 4 * 32 * itb);
  }
  {
    const int grid = cus * 4;
    timed("bitsliced leaf block (1 block), 4 x 256 thr/CU", [&](int warm) {
      hipLaunchKernelGGL(k_bs<1>, dim3(grid), dim3(256), 0, 0, warm ? warm : itb * 2, 1u, out);
    }, (double)grid * 256 / 4 * 32 * itb * 2);
  }
  timed("T-table G(seed) 3 blocks (aes_ctr_row<3,1>), 1024 thr/CU", [&](int warm) {
    hipLaunchKernelGGL(k_tt<3>, dim3(cus), dim3(1024), 0, 0, warm ? warm : itt, 2u, out);
  }, (double)cus * 1024 * itt);
  timed("T-table leaf block (aes_ctr_row<1,1>), 1024 thr/CU", [&](int warm) {
    hipLaunchKernelGGL(k_tt<1>, dim3(cus), dim3(1024), 0, 0, warm ? warm : itt * 2, 2u, out);
  }, (double)cus * 1024 * itt * 2);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
