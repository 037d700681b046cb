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

#include "aes_bs.h"

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
