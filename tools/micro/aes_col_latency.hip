// Micro-benchmark (not part of the product): the dependent chain of k_query's tile-root descent,
// one wave: per level ONE column-shape PRG call (16 lanes = 4 CTR blocks x 4 columns; every
// quad of the wave the same node), the chosen child's 4 key words back to every lane through
// v_readlane (SGPRs), as pir_kernels.hip's descent does.  Variants of the column AES:
//   col  : pir_aes.h aes_col (lane q holds key word q; the key schedule's prefix XOR by DPP)
//   col2 : every lane holds the whole round key (the schedule's word chain as prefixes of the
//          old key, off the critical path; no DPP in the key path), lane q picks word q
// Output: cycles per level (s_memtime) and the 4 key words after `iters` levels (the two
// variants must agree).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../erasurecodedpir_amd/csrc -o aes_col_latency aes_col_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "pir_aes.h"

using namespace pir;

__device__ __forceinline__ uint32_t aes_col2(const Tab& T, uint32_t k0, uint32_t k1, uint32_t k2,
                                             uint32_t k3, uint32_t ptq, uint32_t q) {
  const bool q0 = q == 0, q1 = q == 1, q2 = q == 2;
  auto pick = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return q0 ? a : (q1 ? b : (q2 ? c : d));
  };
  uint32_t w = pick(k0, k1, k2, k3) ^ ptq;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t p1 = k0 ^ k1, p2 = p1 ^ k2, p3 = p2 ^ k3;  // old-key prefixes
    const uint32_t pq = pick(k0, p1, p2, p3);
    const uint32_t t = (T.t2<1>(k3) & 0xffu) | (T.t0<2>(k3) & 0xff00u) |
                       (T.t0<3>(k3) & 0xff0000u) | (T.t2<0>(k3) & 0xff000000u);
    const uint32_t tr = t ^ kRcon[r];
    k0 ^= tr; k1 = p1 ^ tr; k2 = p2 ^ tr; k3 = p3 ^ tr;
    const uint32_t kq = pq ^ tr;
    const uint32_t b = qperm<kQ1230>(w), c = qperm<kQ2301>(w), d = qperm<kQ3012>(w);
    if (r < 9)
      w = xor3(T.t0<0>(w), T.t2<2>(c), rotl8(xor3(T.t0<1>(b), T.t2<3>(d), rotr8(kq))));
    else
      w = last_col(T, w, b, c, d, kq);
  }
  return w;
}

template <int V>
__global__ __launch_bounds__(1024) void k_desc(int iters, uint32_t* out, long long* cyc) {
  __shared__ uint32_t tab[2 * 256 * 32];
  load_tables(tab);
  __syncthreads();
  if (threadIdx.x >= 64) {  // the other waves park at a barrier (as in k_query's descent)
    __syncthreads();
    return;
  }
  const Tab T(tab);
  const uint32_t lane = threadIdx.x & 63u, q = lane & 3u, role = (lane >> 2) & 3u;
  const uint32_t mq1 = q >= 1 ? ~0u : 0u, mq2 = q >= 2 ? ~0u : 0u;
  const uint32_t ptq = q == 3 ? (role << 24) : 0u;
  const uint32_t m0 = q == 0 ? ~0u : 0u, m1 = q == 1 ? ~0u : 0u, m2 = q == 2 ? ~0u : 0u,
                 m3 = q == 3 ? ~0u : 0u;
  uint32_t c0 = 0x03020100u, c1 = 0x07060504u, c2 = 0x0b0a0908u, c3 = 0x0f0e0d0cu;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    uint32_t o;
    if constexpr (V == 0) {
      const uint32_t sq = (c0 & m0) | (c1 & m1) | (c2 & m2) | (c3 & m3);
      o = aes_col(T, sq, ptq, mq1, mq2);
    } else {
      o = aes_col2(T, c0, c1, c2, c3, ptq, q);
    }
    const int bit = i & 1;  // left / right child alternately (block 0 / block 1)
    c0 = (uint32_t)__builtin_amdgcn_readlane((int)o, 4 * bit + 0);
    c1 = (uint32_t)__builtin_amdgcn_readlane((int)o, 4 * bit + 1);
    c2 = (uint32_t)__builtin_amdgcn_readlane((int)o, 4 * bit + 2);
    c3 = (uint32_t)__builtin_amdgcn_readlane((int)o, 4 * bit + 3);
  }
  const long long t1 = clock64();
  if (lane == 0) {
    out[4 * blockIdx.x + 0] = c0; out[4 * blockIdx.x + 1] = c1;
    out[4 * blockIdx.x + 2] = c2; out[4 * blockIdx.x + 3] = c3;
    if (blockIdx.x == 0) *cyc = t1 - t0;
  }
  __syncthreads();
}

int main() {
  uint32_t* d_o;
  long long* d_c;
  (void)hipMalloc(&d_o, 256 * 16);
  (void)hipMalloc(&d_c, 8);
  const int iters = 2000;
  uint32_t h[2][4];
  for (int v = 0; v < 2; ++v) {
    long long best = 1ll << 62;
    for (int r = 0; r < 3; ++r) {
      if (v == 0) hipLaunchKernelGGL(k_desc<0>, dim3(256), dim3(1024), 0, 0, iters, d_o, d_c);
      else hipLaunchKernelGGL(k_desc<1>, dim3(256), dim3(1024), 0, 0, iters, d_o, d_c);
      if (hipDeviceSynchronize() != hipSuccess) return 1;
      long long c;
      (void)hipMemcpy(&c, d_c, 8, hipMemcpyDeviceToHost);
      if (c < best) best = c;
    }
    (void)hipMemcpy(h[v], d_o, 16, hipMemcpyDeviceToHost);
    printf("%-5s %8.1f cycles per level (s_memtime), key %08x %08x %08x %08x\n",
           v == 0 ? "col" : "col2", (double)best / iters, h[v][0], h[v][1], h[v][2], h[v][3]);
  }
  const bool same = h[0][0] == h[1][0] && h[0][1] == h[1][1] && h[0][2] == h[1][2] && h[0][3] == h[1][3];
  printf("variants %s\n", same ? "AGREE" : "DIFFER");
  return same ? 0 : 2;
}
