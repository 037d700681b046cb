// pir_leaves.hip -- the leaf-converting last stage of the DPF tree, depth first per lane.
//
// k_expand builds a stage breadth first in LDS: a workgroup of 1024 threads starts from `tile`
// nodes, so its first levels keep only 4 and 8 of its 16 waves busy (256 and 512 nodes) and
// every level ends at a barrier.  Here every lane owns ONE input node of level L0 and walks its
// subtree of 2^KD leaves depth first in registers (the pending right child of each level waits
// in 5 VGPRs), so all waves are busy from the first level, there is no node traffic through
// LDS and no barrier after the table fill.  The work is the reference's (dpf_tree.cpp:525-580):
// KD levels of G(seed) expansions + correction words, then the leaf conversion
//   c[leaf][a] = AES_{s_leaf}(0)[a] ^ XOR_{k: t_leaf bit k} lastCW[k][a]   (a < nq).
// blockIdx.y = key of a batch (its DevKey, input node range and share slot), as in k_expand.
#include "pir_kernels.h"
#include "pir_tree.h"
#include "pir_aes4.h"

#include <stdlib.h>

namespace pir {

void upload_leaves_aes_table(hipStream_t s) { upload_te0(s); }

constexpr int kLeafThreads = 1024;  // one workgroup (128 KiB of tables) per CU: 16 waves

__device__ __forceinline__ uint4 and_q(const uint4& v, const uint4& m) {
  return make_uint4(v.x & m.x, v.y & m.y, v.z & m.z, v.w & m.w);
}

// G(seed) of an internal node (the 4-table AES; TB valid bytes of the control-bit block)
template <int TB>
__device__ __forceinline__ void expand_node4(const Tab4& T, const DevKey* __restrict__ K, int L,
                                             const Bits& B, uint4 seed, uint32_t t, uint4& sl,
                                             uint4& sr, uint32_t& tl, uint32_t& tr) {
  uint4 o[3];
  aes_ctr_row4<3, TB>(T, seed, o);
  uint4 cs;
  uint32_t ct;
  level_cw(K, L, t, B.pm1, cs, ct);
  sl = xor4(o[0], cs);
  sr = xor4(o[1], cs);
  const uint32_t tb = (o[2].x & B.tb_mask) ^ ct;
  tl = tb & B.tmask;
  tr = (tb >> B.pm1) & B.tmask;
}

// the leaf value's NRP bytes (the rest: don't care; the caller masks to nq)
template <int NRP>
__device__ __forceinline__ uint4 leaf_value4(const Tab4& T, const DevKey* __restrict__ K,
                                             uint32_t pm1, uint4 seed, uint32_t t) {
  uint4 o[1];
  aes_ctr_row4<1, NRP>(T, seed, o);
  for (uint32_t j = 0; j < pm1; ++j) o[0] = xor4(o[0], and4(K->lastcw[j], 0u - ((t >> j) & 1u)));
  return o[0];
}

// the 2^D leaves under node (s, t) of level L, leaf indices [leaf, leaf + 2^D)
template <int NRP, int TB, int D>
__device__ __forceinline__ void leaves_dfs(const Tab4& T, const DevKey* __restrict__ K, int L,
                                           const Bits& B, uint4 s, uint32_t t,
                                           uint8_t* __restrict__ c, uint64_t leaf,
                                           uint32_t cstride, const uint4& qm) {
  uint4 sl, sr;
  uint32_t tl, tr;
  expand_node4<TB>(T, K, L, B, s, t, sl, sr, tl, tr);
  if constexpr (D == 1) {
    const uint4 vl = leaf_value4<NRP>(T, K, B.pm1, sl, tl);
    const uint4 vr = leaf_value4<NRP>(T, K, B.pm1, sr, tr);
    store_leaf<NRP>(c, leaf, and_q(vl, qm), cstride);
    store_leaf<NRP>(c, leaf + 1, and_q(vr, qm), cstride);
  } else {
    // one copy of the subtree code per level: the right child waits in registers
#pragma unroll 1
    for (int i = 0; i < 2; ++i)
      leaves_dfs<NRP, TB, D - 1>(T, K, L + 1, B, i ? sr : sl, i ? tr : tl, c,
                                 leaf + ((uint64_t)i << (D - 1)), cstride, qm);
  }
}

template <int NRP, int TB, int KD>
__global__ __launch_bounds__(kLeafThreads)
void k_leaves(const DevKey* __restrict__ K, const uint4* __restrict__ in_s,
              const uint32_t* __restrict__ in_t, int L0, uint64_t nin, uint64_t in_stride,
              uint8_t* __restrict__ c, uint32_t cstride, uint32_t c_key_off) {
  K += blockIdx.y;
  in_s += blockIdx.y * in_stride;
  in_t += blockIdx.y * in_stride;
  c += (size_t)blockIdx.y * c_key_off;
  __shared__ uint32_t tab[kTab4Bytes / 4];
  load_tables4_n<kLeafThreads>(tab);
  const Bits B(K->p);
  uint4 qm;  // keep the nq output bytes
  {
    const int nq = (int)K->nq;
    uint32_t m[4];
    for (int w = 0; w < 4; ++w) {
      const int nb = nq - 4 * w;
      m[w] = nb >= 4 ? 0xffffffffu : (nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u));
    }
    qm = make_uint4(m[0], m[1], m[2], m[3]);
  }
  __syncthreads();
  const Tab4 T(tab);
  const uint64_t u = (uint64_t)blockIdx.x * kLeafThreads + threadIdx.x;
  if (u >= nin) return;  // no barrier below
  leaves_dfs<NRP, TB, KD>(T, K, L0, B, in_s[u], in_t[u], c, u << KD, cstride, qm);
}

bool leaves_supported(int kd) { return kd >= kLeavesMinK && kd <= kLeavesMaxK; }

template <int NRP, int TB>
static hipError_t leaves_tb(int kd, dim3 grid, const DevKey* d_key, const uint4* is,
                             const uint32_t* it, int L0, uint64_t nin, uint64_t in_stride,
                             uint8_t* c, uint32_t cstride, uint32_t c_key_off, hipStream_t s) {
#define PIR_LV(KD)                                                                            \
  hipLaunchKernelGGL((k_leaves<NRP, TB, KD>), grid, dim3(kLeafThreads), 0, s, d_key, is, it, L0, \
                     nin, in_stride, c, cstride, c_key_off)
  switch (kd) {
    case 4: PIR_LV(4); break;
    case 5: PIR_LV(5); break;
    default: return hipErrorInvalidValue;
  }
#undef PIR_LV
  return hipGetLastError();
}

// TB = bytes of the control-bit block the node reads: 2(p-1) bits
template <int NRP>
static hipError_t leaves_nrp(int p, int kd, dim3 grid, const DevKey* d_key, const uint4* is,
                             const uint32_t* it, int L0, uint64_t nin, uint64_t in_stride,
                             uint8_t* c, uint32_t cstride, uint32_t c_key_off, hipStream_t s) {
  const int tbits = 2 * (p - 1);
  if (tbits <= 8) return leaves_tb<NRP, 1>(kd, grid, d_key, is, it, L0, nin, in_stride, c, cstride, c_key_off, s);
  if (tbits <= 16) return leaves_tb<NRP, 2>(kd, grid, d_key, is, it, L0, nin, in_stride, c, cstride, c_key_off, s);
  return leaves_tb<NRP, 4>(kd, grid, d_key, is, it, L0, nin, in_stride, c, cstride, c_key_off, s);
}

hipError_t launch_leaves(int p, int nrp, int kd, const DevKey* d_key, const uint4* is,
                         const uint32_t* it, int L0, uint64_t nin, int nkeys, uint64_t in_stride,
                         uint8_t* c, uint32_t cstride, uint32_t c_key_off, hipStream_t s) {
  if (!leaves_supported(kd) || nkeys < 1 || nin == 0 || p < 2 || p > 17) return hipErrorInvalidValue;
  const uint64_t blocks = (nin + kLeafThreads - 1) / kLeafThreads;
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  const dim3 grid((unsigned)blocks, (unsigned)nkeys);
  switch (nrp) {
    case 1: return leaves_nrp<1>(p, kd, grid, d_key, is, it, L0, nin, in_stride, c, cstride, c_key_off, s);
    case 2: return leaves_nrp<2>(p, kd, grid, d_key, is, it, L0, nin, in_stride, c, cstride, c_key_off, s);
    case 4: return leaves_nrp<4>(p, kd, grid, d_key, is, it, L0, nin, in_stride, c, cstride, c_key_off, s);
    case 8: return leaves_nrp<8>(p, kd, grid, d_key, is, it, L0, nin, in_stride, c, cstride, c_key_off, s);
    case 16: return leaves_nrp<16>(p, kd, grid, d_key, is, it, L0, nin, in_stride, c, cstride, c_key_off, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pir
