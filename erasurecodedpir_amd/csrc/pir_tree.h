// pir_tree.h -- per-node pieces of the DPF tree shared by the tree kernels (pir_kernels.hip,
// pir_leaves.hip): correction words, one node expansion G(seed) (dpf_tree.cpp:525-559) and the
// leaf conversion (dpf_tree.cpp:567-580).
#pragma once
#include "pir_aes.h"
#include "pir_kernels.h"

namespace pir {

// ------------------------------------------------------------------------------------------
// Correction words of one level for a node with control bits t (dpf_tree.cpp:533-541):
//   cs = XOR_{j: t_j} sCW[L][j]   (applied to both child seeds)
//   ct = XOR_{j: t_j} tCW[L][j]   (applied to the packed child control bits)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void level_cw(const DevKey* __restrict__ K, int L, uint32_t t,
                                         uint32_t pm1, uint4& cs, uint32_t& ct) {
  cs = make_uint4(0, 0, 0, 0);
  ct = 0;
  for (uint32_t j = 0; j < pm1; ++j) {
    const uint32_t m = 0u - ((t >> j) & 1u);
    cs = xor4(cs, and4(K->scw[L * kMaxCW + j], m));
    ct ^= K->tcw[L * kMaxCW + j] & m;
  }
}

struct Bits {
  uint32_t pm1, tmask, tb_mask;
  __device__ explicit Bits(uint32_t p) {
    pm1 = p - 1;
    tmask = (1u << pm1) - 1u;
    tb_mask = 2 * pm1 >= 32 ? 0xffffffffu : ((1u << (2 * pm1)) - 1u);
  }
};

// G(seed) of an internal node with corrections: children seeds and control bits
__device__ __forceinline__ void expand_node(const Tab& T, const DevKey* __restrict__ K, int L,
                                            const Bits& B, uint4 seed, uint32_t t, uint4& sl,
                                            uint4& sr, uint32_t& tl, uint32_t& tr) {
  uint4 o[3];
  aes_ctr_row<3, 1>(T, seed, o);
  uint4 cs;
  uint32_t ct;
  level_cw(K, L, t, B.pm1, cs, ct);
  sl = xor4(o[0], cs);
  sr = xor4(o[1], cs);
  const uint32_t tb = (o[2].x & B.tb_mask) ^ ct;
  tl = tb & B.tmask;
  tr = (tb >> B.pm1) & B.tmask;
}

// NRP bytes of leaf `leaf` at c + leaf * cstride (cstride = NRP, or a multiple of it when the
// shares of several keys are interleaved per leaf for a batched scan)
template <int NRP>
__device__ __forceinline__ void store_leaf(uint8_t* __restrict__ c, uint64_t leaf, uint4 v,
                                           uint32_t cstride = NRP) {
  uint8_t* dst = c + leaf * cstride;
  if constexpr (NRP == 1) *dst = (uint8_t)v.x;
  else if constexpr (NRP == 2) *reinterpret_cast<uint16_t*>(dst) = (uint16_t)v.x;
  else if constexpr (NRP == 4) *reinterpret_cast<uint32_t*>(dst) = v.x;
  else if constexpr (NRP == 8) *reinterpret_cast<uint2*>(dst) = make_uint2(v.x, v.y);
  else *reinterpret_cast<uint4*>(dst) = v;
}

// leaf value (before masking to nq bytes); LASTB 1-3: only that many bytes valid
template <int NW, int LASTB = 0>
__device__ __forceinline__ uint4 leaf_value(const Tab& T, const DevKey* __restrict__ K,
                                            uint32_t pm1, uint4 seed, uint32_t t) {
  uint4 o[1];
  aes_ctr_row<1, NW, LASTB>(T, seed, o);
  for (uint32_t j = 0; j < pm1; ++j) o[0] = xor4(o[0], and4(K->lastcw[j], 0u - ((t >> j) & 1u)));
  return o[0];
}

}  // namespace pir
