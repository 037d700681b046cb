// pir_leaves.hip -- the throughput stages of the DPF tree, depth first per lane (k_subtree).
//
// k_expand builds a stage breadth first in LDS: a workgroup of 1024 threads starts from `tile`
// nodes, so its first levels keep only 4 and 8 of its 16 waves busy (256 and 512 nodes) and
// every level ends at a barrier.  Here every lane owns ONE input node of level L0 and walks its
// subtree of 2^KD leaves depth first in registers (the pending right child of each level waits
// in 5 VGPRs), so all waves are busy from the first level, there is no node traffic through
// LDS and no barrier after the table fill.  The AES is the 4-table T-box of pir_aes4.h (the
// kernel holds nothing else in LDS).  The work is the reference's (dpf_tree.cpp:525-580):
// KD levels of G(seed) expansions + correction words, then either
//   * leaf stage: the leaf conversion c[leaf][a] = AES_{s_leaf}(0)[a] ^ XOR_{k: t_leaf bit k}
//     lastCW[k][a] (a < nq), or
//   * node stage: the 2^KD nodes (seed, control bits) of the stage's last level, for the next.
// blockIdx.y = key of a batch (its DevKey, input node range and outputs), as in k_expand.
#include "pir_kernels.h"
#include "pir_tree.h"
#include "pir_aes4.h"

#include <stdlib.h>

namespace pir {


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

// The AES flavour of a subtree walk: the 4-table T-box (pir_aes4.h, 128 KiB of LDS: one
// 1024-thread workgroup per CU) or, T2, the 2-table T-box of pir_aes.h (64 KiB: two workgroups
// per CU, so kLeaf2Threads x 2 threads at amdgpu_waves_per_eu(kLeaf2WPE) -- more waves in
// flight for an LDS-latency-bound walk at the price of 2 v_alignbit per column).
template <bool T2> struct AesF;
template <> struct AesF<false> {
  using TabT = Tab4;
  template <int TB>
  __device__ __forceinline__ static void node(const Tab4& T, const DevKey* __restrict__ K, int L,
                                              const Bits& B, uint4 s, uint32_t t, uint4& sl,
                                              uint4& sr, uint32_t& tl, uint32_t& tr) {
    expand_node4<TB>(T, K, L, B, s, t, sl, sr, tl, tr);
  }
  template <int NRP>
  __device__ __forceinline__ static uint4 leaf(const Tab4& T, const DevKey* __restrict__ K,
                                               uint32_t pm1, uint4 s, uint32_t t) {
    return leaf_value4<NRP>(T, K, pm1, s, t);
  }
};
template <> struct AesF<true> {
  using TabT = Tab;
  template <int TB>
  __device__ __forceinline__ static void node(const Tab& T, const DevKey* __restrict__ K, int L,
                                              const Bits& B, uint4 s, uint32_t t, uint4& sl,
                                              uint4& sr, uint32_t& tl, uint32_t& tr) {
    expand_node(T, K, L, B, s, t, sl, sr, tl, tr);
  }
  template <int NRP>
  __device__ __forceinline__ static uint4 leaf(const Tab& T, const DevKey* __restrict__ K,
                                               uint32_t pm1, uint4 s, uint32_t t) {
    return leaf_value<NRP <= 4 ? 1 : NRP / 4, (NRP < 4 ? NRP : 0)>(T, K, pm1, s, t);
  }
};
#ifndef PIR_LEAF2_THREADS
#define PIR_LEAF2_THREADS 768
#endif
#ifndef PIR_LEAF2_WPE
#define PIR_LEAF2_WPE 6
#endif
constexpr int kLeaf2Threads = PIR_LEAF2_THREADS;
constexpr int kLeaf2WPE = PIR_LEAF2_WPE;

// Where a subtree's bottom level goes: the DPF shares of its leaves (leaf stage) or its nodes
// (seed, control bits) for the next stage (node stage).
struct DfsOut {
  uint8_t* c;        // leaf stage: leaf i's NRP share bytes at c + i * cstride
  uint32_t cstride;
  uint4 qm;          // ... masked to the nq bytes
  uint4* s;          // node stage: node i at s[i], t[i]
  uint32_t* t;
};

// Packed leaf stores (PACK: leaf i's NRP bytes at c + i * NRP, i.e. one key's shares
// contiguous -- the key-major share layout of batched answers, or a single key): the DFS emits
// a lane's leaves in increasing index order, so they shift into a 16-byte register (newest at
// the top) and every 16 / NRP leaves leave as ONE 16-byte store, instead of a 1-4 byte store
// per leaf (2.25 GB written per 8-key launch for 128 MiB of shares, r03_pmc_c3b.json).
template <int NRP>
__device__ __forceinline__ void pack_leaf(uint4& acc, uint32_t v) {
  constexpr int SH = 8 * NRP;  // bits per leaf (NRP <= 4)
  if constexpr (SH == 32) {
    acc = make_uint4(acc.y, acc.z, acc.w, v);
  } else {
    acc.x = __builtin_amdgcn_alignbit(acc.y, acc.x, SH);
    acc.y = __builtin_amdgcn_alignbit(acc.z, acc.y, SH);
    acc.z = __builtin_amdgcn_alignbit(acc.w, acc.z, SH);
    acc.w = __builtin_amdgcn_alignbit(v, acc.w, SH);
  }
}

// the 2^D leaves (or bottom nodes) under node (s, t) of level L, indices [i0, i0 + 2^D)
template <bool NODES, int NRP, int TB, int D, bool PACK, bool T2>
__device__ __forceinline__ void subtree_dfs(const typename AesF<T2>::TabT& T,
                                            const DevKey* __restrict__ K, int L, const Bits& B,
                                            uint4 s, uint32_t t, uint64_t i0, const DfsOut& o,
                                            uint4& acc) {
  uint4 sl, sr;
  uint32_t tl, tr;
  AesF<T2>::template node<TB>(T, K, L, B, s, t, sl, sr, tl, tr);
  if constexpr (D == 1) {
    if constexpr (NODES) {
      o.s[i0] = sl; o.s[i0 + 1] = sr;
      o.t[i0] = tl; o.t[i0 + 1] = tr;
    } else {
      const uint4 vl = AesF<T2>::template leaf<NRP>(T, K, B.pm1, sl, tl);
      const uint4 vr = AesF<T2>::template leaf<NRP>(T, K, B.pm1, sr, tr);
      if constexpr (PACK) {
        constexpr uint32_t LPS = 16 / NRP;  // leaves per 16-byte store
        pack_leaf<NRP>(acc, vl.x & o.qm.x);
        pack_leaf<NRP>(acc, vr.x & o.qm.x);
        if (((uint32_t)i0 & (LPS - 1)) == LPS - 2)  // leaf i0 + 1 completes the register
          *reinterpret_cast<uint4*>(o.c + (i0 + 2 - LPS) * NRP) = acc;
      } else {
        store_leaf<NRP>(o.c, i0, and_q(vl, o.qm), o.cstride);
        store_leaf<NRP>(o.c, i0 + 1, and_q(vr, o.qm), o.cstride);
      }
    }
  } else {
    // one copy of the subtree code per level: the right child waits in registers
#pragma unroll 1
    for (int i = 0; i < 2; ++i)
      subtree_dfs<NODES, NRP, TB, D - 1, PACK, T2>(T, K, L + 1, B, i ? sr : sl, i ? tr : tl,
                                                   i0 + ((uint64_t)i << (D - 1)), o, acc);
  }
}

// blockIdx.y = key of a batch: its DevKey, input node range (in_stride apart) and outputs
// (shares at c + y * c_key_off, or nodes out_stride apart)
template <bool NODES, int NRP, int TB, int KD, bool PACK = false, bool T2 = false>
__global__ __launch_bounds__(T2 ? kLeaf2Threads : kLeafThreads)
__attribute__((amdgpu_waves_per_eu(T2 ? kLeaf2WPE : 4)))
void k_subtree(const DevKey* __restrict__ K, const uint4* __restrict__ in_s,
               const uint32_t* __restrict__ in_t, int L0, uint64_t nin, uint64_t in_stride,
               uint8_t* __restrict__ c, uint32_t cstride, uint32_t c_key_off,
               uint4* __restrict__ out_s, uint32_t* __restrict__ out_t, uint64_t out_stride) {
  K += blockIdx.y;
  in_s += blockIdx.y * in_stride;
  in_t += blockIdx.y * in_stride;
  constexpr int NT = T2 ? kLeaf2Threads : kLeafThreads;
  __shared__ uint32_t tab[(T2 ? kTablesBytes : kTab4Bytes) / 4];
  if constexpr (T2) load_tables_n<NT>(tab);
  else load_tables4_n<NT>(tab);
  const Bits B(K->p);
  DfsOut o;
  if constexpr (NODES) {
    o.s = out_s + blockIdx.y * out_stride;
    o.t = out_t + blockIdx.y * out_stride;
  } else {
    o.c = c + (size_t)blockIdx.y * c_key_off;
    o.cstride = cstride;
    const int nq = (int)K->nq;  // keep the nq output bytes
    uint32_t m[4];
    for (int w = 0; w < 4; ++w) {
      const int nb = nq - 4 * w;
      m[w] = nb >= 4 ? 0xffffffffu : (nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u));
    }
    o.qm = make_uint4(m[0], m[1], m[2], m[3]);
  }
  __syncthreads();
  const typename AesF<T2>::TabT T(tab);
  const uint64_t u = (uint64_t)blockIdx.x * NT + threadIdx.x;
  if (u >= nin) return;  // no barrier below
  uint4 acc = make_uint4(0, 0, 0, 0);
  subtree_dfs<NODES, NRP, TB, KD, PACK, T2>(T, K, L0, B, in_s[u], in_t[u], u << KD, o, acc);
}

bool leaves_supported(int kd) { return kd >= kLeavesMinK && kd <= kLeavesMaxK; }
bool nodes_dfs_supported(int kd) { return kd >= 1 && kd <= kNodesMaxK; }

struct SubtreeArgs {
  const DevKey* key;
  const uint4* is;
  const uint32_t* it;
  int L0;
  uint64_t nin, in_stride;
  uint8_t* c;
  uint32_t cstride, c_key_off;
  uint4* os;
  uint32_t* ot;
  uint64_t out_stride;
};

template <bool NODES, int NRP, int TB, int KD, bool PACK = false, bool T2 = false>
static hipError_t subtree_launch(dim3 grid, const SubtreeArgs& a, hipStream_t s) {
  constexpr int NT = T2 ? kLeaf2Threads : kLeafThreads;
  grid.x = (unsigned)((a.nin + NT - 1) / NT);
  hipLaunchKernelGGL((k_subtree<NODES, NRP, TB, KD, PACK, T2>), grid, dim3(NT), 0, s,
                     a.key, a.is, a.it, a.L0, a.nin, a.in_stride, a.c, a.cstride, a.c_key_off,
                     a.os, a.ot, a.out_stride);
  return hipGetLastError();
}

// TB = bytes of the control-bit block the node reads: 2(p-1) bits
template <int NRP, int TB>
static hipError_t leaves_kd(int kd, dim3 grid, const SubtreeArgs& a, hipStream_t s) {
  // contiguous shares of <= 4 bytes at 16-byte aligned subtree bases: packed 16-byte stores
  // ($PIR_LEAF_PACK=0: one store per leaf, diagnostics)
  const char* pk = getenv("PIR_LEAF_PACK");
  const bool pack_ok = !(pk && atoi(pk) == 0);
  // $PIR_LEAF_T2=1 (experiment): the 2-table AES at two workgroups per CU (packed stores only)
  const char* t2 = getenv("PIR_LEAF_T2");
  const bool use_t2 = t2 && atoi(t2) == 1;
  if constexpr (NRP <= 4) {
    if (pack_ok && a.cstride == (uint32_t)NRP && (reinterpret_cast<uintptr_t>(a.c) & 15) == 0 &&
        ((uint64_t)a.c_key_off & 15) == 0) {
      if (use_t2) {
        switch (kd) {
          case 4: return subtree_launch<false, NRP, TB, 4, true, true>(grid, a, s);
          case 5: return subtree_launch<false, NRP, TB, 5, true, true>(grid, a, s);
          default: return hipErrorInvalidValue;
        }
      }
      switch (kd) {
        case 4: return subtree_launch<false, NRP, TB, 4, true>(grid, a, s);
        case 5: return subtree_launch<false, NRP, TB, 5, true>(grid, a, s);
        default: return hipErrorInvalidValue;
      }
    }
  }
  switch (kd) {
    case 4: return subtree_launch<false, NRP, TB, 4>(grid, a, s);
    case 5: return subtree_launch<false, NRP, TB, 5>(grid, a, s);
    default: return hipErrorInvalidValue;
  }
}
template <int NRP>
static hipError_t leaves_nrp(int p, int kd, dim3 grid, const SubtreeArgs& a, hipStream_t s) {
  const int tbits = 2 * (p - 1);
  if (tbits <= 8) return leaves_kd<NRP, 1>(kd, grid, a, s);
  if (tbits <= 16) return leaves_kd<NRP, 2>(kd, grid, a, s);
  return leaves_kd<NRP, 4>(kd, grid, a, s);
}
template <int TB>
static hipError_t nodes_kd(int kd, dim3 grid, const SubtreeArgs& a, hipStream_t s) {
  switch (kd) {
    case 1: return subtree_launch<true, 1, TB, 1>(grid, a, s);
    case 2: return subtree_launch<true, 1, TB, 2>(grid, a, s);
    case 3: return subtree_launch<true, 1, TB, 3>(grid, a, s);
    case 4: return subtree_launch<true, 1, TB, 4>(grid, a, s);
    default: return hipErrorInvalidValue;
  }
}

static bool subtree_grid(uint64_t nin, int nkeys, int p, dim3& grid) {
  if (nkeys < 1 || nin == 0 || p < 2 || p > 17) return false;
  const uint64_t blocks = (nin + kLeafThreads - 1) / kLeafThreads;
  if (blocks > 0x7fffffffull || nkeys > 65535) return false;
  grid = dim3((unsigned)blocks, (unsigned)nkeys);
  return true;
}

hipError_t launch_leaves(int p, int nrp, int kd, const DevKey* d_key, const uint4* is,
                         const uint32_t* it, int L0, uint64_t nin, int nkeys, uint64_t in_stride,
                         uint8_t* c, uint32_t cstride, uint32_t c_key_off, hipStream_t s) {
  dim3 grid;
  if (!leaves_supported(kd) || !subtree_grid(nin, nkeys, p, grid)) return hipErrorInvalidValue;
  const SubtreeArgs a{d_key, is, it, L0, nin, in_stride, c, cstride, c_key_off, nullptr, nullptr, 0};
  switch (nrp) {
    case 1: return leaves_nrp<1>(p, kd, grid, a, s);
    case 2: return leaves_nrp<2>(p, kd, grid, a, s);
    case 4: return leaves_nrp<4>(p, kd, grid, a, s);
    case 8: return leaves_nrp<8>(p, kd, grid, a, s);
    case 16: return leaves_nrp<16>(p, kd, grid, a, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_nodes_dfs(int p, int kd, const DevKey* d_key, const uint4* is,
                            const uint32_t* it, int L0, uint64_t nin, int nkeys,
                            uint64_t in_stride, uint4* os, uint32_t* ot, uint64_t out_stride,
                            hipStream_t s) {
  dim3 grid;
  if (!nodes_dfs_supported(kd) || !subtree_grid(nin, nkeys, p, grid)) return hipErrorInvalidValue;
  const SubtreeArgs a{d_key, is, it, L0, nin, in_stride, nullptr, 0, 0, os, ot, out_stride};
  const int tbits = 2 * (p - 1);
  if (tbits <= 8) return nodes_kd<1>(kd, grid, a, s);
  if (tbits <= 16) return nodes_kd<2>(kd, grid, a, s);
  return nodes_kd<4>(kd, grid, a, s);
}

}  // namespace pir
