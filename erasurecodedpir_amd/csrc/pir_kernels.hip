// pir_kernels.hip -- CDNA4 (gfx950) kernels of the tree-DPF PIR answer path.
//
//   k_key_prep   raw genOptimizedDPF key bytes -> DevKey               (dpf_tree.cpp:504-519)
//   k_frontier   root (or partition prefix) -> frontier level F        (dpf_tree.cpp:525-559)
//   k_expand     frontier -> ... -> leaves -> DPF shares c[i][a]       (dpf_tree.cpp:525-580)
//   k_scan       ans[a] ^= c[i][a] * shard[i]  over GF(2^8)            (server.cpp:121-127)
//   k_fused      leaf stage + scan in one persistent kernel (shares stay in LDS)
//   k_reduce     XOR of per-workgroup partial answers                  (server.cpp:553-562)
// k_frontier and k_expand take a batch of keys along gridDim.y (batched answers).
//
// AES-128 (the PRG G of utils.cpp:37-51 re-keys on every node seed) is a T-table cipher:
// Te0 and Te2 = rotl16(Te0) replicated 32x in LDS (pir_aes.h) so every lane of a 32-lane
// ds_read_b32 group hits its own bank; Te1, Te3 are byte rotations of Te0, Te2.
// The GF(2^8) scan keeps, per lane, 8 bit-plane accumulators Z_k (Z_k ^= x when bit k of the
// record's coefficient is set) and folds ans = sum_k alpha^k Z_k once at the end, so the
// HBM stream costs ~1 VALU op per byte.
#include "pir_kernels.h"
#include "pir_aes.h"
#include "pir_tree.h"
#include "pir_m4r.h"
#include "pir_mp.h"

#include <algorithm>
#include <type_traits>
#include <stdlib.h>

namespace pir {

// ------------------------------------------------------------------------------------------
// k_key_prep: raw key bytes -> DevKey (one workgroup per key)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t load_le32(const uint8_t* b) {
  return b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
}
__device__ __forceinline__ uint4 load_le128(const uint8_t* b) {
  return make_uint4(load_le32(b), load_le32(b + 4), load_le32(b + 8), load_le32(b + 12));
}

// sCW[L][j] / tCW[L][j] of the raw key (dpf_tree.cpp:506-513): tCW bytes packed to bits
__device__ __forceinline__ void parse_cw(const uint8_t* key, int p, int L, int j, uint4& scw,
                                         uint32_t& tcw) {
  const int pm1 = p - 1, CWk = 16 + 2 * p - 2, CW = pm1 * CWk;
  const uint8_t* cw = key + 16 + L * CW + j * CWk;
  scw = load_le128(cw);
  uint32_t tb = 0;
  for (int k = 0; k < 2 * pm1; ++k) tb |= (uint32_t)(cw[16 + k] & 1u) << k;
  tcw = tb;
}

// the whole DevKey, parsed by the threads of one workgroup
__device__ void parse_key(const uint8_t* __restrict__ key, int p, int n, int nq, int party0,
                          DevKey* __restrict__ K) {
  const int pm1 = p - 1, CWk = 16 + 2 * p - 2, CW = pm1 * CWk;
  const int tid = threadIdx.x;
  if (tid == 0) {
    K->root_seed = load_le128(key);
    K->root_t = party0 >= 1 ? (1u << (party0 - 1)) : 0u;  // dpf_tree.cpp:496-502
    K->p = p; K->n = n; K->nq = nq;
  }
  for (int e = tid; e < n * pm1; e += blockDim.x) {
    const int L = e / pm1, j = e - L * pm1;
    parse_cw(key, p, L, j, K->scw[L * kMaxCW + j], K->tcw[L * kMaxCW + j]);
  }
  for (int j = tid; j < kMaxCW; j += blockDim.x) {  // dpf_tree.cpp:515-519
    uint32_t w[4] = {0, 0, 0, 0};
    if (j < pm1)
      for (int a = 0; a < nq; ++a)
        w[a >> 2] |= (uint32_t)key[16 + n * CW + a * pm1 + j] << (8 * (a & 3));
    K->lastcw[j] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

#ifndef PIR_QUERY_PART
__global__ __launch_bounds__(256) void k_key_prep(const uint8_t* __restrict__ raw,
                                                  size_t key_stride, int p, int n, int nq,
                                                  int party0, DevKey* __restrict__ out) {
  parse_key(raw + blockIdx.x * key_stride, p, n, nq, party0, out + blockIdx.x);
}
#endif


// ------------------------------------------------------------------------------------------
// k_frontier: the narrow, latency-bound top of the tree.  Each of 2^g workgroups descends from
// the root along (prefix << g | blockIdx.x) for log_parts + g levels, then expands e levels
// breadth-first; the 2^e nodes of the last level go to global memory.  Column-shape AES: a
// node is 16 lanes = 4 quads, quad r computes CTR block r of G(seed) (quad 3 is a spare), so
// one expansion costs ~1/4 of a row-shape block's latency.  During the descent every 16-lane
// group computes the same node (no barrier: the chosen child is fetched with __shfl).
// ------------------------------------------------------------------------------------------
constexpr int kFrontThreads = 512;
constexpr int kFrontCap = 256;  // nodes per LDS level buffer (e <= 9)
constexpr int kFrontCwLevels = 32;  // levels whose CWs are staged in LDS (F <= 16 + parts)
struct FrontSmem {
  uint32_t tab[2 * 256 * 32];
  uint32_t s[2][kFrontCap][4];
  uint32_t t[2][kFrontCap];
  uint4 scw[kFrontCwLevels * kMaxCW];
  uint32_t tcw[kFrontCwLevels * kMaxCW];
};

// level_cw from LDS-staged correction words (frontier: no scalar-cache misses per level)
__device__ __forceinline__ void level_cw_lds(const uint4* scw, const uint32_t* tcw, int L,
                                             uint32_t t, uint32_t pm1, uint4& cs, uint32_t& ct) {
  cs = make_uint4(0, 0, 0, 0);
  ct = 0;
  for (uint32_t j = 0; j < pm1; ++j) {
    const uint32_t m = 0u - ((t >> j) & 1u);
    cs = xor4(cs, and4(scw[L * kMaxCW + j], m));
    ct ^= tcw[L * kMaxCW + j] & m;
  }
}

__device__ __forceinline__ uint32_t word_of(const uint4& v, uint32_t q) {
  return q == 0 ? v.x : (q == 1 ? v.y : (q == 2 ? v.z : v.w));
}

#ifndef PIR_QUERY_PART
__global__ __launch_bounds__(kFrontThreads) void k_frontier(
    const uint8_t* __restrict__ raw, int p, int n, int nq, int party0, DevKey* __restrict__ K,
    uint64_t prefix, int log_parts, int g, int e, uint4* __restrict__ out_s,
    uint32_t* __restrict__ out_t, uint32_t raw_stride, uint64_t out_stride) {
  // raw != nullptr: parse the key here (every workgroup stages the CWs it needs in LDS;
  // workgroup 0 also writes the full DevKey for the later kernels).  raw == nullptr: K was
  // written by k_key_prep.  blockIdx.y = key of a batch (raw_stride bytes, K + y, out_stride
  // nodes apart).
  if (raw) raw += (size_t)blockIdx.y * raw_stride;
  K += blockIdx.y;
  out_s += blockIdx.y * out_stride;
  out_t += blockIdx.y * out_stride;
  __shared__ FrontSmem sm;
  __shared__ uint4 root_seed;
  __shared__ uint32_t root_t;
  load_tables(sm.tab);
  const Tab T(sm.tab);
  const Bits B((uint32_t)p);
  const uint32_t q = threadIdx.x & 3u, role = (threadIdx.x >> 2) & 3u;
  const uint32_t mq1 = q >= 1 ? 0xffffffffu : 0u, mq2 = q >= 2 ? 0xffffffffu : 0u;
  const uint32_t ptq = q == 3 ? (role << 24) : 0u;  // CTR block `role`: BE128(role)
  const int lane = threadIdx.x & 63;
  const int g16 = lane & ~15;
  const int nlev = log_parts + g + e;  // levels this kernel expands
  const bool cw_lds = nlev <= kFrontCwLevels;
  if (raw) {
    if (blockIdx.x == 0) parse_key(raw, p, n, nq, party0, K);
    for (int i = threadIdx.x; i < nlev * (p - 1); i += blockDim.x) {
      const int L = i / (p - 1), j = i - L * (p - 1);
      parse_cw(raw, p, L, j, sm.scw[L * kMaxCW + j], sm.tcw[L * kMaxCW + j]);
    }
    if (threadIdx.x == 0) {
      root_seed = load_le128(raw);
      root_t = party0 >= 1 ? (1u << (party0 - 1)) : 0u;
    }
  } else {
    if (cw_lds)
      for (int i = threadIdx.x; i < nlev * kMaxCW; i += blockDim.x) {
        sm.scw[i] = K->scw[i];
        sm.tcw[i] = K->tcw[i];
      }
    if (threadIdx.x == 0) {
      root_seed = K->root_seed;
      root_t = K->root_t;
    }
  }
  __syncthreads();
  auto cw = [&](int L, uint32_t tv, uint4& cs, uint32_t& ct) {
    if (cw_lds) level_cw_lds(sm.scw, sm.tcw, L, tv, B.pm1, cs, ct);
    else level_cw(K, L, tv, B.pm1, cs, ct);
  };

  // ---- descent: wave 0 only (its 4 groups of 16 lanes compute the same node) -------------
  const int D0 = log_parts + g;
  const uint64_t path = (prefix << g) | blockIdx.x;
  const uint64_t obase = (uint64_t)blockIdx.x << e;
  if (threadIdx.x < 64) {
    uint32_t sq = word_of(root_seed, q), t = root_t;
    for (int L = 0; L < D0; ++L) {
      const uint32_t o = aes_col(T, sq, ptq, mq1, mq2);
      uint4 cs;
      uint32_t ct;
      cw(L, t, cs, ct);
      const uint32_t bit = (uint32_t)((path >> (D0 - 1 - L)) & 1u);
      const uint32_t oc = o ^ word_of(cs, q);
      sq = (uint32_t)__shfl((int)oc, g16 | (int)(bit << 2) | (int)q, 64);
      const uint32_t tb = ((uint32_t)__shfl((int)o, g16 | 8, 64) & B.tb_mask) ^ ct;
      t = (tb >> (bit * B.pm1)) & B.tmask;
    }
    if (e == 0) {
      if (threadIdx.x < 4) reinterpret_cast<uint32_t*>(out_s + blockIdx.x)[q] = sq;
      if (threadIdx.x == 0) out_t[blockIdx.x] = t;
    } else {
      if (threadIdx.x < 4) sm.s[0][0][q] = sq;
      if (threadIdx.x == 0) sm.t[0][0] = t;
    }
  }
  if (e == 0) return;
  __syncthreads();

  // ---- breadth-first expansion, 32 nodes per pass ----------------------------------------
  int cur = 0, W = 1;
  for (int lv = 0; lv < e; ++lv) {
    const int L = D0 + lv;
    const bool last = lv == e - 1;
    for (int u0 = 0; u0 < W; u0 += kFrontThreads / 16) {
      const int u = u0 + (int)(threadIdx.x >> 4);
      if (u < W) {  // uniform per 16-lane group (DPP stays inside a quad)
        const uint32_t s_in = sm.s[cur][u][q], t_in = sm.t[cur][u];
        const uint32_t o = aes_col(T, s_in, ptq, mq1, mq2);
        uint4 cs;
        uint32_t ct;
        cw(L, t_in, cs, ct);
        if (role < 2) {
          const uint32_t v = o ^ word_of(cs, q);
          if (last) reinterpret_cast<uint32_t*>(out_s + obase + 2 * u + role)[q] = v;
          else sm.s[cur ^ 1][2 * u + role][q] = v;
        } else if (role == 2 && q == 0) {
          const uint32_t tb = (o & B.tb_mask) ^ ct;
          const uint32_t tl = tb & B.tmask, tr = (tb >> B.pm1) & B.tmask;
          if (last) {
            out_t[obase + 2 * u] = tl;
            out_t[obase + 2 * u + 1] = tr;
          } else {
            sm.t[cur ^ 1][2 * u] = tl;
            sm.t[cur ^ 1][2 * u + 1] = tr;
          }
        }
      }
    }
    __syncthreads();
    cur ^= 1;
    W *= 2;
  }
}
#endif  // PIR_QUERY_PART

// ------------------------------------------------------------------------------------------
// k_expand: the wide, throughput-bound levels.  A workgroup takes `tile` nodes of level L0 and
// expands k levels breadth-first in LDS, one lane per node (row-shape AES: the 3 CTR blocks of
// G(seed) share one key schedule).  FINAL: the last level is fused with the leaf conversion
// (dpf_tree.cpp:567-580): each lane expands a parent and converts both children,
//   c[leaf][a] = AES_{s_leaf}(0)[a] ^ XOR_{k: t_leaf bit k} lastCW[k][a]   (a < nq),
// written as rows of NRP bytes (nq padded to a power of two, pad bytes zero).
// !FINAL: the last level's nodes go to global memory for the next stage.
// ------------------------------------------------------------------------------------------
constexpr int kExpThreads = 1024;
constexpr int kExpOut = 4096;  // nodes produced per workgroup (tile << k)
struct ExpSmem {
  uint32_t tab[2 * 256 * 32];
  uint4 sa[kExpOut / 2];
  uint32_t ta[kExpOut / 2];
  uint4 sb[kExpOut / 4];
  uint32_t tb[kExpOut / 4];
};


template <bool FINAL, int NRP>
__global__ __launch_bounds__(kExpThreads) void k_expand(
    const DevKey* __restrict__ K, const uint4* __restrict__ in_s, const uint32_t* __restrict__ in_t,
    int L0, int k, int tile, uint4* __restrict__ out_s, uint32_t* __restrict__ out_t,
    uint8_t* __restrict__ c, uint32_t cstride, uint64_t in_stride, uint64_t out_stride,
    uint32_t c_key_off) {
  // blockIdx.y = key of a batch: its DevKey, node ranges and share slot
  K += blockIdx.y;
  in_s += blockIdx.y * in_stride;
  in_t += blockIdx.y * in_stride;
  out_s += blockIdx.y * out_stride;
  out_t += blockIdx.y * out_stride;
  c += (size_t)blockIdx.y * c_key_off;
  constexpr int NW = NRP <= 4 ? 1 : NRP / 4;
  __shared__ ExpSmem sm;
  load_tables(sm.tab);
  const Tab T(sm.tab);
  const Bits B(K->p);
  const uint64_t ibase = (uint64_t)blockIdx.x * tile;
  const uint64_t obase = ibase << k;
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
  if (k == 0) {  // FINAL only: the input nodes are the leaves
    __syncthreads();
    for (int i = threadIdx.x; i < tile; i += blockDim.x) {
      const uint4 v = leaf_value<NW, (NRP < 4 ? NRP : 0)>(T, K, B.pm1, in_s[ibase + i], in_t[ibase + i]);
      store_leaf<NRP>(c, obase + i, make_uint4(v.x & qm.x, v.y & qm.y, v.z & qm.z, v.w & qm.w), cstride);
    }
    return;
  }
  // level i (width tile << i) lives in buffer a when (k-1-i) is even, else b
  int buf = (k - 1) & 1;  // buffer of level 0: 0 = a, 1 = b
  {
    uint4* s0 = buf ? sm.sb : sm.sa;
    uint32_t* t0 = buf ? sm.tb : sm.ta;
    for (int i = threadIdx.x; i < tile; i += blockDim.x) {
      s0[i] = in_s[ibase + i];
      t0[i] = in_t[ibase + i];
    }
  }
  __syncthreads();
  int W = tile;
  for (int lv = 0; lv < k - 1; ++lv) {
    const uint4* is = buf ? sm.sb : sm.sa;
    const uint32_t* it = buf ? sm.tb : sm.ta;
    uint4* os = buf ? sm.sa : sm.sb;
    uint32_t* ot = buf ? sm.ta : sm.tb;
    for (int u = threadIdx.x; u < W; u += blockDim.x) {
      uint4 sl, sr;
      uint32_t tl, tr;
      expand_node(T, K, L0 + lv, B, is[u], it[u], sl, sr, tl, tr);
      os[2 * u] = sl; os[2 * u + 1] = sr;
      ot[2 * u] = tl; ot[2 * u + 1] = tr;
    }
    __syncthreads();
    buf ^= 1;
    W *= 2;
  }
  const int L = L0 + k - 1;
  const uint4* is = buf ? sm.sb : sm.sa;
  const uint32_t* it = buf ? sm.tb : sm.ta;
  for (int u = threadIdx.x; u < W; u += blockDim.x) {
    uint4 sl, sr;
    uint32_t tl, tr;
    expand_node(T, K, L, B, is[u], it[u], sl, sr, tl, tr);
    if constexpr (FINAL) {
      const uint4 vl = leaf_value<NW, (NRP < 4 ? NRP : 0)>(T, K, B.pm1, sl, tl);
      const uint4 vr = leaf_value<NW, (NRP < 4 ? NRP : 0)>(T, K, B.pm1, sr, tr);
      if (NRP == 1 && cstride == 1) {  // both leaves in one 16-bit store
        *reinterpret_cast<uint16_t*>(c + obase + 2 * u) =
            (uint16_t)((vl.x & qm.x & 0xffu) | ((vr.x & qm.x & 0xffu) << 8));
      } else {
        store_leaf<NRP>(c, obase + 2 * u, make_uint4(vl.x & qm.x, vl.y & qm.y, vl.z & qm.z, vl.w & qm.w), cstride);
        store_leaf<NRP>(c, obase + 2 * u + 1, make_uint4(vr.x & qm.x, vr.y & qm.y, vr.z & qm.z, vr.w & qm.w), cstride);
      }
    } else {
      out_s[obase + 2 * u] = sl;
      out_s[obase + 2 * u + 1] = sr;
      out_t[obase + 2 * u] = tl;
      out_t[obase + 2 * u + 1] = tr;
    }
  }
}

// ------------------------------------------------------------------------------------------
// k_scan: per-workgroup partial answers over GF(2^8), poly 0x11d (coding.cpp:9-21)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t gf_xtime4(uint32_t x) {  // 4 packed bytes times alpha
  return ((x & 0x7f7f7f7fu) << 1) ^ (((x >> 7) & 0x01010101u) * 0x1du);
}

template <int VEC>
struct Chunk {
  uint32_t v[VEC];
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int VEC>
__device__ __forceinline__ Chunk<VEC> load_chunk(const uint8_t* p) {
  Chunk<VEC> ch;
  if constexpr (VEC == 4) {
    u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    ch.v[0] = q.x; ch.v[1] = q.y; ch.v[2] = q.z; ch.v[3] = q.w;
  } else if constexpr (VEC == 2) {
    u32x2 q = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
    ch.v[0] = q.x; ch.v[1] = q.y;
  } else {
    ch.v[0] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p));
  }
  return ch;
}

// the same through a buffer resource (nt): soff = the row's byte offset (wave-uniform), voff =
// the lane's chunk offset; a load past num_records reads zeros without touching memory
template <int VEC>
__device__ __forceinline__ Chunk<VEC> load_chunk_buf(__amdgpu_buffer_rsrc_t r, uint32_t voff,
                                                     uint32_t soff) {
  Chunk<VEC> ch;
  if constexpr (VEC == 4) {
    const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 2);
    ch.v[0] = q.x; ch.v[1] = q.y; ch.v[2] = q.z; ch.v[3] = q.w;
  } else if constexpr (VEC == 2) {
    const u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 2);
    ch.v[0] = q.x; ch.v[1] = q.y;
  } else {
    ch.v[0] = __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 2);
  }
  return ch;
}

// Four-Russians plane indices of a group of 4 rows (pir_m4r.h): lane k = plane (k / 8, k % 8)
// takes bit k % 8 of the rows' round-k/8 coefficient bytes -- bit k of each row's 64-bit
// coefficient word (rounds 0-7 little-endian), i.e. the word used as a lane mask: one
// v_cndmask per row.  w_r = row r's word, wave-uniform.
__device__ __forceinline__ uint32_t m4r_index(uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3) {
  uint32_t vi, t;
  asm("v_cndmask_b32_e64 %0, 0, 1, %2\n\t"
      "v_cndmask_b32_e64 %1, 0, 2, %3\n\t"
      "v_or_b32_e32 %0, %0, %1\n\t"
      "v_cndmask_b32_e64 %1, 0, 4, %4\n\t"
      "v_or_b32_e32 %0, %0, %1\n\t"
      "v_cndmask_b32_e64 %1, 0, 8, %5\n\t"
      "v_or_b32_e32 %0, %0, %1"
      : "=&v"(vi), "=&v"(t)
      : "s"(w0), "s"(w1), "s"(w2), "s"(w3));
  return vi;
}
// m4r_fold4p's packed indices: lane 8a + 7 <- the OR of lanes 8a .. 8a + 7's indices, each
// shifted to bits [4b, 4b + 4) (sh = 4 (lane % 8)) -- three row_shr DPP ORs, so a group takes NA
// v_readlane of its indices instead of 8 NA ($PIR_M4R_PACKED=0 at build time: the unpacked fold)
#ifndef PIR_M4R_PACKED
#define PIR_M4R_PACKED 1
#endif
__device__ __forceinline__ uint32_t m4r_pack(uint32_t vi, uint32_t sh) {
  uint32_t t = vi << sh;
  t |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x111, 0xf, 0xf, true);  // row_shr:1
  t |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x112, 0xf, 0xf, true);  // row_shr:2
  t |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x114, 0xf, 0xf, true);  // row_shr:4
  return t;
}
// k_query's four-Russians scan waves build the packed indices of a whole tile at once, one
// group of 4 rows per lane, instead of per group across the wave (8 coefficient readlanes, 7
// lane-mask ops, a shift, 3 DPP ORs and their wait states per group: profiles/r05/fold_phases_*,
// phase "index").  c[r] = row r's coefficient word (bytes = rounds 0-7, the ring layout);
// P[a] = m4r_pack's word for round a: bits [4b, 4b + 4) = bit b of the 4 rows' round-a bytes,
// row r -> bit r of the nibble.  A 4 x 4 byte transpose (v_perm) gathers W_a = byte r of row r
// (bit 8r + b), then four delta swaps of index bits move bit 8r + b to 4b + r.
__device__ __forceinline__ uint32_t m4r_bits_4x8(uint32_t x) {
  auto ds = [](uint32_t v, int d, uint32_t m) {
    const uint32_t t = (v ^ (v >> d)) & m;
    return v ^ t ^ (t << d);
  };
  x = ds(x, 7, 0x00AA00AAu);   // index bits 0 <-> 3
  x = ds(x, 14, 0x0000CCCCu);  // 1 <-> 4
  x = ds(x, 4, 0x00F000F0u);   // 2 <-> 3
  return ds(x, 8, 0x0000FF00u);  // 3 <-> 4
}
template <int NA>
__device__ __forceinline__ void m4r_tile_index(const uint2 (&c)[4], uint32_t (&P)[NA]) {
  static_assert(NA >= 1 && NA <= 5, "rounds 0-4 (coefficient word x: 0-3, y: 4)");
  const uint32_t A = __builtin_amdgcn_perm(c[1].x, c[0].x, 0x05010400u);  // rows 0-1, rounds 0-1
  const uint32_t B = __builtin_amdgcn_perm(c[3].x, c[2].x, 0x05010400u);  // rows 2-3, rounds 0-1
  P[0] = m4r_bits_4x8(__builtin_amdgcn_perm(B, A, 0x05040100u));
  if constexpr (NA > 1) P[1] = m4r_bits_4x8(__builtin_amdgcn_perm(B, A, 0x07060302u));
  if constexpr (NA > 2) {
    const uint32_t C = __builtin_amdgcn_perm(c[1].x, c[0].x, 0x07030602u);  // rounds 2-3
    const uint32_t D = __builtin_amdgcn_perm(c[3].x, c[2].x, 0x07030602u);
    P[2] = m4r_bits_4x8(__builtin_amdgcn_perm(D, C, 0x05040100u));
    if constexpr (NA > 3) P[3] = m4r_bits_4x8(__builtin_amdgcn_perm(D, C, 0x07060302u));
  }
  if constexpr (NA > 4) {
    const uint32_t E = __builtin_amdgcn_perm(c[1].y, c[0].y, 0x0c0c0400u);  // round 4
    const uint32_t F = __builtin_amdgcn_perm(c[3].y, c[2].y, 0x0c0c0400u);
    P[4] = m4r_bits_4x8(__builtin_amdgcn_perm(F, E, 0x05040100u));
  }
}
// $PIR_M4R_TILEIDX=0 at build time: the per-group index build of rounds 2-4 (A/B diagnostics)
#ifndef PIR_M4R_TILEIDX
#define PIR_M4R_TILEIDX 1
#endif
template <int VEC, int NA>
__device__ __forceinline__ void m4r_fold_group(uint32_t (&Z)[NA][8][VEC], const uint32_t* x0,
                                               const uint32_t* x1, const uint32_t* x2,
                                               const uint32_t* x3, uint32_t vi, uint32_t sh) {
#if PIR_M4R_PACKED
  m4r_fold4p<VEC, NA>(Z, x0, x1, x2, x3, m4r_pack(vi, sh));
#else
  (void)sh;
  m4r_fold4<VEC, NA>(Z, x0, x1, x2, x3, vi);
#endif
}
// k_scan_uni's four-Russians groups read their rows' coefficient words by scalar loads
// ($PIR_M4R_SLOAD=0 at build time: lane loads + v_readlane, as k_query does from its LDS ring)
#ifndef PIR_M4R_SLOAD
#define PIR_M4R_SLOAD 1
#endif
// a value the wave holds in every lane, as a wave-uniform (SGPR) value
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
}
// row j's coefficient word from the lanes holding a 64-row block's coefficients (x: rounds 0-3,
// y: rounds 4-7)
__device__ __forceinline__ uint64_t coef_word(const uint4& c4, uint32_t j) {
  // (readlane returns int: through uint32_t, or the low word would sign-extend into the high)
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane(c4.x, j) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(c4.y, j) << 32);
}

// coefficient bytes of record i: nrp bytes at c + i*nrp, as 4 dwords
template <int NRP>
__device__ __forceinline__ uint4 load_coef(const uint8_t* c, uint64_t i) {
  if constexpr (NRP == 1) return make_uint4(c[i], 0, 0, 0);
  else if constexpr (NRP == 2) return make_uint4(reinterpret_cast<const uint16_t*>(c)[i], 0, 0, 0);
  else if constexpr (NRP == 4) return make_uint4(reinterpret_cast<const uint32_t*>(c)[i], 0, 0, 0);
  else if constexpr (NRP == 8) {
    uint2 q = reinterpret_cast<const uint2*>(c)[i];
    return make_uint4(q.x, q.y, 0, 0);
  } else {
    return reinterpret_cast<const uint4*>(c)[i];
  }
}

// z ^ (x & m) in one v_bitop3 (m an all-ones / all-zeros mask: wave-uniform in an SGPR, or a
// per-lane VGPR -- left to itself the compiler emits v_and + v_xor for the per-lane form)
__device__ __forceinline__ uint32_t mxor(uint32_t z, uint32_t x, uint32_t m) {
  return __builtin_amdgcn_bitop3_b32(z, x, m, 0x78);
}

// The 8 bit-plane masks of every coefficient byte: planes[c][k] = bit k of c ? ~0 : 0.  A
// wave-uniform coefficient fetches its 8 masks with ONE s_load_dwordx8 instead of 8 s_bfe_i32:
// the many-round scan issues one SALU op per two v_bitop3 otherwise, and the scalar unit (one
// per CU) paces it (tools/micro/scan_salu.hip: 1.64 -> 2.87 TB/s at 5 rounds).
struct PlaneMasks {
  uint32_t m[256 * 8];
};
constexpr PlaneMasks make_plane_masks() {
  PlaneMasks t{};
  for (int c = 0; c < 256; ++c)
    for (int k = 0; k < 8; ++k) t.m[c * 8 + k] = ((c >> k) & 1) ? 0xffffffffu : 0u;
  return t;
}
static __constant__ PlaneMasks c_planes = make_plane_masks();

typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
#ifndef PIR_PLANE_U
#define PIR_PLANE_U 8
#endif
// k_query: rounds up to which the scan waves fold with scalar branches instead of plane-table
// masks.  Branches measured slower at 5 rounds (c5: 8.36 vs 6.34 ms per query; the k_query scan
// waves are too few per SIMD to hide the scalar issue), so only 1-2 rounds take them.
// k_query scan waves' issue priority over the tree waves (s_setprio)
#ifndef PIR_SCAN_PRIO
#define PIR_SCAN_PRIO 2
#endif
#ifndef PIR_QUERY_BRANCH_MAXNQ
#define PIR_QUERY_BRANCH_MAXNQ 2
#endif

// Many-round scan with wave-uniform coefficients: the 8 masks of coefficient byte c come from
// the table with one s_load_dwordx8, and one asm statement per round folds a row's 2 dwords
// into that round's 8 planes (16 v_bitop3) while the NEXT round's masks load: the scan waves
// are latency-bound (2 per SIMD), so a wait per round would stall them.  Left to the compiler,
// the loads of every round are hoisted ahead and spilled to VGPR lanes (the scan code runs at
// the SGPR limit).  The asm loads are invisible to the compiler's waitcnt bookkeeping: every
// statement that reads masks opens with its own s_waitcnt lgkmcnt(0) (which only ever waits
// longer for the compiler's own LGKM operations), and a loaded tuple is only read by the next
// statement.
__device__ __forceinline__ u32x8 plane_masks_issue(uint32_t c) {
  u32x8 t;
  asm volatile("s_load_dwordx8 %0, %1, %2" : "=s"(t) : "s"(c_planes.m), "s"(c << 5));
  return t;
}

#define PIR_FOLD2_BODY                              \
  "v_bitop3_b32 %0, %0, %17, %19 bitop3:0x78\n\t"   \
  "v_bitop3_b32 %1, %1, %18, %19 bitop3:0x78\n\t"   \
  "v_bitop3_b32 %2, %2, %17, %20 bitop3:0x78\n\t"   \
  "v_bitop3_b32 %3, %3, %18, %20 bitop3:0x78\n\t"   \
  "v_bitop3_b32 %4, %4, %17, %21 bitop3:0x78\n\t"   \
  "v_bitop3_b32 %5, %5, %18, %21 bitop3:0x78\n\t"   \
  "v_bitop3_b32 %6, %6, %17, %22 bitop3:0x78\n\t"   \
  "v_bitop3_b32 %7, %7, %18, %22 bitop3:0x78\n\t"   \
  "v_bitop3_b32 %8, %8, %17, %23 bitop3:0x78\n\t"   \
  "v_bitop3_b32 %9, %9, %18, %23 bitop3:0x78\n\t"   \
  "v_bitop3_b32 %10, %10, %17, %24 bitop3:0x78\n\t" \
  "v_bitop3_b32 %11, %11, %18, %24 bitop3:0x78\n\t" \
  "v_bitop3_b32 %12, %12, %17, %25 bitop3:0x78\n\t" \
  "v_bitop3_b32 %13, %13, %18, %25 bitop3:0x78\n\t" \
  "v_bitop3_b32 %14, %14, %17, %26 bitop3:0x78\n\t" \
  "v_bitop3_b32 %15, %15, %18, %26 bitop3:0x78"
#define PIR_FOLD2_Z                                                                          \
  "+v"(Z[0][0]), "+v"(Z[0][1]), "+v"(Z[1][0]), "+v"(Z[1][1]), "+v"(Z[2][0]), "+v"(Z[2][1]),   \
      "+v"(Z[3][0]), "+v"(Z[3][1]), "+v"(Z[4][0]), "+v"(Z[4][1]), "+v"(Z[5][0]), "+v"(Z[5][1]), \
      "+v"(Z[6][0]), "+v"(Z[6][1]), "+v"(Z[7][0]), "+v"(Z[7][1])
#define PIR_FOLD2_IN                                                                         \
  "v"(x0), "v"(x1), "s"(m[0]), "s"(m[1]), "s"(m[2]), "s"(m[3]), "s"(m[4]), "s"(m[5]), "s"(m[6]), \
      "s"(m[7])

// wait for m, start loading the masks of coefficient byte cn, fold one round (operand 16 is the
// next tuple, so the body's operand numbers match planes_fold2's)
__device__ __forceinline__ u32x8 planes_fold2_next(uint32_t (&Z)[8][2], uint32_t x0, uint32_t x1,
                                                   const u32x8& m, uint32_t cn) {
  u32x8 nx;
  asm volatile("s_waitcnt lgkmcnt(0)\n\t"
               "s_load_dwordx8 %16, %27, %28\n\t" PIR_FOLD2_BODY
               : PIR_FOLD2_Z, "=&s"(nx)
               : PIR_FOLD2_IN, "s"(c_planes.m), "s"(cn << 5));
  return nx;
}
// wait for m and fold one round (no next load)
__device__ __forceinline__ void planes_fold2(uint32_t (&Z)[8][2], uint32_t x0, uint32_t x1,
                                             const u32x8& m) {
  uint32_t pad;  // operand 16 placeholder keeps the body's numbering
  asm volatile("s_waitcnt lgkmcnt(0)\n\t" PIR_FOLD2_BODY : PIR_FOLD2_Z, "=s"(pad) : PIR_FOLD2_IN);
  (void)pad;
}
#undef PIR_FOLD2_BODY
#undef PIR_FOLD2_Z
#undef PIR_FOLD2_IN

// the same for one dword per lane (records of one wave row at VEC = 1): 8 v_bitop3 per round
#define PIR_FOLD1_BODY                            \
  "v_bitop3_b32 %0, %0, %9, %10 bitop3:0x78\n\t" \
  "v_bitop3_b32 %1, %1, %9, %11 bitop3:0x78\n\t" \
  "v_bitop3_b32 %2, %2, %9, %12 bitop3:0x78\n\t" \
  "v_bitop3_b32 %3, %3, %9, %13 bitop3:0x78\n\t" \
  "v_bitop3_b32 %4, %4, %9, %14 bitop3:0x78\n\t" \
  "v_bitop3_b32 %5, %5, %9, %15 bitop3:0x78\n\t" \
  "v_bitop3_b32 %6, %6, %9, %16 bitop3:0x78\n\t" \
  "v_bitop3_b32 %7, %7, %9, %17 bitop3:0x78"
#define PIR_FOLD1_Z                                                                       \
  "+v"(Z[0][0]), "+v"(Z[1][0]), "+v"(Z[2][0]), "+v"(Z[3][0]), "+v"(Z[4][0]), "+v"(Z[5][0]), \
      "+v"(Z[6][0]), "+v"(Z[7][0])
#define PIR_FOLD1_IN                                                                        \
  "v"(x0), "s"(m[0]), "s"(m[1]), "s"(m[2]), "s"(m[3]), "s"(m[4]), "s"(m[5]), "s"(m[6]), "s"(m[7])

__device__ __forceinline__ u32x8 planes_fold1_next(uint32_t (&Z)[8][1], uint32_t x0, const u32x8& m,
                                                   uint32_t cn) {
  u32x8 nx;
  asm volatile("s_waitcnt lgkmcnt(0)\n\t"
               "s_load_dwordx8 %8, %18, %19\n\t" PIR_FOLD1_BODY
               : PIR_FOLD1_Z, "=&s"(nx)
               : PIR_FOLD1_IN, "s"(c_planes.m), "s"(cn << 5));
  return nx;
}
__device__ __forceinline__ void planes_fold1(uint32_t (&Z)[8][1], uint32_t x0, const u32x8& m) {
  uint32_t pad;
  asm volatile("s_waitcnt lgkmcnt(0)\n\t" PIR_FOLD1_BODY : PIR_FOLD1_Z, "=s"(pad) : PIR_FOLD1_IN);
  (void)pad;
}
#undef PIR_FOLD1_BODY
#undef PIR_FOLD1_Z
#undef PIR_FOLD1_IN

__device__ __forceinline__ uint32_t coef_byte(const uint4& c, int a) {
  const uint32_t w = a < 4 ? c.x : (a < 8 ? c.y : (a < 12 ? c.z : c.w));
  return (w >> (8 * (a & 3))) & 0xffu;
}

template <int NQ, int NRP, int VEC, bool UNI>
__global__ __launch_bounds__(kScanThreads) void k_scan(const uint8_t* __restrict__ shard,
                                                       uint64_t nrec, uint32_t pitch,
                                                       uint32_t cpr, const uint8_t* __restrict__ c,
                                                       uint8_t* __restrict__ slabs, int accumulate) {
  constexpr int CH = VEC * 4;  // bytes per lane chunk
  constexpr int GW = kColGroupLanes * VEC;  // words per column group
  __shared__ uint32_t red[NQ * GW];
  for (int i = threadIdx.x; i < NQ * GW; i += blockDim.x) red[i] = 0;

  const int lane = threadIdx.x & 63;
  const uint32_t waves_per_block = blockDim.x >> 6;
  const uint64_t wave = (uint64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * waves_per_block;
  uint32_t rpw, rec_off, chunk;
  bool active;
  if (UNI) {
    rpw = 1; rec_off = 0;
    chunk = blockIdx.y * kColGroupLanes + lane;
    active = chunk < cpr;
  } else {
    rpw = kColGroupLanes / cpr;
    rec_off = lane / cpr;
    chunk = lane - rec_off * cpr;
    active = (uint32_t)lane < rpw * cpr;
  }
  const uint64_t ngroups = (nrec + rpw - 1) / rpw;
  const uint64_t g0 = wave * ngroups / nwaves, g1 = (wave + 1) * ngroups / nwaves;

  uint32_t Z[NQ][8][VEC];
#pragma unroll
  for (int a = 0; a < NQ; ++a)
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int v = 0; v < VEC; ++v) Z[a][k][v] = 0;

  const uint8_t* base = shard + (uint64_t)chunk * CH;
  constexpr int U = 4;
  uint64_t gi = g0;
  for (; gi + U <= g1; gi += U) {
    Chunk<VEC> x[U];
    uint4 cf[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t rec = (gi + u) * rpw + rec_off;
      const bool ok = active && rec < nrec;
      if (ok) x[u] = load_chunk<VEC>(base + rec * pitch);
      else
        for (int v = 0; v < VEC; ++v) x[u].v[v] = 0;
      if (UNI) {
        const uint64_t r = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(gi + u)) |
                           ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)((gi + u) >> 32)) << 32);
        cf[u] = load_coef<NRP>(c, r);
      } else {
        cf[u] = ok ? load_coef<NRP>(c, rec) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int a = 0; a < NQ; ++a) {
        const uint32_t ca = coef_byte(cf[u], a);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t m = 0u - ((ca >> k) & 1u);
#pragma unroll
          for (int v = 0; v < VEC; ++v) Z[a][k][v] = mxor(Z[a][k][v], x[u].v[v], m);
        }
      }
  }
  for (; gi < g1; ++gi) {
    const uint64_t rec = gi * rpw + rec_off;
    const bool ok = active && rec < nrec;
    Chunk<VEC> x;
    if (ok) x = load_chunk<VEC>(base + rec * pitch);
    else
      for (int v = 0; v < VEC; ++v) x.v[v] = 0;
    const uint4 cf = ok ? load_coef<NRP>(c, rec) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int a = 0; a < NQ; ++a) {
      const uint32_t ca = coef_byte(cf, a);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t m = 0u - ((ca >> k) & 1u);
#pragma unroll
        for (int v = 0; v < VEC; ++v) Z[a][k][v] = mxor(Z[a][k][v], x.v[v], m);
      }
    }
  }
  __syncthreads();  // red[] zeroed
  if (active) {
    const uint32_t wbase = (UNI ? (uint32_t)lane : chunk) * VEC;
#pragma unroll
    for (int a = 0; a < NQ; ++a)
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        uint32_t acc = Z[a][7][v];
#pragma unroll
        for (int k = 6; k >= 0; --k) acc = gf_xtime4(acc) ^ Z[a][k][v];
        if (acc) atomicXor(&red[a * GW + wbase + v], acc);
      }
  }
  __syncthreads();
  uint32_t* slab = reinterpret_cast<uint32_t*>(slabs) +
                   ((uint64_t)blockIdx.y * gridDim.x + blockIdx.x) * (NQ * GW);
  if (accumulate)
    for (int i = threadIdx.x; i < NQ * GW; i += blockDim.x) slab[i] ^= red[i];
  else
    for (int i = threadIdx.x; i < NQ * GW; i += blockDim.x) slab[i] = red[i];
}

// k_scan_uni: the scan for records of at least one wave row (one record per wave row,
// wave-uniform coefficients), with the scan-wave inner loop of k_query: a rolling pipeline of U
// rows per lane (row j + U is loaded into x[u] as soon as row j is folded, so U rows stay in
// flight), coefficients read 64 rows ahead (lane l loads row r0 + 64 + l's bytes, broadcast by
// v_readlane), and per round
//   VEC = 4 (NQ <= 3) or NQ <= 2 : scalar branches on the coefficient bits (~4 v_xor of two
//             VGPRs per dword instead of 8 v_bitop3 with an SGPR mask, which issue at 2/3 the
//             rate: profiles/r02_micro/valu_rate.log),
//   VEC <= 2, NQ >= 3 : the 8 plane masks from the table (s_load_dwordx8, one round ahead;
//             per-bit s_bfe masks held the 8-round batched scan to 1.5 TB/s on the scalar unit).
// Wave w folds rows [w * nrec / nwaves, (w + 1) * nrec / nwaves) of its column group.
constexpr uint32_t kScanDynRows = 32;  // k_scan_uni's claimed chunks (four Russians, dyn)
#ifndef PIR_SCAN_DYN_G
#define PIR_SCAN_DYN_G 2  // groups of 4 rows in flight per wave in the four-Russians chunk loop
#endif
template <int NQ, int NRP, int VEC, int NT = kScanThreads>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == kScanThreads ? kScanThreads / 64 * kScanBlocksPerCU / 4 : NT / 256)))
void k_scan_uni(const uint8_t* __restrict__ shard,
                                                           uint64_t nrec, uint32_t pitch,
                                                           uint32_t cpr, const uint8_t* __restrict__ c,
                                                           uint8_t* __restrict__ slabs, int accumulate) {
  constexpr int CH = VEC * 4;
  constexpr int GW = kColGroupLanes * VEC;
#ifndef PIR_SCAN_U3
#define PIR_SCAN_U3 4  // rows in flight per lane for 3 rounds at <= 2 dwords per lane
#endif
  constexpr int U = NQ <= 2 ? 8 : (NQ == 3 && VEC <= 2 ? PIR_SCAN_U3 : 4);  // divides 64
  constexpr bool kBranch = VEC == 4 || NQ <= 2;
  // four Russians over groups of 4 rows (pir_m4r.h): one dword per lane for 4-8 rounds (8 NQ +
  // 16 VGPRs of planes and row combinations fit the 128 of 16 waves per CU), two dwords for 4-5
  // rounds in the 768-thread instance (16 NQ + 32 VGPRs: 168 per wave at 12 waves per CU)
  constexpr bool kM4R = (VEC == 1 && NQ >= 4 && NQ <= 8 && NRP >= 4 && NRP <= 8) ||
                        (VEC == 2 && NQ >= 4 && NQ <= 5 && NT == kScanM4rThreads);
  constexpr bool kAsm = !kBranch && !kM4R && VEC <= 2 && NQ >= 3;
  // accumulate bit 1 (launch_scan, $PIR_SCAN_DYN): the four-Russians waves claim chunks of the
  // workgroup's rows instead of folding a fixed range each
  const bool dyn = (kM4R ? PIR_M4R_SLOAD != 0 : NQ <= 5) && ((accumulate >> 1) & 1);
  accumulate &= 1;
  __shared__ uint32_t red[NQ * GW];
  __shared__ uint32_t next_chunk;
  for (int i = threadIdx.x; i < NQ * GW; i += blockDim.x) red[i] = 0;

  const uint32_t lane = threadIdx.x & 63;
  const uint32_t waves_per_block = blockDim.x >> 6;
  const uint64_t wave = (uint64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * waves_per_block;
  const uint32_t chunk = blockIdx.y * kColGroupLanes + lane;
  const bool active = chunk < cpr;
  const uint64_t r0 = wave * nrec / nwaves, r1 = (wave + 1) * nrec / nwaves;

  uint32_t Z[NQ][8][VEC];
#pragma unroll
  for (int a = 0; a < NQ; ++a)
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int v = 0; v < VEC; ++v) Z[a][k][v] = 0;

  // one row's fold into the planes: row j of the 64-row coefficient block c4 (lane l holds
  // row l's coefficient bytes)
  auto fold_j = [&](const Chunk<VEC>& xr, const uint4& c4, uint32_t j) __attribute__((always_inline)) {
    const uint4 cf = make_uint4(__builtin_amdgcn_readlane(c4.x, j),
                                NRP > 4 ? __builtin_amdgcn_readlane(c4.y, j) : 0u,
                                NRP > 8 ? __builtin_amdgcn_readlane(c4.z, j) : 0u,
                                NRP > 8 ? __builtin_amdgcn_readlane(c4.w, j) : 0u);
    if constexpr (kAsm) {
      u32x8 m = plane_masks_issue(coef_byte(cf, 0));
#pragma unroll
      for (int a = 0; a < NQ; ++a) {
        if constexpr (VEC == 2) {
          auto& Za = reinterpret_cast<uint32_t(&)[8][2]>(Z[a]);
          if (a + 1 < NQ) m = planes_fold2_next(Za, xr.v[0], xr.v[1], m, coef_byte(cf, a + 1));
          else planes_fold2(Za, xr.v[0], xr.v[1], m);
        } else {
          auto& Za = reinterpret_cast<uint32_t(&)[8][1]>(Z[a]);
          if (a + 1 < NQ) m = planes_fold1_next(Za, xr.v[0], m, coef_byte(cf, a + 1));
          else planes_fold1(Za, xr.v[0], m);
        }
      }
    } else {
#pragma unroll
      for (int a = 0; a < NQ; ++a) {
        const uint32_t ca = coef_byte(cf, a);
        if constexpr (kBranch) {
#pragma unroll
          for (int kk = 0; kk < 8; ++kk)
            if (ca & (1u << kk)) {
#pragma unroll
              for (int v = 0; v < VEC; ++v) Z[a][kk][v] ^= xr.v[v];
            }
        } else {
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) {
            const uint32_t m = 0u - ((ca >> kk) & 1u);
#pragma unroll
            for (int v = 0; v < VEC; ++v) Z[a][kk][v] = mxor(Z[a][kk][v], xr.v[v], m);
          }
        }
      }
    }
  };
  if constexpr (!kM4R && NQ <= 5) {  // (6-8 rounds take k_scan_t; the wider instances spill)
    if (dyn) {
      // as the four-Russians chunks below, for the per-row folds: chunks of the 64-row
      // coefficient block, the next chunk's coefficients and first rows in flight
      constexpr uint32_t C = 64;
      if (threadIdx.x == 0) next_chunk = 0;
      __syncthreads();
      const uint64_t wg0 = (uint64_t)blockIdx.x * waves_per_block;
      const uint64_t R0 = rfl64(wg0 * nrec / nwaves);
      const uint32_t nrows = (uint32_t)__builtin_amdgcn_readfirstlane(
          (uint32_t)((wg0 + waves_per_block) * nrec / nwaves - wg0 * nrec / nwaves));
      const uint32_t nch = (nrows + C - 1) / C;
      const uint8_t* base = shard + (uint64_t)(active ? chunk : 0u) * CH + R0 * pitch;
      auto claim = [&]() __attribute__((always_inline)) -> uint32_t {
        uint32_t v = 0;
        if (lane == 0)
          v = __hip_atomic_fetch_add(&next_chunk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return (uint32_t)__builtin_amdgcn_readfirstlane(v);
      };
      auto rowp = [&](uint32_t ch, uint32_t k) __attribute__((always_inline)) -> uint32_t {
        const uint32_t o = ch * C + k;
        return ch < nch && o < nrows ? o : 0u;
      };
      auto coefs_ch = [&](uint32_t ch) __attribute__((always_inline)) {
        const uint32_t o = ch * C + lane;
        return ch < nch && o < nrows ? load_coef<NRP>(c, R0 + o) : make_uint4(0, 0, 0, 0);
      };
      uint32_t cur = claim();
      if (cur < nch) {
        uint32_t nxt = claim();
        Chunk<VEC> x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = load_chunk<VEC>(base + (uint64_t)rowp(cur, u) * pitch);
        uint4 c4 = coefs_ch(cur);
        while (true) {
          const uint4 c4n = coefs_ch(nxt);
          const uint32_t nb = nrows - cur * C < C ? nrows - cur * C : C;
          for (uint32_t j0 = 0; j0 < C; j0 += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const uint32_t j = j0 + u;
              if (j < nb) fold_j(x[u], c4, j);  // wave-uniform
              const uint32_t k = j + U;
              x[u] = load_chunk<VEC>(base + (uint64_t)(k < C ? rowp(cur, k) : rowp(nxt, k - C)) * pitch);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
          cur = nxt;
          c4 = c4n;
          if (cur >= nch) break;
          nxt = claim();
        }
      }
    }
  }
#if PIR_M4R_SLOAD
  if constexpr (kM4R) {
    if (dyn) {
      // Equal-priority waves issue oldest first, so with a fixed row range per wave the oldest
      // waves of a SIMD finish first and the youngest ones fold the tail alone.  Here the
      // workgroup's rows are chunks of kScanDynRows claimed one at a time (an LDS counter, the
      // next chunk claimed while the current one folds, so the rolling row / coefficient loads
      // run ahead across chunk boundaries); every wave's planes are XORed into red[] at the
      // end, so which wave folds a chunk does not matter.  Rows past the workgroup's last take
      // coefficient 0 and re-read its first row.
      constexpr uint32_t C = kScanDynRows % (4 * PIR_SCAN_DYN_G) == 0 ? kScanDynRows : 16 * PIR_SCAN_DYN_G;
      if (threadIdx.x == 0) next_chunk = 0;
      __syncthreads();
      const uint64_t wg0 = (uint64_t)blockIdx.x * waves_per_block;
      const uint64_t R0 = rfl64(wg0 * nrec / nwaves);
      const uint32_t nrows = (uint32_t)__builtin_amdgcn_readfirstlane(
          (uint32_t)((wg0 + waves_per_block) * nrec / nwaves - wg0 * nrec / nwaves));
      const uint32_t nch = (nrows + C - 1) / C;
      using CW = std::conditional_t<NRP == 8, uint64_t, uint32_t>;
      typedef const __attribute__((address_space(4))) CW* ConstCW;
      const ConstCW cwb = (ConstCW)(const CW*)c + R0;
      const uint8_t* base = shard + (uint64_t)(active ? chunk : 0u) * CH + R0 * pitch;
      auto claim = [&]() __attribute__((always_inline)) -> uint32_t {
        uint32_t v = 0;
        if (lane == 0)
          v = __hip_atomic_fetch_add(&next_chunk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return (uint32_t)__builtin_amdgcn_readfirstlane(v);
      };
      uint32_t cur = claim();
      if (cur < nch) {
        uint32_t nxt = claim();
        // G groups of 4 rows in flight (rows and coefficient words loaded G groups ahead)
        constexpr int G = PIR_SCAN_DYN_G;
        static_assert(C % (4 * G) == 0, "whole group batches per chunk");
        // row k of the sequence that runs on from the current chunk into the next: its offset
        // in the workgroup's rows (0 and false past the last row)
        auto pos = [&](uint32_t k, uint32_t& o) __attribute__((always_inline)) -> bool {
          const uint32_t nc = k < C ? cur : nxt;
          o = nc * C + (k < C ? k : k - C);
          const bool v = nc < nch && o < nrows;
          if (!v) o = 0u;
          return v;
        };
        Chunk<VEC> x[4 * G];
        uint64_t w[4 * G];
        bool wv[4 * G];
#pragma unroll
        for (int q = 0; q < 4 * G; ++q) {
          uint32_t o;
          wv[q] = pos((uint32_t)q, o);
          w[q] = (uint64_t)cwb[o];
          x[q] = load_chunk<VEC>(base + (uint64_t)o * pitch);
        }
        while (true) {
          for (uint32_t i = 0; i < C; i += 4 * G) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
              const int q0 = 4 * g;
              const uint32_t vi = m4r_index(rfl64(wv[q0] ? w[q0] : 0), rfl64(wv[q0 + 1] ? w[q0 + 1] : 0),
                                            rfl64(wv[q0 + 2] ? w[q0 + 2] : 0), rfl64(wv[q0 + 3] ? w[q0 + 3] : 0));
              __builtin_amdgcn_sched_barrier(0);
              uint32_t o[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                wv[q0 + r] = pos(i + 4u * G + (uint32_t)(q0 + r), o[r]);
                w[q0 + r] = (uint64_t)cwb[o[r]];
              }
              m4r_fold_group<VEC, NQ>(Z, x[q0].v, x[q0 + 1].v, x[q0 + 2].v, x[q0 + 3].v, vi,
                                      (lane & 7u) * 4u);
#pragma unroll
              for (int r = 0; r < 4; ++r) x[q0 + r] = load_chunk<VEC>(base + (uint64_t)o[r] * pitch);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
          cur = nxt;
          if (cur >= nch) break;
          nxt = claim();
        }
      }
    }
  }
#endif
  if (!dyn && r1 > r0) {
    // inactive lanes read the row's first chunk (their planes are never written out); slots past
    // the wave's last row re-read its first row (never folded)
    const uint8_t* base = shard + (uint64_t)(active ? chunk : 0u) * CH;
    auto load_row = [&](uint64_t r, Chunk<VEC>& dst) __attribute__((always_inline)) {
      dst = load_chunk<VEC>(base + (r < r1 ? r : r0) * pitch);
    };
    auto coefs64 = [&](uint64_t rb) __attribute__((always_inline)) {
      const uint64_t r = rb + lane;
      return r < r1 ? load_coef<NRP>(c, r) : make_uint4(0, 0, 0, 0);
    };
    Chunk<VEC> x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) load_row(r0 + u, x[u]);
#if PIR_M4R_SLOAD
    if constexpr (kM4R) {
      // the 4 rows' coefficient words straight into SGPRs: scalar loads of the wave-uniform rows
      // (constant address space), issued one group ahead, after the group's indices are built --
      // an s_waitcnt lgkmcnt(0) before m4r_index then waits only for loads a whole fold old.
      // Rows past the wave's last read its last row's word and take 0.
      using CW = std::conditional_t<NRP == 8, uint64_t, uint32_t>;
      typedef const __attribute__((address_space(4))) CW* ConstCW;
      const ConstCW cw = (ConstCW)(const CW*)c;
      // 32-bit row offsets in the wave's range: SALU compares (no 64-bit s_cmp_lt on gfx950),
      // and the zeroing select at use, a group after the load
      const uint64_t u0 = rfl64(r0);
      const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(r1 - r0));
      const ConstCW cwb = cw + u0;
      auto raw = [&](uint32_t i) __attribute__((always_inline)) -> uint64_t {
        return (uint64_t)cwb[i < n ? i : n - 1];
      };
      uint64_t w[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = raw(r);
      for (uint32_t i = 0; i < n; i += 4) {
        const uint32_t vi = m4r_index(w[0], i + 1 < n ? w[1] : 0, i + 2 < n ? w[2] : 0,
                                      i + 3 < n ? w[3] : 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = raw(i + 4 + r);
        m4r_fold_group<VEC, NQ>(Z, x[0].v, x[1].v, x[2].v, x[3].v, vi, (lane & 7u) * 4u);
#pragma unroll
        for (int r = 0; r < 4; ++r) load_row(r0 + i + r + U, x[r]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else
#endif
    {
    uint4 c4 = coefs64(r0);
    for (uint64_t rb = r0; rb < r1; rb += 64) {
      const uint4 c4n = coefs64(rb + 64);  // the next 64 rows' coefficients, in flight
      const uint32_t nb = (uint32_t)(r1 - rb < 64 ? r1 - rb : 64);
      if constexpr (kM4R) {
        // groups of 4 rows; rows past the wave's last have zero coefficients (no plane takes
        // them) and re-read its first row
        for (uint32_t j0 = 0; j0 < nb; j0 += 4) {
          const uint32_t vi = m4r_index(coef_word(c4, j0), coef_word(c4, j0 + 1),
                                        coef_word(c4, j0 + 2), coef_word(c4, j0 + 3));
          m4r_fold_group<VEC, NQ>(Z, x[0].v, x[1].v, x[2].v, x[3].v, vi, (lane & 7u) * 4u);
#pragma unroll
          for (int r = 0; r < 4; ++r) load_row(rb + j0 + r + U, x[r]);
          __builtin_amdgcn_sched_barrier(0);
        }
        c4 = c4n;
        continue;
      }
      for (uint32_t j0 = 0; j0 < nb; j0 += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t j = j0 + u;
          if (j < nb) fold_j(x[u], c4, j);  // wave-uniform
          load_row(rb + j + U, x[u]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      c4 = c4n;
    }
    }
  }
  __syncthreads();  // red[] zeroed
  if (active) {
    const uint32_t wbase = lane * VEC;
#pragma unroll
    for (int a = 0; a < NQ; ++a)
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        uint32_t acc = Z[a][7][v];
#pragma unroll
        for (int k = 6; k >= 0; --k) acc = gf_xtime4(acc) ^ Z[a][k][v];
        if (acc) atomicXor(&red[a * GW + wbase + v], acc);
      }
  }
  __syncthreads();
  uint32_t* slab = reinterpret_cast<uint32_t*>(slabs) +
                   ((uint64_t)blockIdx.y * gridDim.x + blockIdx.x) * (NQ * GW);
  if (accumulate)
    for (int i = threadIdx.x; i < NQ * GW; i += blockDim.x) slab[i] ^= red[i];
  else
    for (int i = threadIdx.x; i < NQ * GW; i += blockDim.x) slab[i] = red[i];
}

// ------------------------------------------------------------------------------------------
// k_fused: the leaf stage of the tree and the shard scan in ONE persistent kernel, one
// workgroup per CU, waves specialised by role so the AES tree (VALU + LDS bound) runs under
// the HBM-bound scan on every CU:
//   tree waves [0, TW)   : tile i (TILE_LEAVES leaves) = expand `tile_in` nodes of level L_in
//                          by k levels (row-shape AES, breadth-first in LDS, synchronised by an
//                          LDS counter barrier among the tree waves only) and write the DPF
//                          shares c[leaf][0..NRP) into LDS ring slot i % 2;
//   scan waves [TW, 16)  : stream the shard rows of tile i from HBM and fold them into the
//                          per-lane GF(2^8) bit-plane accumulators with the shares of slot i%2.
// Handshake through two LDS counters: `ready` (tiles produced) and `consumed` (scan-wave
// arrivals), so the tree can run one tile ahead.  The shares never leave the CU.
// ------------------------------------------------------------------------------------------
constexpr int kFusedThreads = 1024;
constexpr int kFusedWaves = kFusedThreads / 64;
constexpr int kM4rThreads = 768;  // k_query, 4-5 rounds: 4 tree + 8 scan waves, 168 VGPRs each
constexpr int kM4rTW = 4;

template <int TILE, int NRP, int NQ, int VEC, int GYMAX>
struct FusedSmem {
  uint32_t tab[2 * 256 * 32];
  uint4 sa[TILE / 2];
  uint32_t ta[TILE / 2];
  uint4 sb[TILE / 4];
  uint32_t tb[TILE / 4];
  uint8_t ring[2][TILE * NRP];
  uint32_t red[GYMAX][NQ * kColGroupLanes * VEC];
  uint32_t bar, ready;
  uint32_t consumed[2];  // per ring slot: scan-wave arrivals (a wave may run a tile ahead)
};

__device__ __forceinline__ uint32_t lds_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait_geq(const uint32_t* p, uint32_t v) {
  while (lds_load(p) < v) __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// the same for a wait expected to be long (a tree wave far ahead of the scan): polls ~0.5 us apart
__device__ __forceinline__ void lds_wait_geq_idle(const uint32_t* p, uint32_t v) {
  while (lds_load(p) < v) __builtin_amdgcn_s_sleep(16);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ void lds_signal(uint32_t* p) {  // one lane per wave
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Diagnostic build only (-DPIR_FOLD_STAMPS=1, tools/fold_phases.py): k_query's four-Russians
// scan waves add the shader cycles of each phase of their loop into per-wave counters, written
// to trace[kFoldStampBase + 8 sw + k] at the end.  s_memtime + its wait costs ~10 % of a wave's
// cycles, so the shares, not the totals, are the finding.  The product build has none of this.
#ifndef PIR_FOLD_STAMPS
#define PIR_FOLD_STAMPS 0
#endif
constexpr int kFoldStampBase = 192;
__device__ __forceinline__ uint64_t fold_stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  return t;
}
// barrier among `nw` waves (not the whole workgroup): generation-counted LDS counter
__device__ __forceinline__ void group_barrier(uint32_t* ctr, uint32_t& gen, uint32_t nw) {
  lds_signal(ctr);
  gen += nw;
  lds_wait_geq(ctr, gen);
}

template <int NQ, int NRP, int VEC, bool UNI, int TW, int TILE, int GYMAX>
__global__ __launch_bounds__(kFusedThreads) void k_fused(
    const DevKey* __restrict__ K, const uint4* __restrict__ in_s, const uint32_t* __restrict__ in_t,
    int L_in, int k, uint64_t ntiles, const uint8_t* __restrict__ shard, uint32_t pitch,
    uint32_t cpr, uint32_t gy, uint8_t* __restrict__ slabs) {
  constexpr int SW = kFusedWaves - TW;
  constexpr int CH = VEC * 4;
  constexpr int GW = kColGroupLanes * VEC;
  constexpr int NW = NRP <= 4 ? 1 : NRP / 4;
  using Smem = FusedSmem<TILE, NRP, NQ, VEC, GYMAX>;
  __shared__ Smem sm;
  load_tables(sm.tab);
  for (int i = threadIdx.x; i < GYMAX * NQ * GW; i += blockDim.x) (&sm.red[0][0])[i] = 0;
  if (threadIdx.x == 0) { sm.bar = 0; sm.ready = 0; sm.consumed[0] = 0; sm.consumed[1] = 0; }
  __syncthreads();

  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t G = gridDim.x, b = blockIdx.x;
  const uint32_t my_tiles = ntiles > b ? (uint32_t)((ntiles - 1 - b) / G + 1) : 0u;
  const int tile_in = TILE >> k;

  if (wave < (uint32_t)TW) {
    // ===================================== tree role ======================================
    const Tab T(sm.tab);
    const Bits B(K->p);
    const int tt = threadIdx.x, nt = TW * 64;
    uint32_t gen = 0;
    uint4 qm;
    {
      const int nq = (int)K->nq;
      uint32_t m[4];
      for (int w = 0; w < 4; ++w) {
        const int nb = nq - 4 * w;
        m[w] = nb >= 4 ? 0xffffffffu : (nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u));
      }
      qm = make_uint4(m[0], m[1], m[2], m[3]);
    }
    for (uint32_t i = 0; i < my_tiles; ++i) {
      const uint64_t tile = b + (uint64_t)i * G;
      const uint64_t ibase = tile * tile_in;
      uint8_t* ring = sm.ring[i & 1];
      // slot i&1 free: every scan wave finished tile i-2 (per-slot count: no wave can arrive
      // twice on a slot before the tree refills it)
      if (i >= 2) lds_wait_geq(&sm.consumed[i & 1], (i >> 1) * SW);
      int buf = (k - 1) & 1;
      {
        uint4* s0 = buf ? sm.sb : sm.sa;
        uint32_t* t0 = buf ? sm.tb : sm.ta;
        for (int u = tt; u < tile_in; u += nt) {
          s0[u] = in_s[ibase + u];
          t0[u] = in_t[ibase + u];
        }
      }
      group_barrier(&sm.bar, gen, TW);
      int W = tile_in;
      for (int lv = 0; lv < k - 1; ++lv) {
        const uint4* is = buf ? sm.sb : sm.sa;
        const uint32_t* it = buf ? sm.tb : sm.ta;
        uint4* os = buf ? sm.sa : sm.sb;
        uint32_t* ot = buf ? sm.ta : sm.tb;
        for (int u = tt; u < W; u += nt) {
          uint4 sl, sr;
          uint32_t tl, tr;
          expand_node(T, K, L_in + lv, B, is[u], it[u], sl, sr, tl, tr);
          os[2 * u] = sl; os[2 * u + 1] = sr;
          ot[2 * u] = tl; ot[2 * u + 1] = tr;
        }
        group_barrier(&sm.bar, gen, TW);
        buf ^= 1;
        W *= 2;
      }
      {
        const uint4* is = buf ? sm.sb : sm.sa;
        const uint32_t* it = buf ? sm.tb : sm.ta;
        const int L = L_in + k - 1;
        for (int u = tt; u < W; u += nt) {
          uint4 sl, sr;
          uint32_t tl, tr;
          expand_node(T, K, L, B, is[u], it[u], sl, sr, tl, tr);
          uint4 vl = leaf_value<NW, (NRP < 4 ? NRP : 0)>(T, K, B.pm1, sl, tl);
          uint4 vr = leaf_value<NW, (NRP < 4 ? NRP : 0)>(T, K, B.pm1, sr, tr);
          vl = make_uint4(vl.x & qm.x, vl.y & qm.y, vl.z & qm.z, vl.w & qm.w);
          vr = make_uint4(vr.x & qm.x, vr.y & qm.y, vr.z & qm.z, vr.w & qm.w);
          if constexpr (NRP == 1) {
            *reinterpret_cast<uint16_t*>(ring + 2 * u) = (uint16_t)((vl.x & 0xffu) | ((vr.x & 0xffu) << 8));
          } else {
            store_leaf<NRP>(ring, 2 * u, vl);
            store_leaf<NRP>(ring, 2 * u + 1, vr);
          }
        }
      }
      group_barrier(&sm.bar, gen, TW);  // every share of tile i is in the ring
      if (wave == 0) lds_signal(&sm.ready);
    }
  } else {
    // ===================================== scan role ======================================
    const uint32_t sw = wave - TW;
    uint32_t gcol, wi, nwg, rpw, rec_off, chunk;
    bool active;
    if (UNI) {  // gy column groups share the SW waves
      gcol = sw % gy;
      wi = sw / gy;
      nwg = SW / gy;
      rpw = 1; rec_off = 0;
      chunk = gcol * kColGroupLanes + lane;
      active = chunk < cpr && wi < nwg;
    } else {
      gcol = 0; wi = sw; nwg = SW;
      rpw = kColGroupLanes / cpr;
      rec_off = lane / cpr;
      chunk = lane - rec_off * cpr;
      active = lane < rpw * cpr;
    }
    uint32_t Z[NQ][8][VEC];
#pragma unroll
    for (int a = 0; a < NQ; ++a)
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
#pragma unroll
        for (int v = 0; v < VEC; ++v) Z[a][kk][v] = 0;
    const uint32_t ngroups = (TILE + rpw - 1) / rpw;
    constexpr int U = SW >= 8 ? 8 : 16;
    // memory-bound waves go first: their few VALU ops gate the next loads
    __builtin_amdgcn_s_setprio(2);
    for (uint32_t i = 0; i < my_tiles; ++i) {
      const uint64_t tile = b + (uint64_t)i * G;
      const uint8_t* ring = sm.ring[i & 1];
      lds_wait_geq(&sm.ready, i + 1);
      if (wi < nwg) {
        const uint8_t* base = shard + (tile * TILE) * pitch + (uint64_t)chunk * CH;
        // this wave's row groups: wi, wi + nwg, ...  (U rows in flight per lane)
        for (uint32_t g0 = wi; g0 < ngroups; g0 += U * nwg) {
          Chunk<VEC> x[U];
          uint4 cf[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const uint32_t gi = g0 + u * nwg;
            const uint32_t rl = gi * rpw + rec_off;
            const bool ok = active && gi < ngroups && rl < TILE;
            if (ok) x[u] = load_chunk<VEC>(base + (uint64_t)rl * pitch);
            else
              for (int v = 0; v < VEC; ++v) x[u].v[v] = 0;
            if (UNI) {  // one record per wave row: the coefficients are wave-uniform
              const uint32_t gu = __builtin_amdgcn_readfirstlane(gi);
              uint4 c4 = gu < ngroups ? load_coef<NRP>(ring, gu) : make_uint4(0, 0, 0, 0);
              cf[u] = make_uint4(__builtin_amdgcn_readfirstlane(c4.x), __builtin_amdgcn_readfirstlane(c4.y),
                                 __builtin_amdgcn_readfirstlane(c4.z), __builtin_amdgcn_readfirstlane(c4.w));
            } else {
              cf[u] = ok ? load_coef<NRP>(ring, rl) : make_uint4(0, 0, 0, 0);
            }
          }
#pragma unroll
          for (int u = 0; u < U; ++u)
#pragma unroll
            for (int a = 0; a < NQ; ++a) {
              const uint32_t ca = coef_byte(cf[u], a);
              if (UNI && NQ <= 2) {  // scalar branches: ~4 XORs per dword instead of 8 masked
#pragma unroll
                for (int kk = 0; kk < 8; ++kk)
                  if (ca & (1u << kk)) {
#pragma unroll
                    for (int v = 0; v < VEC; ++v) Z[a][kk][v] ^= x[u].v[v];
                  }
              } else if (UNI) {  // many rounds: branch-free, SGPR masks (no 8*NQ branches)
#pragma unroll
                for (int kk = 0; kk < 8; ++kk) {
                  const uint32_t m = 0u - ((ca >> kk) & 1u);
#pragma unroll
                  for (int v = 0; v < VEC; ++v) Z[a][kk][v] = mxor(Z[a][kk][v], x[u].v[v], m);
                }
              } else {
#pragma unroll
                for (int kk = 0; kk < 8; ++kk) {
                  const uint32_t m = 0u - ((ca >> kk) & 1u);
#pragma unroll
                  for (int v = 0; v < VEC; ++v) Z[a][kk][v] = mxor(Z[a][kk][v], x[u].v[v], m);
                }
              }
            }
        }
      }
      lds_signal(&sm.consumed[i & 1]);
    }
    if (active) {
      const uint32_t wbase = (UNI ? lane : chunk) * VEC;
#pragma unroll
      for (int a = 0; a < NQ; ++a)
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          uint32_t acc = Z[a][7][v];
#pragma unroll
          for (int kk = 6; kk >= 0; --kk) acc = gf_xtime4(acc) ^ Z[a][kk][v];
          if (acc) atomicXor(&sm.red[gcol][a * GW + wbase + v], acc);
        }
    }
  }
  __syncthreads();
  for (uint32_t g = 0; g < gy; ++g) {
    uint32_t* slab = reinterpret_cast<uint32_t*>(slabs) + ((uint64_t)g * gridDim.x + blockIdx.x) * (NQ * GW);
    for (int i = threadIdx.x; i < NQ * GW; i += blockDim.x) slab[i] = sm.red[g][i];
  }
}

// ------------------------------------------------------------------------------------------
// k_query: ONE launch answers a queue of `nk` independent queries, each its own DPF tree and
// its own full pass over the shard (no frontier / expand kernels before it).  Workgroup b owns
// region b of the partition (R = 2^(nr - lr) leaves, nr = n - log_parts) = T tiles of TILE
// leaves, and walks the tiles of query 0, then of query 1, ... .  Tree waves:
//   * key: the correction words of all levels and lastCW of the current query, in LDS;
//   * tile root: wave 0 walks the tree depth-first in column shape (16 lanes per node) from the
//     root along (prefix, b, tile) -- tile 0 descends all Lt = log_parts + lr + log2 T levels;
//     tile i > 0 pops the right sibling stored when its ancestor was expanded and descends
//     ctz(i) levels, so the T tile roots cost T - 1 expansions in all;
//   * tile: expand the root breadth-first in LDS and write the DPF shares into the LDS ring
//     (RING slots, so the tree runs up to RING - 1 tiles ahead of the scan).
// Tile 0 of query 0 is built by all 16 waves (nothing to scan before it).  Later tiles -- and
// the descent and first tile of the next query -- are built by the TW tree waves while the
// scan waves stream the previous ones, so in a queue only the first query waits for its tree.
// Scan waves are k_fused's; at the end of a query they fold their bit planes into LDS and
// write the workgroup's partial answer (slab) of that query.
// ------------------------------------------------------------------------------------------
// k_query tree waves: nodes per lane in flight on the wide row-shape levels and the leaf level
// (1 = one AES chain per lane, the round-3 form; PIR_TREE_ILP at build time)
#ifndef PIR_TREE_ILP
#define PIR_TREE_ILP 2
#endif
constexpr int kTreeIlp = PIR_TREE_ILP;
constexpr int kQueryCwCap = 256;  // (levels x (p-1)) correction words staged in LDS
#ifndef PIR_TRACE_TREE_TILES
// diagnostics build only: wave 0 of the tree team stamps two chosen queue tiles' phases into
// trace[224 + 16 t + k] (tiles from the trace flags' bits 8-15 and 16-23, 0 = off)
#define PIR_TRACE_TREE_TILES 0
#endif
constexpr int kQueryKin = 6;      // a tile's input nodes sit 6 levels below its root (64 of them)

template <int TILE, int NRP, int NQ, int VEC, int GYMAX, int RING>
struct QuerySmem {
  uint32_t tab[2 * 256 * 32];
  uint4 sa[TILE / 2];
  uint32_t ta[TILE / 2];
  uint4 sb[TILE / 4];
  uint32_t tb[TILE / 4];
  uint8_t ring[RING][TILE * NRP];
  uint32_t red[GYMAX][NQ * kColGroupLanes * VEC];
  uint4 scw[kQueryCwCap];           // sCW[L][j] at L * (p-1) + j
  uint32_t tcw[kQueryCwCap];
  uint4 lastcw[kMaxCW];
  uint4 stk_s[kMaxLevels + 1];      // right siblings on the current root-to-tile path
  uint32_t stk_t[kMaxLevels + 1];
  uint32_t bar, sbar, ready, lastq;
  uint32_t consumed[RING];
  uint32_t prog[8];  // tiles each scan wave has consumed (scan_even mode 2)
};

__device__ __forceinline__ void cw_lds(const uint4* scw, const uint32_t* tcw, int L, uint32_t t,
                                       uint32_t pm1, uint4& cs, uint32_t& ct) {
  cs = make_uint4(0, 0, 0, 0);
  ct = 0;
  const int base = L * (int)pm1;
  for (uint32_t j = 0; j < pm1; ++j) {
    const uint32_t m = 0u - ((t >> j) & 1u);
    cs = xor4(cs, and4(scw[base + j], m));
    ct ^= tcw[base + j] & m;
  }
}

// the key's correction words (dpf_tree.cpp:504-519) into LDS, by threads [0, nt)
__device__ __forceinline__ void stage_key(const uint8_t* __restrict__ raw, int p, int n, int nq,
                                          int tid, int nt, uint4* scw, uint32_t* tcw,
                                          uint4* lastcw) {
  const int pm1 = p - 1;
  for (int i = tid; i < n * pm1; i += nt) {
    const int L = i / pm1, j = i - L * pm1;
    parse_cw(raw, p, L, j, scw[i], tcw[i]);
  }
  for (int j = tid; j < kMaxCW; j += nt) {
    uint32_t w[4] = {0, 0, 0, 0};
    if (j < pm1)
      for (int a = 0; a < nq; ++a)
        w[a >> 2] |= (uint32_t)raw[16 + n * pm1 * (16 + 2 * p - 2) + a * pm1 + j] << (8 * (a & 3));
    lastcw[j] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// The shares of records [rec0, rec0 + TILE) of a sqrt(N) DPF key (multiparty or covering
// design, the layout of pir_mp.h: share a of record i*mu + x = XOR over the row's seeds j with
// toggle (a, i, j) set of G(s[i][j], mu)[x] ^ cw[j][x]; multiparty_dpf.cpp:590-601, :665-675)
// into a k_query ring slot ([record][NRP] bytes), by the first nt threads: lpi lanes per CTR
// block of the tile (16 records) split the row's seeds, then XOR their partials.  TILE | mu.
// nt >= TILE / 16 is required (one block per thread at most; query_nq_mp static_asserts it).
template <int TILE, int NRP>
__device__ __forceinline__ void mp_tile(const Tab& T, const uint8_t* __restrict__ key,
                                        const MpLayout& L, uint64_t rec0, uint8_t* ring, int tt,
                                        int nt) {
  constexpr int NB = TILE / 16;
  int lpi = 1;
  while (lpi * 2 * NB <= nt) lpi *= 2;
  const int blk = tt / lpi, sub = tt & (lpi - 1);
  const bool act = blk < NB;
  const uint64_t ri = rec0 / L.mu;
  const uint32_t bc = (uint32_t)((rec0 - ri * L.mu) >> 4) + (uint32_t)(act ? blk : 0);
  const uint64_t row_tog = L.nu * L.p2;
  const bool cw_al = (L.cw_off & 15) == 0;
  uint4 acc[NRP];
#pragma unroll
  for (int a = 0; a < NRP; ++a) acc[a] = make_uint4(0, 0, 0, 0);
  if (act) {
    for (uint32_t j = (uint32_t)sub; j < L.p2; j += (uint32_t)lpi) {
      uint32_t m[NRP];
      uint32_t any = 0;
#pragma unroll
      for (int a = 0; a < NRP; ++a) {
        m[a] = (a < L.nrk && key[L.tog_off + a * row_tog + ri * L.p2 + j]) ? ~0u : 0u;
        any |= m[a];
      }
      if (!any) continue;
      const uint4 seed = *reinterpret_cast<const uint4*>(key + ri * 16ull * L.p2 + 16ull * j);
      uint4 o[1];
      aes_ctr_row<1, 4>(T, seed, o, __builtin_bswap32(bc));
      const uint8_t* cwp = key + L.cw_off + (uint64_t)j * L.mu + 16ull * bc;
      uint4 cw;
      if (cw_al) {
        cw = *reinterpret_cast<const uint4*>(cwp);
      } else {
        uint32_t w[4] = {0, 0, 0, 0};
        for (int k = 0; k < 16; ++k) w[k >> 2] |= (uint32_t)cwp[k] << (8 * (k & 3));
        cw = make_uint4(w[0], w[1], w[2], w[3]);
      }
      const uint4 v = xor4(o[0], cw);
#pragma unroll
      for (int a = 0; a < NRP; ++a) acc[a] = xor4(acc[a], and4(v, m[a]));
    }
  }
  for (int off = 1; off < lpi; off <<= 1) {  // the lpi lanes of a block are adjacent
#pragma unroll
    for (int a = 0; a < NRP; ++a) {
      acc[a].x ^= (uint32_t)__shfl_xor((int)acc[a].x, off, 64);
      acc[a].y ^= (uint32_t)__shfl_xor((int)acc[a].y, off, 64);
      acc[a].z ^= (uint32_t)__shfl_xor((int)acc[a].z, off, 64);
      acc[a].w ^= (uint32_t)__shfl_xor((int)acc[a].w, off, 64);
    }
  }
  if (act && sub == 0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
      for (int a = 0; a < NRP; ++a) {
        const uint32_t wd = (k >> 2) == 0 ? acc[a].x : (k >> 2) == 1 ? acc[a].y
                          : (k >> 2) == 2 ? acc[a].z : acc[a].w;
        w[a >> 2] |= ((wd >> (8 * (k & 3))) & 0xffu) << (8 * (a & 3));
      }
      store_leaf<NRP>(ring, (uint64_t)(16 * blk + k), make_uint4(w[0], w[1], w[2], w[3]));
    }
  }
}

template <int NQ, int NRP, int VEC, bool UNI, int TW, int TILE, int GYMAX, int RING,
          int NT = kFusedThreads, bool MPK = false>
__global__ __launch_bounds__(NT) void k_query(
    const uint8_t* __restrict__ raw0, uint32_t key_stride, int nk, int p, int n, int nq,
    int party0, int log_parts, uint64_t prefix, int lr, int lt, int ls,
    uint4* __restrict__ fr_s, uint32_t* __restrict__ fr_t, const uint8_t* __restrict__ shard,
    uint32_t pitch, uint32_t cpr, uint32_t gy, uint8_t* __restrict__ slabs,
    uint64_t* __restrict__ trace, uint8_t* __restrict__ out, uint32_t* __restrict__ qcnt,
    uint32_t efs, uint32_t red_mode, MpLayout mpl, StealArgs stl) {
  // MPK: the queue's keys are sqrt(N) DPF keys of layout mpl (key_stride bytes apart; multiparty
  // or covering design), and the tree waves build each tile's shares with mp_tile instead of a
  // DPF tree; the scan waves, slabs and reduce are the same
  // out != nullptr: the slabs of each query are reduced in-kernel into out (query k at
  // out + k * nq * efs); else the host launches k_reduce.  red_mode 1: the last workgroup to
  // add to qcnt[k] (zero on entry, left zero) XORs every slab.  Modes 2 and 3 (efs % 4 == 0,
  // out 4-byte aligned) XOR into answers the host zeroed (hipMemsetAsync on the launch's
  // stream) with memory-side atomics: 2 = every workgroup its own partial (no slab traffic, no
  // single-workgroup tail); 3 = per group of the workgroups b = x mod 8 (one XCD each under
  // round-robin dispatch), the last of the group to add to qcnt[8k + x] XORs the group's slabs
  // and adds that ONE partial (8 atomic adds per answer word instead of 2^lr).
  // trace != nullptr: per-workgroup wall-clock stamps (100 MHz) of query 0's phases,
  // kQueryTraceSlots apart (layout: pir_engine_trace_query, include/pir_engine.h)
  // diagnostics only: trace[kQueryTraceSlots * gridDim.x] bit 0 = scan waves skip their rows
  // (wrong answers; isolates the tree's rate beside the scan)
  const bool trace_flags_noscan = trace && (trace[(uint64_t)kQueryTraceSlots * gridDim.x] & 1u);
#if PIR_TRACE_TREE_TILES
  uint32_t tr_tile[2] = {0u, 0u};
  if (trace) {
    const uint64_t f = trace[(uint64_t)kQueryTraceSlots * gridDim.x];
    tr_tile[0] = (uint32_t)(f >> 8) & 0xffu;
    tr_tile[1] = (uint32_t)(f >> 16) & 0xffu;
  }
#endif
  if (trace) trace += (uint64_t)blockIdx.x * kQueryTraceSlots;
  if (trace && threadIdx.x == 0) { trace[0] = wall_clock64(); trace[56] = clock64(); }
  constexpr int NWV = NT / 64;  // waves per workgroup
  constexpr int SW = NWV - TW;
  constexpr int CH = VEC * 4;
  constexpr int GW = kColGroupLanes * VEC;
  constexpr int KT = TILE == 4096 ? 12 : (TILE == 1024 ? 10 : (TILE == 512 ? 9 : 8));  // log2 TILE
  static_assert((1 << KT) == TILE, "TILE: 256, 512, 1024 or 4096 leaves");
  using Smem = QuerySmem<TILE, NRP, NQ, VEC, GYMAX, RING>;
  static_assert(sizeof(Smem) <= 160 * 1024, "LDS");
  __shared__ Smem sm;
  const uint32_t pm1 = (uint32_t)p - 1;
  load_tables_n<NT>(sm.tab);
  for (int i = threadIdx.x; i < GYMAX * NQ * GW; i += blockDim.x) (&sm.red[0][0])[i] = 0;
  if constexpr (!MPK) stage_key(raw0, p, n, nq, threadIdx.x, NT, sm.scw, sm.tcw, sm.lastcw);
  if (threadIdx.x == 0) {
    sm.bar = 0; sm.sbar = 0; sm.ready = 0;
    for (int r = 0; r < RING; ++r) sm.consumed[r] = 0;
    for (int r = 0; r < 8; ++r) sm.prog[r] = 0;
  }
  // atomic_red: the answers were zeroed by a memset the host enqueued before this launch (on
  // the same stream), so no workgroup waits on another's progress
  const uint32_t tree_prio = (red_mode >> 8) & 3u;  // launch_query: $PIR_QUERY_TREE_PRIO
  const uint32_t scan_even = (red_mode >> 10) & 3u;  // launch_query: $PIR_QUERY_SCAN_EVEN
  const bool tree_rot = (red_mode >> 12) & 1u;       // launch_query: $PIR_QUERY_TREE_ROT
  red_mode &= 0xffu;
  const bool atomic_red = out && red_mode == 2;
  const uint32_t red_groups = red_mode == 3 ? 8u : 1u;  // slab groups of the last-add reduce
  __syncthreads();
  if (trace && threadIdx.x == 0) trace[1] = wall_clock64();

  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b = blockIdx.x;
  const uint32_t ntiles = 1u << lt;
  const uint32_t total = ntiles * (uint32_t)nk;  // tiles of the whole queue
  if (ls) {  // this workgroup's super-tile scratch (64 << ls nodes)
    fr_s += (size_t)b << (kQueryKin + ls);
    fr_t += (size_t)b << (kQueryKin + ls);
  }
  const uint64_t region_rows = (uint64_t)TILE << lt;
  // end-of-query work stealing (StealArgs, pir_kernels.h): a lone whole answer, 1-2 rounds,
  // records of one wave row
  constexpr bool kSteal = PIR_QUERY_STEAL && UNI && !MPK && NQ <= 2 && NWV - TW >= 8;
  const bool steal_on = kSteal && stl.buf && stl.gen && nk == 1 && gy == 1;
  // first row (in this engine's rows) of tile i of this workgroup
  auto tile_row0 = [&](uint32_t i) __attribute__((always_inline)) -> uint64_t {
    return (uint64_t)blockIdx.x * region_rows + (uint64_t)i * TILE;
  };
  const size_t slab_words = (size_t)NQ * GW;
  const size_t slab_q_words = (size_t)gy * gridDim.x * slab_words;  // one query's slabs

  // ================================ end-of-query work stealing ==============================
  // The lone query's last tile (every workgroup's) is split: its first kStealPre rows go to the
  // scan waves' static slots, the rest are chunks of kStealRows rows claimed one at a time
  // with an agent-scope atomic add on the owning workgroup's counter (StealArgs).  A claimed
  // chunk is folded by ONE wave into its own planes Zs (the chunk's rows x its shares): the
  // scan waves claim only their own workgroup's chunks (shares in the LDS ring); the tree
  // waves, idle once the last tile is built, claim their own and then, with `search`, those
  // of any workgroup that has published its last tile (shares from global memory) -- so the
  // workgroups that finish early fold the late ones' rows.  A wave leaves when no published
  // tile has chunks left and every tile is published (or the bounded wait ran out: a
  // workgroup not yet resident cannot publish; the late ones then fold their own chunks).
  // Each fold lands in the folding workgroup's slab; the answer is the XOR of all slabs.
  constexpr int kStealU = 8;                    // rows per batch (the scan waves' U)
  constexpr uint32_t kStealPre = kStealU * (NWV - TW);  // rows of the static prefix (gy == 1)
  constexpr uint32_t kStealRows = 32;
  constexpr uint32_t kStealChunks = TILE > kStealPre ? (TILE - kStealPre) / kStealRows : 0u;
  static_assert(!kSteal || (TILE - kStealPre) % kStealRows == 0, "whole chunks");
  constexpr uint64_t kStealWaitTicks = 6000;   // 60 us of the 100 MHz wall clock
  constexpr uint32_t kStealVictims = 16;       // neighbours a workgroup's tree waves help
  constexpr uint32_t kStealSearchWaves = 2;    // tree waves that help them (all fold own chunks)
  auto steal_chunks = [&](uint32_t (&Zs)[NQ][8][VEC], auto& xs, const uint8_t* own_ring,
                          bool search) __attribute__((always_inline)) {
    constexpr int SU = (int)(sizeof(xs) / sizeof(xs[0]));  // rows per batch
    static_assert(kStealRows % SU == 0 && SU <= kStealU, "batches of a chunk");
    const uint32_t G = gridDim.x, b32 = (uint32_t)b, C = kStealChunks;
    constexpr uint32_t CW = TILE * NRP / 4;  // share dwords of one tile
    const uint32_t xoff = lane < cpr ? lane * (uint32_t)CH : 0u;
    const uint64_t give_up = wall_clock64() + kStealWaitTicks;
    uint32_t v = b32, folded = 0;  // chunks folded: own in the low half, others' in the high
    for (;;) {
      uint32_t k = 0;
      if (lane == 0)
        k = __hip_atomic_fetch_add(stl.buf + 2 * v, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      k = (uint32_t)__builtin_amdgcn_readfirstlane((int)k);
      if (k >= C) {
        if (!search) break;
        // a neighbour with chunks left: workgroups b + 1 .. b + kStealVictims (mod G: every
        // XCD under round-robin dispatch), lane d - 1 checks b + d's flag (== gen: published)
        // and counter (< C: chunks left) -- two cache lines per probe, one probe per ~1 us
        // while a neighbour is unpublished (polling every workgroup's flags flooded the fabric
        // and slowed the late trees: profiles/r05/steal_trace_v1.txt)
        const uint32_t NV = G - 1 < kStealVictims ? G - 1 : kStealVictims;
        uint32_t nv = G;
        for (;;) {
          uint32_t cand = b32 + lane + 1;
          if (cand >= G) cand -= G;
          const bool live = lane < NV;
          uint32_t fl = 0, nx = C;
          if (live) {
            fl = __hip_atomic_load(stl.buf + 2 * cand + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            nx = __hip_atomic_load(stl.buf + 2 * cand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          const uint64_t am = __ballot(live && fl == stl.gen && nx < C);
          if (am) {  // the stealing waves of a workgroup start at different neighbours
            const uint64_t hi = am & (~0ull << ((wave * 5u) % NV));
            nv = (uint32_t)__builtin_amdgcn_readlane((int)cand, (int)__builtin_ctzll(hi ? hi : am));
            break;
          }
          if (!__ballot(live && fl != stl.gen) || wall_clock64() > give_up) break;
          __builtin_amdgcn_s_sleep(32);  // a neighbour's last tile is not published yet
        }
        if (nv >= G) break;
        // no acquire fence (an L2 invalidate at agent scope): the shares are read with
        // agent-scope loads issued after the flag's value came back
        v = nv;
        continue;
      }
      const bool own = v == b32;
      folded += own ? 1u : 0x10000u;
      const uint32_t r0 = kStealPre + k * kStealRows;  // rows of workgroup v's last tile
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(shard + ((uint64_t)v * region_rows + (uint64_t)(ntiles - 1) * TILE) * pitch),
          (short)0, (int)(TILE * pitch), kBufRsrcWord3);
      const uint32_t* cgl = stl.buf + 2 * (uint64_t)G + (uint64_t)v * CW;
#pragma unroll 1
      for (uint32_t u0 = 0; u0 < kStealRows; u0 += SU) {
#pragma unroll
        for (int u = 0; u < SU; ++u) xs[u] = load_chunk_buf<VEC>(rs, xoff, (r0 + u0 + u) * pitch);
        // lane u < SU reads row u's shares, v_readlane broadcasts them
        const uint32_t rr = r0 + u0 + (lane < (uint32_t)SU ? lane : 0u);
        uint32_t cw;
        if (own) {
          cw = load_coef<NRP>(own_ring, rr).x;
        } else {
          const uint32_t w = __hip_atomic_load(cgl + rr * NRP / 4, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
          cw = NRP == 1 ? (w >> (8 * (rr & 3u))) & 0xffu : (w >> (16 * (rr & 1u))) & 0xffffu;
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const uint32_t cu = (uint32_t)__builtin_amdgcn_readlane((int)cw, u);
#pragma unroll
          for (int a = 0; a < NQ; ++a) {
            const uint32_t ca = (cu >> (8 * a)) & 0xffu;
#pragma unroll
            for (int kk = 0; kk < 8; ++kk)
              if (ca & (1u << kk)) {
#pragma unroll
                for (int vv = 0; vv < VEC; ++vv) Zs[a][kk][vv] ^= xs[u].v[vv];
              }
          }
        }
      }
    }
    return folded;
  };
  // trace: chunk counts ([59] others' by the tree waves, [60] own by the tree waves, [61] own
  // by the scan waves) and the tree waves' last stealing stamp ([58])
  auto steal_trace = [&](uint32_t folded, bool tree) __attribute__((always_inline)) {
    if (trace && lane == 0) {
      if (tree) {
        __hip_atomic_fetch_add(trace + 59, (uint64_t)(folded >> 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(trace + 60, (uint64_t)(folded & 0xffffu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_max(trace + 58, wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        __hip_atomic_fetch_add(trace + 61, (uint64_t)(folded & 0xffffu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  };

  // ======================================= tree work =======================================
  // tree_tile(g, nt, team): the shares of queue tile g (query g / T, tile g % T) into ring slot
  // g % RING, by the first nt threads (team = their waves)
  const Tab T(sm.tab);
  const Bits B((uint32_t)p);
  const int tt = threadIdx.x;
  const uint32_t q = tt & 3u, role = (tt >> 2) & 3u;
  const uint32_t mq1 = q >= 1 ? 0xffffffffu : 0u, mq2 = q >= 2 ? 0xffffffffu : 0u;
  const uint32_t ptq = q == 3 ? (role << 24) : 0u;  // column shape: CTR block `role`
  const int Lr = log_parts + lr;  // region root level
  const int Lt = Lr + lt;         // tile root level
  const int L_leaf_parent = Lt + KT - 1;
  uint32_t gen = 0;
  uint4 qm;
  {
    uint32_t m[4];
    for (int w = 0; w < 4; ++w) {
      const int nb = nq - 4 * w;
      m[w] = nb >= 4 ? 0xffffffffu : (nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u));
    }
    qm = make_uint4(m[0], m[1], m[2], m[3]);
  }
  auto cw = [&](int L, uint32_t tv, uint4& cs, uint32_t& ct) {
    cw_lds(sm.scw, sm.tcw, L, tv, pm1, cs, ct);
  };
  auto tree_tile = [&](uint32_t g, int nt, uint32_t team) __attribute__((always_inline)) {
    const uint32_t i = g % ntiles;
    // levels narrower than the team run on its first waves; with tree_rot the team's waves take
    // turns tile by tile (whole-wave rotation: lane positions, and so q / role, are unchanged),
    // so that each SIMD's tree wave carries the same share and its scan waves the same slowdown
    const int tt = (tree_rot && team != (uint32_t)NWV)
                       ? (int)((threadIdx.x + 64u * (g % team)) % (uint32_t)nt) : (int)threadIdx.x;
#if PIR_TRACE_TREE_TILES
    uint64_t* tts = nullptr;  // this tile's stamp slots, if traced
    if (trace && tt == 0 && g && (g == tr_tile[0] || g == tr_tile[1])) tts = trace + 224 + (g == tr_tile[0] ? 0 : 16);
    if (tts) tts[0] = wall_clock64();
#define PIR_TTS(k) do { if (tts) tts[k] = wall_clock64(); } while (0)
#else
#define PIR_TTS(k) do {} while (0)
#endif
    const uint8_t* raw = raw0 + (size_t)(g / ntiles) * key_stride;
    uint8_t* ring = sm.ring[g % RING];
    // the whole workgroup: hardware barrier (waiting waves sleep); the tree waves alone: LDS
    // counter barrier (the scan waves keep streaming)
    auto sync = [&]() __attribute__((always_inline)) {
      if (team == (uint32_t)NWV) __syncthreads();
      else group_barrier(&sm.bar, gen, team);
    };
    if constexpr (MPK) {  // a sqrt(N) DPF key's shares instead of a DPF tree
      mp_tile<TILE, NRP>(T, raw, mpl, ((uint64_t)prefix << (n - log_parts)) + tile_row0(i), ring,
                         tt, nt);
      sync();  // every share of tile g is in the ring
      if (wave == 0) lds_signal(&sm.ready);
      return;
    }
    if (i == 0 && g > 0) {  // next query: its key replaces the previous one's (all tree waves
      stage_key(raw, p, n, nq, tt, nt, sm.scw, sm.tcw, sm.lastcw);  // are past its last use)
      sync();
    }
    // ---- breadth-first expansion of a subtree, relative levels m0 -> mlast ----------------
    // (level m of the span, width 2^m, lives in buffer a when (mlast - m) is even, else b, so
    // the span's last level ends in a; absolute level = Lspan + m)
    int tl = 0;  // levels expanded so far in this tile (trace)
    auto expand_span = [&](int Lspan, int m0, int mlast) __attribute__((always_inline)) {
      for (int m = m0; m < mlast; ++m) {
        const int W = 1 << m, L = Lspan + m;
        const bool inb = (mlast - m) & 1;
        const uint4* is = inb ? sm.sb : sm.sa;
        const uint32_t* it = inb ? sm.tb : sm.ta;
        uint4* os = inb ? sm.sa : sm.sb;
        uint32_t* ot = inb ? sm.ta : sm.tb;
        if (W * 16 <= nt) {  // column shape: 16 lanes per node
          const int u = tt >> 4;
          if (u < W) {  // uniform per 16-lane group
            const uint32_t s_in = reinterpret_cast<const uint32_t*>(&is[u])[q], t_in = it[u];
            uint4 cs;
            uint32_t ct;
            cw(L, t_in, cs, ct);
            const uint32_t o = aes_col(T, s_in, ptq, mq1, mq2);
            if (role < 2) {
              reinterpret_cast<uint32_t*>(&os[2 * u + role])[q] = o ^ word_of(cs, q);
            } else if (role == 2 && q == 0) {
              const uint32_t tb = (o & B.tb_mask) ^ ct;
              ot[2 * u] = tb & B.tmask;
              ot[2 * u + 1] = (tb >> B.pm1) & B.tmask;
            }
          }
        } else if (W <= (nt >> 6) * 21) {
          // 3 lanes per node, lane r runs CTR block r with its own key schedule: two thirds of
          // the row-shape latency for a level that fits the team in one pass
          const int l = tt & 63, ul = l / 3, r = l - 3 * ul;
          const int npp = (nt >> 6) * 21;
          for (int u = (tt >> 6) * 21 + ul; l < 63 && u < W; u += npp) {
            uint4 cs;
            uint32_t ct;
            cw(L, it[u], cs, ct);
            const uint4 o = aes_ctr_block(T, is[u], (uint32_t)r);
            if (r < 2) {
              os[2 * u + r] = xor4(o, cs);
            } else {
              const uint32_t tb = (o.x & B.tb_mask) ^ ct;
              ot[2 * u] = tb & B.tmask;
              ot[2 * u + 1] = (tb >> B.pm1) & B.tmask;
            }
          }
        } else if (kTreeIlp > 1 && W >= 2 * nt) {
          // row shape, two nodes per lane with their AES rounds interleaved: the tree waves
          // beside the scan are few, so one dependent AES chain per lane leaves the LDS idle
          // (the second node of a lane past W repeats the first and stores nothing)
          for (int u0 = tt; u0 < W; u0 += 2 * nt) {
            const bool ok1 = u0 + nt < W;
            const int uu[2] = {u0, ok1 ? u0 + nt : u0};
            uint4 cs[2], key[2];
            uint32_t ct[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              cw(L, it[uu[k]], cs[k], ct[k]);
              key[k] = is[uu[k]];
            }
            uint4 o[2][3];
            aes_ctr_rowk<2, 3, 1>(T, key, o);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              if (k == 1 && !ok1) break;
              const int u = uu[k];
              const uint32_t tb = (o[k][2].x & B.tb_mask) ^ ct[k];
              os[2 * u] = xor4(o[k][0], cs[k]);
              os[2 * u + 1] = xor4(o[k][1], cs[k]);
              ot[2 * u] = tb & B.tmask;
              ot[2 * u + 1] = (tb >> B.pm1) & B.tmask;
            }
          }
        } else {  // row shape: one lane per node, 3 CTR blocks on one key schedule
          for (int u = tt; u < W; u += nt) {
            uint4 cs;
            uint32_t ct;
            cw(L, it[u], cs, ct);
            uint4 o[3];
            aes_ctr_row<3, 1>(T, is[u], o);
            const uint32_t tb = (o[2].x & B.tb_mask) ^ ct;
            os[2 * u] = xor4(o[0], cs);
            os[2 * u + 1] = xor4(o[1], cs);
            ot[2 * u] = tb & B.tmask;
            ot[2 * u + 1] = (tb >> B.pm1) & B.tmask;
          }
        }
        sync();
        if (trace && g == 0 && tt == 0 && tl < 16) trace[40 + tl] = wall_clock64();
        if (trace && g == 1 && tt == 0 && tl < 16) trace[160 + tl] = wall_clock64();
        ++tl;
        if (tl < 12) PIR_TTS(1 + tl);
      }
    };
    // ---- super-tile root (wave 0, column shape, depth-first) ------------------------------
    // Super-tile j = i >> ls (2^ls tiles, root at level Ls) is expanded once down to the 64
    // input nodes of each of its tiles; j == 0 descends all Ls levels from the root along
    // (prefix, b, 0); j > 0 pops the right sibling stored when its ancestor was expanded and
    // descends ctz(j) levels, so the super-tile roots cost (#super-tiles - 1) expansions.
    const uint32_t smask = (1u << ls) - 1u;
    const int Ls = Lt - ls;
    const int span_last = ls ? ls + kQueryKin : KT - 1;  // relative last level of the root span
    if ((i & smask) == 0) {
      const uint32_t j = i >> ls;
      if (wave == 0) {
        int L0, depth;
        uint32_t sq, t;
        uint64_t path;  // bits of the levels still to descend (MSB first)
        if (j == 0) {
          L0 = 0;
          depth = Ls;
          sq = load_le32(raw + 4 * q);
          t = party0 >= 1 ? (1u << (party0 - 1)) : 0u;  // dpf_tree.cpp:496-502
          path = (((prefix << lr) | b) << (lt - ls));
        } else {
          const int c = __builtin_ctz(j);
          L0 = Ls - c;  // the right sibling popped at level L0, then c left turns
          depth = c;
          sq = reinterpret_cast<const uint32_t*>(&sm.stk_s[L0])[q];
          t = sm.stk_t[L0];
          path = 0;
        }
        // the 4 groups of 16 lanes compute the same node; the path bit is wave-uniform, so the
        // chosen child moves to every lane through SGPRs (v_readlane), not through the LDS
        const uint32_t m0 = q == 0 ? ~0u : 0u, m1 = q == 1 ? ~0u : 0u;
        const uint32_t m2 = q == 2 ? ~0u : 0u, m3 = q == 3 ? ~0u : 0u;
        for (int d = 0; d < depth; ++d) {
          const int L = L0 + d;
          // word q of the correction word (t is wave-uniform here); issued before the rounds
          uint32_t csq = 0, ct = 0;
          for (uint32_t jj = 0; jj < pm1; ++jj) {
            const uint32_t m = 0u - ((t >> jj) & 1u);
            csq ^= reinterpret_cast<const uint32_t*>(&sm.scw[L * (int)pm1 + (int)jj])[q] & m;
            ct ^= sm.tcw[L * (int)pm1 + (int)jj] & m;
          }
          const uint32_t o = aes_col(T, sq, ptq, mq1, mq2);
          const uint32_t bit = (uint32_t)((path >> (depth - 1 - d)) & 1u);
          const uint32_t oc = o ^ csq;
          const uint32_t tbits = (__builtin_amdgcn_readlane(o, 8) & B.tb_mask) ^
                                 __builtin_amdgcn_readfirstlane(ct);
          if (L >= Lr && bit == 0) {  // inside the region: keep the right child for later
            if (lane >= 4 && lane < 8) reinterpret_cast<uint32_t*>(&sm.stk_s[L + 1])[lane - 4] = oc;
            if (lane == 0) sm.stk_t[L + 1] = (tbits >> pm1) & B.tmask;
          }
          const uint32_t c0 = __builtin_amdgcn_readlane(oc, (int)(4 * bit + 0));
          const uint32_t c1 = __builtin_amdgcn_readlane(oc, (int)(4 * bit + 1));
          const uint32_t c2 = __builtin_amdgcn_readlane(oc, (int)(4 * bit + 2));
          const uint32_t c3 = __builtin_amdgcn_readlane(oc, (int)(4 * bit + 3));
          sq = (c0 & m0) | (c1 & m1) | (c2 & m2) | (c3 & m3);
          t = (tbits >> (bit * pm1)) & B.tmask;
          if (trace && g == 0 && lane == 0 && d < 32) trace[8 + d] = wall_clock64();
        }
        uint4* s0 = (span_last & 1) ? sm.sb : sm.sa;
        uint32_t* t0 = (span_last & 1) ? sm.tb : sm.ta;
        if (lane < 4) reinterpret_cast<uint32_t*>(&s0[0])[lane] = sq;
        if (lane == 0) t0[0] = t;
        if (trace && g == 0 && lane == 0) { trace[2] = wall_clock64(); trace[57] = clock64(); }
      }
      sync();
      if (trace && g == 1 && tt == 0) trace[176] = wall_clock64();
      if (ls) {  // the super-tile's top: 2^ls x 64 tile inputs, once, to the scratch
        expand_span(Ls, 0, span_last);
        const int nf = 64 << ls;
        for (int u = tt; u < nf; u += nt) {
          fr_s[u] = sm.sa[u];
          fr_t[u] = sm.ta[u];
        }
        sync();
      }
    }
    if (ls) {  // this tile's 64 input nodes (relative level kQueryKin) from the scratch
      const bool inb = (KT - 1 - kQueryKin) & 1;
      uint4* s0 = inb ? sm.sb : sm.sa;
      uint32_t* t0 = inb ? sm.tb : sm.ta;
      const int base = (int)(i & smask) * 64;
      for (int u = tt; u < 64; u += nt) {
        s0[u] = fr_s[base + u];
        t0[u] = fr_t[base + u];
      }
      sync();
      PIR_TTS(1);
      expand_span(Lt, kQueryKin, KT - 1);
    } else {
      expand_span(Lt, 0, KT - 1);
    }
    const int buf = 0;            // the leaf parents (relative level KT - 1) are in buffer a
    const int W = 1 << (KT - 1);  // ... TILE / 2 of them
    // ---- last level + leaf conversion (dpf_tree.cpp:567-580) into the ring -----------------
    // c[leaf][a] = AES_{s_leaf}(0)[a] ^ XOR_{k: t_leaf bit k} lastCW[k][a]   (a < nq)
    {
      const uint4* is = buf ? sm.sb : sm.sa;
      const uint32_t* it = buf ? sm.tb : sm.ta;
      if (team == (uint32_t)NWV && !(kTreeIlp > 1 && W <= 2 * nt)) {
        // 3 lanes per parent; the child lanes convert (with kTreeIlp > 1 only for levels wider
        // than two parents per lane: a narrower last level takes the row shape below, one or
        // two parents per lane with their leaves' AES interleaved)
        const int l = tt & 63, ul = l / 3, r = l - 3 * ul;
        const int npp = (nt >> 6) * 21;
        const int u0 = (tt >> 6) * 21 + ul;
        const int src = (l < 63 ? l - r + 2 : l);  // the node's control-bit lane
        for (int ub = 0; ub < W; ub += npp) {  // uniform trip count: every lane joins the shuffle
          const int u = u0 + ub;
          const bool act = l < 63 && u < W;
          uint4 cs = make_uint4(0, 0, 0, 0);
          uint32_t ct = 0;
          uint4 o = make_uint4(0, 0, 0, 0);
          if (act) {
            cw(L_leaf_parent, it[u], cs, ct);
            o = aes_ctr_block(T, is[u], (uint32_t)r);
          }
          const uint32_t tb = (uint32_t)__shfl((int)((o.x & B.tb_mask) ^ ct), src, 64);
          if (act && r < 2) {
            const uint32_t tc = (tb >> (r * pm1)) & B.tmask;
            uint4 v = aes_ctr_block(T, xor4(o, cs), 0u);
            for (uint32_t j = 0; j < pm1; ++j) v = xor4(v, and4(sm.lastcw[j], 0u - ((tc >> j) & 1u)));
            store_leaf<NRP>(ring, 2 * u + r, make_uint4(v.x & qm.x, v.y & qm.y, v.z & qm.z, v.w & qm.w));
          }
        }
      } else if (kTreeIlp > 1 && W >= 2 * nt) {
        // two parents per lane, their AES rounds interleaved, then their four leaf blocks
        constexpr int NW = NRP <= 4 ? 1 : NRP / 4;
        for (int u0 = tt; u0 < W; u0 += 2 * nt) {
          const bool ok1 = u0 + nt < W;
          const int uu[2] = {u0, ok1 ? u0 + nt : u0};
          uint4 cs[2], key[2];
          uint32_t ct[2];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            cw(L_leaf_parent, it[uu[k]], cs[k], ct[k]);
            key[k] = is[uu[k]];
          }
          uint4 o[2][3];
          aes_ctr_rowk<2, 3, 1>(T, key, o);
          uint4 lk[4];
          uint32_t tc[4];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const uint32_t tb = (o[k][2].x & B.tb_mask) ^ ct[k];
            tc[2 * k] = tb & B.tmask;
            tc[2 * k + 1] = (tb >> B.pm1) & B.tmask;
            lk[2 * k] = xor4(o[k][0], cs[k]);
            lk[2 * k + 1] = xor4(o[k][1], cs[k]);
          }
          uint4 v[4][1];
          aes_ctr_rowk<4, 1, NW, (NRP < 4 ? NRP : 0)>(T, lk, v);
#pragma unroll
          for (int c = 0; c < 4; ++c)
            for (uint32_t j = 0; j < pm1; ++j)
              v[c][0] = xor4(v[c][0], and4(sm.lastcw[j], 0u - ((tc[c] >> j) & 1u)));
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            if (k == 1 && !ok1) break;
            const int u = uu[k];
            const uint4 a = make_uint4(v[2 * k][0].x & qm.x, v[2 * k][0].y & qm.y,
                                       v[2 * k][0].z & qm.z, v[2 * k][0].w & qm.w);
            const uint4 c = make_uint4(v[2 * k + 1][0].x & qm.x, v[2 * k + 1][0].y & qm.y,
                                       v[2 * k + 1][0].z & qm.z, v[2 * k + 1][0].w & qm.w);
            if constexpr (NRP == 1) {
              *reinterpret_cast<uint16_t*>(ring + 2 * u) = (uint16_t)((a.x & 0xffu) | ((c.x & 0xffu) << 8));
            } else {
              store_leaf<NRP>(ring, 2 * u, a);
              store_leaf<NRP>(ring, 2 * u + 1, c);
            }
          }
        }
      } else {
        constexpr int NW = NRP <= 4 ? 1 : NRP / 4;
        for (int u = tt; u < W; u += nt) {
          uint4 cs;
          uint32_t ct;
          cw(L_leaf_parent, it[u], cs, ct);
          uint4 o[3];
          aes_ctr_row<3, 1>(T, is[u], o);
          const uint32_t tb = (o[2].x & B.tb_mask) ^ ct;
          const uint32_t tl = tb & B.tmask, tr = (tb >> B.pm1) & B.tmask;
          uint4 vl[1], vr[1];
          if constexpr (kTreeIlp > 1) {  // the two leaf blocks' rounds interleaved
            const uint4 lk[2] = {xor4(o[0], cs), xor4(o[1], cs)};
            uint4 v2[2][1];
            aes_ctr_rowk<2, 1, NW, (NRP < 4 ? NRP : 0)>(T, lk, v2);
            vl[0] = v2[0][0];
            vr[0] = v2[1][0];
          } else {
            aes_ctr_row<1, NW, (NRP < 4 ? NRP : 0)>(T, xor4(o[0], cs), vl);
            aes_ctr_row<1, NW, (NRP < 4 ? NRP : 0)>(T, xor4(o[1], cs), vr);
          }
          for (uint32_t j = 0; j < pm1; ++j) {
            vl[0] = xor4(vl[0], and4(sm.lastcw[j], 0u - ((tl >> j) & 1u)));
            vr[0] = xor4(vr[0], and4(sm.lastcw[j], 0u - ((tr >> j) & 1u)));
          }
          const uint4 a = make_uint4(vl[0].x & qm.x, vl[0].y & qm.y, vl[0].z & qm.z, vl[0].w & qm.w);
          const uint4 c = make_uint4(vr[0].x & qm.x, vr[0].y & qm.y, vr[0].z & qm.z, vr[0].w & qm.w);
          if constexpr (NRP == 1) {
            *reinterpret_cast<uint16_t*>(ring + 2 * u) = (uint16_t)((a.x & 0xffu) | ((c.x & 0xffu) << 8));
          } else {
            store_leaf<NRP>(ring, 2 * u, a);
            store_leaf<NRP>(ring, 2 * u + 1, c);
          }
        }
      }
    }
    PIR_TTS(14);
    sync();  // every share of tile g is in the ring
#undef PIR_TTS
    if constexpr (kSteal) {
      if (steal_on && g + 1 == total) {
        // the last tile's shares and the chunk counter reset as agent-scope (write-through)
        // stores, each thread's complete (vmcnt 0) before the barrier, then the generation
        // published: other workgroups may now claim chunks of this tile (the reset is also
        // ordered before this workgroup's own claims by the ready signal below).  No release
        // FENCE: at agent scope that is an L2 writeback, and 32 of them per XCD (every
        // workgroup's last tile) stalled the XCD's L2 for ~100 us (profiles/r05/steal_trace_v2.txt)
        constexpr uint32_t CW = TILE * NRP / 4;
        uint32_t* hdr = stl.buf + 2 * b;
        uint32_t* cg = stl.buf + 2 * (uint64_t)gridDim.x + b * CW;
        const uint32_t* r32 = reinterpret_cast<const uint32_t*>(ring);
        for (int w = tt; w < (int)CW; w += nt)
          __hip_atomic_store(cg + w, r32[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (tt == 0) __hip_atomic_store(hdr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (also a compiler barrier)
        sync();
        if (tt == 0) __hip_atomic_store(hdr + 1, stl.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (wave == 0) lds_signal(&sm.ready);
    if (trace && tt == 0 && (g == 0 || g == ntiles - 1)) trace[g == 0 ? 3 : 4] = wall_clock64();
    if (trace && tt == 0 && g < 32) { trace[64 + g] = wall_clock64(); trace[128 + g] = clock64(); }
  };

  tree_tile(0, NT, NWV);  // every wave builds the first tile
  if (wave < (uint32_t)TW) {
    // ===================================== tree role ======================================
    if (tree_prio == 3) __builtin_amdgcn_s_setprio(3);
    else if (tree_prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (tree_prio == 1) __builtin_amdgcn_s_setprio(1);
    for (uint32_t g = 1; g < total; ++g) {
      // slot g % RING free: every scan wave has consumed tile g - RING (per-slot counts)
#if PIR_TRACE_TREE_TILES
      if (trace && tt == 0 && (g == tr_tile[0] || g == tr_tile[1])) trace[224 + (g == tr_tile[0] ? 0 : 16) + 15] = wall_clock64();
#endif
      if (g >= (uint32_t)RING) lds_wait_geq_idle(&sm.consumed[g % RING], (g / RING) * SW);
      tree_tile(g, TW * 64, TW);
    }
    if constexpr (kSteal) {
      if (steal_on) {  // chunks of the last tiles, then the planes into red[] (ready += 1)
        uint32_t Zt[NQ][8][VEC];
#pragma unroll
        for (int a = 0; a < NQ; ++a)
#pragma unroll
          for (int kk = 0; kk < 8; ++kk)
#pragma unroll
            for (int vv = 0; vv < VEC; ++vv) Zt[a][kk][vv] = 0;
        Chunk<VEC> xt[NQ == 1 ? kStealU : kStealU / 2];  // (two rounds: 64 plane VGPRs)
        if (stl.mode & 1u)
          steal_trace(steal_chunks(Zt, xt, sm.ring[(total - 1) % RING],
                                   (stl.mode & 2u) && wave < kStealSearchWaves), true);
        if (lane < cpr) {
#pragma unroll
          for (int a = 0; a < NQ; ++a)
#pragma unroll
            for (int vv = 0; vv < VEC; ++vv) {
              uint32_t acc = Zt[a][7][vv];
#pragma unroll
              for (int kk = 6; kk >= 0; --kk) acc = gf_xtime4(acc) ^ Zt[a][kk][vv];
              if (acc) atomicXor(&sm.red[0][a * GW + lane * VEC + vv], acc);
            }
        }
        lds_signal(&sm.ready);  // the scan waves reduce red[] once every tree wave is in
      }
    }
  } else {
    // ===================================== scan role ======================================
    const uint32_t sw = wave - TW;
    uint32_t sgen = 0;  // scan-wave barrier generation
    uint32_t gcol, wi, nwg, rpw, rec_off, chunk;
    bool active;
    if (UNI) {
      gcol = sw % gy;
      wi = sw / gy;
      nwg = SW / gy;
      rpw = 1; rec_off = 0;
      chunk = gcol * kColGroupLanes + lane;
      active = chunk < cpr && wi < nwg;
    } else {
      gcol = 0; wi = sw; nwg = SW;
      rpw = kColGroupLanes / cpr;
      rec_off = lane / cpr;
      chunk = lane - rec_off * cpr;
      active = lane < rpw * cpr;
    }
    uint32_t Z[NQ][8][VEC];
#pragma unroll
    for (int a = 0; a < NQ; ++a)
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
#pragma unroll
        for (int v = 0; v < VEC; ++v) Z[a][kk][v] = 0;
    const uint32_t ngroups = (TILE + rpw - 1) / rpw;
    // many rounds, wave-uniform coefficients, 2 dwords per lane: scalar branches on the
    // coefficient bits (avg 4 two-VGPR v_xor per dword and round) up to PIR_QUERY_BRANCH_MAXNQ
    // rounds, else masks from the plane table (8 v_bitop3 with an SGPR mask, 2/3 the issue rate)
    // 768-thread workgroups (4 to 5 rounds): four Russians over groups of 4 rows (pir_m4r.h:
    // 2.5x fewer VALU ops than the masks, 32 more VGPRs -- which 16 waves per CU do not have)
    constexpr bool kM4R = UNI && VEC == 2 && NQ >= 3 && NQ <= 5 && NT == kM4rThreads;
    constexpr bool kPlaneAsm = !kM4R && UNI && VEC == 2 && NQ >= 3 && NQ > PIR_QUERY_BRANCH_MAXNQ;
    // rows in flight per lane (one record per wave row: a rolling pipeline whose x[] stays live
    // across tiles; several records per row: U rows loaded, then folded, per batch)
    constexpr int U = (kPlaneAsm || kM4R) ? PIR_PLANE_U : (SW >= 8 ? 8 : 16);
    static_assert(!kM4R || U % 4 == 0, "four Russians: groups of 4 rows");
    // row slot j of a tile = row group wi + j * nwg; rpt slots per tile, a multiple of U (slots
    // past the tile's row groups are masked)
    const uint32_t rpt = ((ngroups + nwg - 1) / nwg + U - 1) / U * U;
    constexpr bool kM4RExact = kM4R && SW == 8 && TILE == 1024 && 128 % U == 0;
    // the tile's packed indices one group per lane: 8 scan waves, 2 column groups -> 4 row
    // waves x 64 groups of 4 rows = the 1024 rows of a tile
    constexpr bool kM4RLane = kM4RExact && PIR_M4R_TILEIDX && NQ <= 5;
    const bool lane_tile = kM4RLane && rpt <= 256;  // records of 512 B and 1 KiB (gy <= 2)
    const bool scan = wi < nwg && !(trace && trace_flags_noscan);
    __builtin_amdgcn_s_setprio(PIR_SCAN_PRIO);
    const uint8_t* rbase = shard + (uint64_t)chunk * CH;  // + tile_row0(i) rows
    // Rolling load pipeline: x[u] holds slot j0 + u; once it is folded, slot j0 + U + u is loaded
    // into it -- at the end of a tile, from the next tile (of this or the next query).  Shard rows
    // do not depend on the tree, so U rows per lane stay in flight across tiles and queries; only
    // the coefficients wait for the tree.
    Chunk<VEC> x[UNI ? U : 1];
    // Unconditional loads (straight-line code keeps each refill behind its fold): a slot with
    // no row reads the shard's first bytes instead, and its coefficient is 0 (or, past the last
    // tile, it is never folded; inactive lanes' planes are never written out).
    // one record per wave row: buffer loads over the tile's rows (resource in SGPRs, num_records
    // 0 past the queue's last tile), the row's byte offset in soffset (wave-uniform), the lane's
    // chunk offset in voffset (lanes past the record read its first chunk) -- no per-lane 64-bit
    // address arithmetic, exec masking or branch per row.  TILE * pitch < 2^31 (make_query_plan).

    const uint32_t lane_off = chunk < cpr ? chunk * CH : 0u;
    const uint32_t tile_bytes = (uint32_t)TILE * pitch;
    // the buffer resource of tile g's rows (num_records 0 past the queue's last tile)
    auto tile_rsrc = [&](uint32_t g) __attribute__((always_inline)) {
      return __builtin_amdgcn_make_buffer_rsrc(
          (void*)(shard + tile_row0(g & (ntiles - 1)) * pitch), (short)0,
          g < total ? (int)tile_bytes : 0, kBufRsrcWord3);
    };
    auto load_slot = [&](uint32_t g, uint32_t j, Chunk<VEC>& dst) __attribute__((always_inline)) {
      const uint32_t gi = wi + j * nwg;
      if constexpr (UNI) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(shard + tile_row0(g & (ntiles - 1)) * pitch), (short)0,
            g < total ? (int)tile_bytes : 0, kBufRsrcWord3);
        // four-Russians scan waves at 8 per workgroup: nwg = 8 / gy divides 8, so with TILE =
        // 1024 rows and U | 128 every slot holds a row -- no guard, two SALU fewer per row
        dst = load_chunk_buf<VEC>(rs, lane_off, (kM4RExact || gi < ngroups) ? gi * pitch : 0u);
      } else {
        const uint32_t rl = gi * rpw + rec_off;
        const bool ok = g < total && active && gi < ngroups && rl < TILE;
        dst = load_chunk<VEC>(ok ? rbase + (tile_row0(g & (ntiles - 1)) + rl) * pitch : shard);
      }
    };
    auto fold_row = [&](const Chunk<VEC>& xr, const uint4& c4) __attribute__((always_inline)) {
#pragma unroll
      for (int a = 0; a < NQ; ++a) {
        const uint32_t ca = coef_byte(c4, a);
        if (UNI && NQ <= (PIR_QUERY_BRANCH_MAXNQ > 2 ? PIR_QUERY_BRANCH_MAXNQ : 2)) {  // scalar branches: ~4 XORs per dword instead of 8 masked
#pragma unroll
          for (int kk = 0; kk < 8; ++kk)
            if (ca & (1u << kk)) {
#pragma unroll
              for (int v = 0; v < VEC; ++v) Z[a][kk][v] ^= xr.v[v];
            }
        } else if (UNI) {  // many rounds, 1 dword per lane: branch-free, SGPR masks
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) {
            const uint32_t m = 0u - ((ca >> kk) & 1u);
#pragma unroll
            for (int v = 0; v < VEC; ++v) Z[a][kk][v] = mxor(Z[a][kk][v], xr.v[v], m);
          }
        } else {
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) {
            const uint32_t m = 0u - ((ca >> kk) & 1u);
#pragma unroll
            for (int v = 0; v < VEC; ++v) Z[a][kk][v] = mxor(Z[a][kk][v], xr.v[v], m);
          }
        }
      }
    };
    if constexpr (UNI) {
      if (scan) {
#pragma unroll
        for (int u = 0; u < U; ++u) load_slot(0, u, x[u]);
      }
    }
#if PIR_FOLD_STAMPS
    uint32_t fs[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // per-phase cycles of this wave (fold_stamp)
    uint64_t fs_t = fold_stamp();
#define PIR_FS(k)                                          \
  do {                                                     \
    if constexpr (kM4R) {                                  \
      const uint64_t t_ = fold_stamp();                    \
      fs[k] += (uint32_t)(t_ - fs_t);                      \
      fs_t = t_;                                           \
    }                                                      \
  } while (0)
#else
#define PIR_FS(k) do {} while (0)
#endif
    for (uint32_t g = 0; g < total; ++g) {
      const uint32_t i = g % ntiles;
      const uint8_t* ring = sm.ring[g % RING];
      PIR_FS(6);  // the previous tile's bookkeeping, end-of-query fold and slab
      // Equal-priority waves issue oldest first, so of a SIMD's two scan waves the older one
      // runs ahead and the younger one falls tiles behind -- and the slowest scan wave holds
      // the ring slot the tree needs next.  A wave that starts tile g while another scan wave
      // has not finished tile g - 1 drops one priority level for this tile.
      if (scan_even == 1 && g > 0) {
        if (lds_load(&sm.consumed[(g - 1) % RING]) < ((g - 1) / RING + 1) * SW)
          __builtin_amdgcn_s_setprio(PIR_SCAN_PRIO - 1);
        else
          __builtin_amdgcn_s_setprio(PIR_SCAN_PRIO);
      } else if (scan_even == 2 && g > 0 && SW >= 2 && SW <= 8) {
        // the other scan wave on this wave's SIMD (waves are dealt to SIMDs round robin)
        if (lds_load(&sm.prog[sw ^ (uint32_t)(SW / 2)]) < g)
          __builtin_amdgcn_s_setprio(PIR_SCAN_PRIO - 1);
        else
          __builtin_amdgcn_s_setprio(PIR_SCAN_PRIO);
      }
      lds_wait_geq(&sm.ready, g + 1);
      PIR_FS(0);  // waiting for the tree (tile g's shares)
      if (!UNI && scan) {  // per-lane coefficients: batches of U rows of this tile
        const uint8_t* base = rbase + tile_row0(i) * pitch;
        for (uint32_t g0 = wi; g0 < ngroups; g0 += U * nwg) {
          Chunk<VEC> xb[U];
          uint4 cb[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const uint32_t gi = g0 + u * nwg, rl = gi * rpw + rec_off;
            const bool ok = active && gi < ngroups && rl < TILE;
            if (ok) xb[u] = load_chunk<VEC>(base + (uint64_t)rl * pitch);
            else
              for (int v = 0; v < VEC; ++v) xb[u].v[v] = 0;
            cb[u] = ok ? load_coef<NRP>(ring, rl) : make_uint4(0, 0, 0, 0);
          }
#pragma unroll
          for (int u = 0; u < U; ++u) fold_row(xb[u], cb[u]);
        }
      }
      if (UNI && scan) {
        if constexpr (kM4RLane) if (lane_tile) {
          // four Russians, per tile: lane l builds the packed indices of the wave's group l
          // (slots 4l .. 4l + 3: rows wi + (4l + r) nwg of the tile; rpt / 4 <= 64 groups)
          uint2 cr[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t j = 4u * lane + (uint32_t)r;
            const uint4 c = load_coef<NRP>(ring, j < rpt ? wi + j * nwg : 0u);
            cr[r] = make_uint2(c.x, c.y);
          }
          uint32_t P[NQ];
          m4r_tile_index<NQ>(cr, P);
          PIR_FS(5);  // the tile's packed indices (one group per lane)
          // the refills read this tile's rows, then (the last batch) the next tile's: both
          // buffer resources once per tile, row offsets as running sums (no per-load address
          // arithmetic beyond one s_add)
          const uint32_t rstep = nwg * pitch;
          auto batch = [&](uint32_t j0, __amdgpu_buffer_rsrc_t rs, uint32_t soff)
              __attribute__((always_inline)) {
#pragma unroll
            for (int g4 = 0; g4 < U; g4 += 4) {
              uint32_t pk[NQ];
#pragma unroll
              for (int a = 0; a < NQ; ++a)
                pk[a] = (uint32_t)__builtin_amdgcn_readlane((int)P[a], (int)((j0 + g4) >> 2));
#if PIR_FOLD_STAMPS
              PIR_FS(1);
              asm volatile("" ::"v"(x[g4].v[0]), "v"(x[g4].v[1]), "v"(x[g4 + 1].v[0]),
                           "v"(x[g4 + 1].v[1]), "v"(x[g4 + 2].v[0]), "v"(x[g4 + 2].v[1]),
                           "v"(x[g4 + 3].v[0]), "v"(x[g4 + 3].v[1]));
              PIR_FS(2);
              ++fs[7];
#endif
              m4r_fold4s<VEC, NQ>(Z, x[g4].v, x[g4 + 1].v, x[g4 + 2].v, x[g4 + 3].v, pk);
              PIR_FS(3);
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                x[g4 + r] = load_chunk_buf<VEC>(rs, lane_off, soff);
                soff += rstep;
              }
              PIR_FS(4);
              __builtin_amdgcn_sched_barrier(0);
            }
          };
          const __amdgpu_buffer_rsrc_t rs_here = tile_rsrc(g), rs_next = tile_rsrc(g + 1);
          const uint32_t row_off = wi * pitch;  // slot j at row_off + j * rstep
          for (uint32_t j0 = 0; j0 + U < rpt; j0 += U) batch(j0, rs_here, row_off + (j0 + U) * rstep);
          batch(rpt - U, rs_next, row_off);  // refills from the next tile (of this or the next query)
        }
        // the lone query's last tile with stealing: only the first U slots statically (they were
        // loaded at the end of the previous tile), the rest in claimed chunks (steal_tail)
        const bool dyn = kSteal && steal_on && g + 1 == total;
        const uint32_t rpt_g = dyn ? (uint32_t)U : rpt;
        for (uint32_t j0 = 0; j0 < (lane_tile ? 0u : rpt_g); j0 += U) {
          // wave-uniform coefficients: lane u reads row u's (one LDS read), v_readlane broadcasts
          uint4 cf[U];
          const uint32_t gl = wi + (j0 + (lane < (uint32_t)U ? lane : 0u)) * nwg;
          uint4 c4 = load_coef<NRP>(ring, gl < ngroups ? gl : 0u);
          if (gl >= ngroups) c4 = make_uint4(0, 0, 0, 0);
          const bool last = j0 + U == rpt_g;
          const uint32_t gn = last ? g + 1 : g, jn = last ? 0u : j0 + U;
          if constexpr (kM4R) {
#pragma unroll
            for (int g4 = 0; g4 < U; g4 += 4) {
              const uint32_t vi = m4r_index(coef_word(c4, g4), coef_word(c4, g4 + 1),
                                            coef_word(c4, g4 + 2), coef_word(c4, g4 + 3));
#if PIR_FOLD_STAMPS
              const uint32_t vp = m4r_pack(vi, (lane & 7u) * 4u);
              PIR_FS(1);  // coefficient words (the ring read at g4 = 0), index, pack
              asm volatile("" ::"v"(x[g4].v[0]), "v"(x[g4].v[1]), "v"(x[g4 + 1].v[0]),
                           "v"(x[g4 + 1].v[1]), "v"(x[g4 + 2].v[0]), "v"(x[g4 + 2].v[1]),
                           "v"(x[g4 + 3].v[0]), "v"(x[g4 + 3].v[1]));
              PIR_FS(2);  // the group's rows (s_waitcnt vmcnt)
              m4r_fold4p<VEC, NQ>(Z, x[g4].v, x[g4 + 1].v, x[g4 + 2].v, x[g4 + 3].v, vp);
              PIR_FS(3);  // combinations + 40 indexed planes
              ++fs[7];
#else
              m4r_fold_group<VEC, NQ>(Z, x[g4].v, x[g4 + 1].v, x[g4 + 2].v, x[g4 + 3].v, vi,
                                      (lane & 7u) * 4u);
#endif
#pragma unroll
              for (int r = 0; r < 4; ++r) load_slot(gn, jn + g4 + r, x[g4 + r]);
              PIR_FS(4);  // the 4 refill loads
              __builtin_amdgcn_sched_barrier(0);
            }
            continue;
          }
          u32x8 mrow;  // kPlaneAsm: masks of the next row's round 0, in flight
          if constexpr (kPlaneAsm) mrow = plane_masks_issue(__builtin_amdgcn_readlane(c4.x, 0) & 0xffu);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            cf[u] = make_uint4(__builtin_amdgcn_readlane(c4.x, u),
                               NRP > 4 ? __builtin_amdgcn_readlane(c4.y, u) : 0u,
                               NRP > 8 ? __builtin_amdgcn_readlane(c4.z, u) : 0u,
                               NRP > 8 ? __builtin_amdgcn_readlane(c4.w, u) : 0u);
            if constexpr (kPlaneAsm) {
              u32x8 m = mrow;
#pragma unroll
              for (int a = 0; a < NQ; ++a) {
                auto& Za = reinterpret_cast<uint32_t(&)[8][2]>(Z[a]);
                if (a + 1 < NQ)
                  m = planes_fold2_next(Za, x[u].v[0], x[u].v[VEC - 1], m, coef_byte(cf[u], a + 1));
                else if (u + 1 < U)
                  mrow = planes_fold2_next(Za, x[u].v[0], x[u].v[VEC - 1], m,
                                           __builtin_amdgcn_readlane(c4.x, u + 1) & 0xffu);
                else
                  planes_fold2(Za, x[u].v[0], x[u].v[VEC - 1], m);
              }
            } else {
              fold_row(x[u], cf[u]);
            }
            load_slot(gn, jn + u, x[u]);
            // keep the refill behind its fold: x[u]'s registers are reused (no second buffer),
            // and the wait before the next fold is vmcnt(U - 1), not a drain
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        if constexpr (kSteal) {
          static_assert(!kSteal || U == kStealU, "the scan waves' batch");
          if (dyn) steal_trace(steal_chunks(Z, x, ring, false), false);  // x: holds nothing now
        }
      }
      lds_signal(&sm.consumed[g % RING]);
      if (scan_even == 2 && lane == 0 && sw < 8) __hip_atomic_store(&sm.prog[sw], g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#if PIR_TRACE_TREE_TILES
      // every scan wave's consumed stamp of the two traced tiles (slots 208 + 8 t + sw)
      if (trace && lane == 0 && (g == tr_tile[0] || g == tr_tile[1])) trace[208 + (g == tr_tile[0] ? 0 : 8) + sw] = wall_clock64();
#endif
      if (trace && sw == 0 && lane == 0 && g < 32) trace[96 + g] = wall_clock64();
      if (i == ntiles - 1) {  // end of a query: sum_k alpha^k Z_k into LDS, then the slab
        const uint32_t qy = g / ntiles;
        if (trace && qy == 0 && sw == 0 && lane == 0) trace[5] = wall_clock64();
        if (active) {
          const uint32_t wbase = (UNI ? lane : chunk) * VEC;
#pragma unroll
          for (int a = 0; a < NQ; ++a)
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
              uint32_t acc = Z[a][7][v];
#pragma unroll
              for (int kk = 6; kk >= 0; --kk) acc = gf_xtime4(acc) ^ Z[a][kk][v];
              if (acc) atomicXor(&sm.red[gcol][a * GW + wbase + v], acc);
            }
        }
#pragma unroll
        for (int a = 0; a < NQ; ++a)
#pragma unroll
          for (int kk = 0; kk < 8; ++kk)
#pragma unroll
            for (int v = 0; v < VEC; ++v) Z[a][kk][v] = 0;
        if constexpr (kSteal) {
          if (steal_on) lds_wait_geq(&sm.ready, total + (uint32_t)TW);  // the tree waves' chunks
        }
        group_barrier(&sm.sbar, sgen, SW);  // every scan wave's planes are in red[]
        uint32_t* qslab = reinterpret_cast<uint32_t*>(slabs) + qy * slab_q_words;
        const int st = (int)threadIdx.x - TW * 64;
        if (atomic_red) {
          // the workgroup's partial answer straight into the zeroed out (memory-side atomics)
          uint32_t* o32 = reinterpret_cast<uint32_t*>(out + (size_t)qy * NQ * efs);
          const uint32_t wpr = efs / 4;  // answer words per round
          for (uint32_t gg = 0; gg < gy; ++gg)
            for (int k = st; k < (int)slab_words; k += SW * 64) {
              const uint32_t a = (uint32_t)k / GW, w = gg * GW + (uint32_t)k % GW;
              const uint32_t v = sm.red[gg][k];
              sm.red[gg][k] = 0;
              if (v && w < wpr) atomicXor(o32 + a * wpr + w, v);
            }
          group_barrier(&sm.sbar, sgen, SW);  // red[] is clear for the next query
          if (trace && qy == 0 && sw == 0 && lane == 0) trace[6] = wall_clock64();
          continue;
        }
        for (uint32_t gg = 0; gg < gy; ++gg) {
          uint32_t* slab = qslab + ((uint64_t)gg * gridDim.x + blockIdx.x) * slab_words;
          for (int k = st; k < (int)slab_words; k += SW * 64) {
            if (out)  // read back by another workgroup below: stored past this XCD's L2 (sc1)
              __hip_atomic_store(&slab[k], sm.red[gg][k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
              slab[k] = sm.red[gg][k];
            sm.red[gg][k] = 0;
          }
        }
        if (out) {
          // Fused reduce (no k_reduce launch): every scan wave's sc1 slab stores complete
          // (vmcnt(0)) before the workgroup's ONE agent-scope counter add (one lane, after the
          // scan waves' barrier); the workgroup whose add comes last XORs the slabs of every
          // workgroup with sc1 loads, issued after that add returned (the other scan waves: after
          // the barrier that follows its LDS word) -- the fence-free hand-off of
          // MI355X_MICROARCH.md's sc1 table (agent-scope atomic add row).  Round 5 dropped the
          // release / acquire fences this hand-off does not need: each was an XCD-wide L2
          // write-back or invalidate, 256 of them at the kernel's tail.
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          group_barrier(&sm.sbar, sgen, SW);
          const uint32_t gx = gridDim.x, xg = (uint32_t)b % red_groups;  // this slab group
          uint32_t* const cnt = qcnt + (size_t)qy * red_groups + xg;
          if (st == 0)
            sm.lastq = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) == gx / red_groups - 1;
          group_barrier(&sm.sbar, sgen, SW);
          if (lds_load(&sm.lastq)) {
            const uint32_t words = pitch / 4, P = (uint32_t)NQ * words, nth = SW * 64;
            const uint32_t S = P >= nth ? 1u : nth / P;  // threads per output word
            for (uint32_t idx = (uint32_t)st; idx < P * S; idx += nth) {
              const uint32_t pw = idx % P, part = idx / P;
              const uint32_t a = pw / words, w = pw - a * words;
              const uint32_t grp = w / GW, win = w - grp * GW;
              const uint32_t* src = qslab + (uint64_t)grp * gx * slab_words + a * GW + win;
              uint32_t acc = 0;
              for (uint32_t x = xg + part * red_groups; x < gx; x += S * red_groups)
                acc ^= __hip_atomic_load(src + (uint64_t)x * slab_words, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
              if (acc) atomicXor(&sm.red[grp][a * GW + win], acc);
            }
            group_barrier(&sm.sbar, sgen, SW);
            uint8_t* qout = out + (size_t)qy * NQ * efs;
            for (uint32_t pw = (uint32_t)st; pw < P; pw += nth) {  // pitch -> record bytes
              const uint32_t a = pw / words, w = pw - a * words;
              const uint32_t grp = w / GW, win = w - grp * GW;
              const uint32_t v = sm.red[grp][a * GW + win];
              sm.red[grp][a * GW + win] = 0;
              if (red_groups > 1) {  // one of the groups' partials: add it to the zeroed answer
                if (v && 4 * w < efs) atomicXor(reinterpret_cast<uint32_t*>(qout + (size_t)a * efs) + w, v);
              } else {
                for (uint32_t t = 0; t < 4; ++t)
                  if (4 * w + t < efs) qout[(size_t)a * efs + 4 * w + t] = (uint8_t)(v >> (8 * t));
              }
            }
            if (st == 0)  // ready for the next launch that answers a query in this slot
              __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
        group_barrier(&sm.sbar, sgen, SW);  // red[] is clear for the next query
        if (trace && qy == 0 && sw == 0 && lane == 0) trace[6] = wall_clock64();
      }
    }
#if PIR_FOLD_STAMPS
    PIR_FS(6);
    if constexpr (kM4R) {
      static_assert(kFoldStampBase + 64 <= kQueryTraceSlots, "fold stamps: trace slots");
      if (trace && lane == 0 && sw < 8)  // the first 8 scan waves
        for (int k = 0; k < 8; ++k) trace[kFoldStampBase + 8 * sw + k] = fs[k];
    }
#endif
#undef PIR_FS
  }
}

// ---- fused leaf stage + scan -----------------------------------------------------------------
constexpr int kFusedTW = 8;       // tree waves per workgroup (the other 8 scan)
constexpr int kQueryTreeHeavyTW = 12;  // k_query for small records: 12 tree + 4 scan waves
constexpr int kLoneTile = 1024;        // leaves per tile of a lone query (nk == 1) of large records
constexpr int kFusedTileIn = 64;  // tree nodes entering a tile

template <int NQ, int TILE>
hipError_t query_nq(const QueryPlan& qp, const uint8_t* d_raw, uint32_t key_stride, int nk,
                           int p, int n, int party0, int log_parts, uint64_t prefix,
                           const uint8_t* shard, uint8_t* slabs, uint8_t* scratch, hipStream_t s,
                           uint64_t* trace, uint8_t* out, uint32_t* qcnt, uint32_t efs,
                           uint32_t red_mode, StealArgs stl) {
  uint4* fr_s = reinterpret_cast<uint4*>(scratch);
  uint32_t* fr_t = reinterpret_cast<uint32_t*>(scratch + ((size_t)qp.shape.grid.x << (kQueryKin + qp.ls)) * sizeof(uint4));
  constexpr int NRP = NQ == 1 ? 1 : (NQ == 2 ? 2 : (NQ <= 4 ? 4 : 8));
  constexpr int VEC = NQ <= 2 ? 4 : 2;
  constexpr int RING = TILE == 4096 ? 2 : 4;  // share slots: the tree runs RING-1 tiles ahead
  const ScanShape& sh = qp.shape;
#define PIR_QLN(UNI, TW, GY, gy, NTH)                                                            \
  hipLaunchKernelGGL((k_query<NQ, NRP, VEC, UNI, TW, TILE, GY, RING, NTH>), dim3(sh.grid.x),     \
                     dim3(NTH), 0, s, d_raw, key_stride, nk, p, n, NQ, party0,                    \
                     log_parts, prefix, qp.lr, qp.lt, qp.ls, fr_s, fr_t, shard, sh.pitch, sh.cpr,  \
                     gy, slabs, trace, out, qcnt, efs, red_mode, MpLayout{}, stl)
#define PIR_QL(UNI, TW, GY, gy) PIR_QLN(UNI, TW, GY, gy, kFusedThreads)
  if constexpr (VEC == 2 && NQ >= 3 && NQ <= 5 && NQ > PIR_QUERY_BRANCH_MAXNQ && TILE == 1024) {
    if (sh.uniform && qp.m4r) {  // four-Russians scan waves (k_query's kM4R)
      if (qp.m4r == 2) PIR_QLN(true, 2, 4, sh.grid.y, kM4rThreads);  // diagnostics: 2 tree waves
      else PIR_QLN(true, kM4rTW, 4, sh.grid.y, kM4rThreads);
      return hipGetLastError();
    }
  }
  if constexpr (NQ <= 2) {
    if (qp.tw == kQueryTreeHeavyTW) {  // small records: the tree is the bottleneck
      if (sh.uniform) PIR_QL(true, kQueryTreeHeavyTW, 4, sh.grid.y);
      else PIR_QL(false, kQueryTreeHeavyTW, 1, 1u);
      return hipGetLastError();
    }
  }
  if (sh.uniform) PIR_QL(true, kFusedTW, 4, sh.grid.y);
  else PIR_QL(false, kFusedTW, 1, 1u);
#undef PIR_QL
#undef PIR_QLN
  return hipGetLastError();
}

// k_query in its sqrt(N) DPF mode (MPK): mp_tile builds each tile's shares from the key
template <int NQ, int TILE>
hipError_t query_nq_mp(const QueryPlan& qp, const uint8_t* d_key, uint32_t key_stride,
                              int nk, const MpLayout& L, int n, int log_parts, uint64_t prefix,
                              const uint8_t* shard, uint8_t* slabs, hipStream_t s) {
  constexpr int NRP = NQ == 1 ? 1 : (NQ == 2 ? 2 : (NQ <= 4 ? 4 : 8));
  constexpr int VEC = NQ <= 2 ? 4 : 2;
  constexpr int RING = TILE == 4096 ? 2 : 4;
  const ScanShape& sh = qp.shape;
  if (!sh.uniform) return hipErrorInvalidValue;
  // tree-wave priority as launch_query (a lone query's share waves at 3)
  const char* tp = getenv("PIR_QUERY_TREE_PRIO");
  uint32_t rm = ((tp ? (uint32_t)atoi(tp) : (nk == 1 ? 3u : 0u)) & 3u) << 8;
  {  // the four-Russians shape's 8 scan waves: evened and rotated as in launch_query
    const char* se = getenv("PIR_QUERY_SCAN_EVEN");
    rm |= ((se ? (uint32_t)atoi(se) : (qp.m4r ? 2u : 0u)) & 3u) << 10;
    const char* tr = getenv("PIR_QUERY_TREE_ROT");
    if (tr ? atoi(tr) != 0 : qp.m4r) rm |= 1u << 12;
  }
  // mp_tile gives each of its threads at most ONE 16-record CTR block of the tile (no loop
  // over blocks): the share waves (TW * 64 threads; tile 0: all NTH) must cover TILE / 16 blocks
#define PIR_QMP(TW, NTH)                                                                         \
  static_assert((TW) * 64 >= TILE / 16, "mp_tile: one thread per CTR block of the tile");      \
  hipLaunchKernelGGL((k_query<NQ, NRP, VEC, true, TW, TILE, 4, RING, NTH, true>),               \
                     dim3(sh.grid.x), dim3(NTH), 0, s, d_key, key_stride, nk, 2, n, NQ, 0,       \
                     log_parts, prefix, qp.lr, qp.lt, 0, nullptr, nullptr, shard, sh.pitch,      \
                     sh.cpr, sh.grid.y, slabs, nullptr, nullptr, nullptr, 0u, rm, L, StealArgs{})
  if constexpr (VEC == 2 && NQ >= 3 && NQ <= 5 && NQ > PIR_QUERY_BRANCH_MAXNQ && TILE == 1024) {
    if (qp.m4r) {
      PIR_QMP(kM4rTW, kM4rThreads);
      return hipGetLastError();
    }
  }
  // 1-2 shares: few seeds per row (p2 <= 8) build a tile's shares in a fraction of the scan's
  // time, so 4 share waves + 12 scan waves ($PIR_MP_TW=8: the tree DPF's 8 + 8)
  if constexpr (NQ <= 2) {
    const char* tv = getenv("PIR_MP_TW");
    if (L.p2 <= 8 && !(tv && atoi(tv) == 8)) {
      PIR_QMP(4, kFusedThreads);
      return hipGetLastError();
    }
  }
  PIR_QMP(kFusedTW, kFusedThreads);
#undef PIR_QMP
  return hipGetLastError();
}

// ---- where the k_query instantiations are compiled ---------------------------------------
// Every (rounds, tile) instance of query_nq / query_nq_mp (each a few k_query kernels) is
// compiled in one of kQueryParts objects: this file built again with -DPIR_QUERY_PART=k (the
// Makefile's pir_query_k.o), which keeps only the templates and the instances of part k, so the
// parts compile in parallel.  The main object declares them extern.
#define PIR_QNQ_ARGS                                                                            \
  (const QueryPlan&, const uint8_t*, uint32_t, int, int, int, int, int, uint64_t, const uint8_t*, \
   uint8_t*, uint8_t*, hipStream_t, uint64_t*, uint8_t*, uint32_t*, uint32_t, uint32_t, StealArgs)
#define PIR_QMP_ARGS                                                                            \
  (const QueryPlan&, const uint8_t*, uint32_t, int, const MpLayout&, int, int, uint64_t,         \
   const uint8_t*, uint8_t*, hipStream_t)
// X(function, rounds, tile, part)
#define PIR_QUERY_INSTANCES(X)                                                                   \
  X(query_nq, 5, 1024, 0) X(query_nq, 4, 1024, 1) X(query_nq, 3, 1024, 2)                        \
  X(query_nq, 1, 4096, 3) X(query_nq, 2, 4096, 3) X(query_nq, 1, 1024, 4) X(query_nq, 2, 1024, 4) \
  X(query_nq, 1, 512, 5) X(query_nq, 2, 512, 5) X(query_nq, 1, 256, 5) X(query_nq, 2, 256, 5)     \
  X(query_nq, 6, 1024, 6) X(query_nq, 7, 1024, 6) X(query_nq, 8, 1024, 6)                        \
  X(query_nq_mp, 1, 4096, 7) X(query_nq_mp, 2, 4096, 7) X(query_nq_mp, 1, 1024, 7)               \
  X(query_nq_mp, 2, 1024, 7) X(query_nq_mp, 3, 1024, 2) X(query_nq_mp, 4, 1024, 1)              \
  X(query_nq_mp, 5, 1024, 0)
constexpr int kQueryParts = 8;
#define PIR_ARGS_query_nq PIR_QNQ_ARGS
#define PIR_ARGS_query_nq_mp PIR_QMP_ARGS
#ifdef PIR_QUERY_PART
static_assert(PIR_QUERY_PART >= 0 && PIR_QUERY_PART < kQueryParts, "PIR_QUERY_PART");
#define PIR_QI(F, NQ, TL, PART) \
  PIR_QI_##PART(template hipError_t F<NQ, TL> PIR_ARGS_##F;)
#else
#define PIR_QI(F, NQ, TL, PART) extern template hipError_t F<NQ, TL> PIR_ARGS_##F;
#endif
#if defined(PIR_QUERY_PART) && PIR_QUERY_PART == 0
#define PIR_QI_0(...) __VA_ARGS__
#else
#define PIR_QI_0(...)
#endif
#if defined(PIR_QUERY_PART) && PIR_QUERY_PART == 1
#define PIR_QI_1(...) __VA_ARGS__
#else
#define PIR_QI_1(...)
#endif
#if defined(PIR_QUERY_PART) && PIR_QUERY_PART == 2
#define PIR_QI_2(...) __VA_ARGS__
#else
#define PIR_QI_2(...)
#endif
#if defined(PIR_QUERY_PART) && PIR_QUERY_PART == 3
#define PIR_QI_3(...) __VA_ARGS__
#else
#define PIR_QI_3(...)
#endif
#if defined(PIR_QUERY_PART) && PIR_QUERY_PART == 4
#define PIR_QI_4(...) __VA_ARGS__
#else
#define PIR_QI_4(...)
#endif
#if defined(PIR_QUERY_PART) && PIR_QUERY_PART == 5
#define PIR_QI_5(...) __VA_ARGS__
#else
#define PIR_QI_5(...)
#endif
#if defined(PIR_QUERY_PART) && PIR_QUERY_PART == 6
#define PIR_QI_6(...) __VA_ARGS__
#else
#define PIR_QI_6(...)
#endif
#if defined(PIR_QUERY_PART) && PIR_QUERY_PART == 7
#define PIR_QI_7(...) __VA_ARGS__
#else
#define PIR_QI_7(...)
#endif
PIR_QUERY_INSTANCES(PIR_QI)
#undef PIR_QI

#ifndef PIR_QUERY_PART  // the rest: the main object only
// slabs: [grid.y][gx_all][nq][GW words]; out[a*efs + b] for b < efs.
// One 1024-thread block per 64 output words: 16 lane groups split the gx slabs, then LDS.
// blockIdx.y = query of a queue: slabs q_words apart, answers gridDim.z*nq*efs bytes apart.
// blockIdx.z = slice: the slabs [z*gx, (z+1)*gx) of gx_all = gridDim.z*gx (k_query's workgroup
// b owns rows [b*R, (b+1)*R), so slice z of gridDim.z is the partial answer over the rows
// [z*N/Z, (z+1)*N/Z) -- runOptimizedDPFTreeQueryThread's slice, server.cpp:519-541),
// answer (y, z) at out + (y*gridDim.z + z)*nq*efs.
__global__ __launch_bounds__(kReduceThreads) void k_reduce(const uint32_t* __restrict__ slabs,
                                                           int nq, uint32_t gw, uint32_t gx,
                                                           uint32_t pitch, uint32_t efs,
                                                           uint8_t* __restrict__ out,
                                                           uint64_t q_words) {
  const uint32_t gx_all = gx * gridDim.z;
  slabs += blockIdx.y * q_words + (uint64_t)blockIdx.z * gx * nq * gw;
  out += ((uint64_t)blockIdx.y * gridDim.z + blockIdx.z) * nq * efs;
  __shared__ uint32_t part[kReduceThreads / 64][64];
  const uint32_t words = pitch / 4;
  const uint32_t lane = threadIdx.x & 63, grp16 = threadIdx.x >> 6, ngrp = blockDim.x >> 6;
  const uint32_t idx = blockIdx.x * 64 + lane;
  uint32_t acc = 0;
  if (idx < (uint32_t)nq * words) {
    const uint32_t a = idx / words, w = idx - a * words;
    const uint32_t grp = w / gw, win = w - grp * gw;
    const uint32_t* p = slabs + ((uint64_t)grp * gx_all) * nq * gw + (uint64_t)a * gw + win;
    const uint64_t stride = (uint64_t)nq * gw;
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    uint32_t x = grp16;
    for (; x + 3 * ngrp < gx; x += 4 * ngrp) {
      a0 ^= p[x * stride];
      a1 ^= p[(x + ngrp) * stride];
      a2 ^= p[(x + 2 * ngrp) * stride];
      a3 ^= p[(x + 3 * ngrp) * stride];
    }
    for (; x < gx; x += ngrp) a0 ^= p[x * stride];
    acc = a0 ^ a1 ^ a2 ^ a3;
  }
  part[grp16][lane] = acc;
  __syncthreads();
  if (grp16 != 0 || idx >= (uint32_t)nq * words) return;
  for (uint32_t gi = 1; gi < ngrp; ++gi) acc ^= part[gi][lane];
  const uint32_t a = idx / words, w = idx - a * words;
  const uint32_t b0 = 4 * w;
  uint8_t* dst = out + (uint64_t)a * efs;
  if ((efs & 3u) == 0 && b0 + 4 <= efs) {
    *reinterpret_cast<uint32_t*>(dst + b0) = acc;
  } else {
    for (uint32_t k = 0; k < 4; ++k)
      if (b0 + k < efs) dst[b0 + k] = (uint8_t)(acc >> (8 * k));
  }
}

__global__ void k_xor_fold(const uint8_t* __restrict__ in, int nranks, size_t len,
                           uint8_t* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < len;
       i += (size_t)gridDim.x * blockDim.x) {
    uint8_t acc = 0;
    for (int r = 0; r < nranks; ++r) acc ^= in[(size_t)r * len + i];
    out[i] = acc;
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_fill_random(uint8_t* __restrict__ d, size_t bytes, uint64_t seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < bytes;
       i += (size_t)gridDim.x * blockDim.x)
    d[i] = (uint8_t)splitmix64(seed ^ (i * 0xD1B54A32D192ED03ull));
}

// byte b of global row i = byte (b & 7) of splitmix64(seed ^ (i << 20 | b >> 3)); padding 0
__global__ void k_fill_shard(uint8_t* __restrict__ shard, uint64_t rows, uint32_t pitch,
                             uint32_t efs, uint64_t row0, uint64_t seed) {
  const uint32_t cpr = pitch / 16;
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < rows * cpr;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = idx / cpr;
    const uint32_t ch = (uint32_t)(idx - r * cpr);
    const uint64_t gr = row0 + r;
    uint32_t w[4];
    for (int h = 0; h < 2; ++h) {
      const uint32_t b = ch * 16 + h * 8;
      const uint64_t z = splitmix64(seed ^ ((gr << 20) | (b >> 3)));
      w[2 * h] = (uint32_t)z;
      w[2 * h + 1] = (uint32_t)(z >> 32);
    }
    for (int k = 0; k < 16; ++k) {
      const uint32_t b = ch * 16 + k;
      if (b >= efs) w[k >> 2] &= ~(0xffu << (8 * (k & 3)));
    }
    *reinterpret_cast<uint4*>(shard + r * pitch + ch * 16) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// ------------------------------------------------------------------------------------------
// k_encode_across: the server's erasure-coded shard (client.cpp:70-97, every row of
// generate_encoded_across_file): row r of party q = XOR_{j<k, src = encdb*j + r < nfiles}
// gf_pow(q, j) * file[src] over GF(2^8)/0x11d.  One lane per 16-byte chunk of a row; the k
// coefficients are wave-uniform (scalar branches over their bits, x * alpha^b by xtime).
// files == nullptr: the reference's synthetic database (client.cpp:16-33): file v holds the
// byte (v & 0xff) in every position, file 1 holds 0, 1, 2, ....
// ------------------------------------------------------------------------------------------
struct EncodeCoefs {
  uint8_t c[16];
};

__device__ __forceinline__ uint4 gf_mul_const4(uint4 x, uint32_t c) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int b = 0; b < 8; ++b) {
    if (c & (1u << b)) acc = xor4(acc, x);
    x = make_uint4(gf_xtime4(x.x), gf_xtime4(x.y), gf_xtime4(x.z), gf_xtime4(x.w));
  }
  return acc;
}

__device__ __forceinline__ uint32_t synth_word(uint64_t v, uint32_t b0) {  // bytes b0..b0+3
  if (v == 1) {
    uint32_t w = 0;
    for (int t = 0; t < 4; ++t) w |= ((b0 + t) & 0xffu) << (8 * t);
    return w;
  }
  return (uint32_t)(v & 0xff) * 0x01010101u;
}

__global__ void k_encode_across(const uint8_t* __restrict__ files, uint64_t fpitch,
                                uint64_t nfiles, uint64_t encdb, int k, EncodeCoefs co,
                                uint8_t* __restrict__ shard, uint64_t rows, uint64_t row0,
                                uint32_t pitch, uint32_t efs) {
  const uint32_t cpr = pitch / 16;
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < rows * cpr;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = idx / cpr;
    const uint32_t ch = (uint32_t)(idx - r * cpr);
    const uint64_t gr = row0 + r;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int j = 0; j < k; ++j) {
      const uint64_t src = encdb * (uint64_t)j + gr;
      if (src >= nfiles) continue;
      uint4 x;
      if (files && (fpitch & 15u) == 0 && ch * 16u + 16u <= efs) {  // aligned whole chunk
        x = *reinterpret_cast<const uint4*>(files + src * fpitch + ch * 16u);
      } else if (files) {
        uint32_t w[4];
        const uint8_t* f = files + src * fpitch + ch * 16u;
        for (int t = 0; t < 4; ++t) {
          uint32_t v = 0;
          for (int u = 0; u < 4; ++u) {
            const uint32_t bi = ch * 16u + 4u * t + u;
            if (bi < efs) v |= (uint32_t)f[4 * t + u] << (8 * u);
          }
          w[t] = v;
        }
        x = make_uint4(w[0], w[1], w[2], w[3]);
      } else {
        x = make_uint4(synth_word(src, ch * 16u), synth_word(src, ch * 16u + 4),
                       synth_word(src, ch * 16u + 8), synth_word(src, ch * 16u + 12));
      }
      acc = xor4(acc, gf_mul_const4(x, co.c[j]));
    }
    uint32_t w[4] = {acc.x, acc.y, acc.z, acc.w};
    for (int t = 0; t < 16; ++t)
      if (ch * 16u + t >= efs) w[t >> 2] &= ~(0xffu << (8 * (t & 3)));  // zero pad bytes
    *reinterpret_cast<uint4*>(shard + r * pitch + ch * 16u) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// ------------------------------------------------------------------------------------------
// host side: tables, plans, launchers
// ------------------------------------------------------------------------------------------
TreePlan make_plan(int n, int log_parts, uint64_t prefix, int k_last, int p, int max_front) {
  TreePlan pl{};
  pl.p = p;
  pl.n = n;
  pl.log_parts = log_parts;
  pl.prefix = prefix;
  const int nr = n - log_parts;  // depth of this partition's subtree
  pl.nleaves = 1ull << nr;
  // frontier (latency-bound, column-shape AES) down to F, row-shape stages of <= 4 levels,
  // and a last stage of k_last levels that converts the leaves (k_expand<FINAL> or k_fused)
  if (k_last < 0) k_last = 4;
  k_last = std::min(k_last, nr);
  const int L_last = nr - k_last;
  int F = std::min(16, L_last);
  if (max_front < 16 && leaf_dfs_enabled())
    F = L_last <= max_front ? L_last : max_front + (L_last - max_front) % 4;
  pl.F = F;
  pl.g = std::min(F, 8);
  pl.e = F - pl.g;
  pl.nfront = 1ull << F;
  int rem = L_last - F, L = log_parts + F;
  uint64_t nin = pl.nfront;
  int ks[8], ns = 0;
  while (rem > 0) {
    const int k = rem % 4 ? rem % 4 : 4;  // remainder first, then full 4-level stages
    ks[ns++] = k;
    rem -= k;
  }
  ks[ns++] = k_last;
  uint64_t maxnodes = pl.nfront;
  for (int i = 0; i < ns; ++i) {
    Stage& st = pl.st[i];
    st.L_in = L;
    st.k = ks[i];
    st.nin = nin;
    // <= 4096 outputs per workgroup, but >= 256 workgroups when the level is wide enough
    uint64_t tl = std::min<uint64_t>(nin, (uint64_t)(kExpOut >> std::min(st.k, 12)));
    while (tl > 64 && nin / tl < 256) tl >>= 1;
    st.tile = (int)tl;
    st.final = i == ns - 1;
    L += st.k;
    nin <<= st.k;
    if (!st.final) maxnodes = std::max(maxnodes, nin);
  }
  pl.nstages = ns;
  pl.max_nodes = maxnodes;
  return pl;
}

int fused_tile(int nq, uint32_t pitch, uint64_t nleaves, int num_cus) {
  if (nq > 8) return 0;
  const int vec = nq <= 2 ? 4 : 2;
  const uint32_t cpr = pitch / (vec * 4);
  const uint32_t gy = (cpr + kColGroupLanes - 1) / kColGroupLanes;
  if (gy > 4) return 0;  // > 4 column groups: more than the scan waves can split
  // >= 4 tiles per CU so the tree runs under the scan; 4096-leaf tiles only for nrp <= 2
  if (nq <= 2 && nleaves >= (uint64_t)4096 * num_cus * 4) return 4096;
  if (nleaves >= (uint64_t)1024 * num_cus * 2) return 1024;
  return 0;
}

template <int NQ, int TILE>
static hipError_t fused_nq(const TreePlan& pl, const DevKey* d_key, const NodeBufs& nb,
                           const uint8_t* shard, const ScanShape& sh, uint8_t* slabs, int buf,
                           hipStream_t s) {
  constexpr int NRP = NQ == 1 ? 1 : (NQ == 2 ? 2 : (NQ <= 4 ? 4 : 8));
  constexpr int VEC = NQ <= 2 ? 4 : 2;
  const Stage& st = pl.st[pl.nstages - 1];
  const uint64_t ntiles = pl.nleaves / TILE;
  if (sh.uniform)
    hipLaunchKernelGGL((k_fused<NQ, NRP, VEC, true, kFusedTW, TILE, 4>), dim3(sh.grid.x),
                       dim3(kFusedThreads), 0, s, d_key, nb.s[buf], nb.t[buf], st.L_in, st.k,
                       ntiles, shard, sh.pitch, sh.cpr, sh.grid.y, slabs);
  else  // several records per wave row: per-lane coefficients
    hipLaunchKernelGGL((k_fused<NQ, NRP, VEC, false, kFusedTW, TILE, 1>), dim3(sh.grid.x),
                       dim3(kFusedThreads), 0, s, d_key, nb.s[buf], nb.t[buf], st.L_in, st.k,
                       ntiles, shard, sh.pitch, sh.cpr, 1u, slabs);
  return hipGetLastError();
}

ScanShape make_fused_shape(uint64_t nleaves, uint32_t pitch, int nq, int num_cus, int tile) {
  ScanShape sh{};
  sh.nq = nq;
  sh.nrp = nq == 1 ? 1 : (nq == 2 ? 2 : (nq <= 4 ? 4 : 8));
  sh.vec = nq <= 2 ? 4 : 2;
  sh.pitch = pitch;
  sh.cpr = pitch / (sh.vec * 4);
  sh.uniform = sh.cpr >= (uint32_t)kColGroupLanes;
  const uint32_t gy = sh.uniform ? (sh.cpr + kColGroupLanes - 1) / kColGroupLanes : 1;
  const uint64_t ntiles = nleaves / tile;
  sh.grid = dim3((unsigned)std::min<uint64_t>(ntiles, (uint64_t)num_cus), gy);
  sh.slab_bytes = (uint32_t)(nq * kColGroupLanes * sh.vec * 4);
  return sh;
}

hipError_t launch_fused(const TreePlan& pl, const DevKey* d_key, const NodeBufs& nb,
                        const uint8_t* shard, const ScanShape& sh, uint8_t* slabs, int tile,
                        hipStream_t s) {
  const int buf = (pl.nstages - 1) & 1;  // node buffer holding the last stage's input
  if (tile == 4096) {
    switch (sh.nq) {
      case 1: return fused_nq<1, 4096>(pl, d_key, nb, shard, sh, slabs, buf, s);
      case 2: return fused_nq<2, 4096>(pl, d_key, nb, shard, sh, slabs, buf, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (tile != 1024) return hipErrorInvalidValue;
  switch (sh.nq) {
    case 1: return fused_nq<1, 1024>(pl, d_key, nb, shard, sh, slabs, buf, s);
    case 2: return fused_nq<2, 1024>(pl, d_key, nb, shard, sh, slabs, buf, s);
    case 3: return fused_nq<3, 1024>(pl, d_key, nb, shard, sh, slabs, buf, s);
    case 4: return fused_nq<4, 1024>(pl, d_key, nb, shard, sh, slabs, buf, s);
    case 5: return fused_nq<5, 1024>(pl, d_key, nb, shard, sh, slabs, buf, s);
    case 6: return fused_nq<6, 1024>(pl, d_key, nb, shard, sh, slabs, buf, s);
    case 7: return fused_nq<7, 1024>(pl, d_key, nb, shard, sh, slabs, buf, s);
    case 8: return fused_nq<8, 1024>(pl, d_key, nb, shard, sh, slabs, buf, s);
    default: return hipErrorInvalidValue;
  }
}

int fused_k(int tile) { return tile == 4096 ? 6 : (tile == 1024 ? 4 : 0); }

// ---- single-launch query ---------------------------------------------------------------------
QueryPlan make_query_plan(int n, int log_parts, int p, int nq, uint32_t pitch, int num_cus,
                          int nk) {
  QueryPlan qp{};
  const int nr = n - log_parts;
  if (nr < 0 || (uint64_t)n * (uint64_t)(p - 1) > (uint64_t)kQueryCwCap) return qp;
  const uint64_t nleaves = 1ull << nr;
  int tile = fused_tile(nq, pitch, nleaves, num_cus);
  if (!tile) return qp;
  // a queue: 4096-leaf tiles whenever each workgroup gets at least one -- the tree of the next
  // tile is built during the scan of the previous one, and wide tiles spend a smaller share of
  // their tree in latency-bound narrow levels (a lone query keeps 1024: shorter first tile)
  if (nk > 1 && nq <= 2 && nleaves >= (uint64_t)4096 * 256) tile = 4096;
  if (const char* tq = getenv("PIR_QUERY_TILEQ")) {  // diagnostics: a queue's tile size
    const int t = atoi(tq);
    if (nk > 1 && (t == 1024 || (t == 4096 && nq <= 2 && nleaves >= (uint64_t)4096 * 256))) tile = t;
  }
  // a lone query of large records waits for its first tile before any row is scanned: smaller
  // tiles (fewer, cheaper levels under a deeper root) start the scan sooner ($PIR_QUERY_TILE1)
  if (nk == 1 && nq <= 2 && pitch > 256 && tile == 1024) {
    int t1 = kLoneTile;
    if (const char* tv = getenv("PIR_QUERY_TILE1")) t1 = atoi(tv);
    if (t1 == 256 || t1 == 512 || t1 == 1024 || (t1 == 4096 && nleaves >= (uint64_t)4096 * 256))
      tile = t1;
  }
  // records of <= 256 B: a tile's rows stream in a quarter of the time its tree takes, so 12 of
  // the 16 waves build trees and 4 scan ($PIR_QUERY_TW = 8 or 12 overrides)
  qp.tw = (nq <= 2 && pitch <= 256) ? kQueryTreeHeavyTW : kFusedTW;
  if (const char* tw = getenv("PIR_QUERY_TW")) {
    const int v = atoi(tw);
    if (v == kFusedTW || (v == kQueryTreeHeavyTW && nq <= 2)) qp.tw = v;
  }
  // 3-5 rounds at VEC 2 with one record per wave row: the four-Russians k_query (768 threads:
  // 4 tree + 8 scan waves) unless $PIR_QUERY_M4R=0.  Round 4 added 3 rounds: the plane-mask
  // k_query ran a 2^24 x 1 KiB query at 4.40 ms (3.9 TB/s) against 3.44 at 4 rounds with the
  // fold (profiles/r04/probe_rounds*.txt)
  if ((uint64_t)tile * pitch >= (1ull << 31)) return qp;  // a tile's rows: one buffer resource
  qp.m4r = nq >= 3 && nq <= 5 && nq > PIR_QUERY_BRANCH_MAXNQ && tile == 1024 &&
           pitch / 8 >= (uint32_t)kColGroupLanes;
  if (const char* mv = getenv("PIR_QUERY_M4R")) qp.m4r = qp.m4r && atoi(mv) != 0;
  // diagnostics: $PIR_QUERY_M4R_TW=2 -> 2 tree + 10 scan waves (default 4 + 8)
  if (const char* mt = getenv("PIR_QUERY_M4R_TW")) qp.m4r = qp.m4r ? (atoi(mt) == 2 ? 2 : 1) : 0;
  int kt = 0;
  while ((1 << kt) < tile) ++kt;
  int lr = 0;
  while ((2ll << lr) <= num_cus) ++lr;  // regions = largest power of two <= CUs
  lr = std::min(lr, nr - kt);
  if (lr < 0) return qp;
  qp.tile = tile;
  qp.lr = lr;
  qp.lt = nr - kt - lr;
  // super-tiles of 2^ls tiles share their narrow top levels (expanded once, to 64 input nodes
  // per tile); 64 << ls nodes must fit the LDS level buffer of TILE / 2 ($PIR_QUERY_SUPER=0: off)
  // Only where the tree, not the scan, paces the launch (small records, or a queue): a lone
  // query of large records waits for its first tile, and a super-tile's top is wider than one
  // tile's.
  qp.ls = std::min(qp.lt, kt - 1 - kQueryKin);
  const int ls_max = qp.ls;
  if (nk == 1 && !(nq <= 2 && pitch <= 256)) qp.ls = 0;
  if (const char* sv = getenv("PIR_QUERY_SUPER")) {
    if (sv[0] == '0') qp.ls = 0;
    if (sv[0] == '1') qp.ls = ls_max;
  }
  qp.shape = make_fused_shape(nleaves, pitch, nq, num_cus, tile);
  qp.shape.grid.x = 1u << lr;
  return qp;
}

hipError_t launch_query_mp(const QueryPlan& qp, const uint8_t* d_key, uint32_t key_stride,
                           int nk, const MpLayout& L, int n, int log_parts, uint64_t prefix,
                           const uint8_t* shard, uint8_t* slabs, hipStream_t s) {
  if (nk < 1 || !qp.tile || !L.nu || L.mu % (uint64_t)qp.tile != 0 || L.nrk != qp.shape.nq)
    return hipErrorInvalidValue;
#define PIR_QM(NQ, TL) query_nq_mp<NQ, TL>(qp, d_key, key_stride, nk, L, n, log_parts, prefix, shard, slabs, s)
  const int nq = qp.shape.nq;
  if (qp.tile == 4096) {
    if (nq == 1) return PIR_QM(1, 4096);
    if (nq == 2) return PIR_QM(2, 4096);
    return hipErrorInvalidValue;
  }
  if (qp.tile != 1024) return hipErrorInvalidValue;
  switch (nq) {
    case 1: return PIR_QM(1, 1024);
    case 2: return PIR_QM(2, 1024);
    case 3: return PIR_QM(3, 1024);
    case 4: return PIR_QM(4, 1024);
    case 5: return PIR_QM(5, 1024);
    default: return hipErrorInvalidValue;
  }
#undef PIR_QM
}

size_t query_steal_bytes(const QueryPlan& qp) {
  const size_t nrp = qp.shape.nq == 1 ? 1 : 2;  // the rounds the stealing path serves (1-2)
  return ((size_t)2 * qp.shape.grid.x + (size_t)qp.shape.grid.x * qp.tile * nrp / 4) * 4;
}

size_t query_scratch_bytes(const QueryPlan& qp) {
  return qp.ls ? ((size_t)qp.shape.grid.x << (kQueryKin + qp.ls)) * (sizeof(uint4) + sizeof(uint32_t)) : 0;
}

hipError_t launch_query(const QueryPlan& qp, const uint8_t* d_raw, uint32_t key_stride, int nk,
                        int p, int n, int party0, int log_parts, uint64_t prefix,
                        const uint8_t* shard, uint8_t* slabs, uint8_t* scratch, hipStream_t s,
                        uint64_t* trace, uint8_t* out, uint32_t* qcnt, uint32_t efs,
                        uint32_t red_mode, StealArgs steal) {
  if (nk < 1 || (qp.ls && !scratch) || (out && !qcnt)) return hipErrorInvalidValue;
  if (nk != 1 || !steal.buf) steal = StealArgs{};
  if (out && (red_mode < 1 || red_mode > 3 || (qp.lr < 3 && red_mode == 3))) return hipErrorInvalidValue;
  if (out && red_mode >= 2 && (efs % 4 != 0 || reinterpret_cast<uintptr_t>(out) % 4 != 0))
    return hipErrorInvalidValue;
  // the tree waves' s_setprio after the first tile (0-3; the scan waves run at PIR_SCAN_PRIO),
  // passed in red_mode's bits 8-9; $PIR_QUERY_TREE_PRIO (read per launch) overrides
  // A lone query (nk == 1) is paced by its tree after the first tile, a queue by the scan:
  // prio 3 for a lone query's tree waves, the default 0 in a queue (same box, configs[1] lone
  // 0.2500 -> 0.2423 ms; a 2^24 x 1 KiB queue 2.55 -> 2.68 ms at prio 3:
  // profiles/r04/bench_tree_prio.jsonl)
  // Round 5: the four-Russians k_query (3-5 rounds) is paced by its 4 tree waves even in a
  // queue -- its scan waves spent 28 % of their cycles waiting for shares at prio 0
  // (profiles/r05/fold_phases_c5_prio0.txt) -- so its tree waves run at 3 there too (configs[4]
  // queue 3.741 -> 3.488 ms per query, same box: profiles/r05/r5b_c5_tree_prio.jsonl)
  {
    const char* tp = getenv("PIR_QUERY_TREE_PRIO");
    red_mode |= ((tp ? (uint32_t)atoi(tp) : ((nk == 1 || qp.m4r) ? 3u : 0u)) & 3u) << 8;
    // Round 6: with 8 scan waves (two per SIMD), the older of a SIMD's two equal-priority scan
    // waves ran 2-3 tiles ahead of the younger one and the younger one held the ring slot the
    // tree needed next (configs[4] trace: the tree waited 11-15 us per tile for a slot).  The
    // scan waves now yield to a lagging SIMD mate (mode 2; 1 = to any lagging wave), and the
    // tree team's waves take turns at the levels narrower than the team (tree_rot), so every
    // SIMD carries the same tree share: configs[4] queue 3.27-3.37 -> 3.16-3.23 ms, 3-4 round
    // queues -3 %, configs[1] lone -1-2 %, the north_star queue -0.5 %; the 12-tree-wave shape
    // of small records (4 scan waves, one per SIMD) lost 5 % and keeps both off
    // (profiles/r06/r6p_c5_even_ab.log, r6q_*, r6s_shapes_ab.log).  $PIR_QUERY_SCAN_EVEN = 0-2
    // and $PIR_QUERY_TREE_ROT = 0/1 override.
    const bool even_def = qp.m4r || qp.tw == kFusedTW;
    const char* se = getenv("PIR_QUERY_SCAN_EVEN");
    red_mode |= ((se ? (uint32_t)atoi(se) : (even_def ? 2u : 0u)) & 3u) << 10;
    const char* tr = getenv("PIR_QUERY_TREE_ROT");
    if (tr ? atoi(tr) != 0 : even_def) red_mode |= 1u << 12;
  }
#define PIR_Q(NQ, TL) query_nq<NQ, TL>(qp, d_raw, key_stride, nk, p, n, party0, log_parts, prefix, shard, slabs, scratch, s, trace, out, qcnt, efs, red_mode, steal)
#ifdef PIR_DEV_NQ  // development builds only (ISA / register checks): one round count
  return qp.shape.nq == PIR_DEV_NQ && qp.tile == 1024 ? PIR_Q(PIR_DEV_NQ, 1024) : hipErrorInvalidValue;
#else
  if (qp.tile == 4096 || qp.tile == 512 || qp.tile == 256) {
    const int t = qp.tile, nq = qp.shape.nq;
    if (t == 4096 && nq == 1) return PIR_Q(1, 4096);
    if (t == 4096 && nq == 2) return PIR_Q(2, 4096);
    if (t == 512 && nq == 1) return PIR_Q(1, 512);
    if (t == 512 && nq == 2) return PIR_Q(2, 512);
    if (t == 256 && nq == 1) return PIR_Q(1, 256);
    if (t == 256 && nq == 2) return PIR_Q(2, 256);
    return hipErrorInvalidValue;
  }
  if (qp.tile != 1024) return hipErrorInvalidValue;
  switch (qp.shape.nq) {
    case 1: return PIR_Q(1, 1024);
    case 2: return PIR_Q(2, 1024);
    case 3: return PIR_Q(3, 1024);
    case 4: return PIR_Q(4, 1024);
    case 5: return PIR_Q(5, 1024);
    case 6: return PIR_Q(6, 1024);
    case 7: return PIR_Q(7, 1024);
    case 8: return PIR_Q(8, 1024);
    default: return hipErrorInvalidValue;
  }
#endif
#undef PIR_Q
}

hipError_t launch_key_prep(const uint8_t* d_raw, size_t key_stride, int num_keys, int p, int n,
                           int nq, int party0, DevKey* d_keys, hipStream_t s) {
  hipLaunchKernelGGL(k_key_prep, dim3(num_keys), dim3(256), 0, s, d_raw, key_stride, p, n, nq,
                     party0, d_keys);
  return hipGetLastError();
}

hipError_t launch_frontier(const TreePlan& pl, const KeySrc& ks, const NodeBufs& nb,
                           hipStream_t s, int nkeys, size_t raw_stride, uint64_t node_stride) {
  const int nlev = pl.log_parts + pl.g + pl.e;
  const uint8_t* raw = ks.raw;
  if (raw && nlev > kFrontCwLevels) {  // CWs read from global: parse in a kernel of its own
    hipError_t err = launch_key_prep(raw, raw_stride, nkeys, ks.p, ks.n, ks.nq, ks.party0,
                                     ks.key, s);
    if (err != hipSuccess) return err;
    raw = nullptr;
  }
  hipLaunchKernelGGL(k_frontier, dim3(1u << pl.g, nkeys), dim3(kFrontThreads), 0, s, raw, ks.p,
                     ks.n, ks.nq, ks.party0, ks.key, pl.prefix, pl.log_parts, pl.g, pl.e,
                     nb.s[0], nb.t[0], (uint32_t)raw_stride, node_stride);
  return hipGetLastError();
}

bool leaf_dfs_enabled() {
  static const bool on = [] {
    const char* v = getenv("PIR_LEAF_DFS");
    return !(v && v[0] == '0');
  }();
  return on;
}

template <int NRP>
static hipError_t launch_stage(int p, const Stage& st, const DevKey* d_key, const uint4* is,
                               const uint32_t* it, uint4* os, uint32_t* ot, uint8_t* c,
                               uint32_t cstride, unsigned blocks, int nkeys, uint64_t in_stride,
                               uint64_t out_stride, uint32_t c_key_off, hipStream_t s) {
  const dim3 grid(blocks, nkeys);
  if (st.final && leaf_dfs_enabled() && leaves_supported(st.k))
    return launch_leaves(p, NRP, st.k, d_key, is, it, st.L_in, (uint64_t)blocks * st.tile, nkeys,
                         in_stride, c, cstride, c_key_off, s);
  if (!st.final && leaf_dfs_enabled() && nodes_dfs_supported(st.k) &&
      (uint64_t)blocks * st.tile * nkeys >= (1u << 18))  // >= 256 workgroups of one node per lane
    return launch_nodes_dfs(p, st.k, d_key, is, it, st.L_in, (uint64_t)blocks * st.tile, nkeys,
                            in_stride, os, ot, out_stride, s);
  if (st.final)
    hipLaunchKernelGGL((k_expand<true, NRP>), grid, dim3(kExpThreads), 0, s, d_key, is, it,
                       st.L_in, st.k, st.tile, os, ot, c, cstride, in_stride, out_stride,
                       c_key_off);
  else
    hipLaunchKernelGGL((k_expand<false, 1>), grid, dim3(kExpThreads), 0, s, d_key, is, it,
                       st.L_in, st.k, st.tile, os, ot, c, cstride, in_stride, out_stride,
                       c_key_off);
  return hipGetLastError();
}

// stages [i0, i1) of chunk j of C (each stage's input range split evenly); the final stage
// writes leaf i's nrp share bytes at d_c + i * cstride (cstride <= 0: nrp)
hipError_t launch_stages(const TreePlan& pl, const DevKey* d_key, const NodeBufs& nb, int j, int C,
                         uint8_t* d_c, int nrp, hipStream_t s, int i0s, int i1s, int cstride,
                         const StageBatch* batch) {
  if (i1s < 0) i1s = pl.nstages;
  const uint32_t cs = cstride > 0 ? (uint32_t)cstride : (uint32_t)nrp;
  const int nkeys = batch ? batch->nkeys : 1;
  const uint64_t stride = batch ? batch->node_stride : 0;
  const uint32_t c_key_off = batch ? batch->c_key_off : 0;
  for (int i = i0s; i < i1s; ++i) {
    const Stage& st = pl.st[i];
    const uint64_t nin = st.nin / C, i0 = nin * j, o0 = i0 << st.k;
    const uint4* is = nb.s[i & 1] + i0;
    const uint32_t* it = nb.t[i & 1] + i0;
    uint64_t in_stride = stride;
    if (batch && batch->in0_s && i == i0s) {  // first stage input from a separate array
      is = batch->in0_s + i0;
      it = batch->in0_t + i0;
      in_stride = batch->in0_stride;
    }
    uint4* os = nb.s[(i + 1) & 1] + o0;
    uint32_t* ot = nb.t[(i + 1) & 1] + o0;
    uint8_t* c = d_c ? d_c + o0 * cs : nullptr;
    const unsigned blocks = (unsigned)(nin / st.tile);
    hipError_t e;
#define PIR_STAGE(N) launch_stage<N>(pl.p >= 2 ? pl.p : 17, st, d_key, is, it, os, ot, c, cs, blocks, nkeys, in_stride, stride, c_key_off, s)
    switch (nrp) {
      case 1: e = PIR_STAGE(1); break;
      case 2: e = PIR_STAGE(2); break;
      case 4: e = PIR_STAGE(4); break;
      case 8: e = PIR_STAGE(8); break;
      case 16: e = PIR_STAGE(16); break;
      default: return hipErrorInvalidValue;
    }
#undef PIR_STAGE
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

int final_stage_blocks(const TreePlan& pl) {
  const Stage& st = pl.st[pl.nstages - 1];
  return (int)(st.nin / st.tile);
}

static int vec_for(int nq) { return nq <= 3 ? 4 : (nq <= 8 ? 2 : 1); }

ScanShape make_scan_shape(uint64_t nrec, uint32_t pitch, int nq, int num_cus, int blocks_per_cu) {
  ScanShape sh{};
  sh.nq = nq;
  sh.nrp = nq == 1 ? 1 : (nq == 2 ? 2 : (nq <= 4 ? 4 : (nq <= 8 ? 8 : 16)));
  sh.vec = vec_for(nq);
  // a record narrower than a VEC=2 wave row but at least a VEC=1 row: one record per row
  // (wave-uniform coefficients, SGPR masks) beats per-lane coefficients for several records
  if (sh.vec == 2 && pitch / 8 < (uint32_t)kColGroupLanes && pitch / 4 >= (uint32_t)kColGroupLanes)
    sh.vec = 1;
  if (nq == 3 && sh.vec == 4 && pitch / 16 < (uint32_t)kColGroupLanes &&
      pitch / 8 >= (uint32_t)kColGroupLanes)
    sh.vec = 2;  // 3 rounds: a record per wave row at VEC = 2 (as before VEC = 4 took them)
  else if (nq == 3 && sh.vec == 4 && pitch / 8 < (uint32_t)kColGroupLanes &&
           pitch / 4 >= (uint32_t)kColGroupLanes)
    sh.vec = 1;  // 3 rounds, 256-511 B: a record per wave row at VEC = 1
  sh.tfold = scan_t_shape(nq, sh.nrp, pitch);
  if (sh.tfold) sh.vec = 1;  // the transposed fold: one dword per lane, any record width
  sh.pitch = pitch;
  sh.cpr = pitch / (sh.vec * 4);
  sh.uniform = sh.cpr >= (uint32_t)kColGroupLanes;
  const uint32_t gy = sh.uniform ? (sh.cpr + kColGroupLanes - 1) / kColGroupLanes : 1;
  const uint32_t rpw = sh.uniform ? 1 : kColGroupLanes / sh.cpr;
  const uint64_t groups = (nrec + rpw - 1) / rpw;
  // 16 waves per CU with 4 x 16 B loads in flight per lane (~64 KiB per CU), few slabs
  const uint64_t want_blocks = (uint64_t)num_cus * (blocks_per_cu > 0 ? blocks_per_cu : kScanBlocksPerCU);
  const uint64_t waves_per_block = kScanThreads / 64;
  uint64_t gx = std::max<uint64_t>(1, std::min<uint64_t>(want_blocks / gy, (groups + 4 * waves_per_block - 1) / (4 * waves_per_block)));
  sh.grid = dim3((unsigned)gx, gy);
  sh.threads = kScanThreads;
  if (!sh.tfold && blocks_per_cu <= 0 && sh.uniform && sh.vec == 2 && (nq == 4 || nq == 5) &&
      !(getenv("PIR_SCAN_M4R") && atoi(getenv("PIR_SCAN_M4R")) == 0)) {
    // the four-Russians k_scan_uni: one 768-thread workgroup per CU and column group
    const uint64_t wpb = kScanM4rThreads / 64;
    gx = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)num_cus / gy, (groups + 4 * wpb - 1) / (4 * wpb)));
    sh.grid = dim3((unsigned)gx, gy);
    sh.threads = kScanM4rThreads;
  }
  // k_scan_t: its own workgroup size and blocks per CU; it addresses a wave's rows through one
  // buffer resource, < 2^31 bytes of rows per wave (only shards of tens of GiB reach it)
  if (sh.tfold) {
    const uint64_t wpb = kScanTThreads / 64;
    int bpc = kScanTBlocksPerCU;
    if (const char* v = getenv("PIR_SCAN_T_BPC")) bpc = std::max(1, std::min(kScanTBlocksPerCU, atoi(v)));
    const uint64_t want = (uint64_t)num_cus * bpc;  // ($PIR_SCAN_T_BPC: diagnostics)
    uint64_t gxt = std::max<uint64_t>(1, std::min<uint64_t>(want / gy, (groups + 4 * wpb - 1) / (4 * wpb)));
    while ((groups / (gxt * wpb) + 1) * pitch >= (1ull << 31) && gxt < (1u << 30)) gxt *= 2;
    sh.grid = dim3((unsigned)gxt, gy);
    sh.threads = kScanTThreads;
  }
  sh.slab_bytes = (uint32_t)(nq * kColGroupLanes * sh.vec * 4);
  return sh;
}

template <int NQ>
static hipError_t scan_nq(const ScanShape& sh, const uint8_t* d_shard, uint64_t nrec,
                          const uint8_t* d_c, uint8_t* d_slabs, int acc, hipStream_t s) {
  constexpr int NRP = NQ == 1 ? 1 : (NQ == 2 ? 2 : (NQ <= 4 ? 4 : (NQ <= 8 ? 8 : 16)));
  constexpr int VEC = NQ <= 3 ? 4 : (NQ <= 8 ? 2 : 1);
  if constexpr (VEC == 4) {
    if (sh.vec == 1) {  // 3 rounds, 256-511 B records: one per wave row at one dword per lane
      if (!sh.uniform) return hipErrorInvalidValue;
      hipLaunchKernelGGL((k_scan_uni<NQ, NRP, 1>), sh.grid, dim3(kScanThreads), 0, s, d_shard,
                         nrec, sh.pitch, sh.cpr, d_c, d_slabs, acc);
      return hipGetLastError();
    }
  }
  if constexpr (VEC > 1) {
    if (sh.vec == VEC / 2) {  // narrower records: one per wave row at half the width
      if (!sh.uniform) return hipErrorInvalidValue;
      hipLaunchKernelGGL((k_scan_uni<NQ, NRP, VEC / 2>), sh.grid, dim3(kScanThreads), 0, s, d_shard,
                         nrec, sh.pitch, sh.cpr, d_c, d_slabs, acc);
      return hipGetLastError();
    }
  }
  if (sh.vec != VEC) return hipErrorInvalidValue;
  if constexpr (VEC == 2 && NQ >= 4 && NQ <= 5) {
    if (sh.uniform && sh.threads == kScanM4rThreads) {
      hipLaunchKernelGGL((k_scan_uni<NQ, NRP, VEC, kScanM4rThreads>), sh.grid,
                         dim3(kScanM4rThreads), 0, s, d_shard, nrec, sh.pitch, sh.cpr, d_c,
                         d_slabs, acc);
      return hipGetLastError();
    }
  }
  if (sh.uniform)
    hipLaunchKernelGGL((k_scan_uni<NQ, NRP, VEC>), sh.grid, dim3(kScanThreads), 0, s, d_shard,
                       nrec, sh.pitch, sh.cpr, d_c, d_slabs, acc);
  else
    hipLaunchKernelGGL((k_scan<NQ, NRP, VEC, false>), sh.grid, dim3(kScanThreads), 0, s, d_shard,
                       nrec, sh.pitch, sh.cpr, d_c, d_slabs, acc & 1);
  return hipGetLastError();
}

hipError_t launch_scan(const ScanShape& sh, const uint8_t* d_shard, uint64_t nrec,
                       const uint8_t* d_c, uint8_t* d_slabs, bool accumulate, hipStream_t s) {
  // bit 1: the waves of a k_scan_uni / k_scan_t workgroup claim row chunks instead of folding a
  // fixed range each (round 6: Hollanti 5 rounds 3.60 -> 3.12-3.30 ms, 3 rounds -1.5 %,
  // profiles/r06/r6w_*, r6x_*; $PIR_SCAN_DYN=0 restores the fixed ranges)
  const char* dv = getenv("PIR_SCAN_DYN");
  const int acc = (accumulate ? 1 : 0) | ((dv ? atoi(dv) != 0 : true) ? 2 : 0);
  if (sh.tfold) {
    // k_scan_t addresses a workgroup's rows through one buffer resource when they claim chunks
    const bool wg_fits = (nrec / sh.grid.x + 1) * (uint64_t)sh.pitch < (1ull << 31);
    return launch_scan_t(sh, d_shard, nrec, d_c, d_slabs, wg_fits ? acc : (acc & 1), s);
  }
  switch (sh.nq) {
    case 1: return scan_nq<1>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 2: return scan_nq<2>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 3: return scan_nq<3>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 4: return scan_nq<4>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 5: return scan_nq<5>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 6: return scan_nq<6>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 7: return scan_nq<7>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 8: return scan_nq<8>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 9: return scan_nq<9>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 10: return scan_nq<10>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 11: return scan_nq<11>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 12: return scan_nq<12>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 13: return scan_nq<13>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 14: return scan_nq<14>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 15: return scan_nq<15>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    case 16: return scan_nq<16>(sh, d_shard, nrec, d_c, d_slabs, acc, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_reduce(const ScanShape& sh, const uint8_t* d_slabs, uint32_t efs,
                         uint8_t* d_out, hipStream_t s, int nk, int nslices) {
  const uint32_t words = sh.pitch / 4;
  const uint32_t total = (uint32_t)sh.nq * words;
  const uint32_t gw = kColGroupLanes * sh.vec;
  const uint64_t q_words = (uint64_t)sh.grid.x * sh.grid.y * (sh.slab_bytes / 4);
  if (nslices < 1 || sh.grid.x % (uint32_t)nslices != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_reduce, dim3((total + 63) / 64, nk, nslices), dim3(kReduceThreads), 0, s,
                     reinterpret_cast<const uint32_t*>(d_slabs), sh.nq, gw,
                     sh.grid.x / (uint32_t)nslices, sh.pitch, efs, d_out, q_words);
  return hipGetLastError();
}

// grid-stride kernels of 256 threads: enough workgroups to fill the chip many times over, and
// never past the 2^32 threads a launch may have (a 2^27-row shard has 2^33 16-byte chunks)
static unsigned grid_1d(uint64_t items) {
  return (unsigned)std::min<uint64_t>((items + 255) / 256, 1u << 16);
}

hipError_t launch_xor_fold(const uint8_t* d_in, int nranks, size_t len, uint8_t* d_out,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_xor_fold, dim3(grid_1d(len)), dim3(256), 0, s, d_in,
                     nranks, len, d_out);
  return hipGetLastError();
}

hipError_t launch_fill_random(uint8_t* d, size_t bytes, uint64_t seed, hipStream_t s) {
  hipLaunchKernelGGL(k_fill_random, dim3(grid_1d(bytes)), dim3(256), 0, s, d,
                     bytes, seed);
  return hipGetLastError();
}

hipError_t launch_encode_across(const uint8_t* d_files, uint64_t file_pitch, uint64_t nfiles,
                               int k, int party, uint8_t* d_shard, uint64_t rows, uint64_t row0,
                               uint32_t pitch, uint32_t efs, hipStream_t s) {
  if (k < 1 || k > 16) return hipErrorInvalidValue;
  EncodeCoefs co{};
  for (int j = 0; j < k; ++j) {  // gf_pow(party, j) (coding.cpp:46-60; pow(0, e) == 1)
    uint32_t r = 1;
    for (int t = 0; t < j && party; ++t) {
      uint32_t a = r, b = (uint32_t)party, m = 0;
      while (b) {
        if (b & 1) m ^= a;
        a = ((a << 1) ^ ((a & 0x80) ? 0x11d : 0)) & 0xff;
        b >>= 1;
      }
      r = m;
    }
    co.c[j] = (uint8_t)r;
  }
  const uint64_t encdb = (nfiles + k - 1) / k;
  const uint64_t total = rows * (pitch / 16);
  hipLaunchKernelGGL(k_encode_across, dim3(grid_1d(total)), dim3(256), 0, s,
                     d_files, file_pitch, nfiles, encdb, k, co, d_shard, rows, row0, pitch, efs);
  return hipGetLastError();
}

hipError_t launch_fill_shard(uint8_t* d_shard, uint64_t rows, uint32_t pitch, uint32_t efs,
                             uint64_t global_row0, uint64_t seed, hipStream_t s) {
  const uint64_t total = rows * (pitch / 16);
  hipLaunchKernelGGL(k_fill_shard, dim3(grid_1d(total)), dim3(256), 0, s,
                     d_shard, rows, pitch, efs, global_row0, seed);
  return hipGetLastError();
}

#endif  // !PIR_QUERY_PART

}  // namespace pir
