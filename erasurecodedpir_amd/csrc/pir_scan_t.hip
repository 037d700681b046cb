// pir_scan_t.hip -- the many-round GF(2^8) scan as a transposed four-Russians fold (k_scan_t).
//
// The answer of round a is ans_a = sum_i c_a[i] * x_i over GF(2^8) (server.cpp:121-127).  Over
// bit planes (coding.cpp:9-21, poly 0x11d): ans_a = sum_b alpha^b Z_{a,b}, Z_{a,b} = XOR of the
// rows whose round-a coefficient has bit b set.  With one record per wave row the coefficient
// word w_i (the record's NRP <= 8 coefficient bytes, round a = byte a, as 64 bits: plane
// p = 8a + b) is wave-uniform, and the scans of pir_kernels.hip select each plane's row
// combination by GPR index (pir_m4r.h): one index switch per plane per 4 rows, whose cost grows
// with the number of planes (2.2 TB/s at 64 planes, 3.4 at 40: profiles/r02_micro/).
//
// Here the roles are swapped.  Per lane and 8 rows, bit j of the lane's 8 row dwords forms an
// 8-bit index n_j (an 8 x 32 bit transpose of the rows, pir_bits.h), and the wave keeps in LDS a
// table of the 256 XOR combinations of the 8 rows' coefficient words, T[v] = XOR_{r: bit r of v}
// w_r.  Then for every bit position j: Zt[j] ^= T[n_j] -- one ds_read_b64 and two v_xor --
// where Zt[j] (64 bits) is bit j of the lane's dword in every plane at once.  The cost per row
// no longer depends on the number of planes (up to 64), and no scalar index setting is left in
// the loop.  At the end Zt is transposed back to planes (32 x 32 bit transposes) and folded by
// the alpha powers as in k_scan_uni; slabs and k_reduce are unchanged.
//
// One record per wave row at one dword per lane (pitch >= 256 B; column groups of 64 dwords
// along grid y), NRP = 4 or 8 coefficient bytes per record (NQ <= NRP rounds), rows of a wave
// through one buffer resource with the row offset in soffset (< 2^31 B of rows per wave: host).
#include "pir_bits.h"
#include <stdlib.h>
#include <type_traits>
#include "pir_kernels.h"

namespace pir {

constexpr int kScanTWaves = kScanTThreads / 64;

__device__ __forceinline__ uint32_t gf_xtime4_t(uint32_t x) {  // 4 packed bytes times alpha
  return ((x & 0x7f7f7f7fu) << 1) ^ (((x >> 7) & 0x01010101u) * 0x1du);
}

template <int NQ, int NRP>
__global__ __launch_bounds__(kScanTThreads) __attribute__((amdgpu_waves_per_eu(kScanTWavesPerEU)))
void k_scan_t(const uint8_t* __restrict__ shard, uint64_t nrec, uint32_t pitch, uint32_t cpr,
              const uint8_t* __restrict__ c, uint8_t* __restrict__ slabs, int accumulate,
              uint32_t ckey, uint64_t ckoff) {
  static_assert(NRP == 4 || NRP == 8, "coefficient words of 32 or 64 bits");
  static_assert(NQ >= 1 && NQ <= NRP, "rounds");
  constexpr int WD = NRP / 4;  // coefficient words per record (rounds 0-3, 4-7)
  constexpr int GW = kColGroupLanes;
  // per wave: T[v] at [v * WD]; read as uint2 (ds_read_b64) when WD == 2, hence 8-aligned
  __shared__ alignas(8) uint32_t tab[kScanTWaves][256 * WD];
  __shared__ uint32_t red[NQ * GW];
  __shared__ uint32_t next_chunk;
  for (int i = threadIdx.x; i < NQ * GW; i += blockDim.x) red[i] = 0;
  // accumulate bit 1 (launch_scan_t, $PIR_SCAN_DYN): the waves claim 64-row chunks of the
  // workgroup's rows (as k_scan_uni: equal-priority waves issue oldest first, so fixed ranges
  // leave the youngest waves folding the tail alone)
  const bool dyn = (accumulate >> 1) & 1;
  accumulate &= 1;

  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t wave = (uint64_t)blockIdx.x * kScanTWaves + wv;
  const uint64_t nwaves = (uint64_t)gridDim.x * kScanTWaves;
  const uint32_t chunk = blockIdx.y * kColGroupLanes + lane;
  const bool active = chunk < cpr;
  // the wave's rows, or (dyn) the workgroup's
  const uint64_t r0 = dyn ? (uint64_t)blockIdx.x * kScanTWaves * nrec / nwaves : wave * nrec / nwaves;
  const uint64_t r1 = dyn ? ((uint64_t)blockIdx.x + 1) * kScanTWaves * nrec / nwaves : (wave + 1) * nrec / nwaves;
  uint32_t* const tw = &tab[wv][0];
  if (dyn) {
    if (threadIdx.x == 0) next_chunk = 0;
    __syncthreads();
  }

  uint32_t Zt[32][WD];
#pragma unroll
  for (int j = 0; j < 32; ++j)
#pragma unroll
    for (int d = 0; d < WD; ++d) Zt[j][d] = 0;

  if (r1 > r0) {
    const uint32_t nrows = (uint32_t)(r1 - r0);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(shard + r0 * pitch), (short)0, (int)(nrows * pitch), kBufRsrcWord3);
    const uint32_t voff = (active ? chunk : 0u) * 4u;  // inactive lanes: the row's first dword
    // rows past the wave's last re-read row r0 and have zero coefficient words
    auto load_rel = [&](uint32_t rel) __attribute__((always_inline)) {
      return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, voff, rel < nrows ? rel * pitch : 0u, 2);
    };
    // lane l: the coefficient words of row rb + l (zero past the wave's rows); key-major
    // coefficients (ckey bytes per key) are gathered key by key: one ckey-byte load per key,
    // coalesced across the wave's 64 rows
    auto coefs64 = [&](uint32_t rb) __attribute__((always_inline)) {
      const uint32_t rl = rb + lane;
      uint2 cw = make_uint2(0, 0);
      if (rl < nrows) {
        const uint64_t row = r0 + rl;
        if (ckey == 0) {
          const uint8_t* p = c + row * NRP;
          if constexpr (NRP == 8) cw = *reinterpret_cast<const uint2*>(p);
          else cw.x = *reinterpret_cast<const uint32_t*>(p);
        } else {
          uint64_t w = 0;
          for (uint32_t g = 0; g * ckey < (uint32_t)NRP; ++g) {
            const uint8_t* p = c + g * ckoff + row * ckey;
            const uint64_t v = ckey == 1 ? *p : (ckey == 2 ? *reinterpret_cast<const uint16_t*>(p)
                                                           : *reinterpret_cast<const uint32_t*>(p));
            w |= v << (8 * g * ckey);
          }
          cw = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
        }
      }
      return cw;
    };
    // table entries lane + 64 k: the XOR of w_r over the set bits r < 6 of the lane, then w6, w7
    uint32_t lm[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) lm[r] = ((lane >> r) & 1u) ? 0xffffffffu : 0u;

    // chunk claims (dyn): rb walks the claimed chunks' first rows; the rows and coefficient words
    // loaded ahead come from the next claimed chunk past the current one's end
    const uint32_t nch = (nrows + 63) / 64;
    auto claim = [&]() __attribute__((always_inline)) -> uint32_t {
      uint32_t v = 0;
      if (lane == 0)
        v = __hip_atomic_fetch_add(&next_chunk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return (uint32_t)__builtin_amdgcn_readfirstlane(v);
    };
    uint32_t cur = dyn ? claim() : 0u;
    uint32_t nxt = dyn ? (cur < nch ? claim() : nch) : 1u;
    // row k >= 0 of the sequence that continues past the current chunk into the next
    auto seq_row = [&](uint32_t k) __attribute__((always_inline)) -> uint32_t {
      return k < 64 ? cur * 64 + k : (nxt < nch ? nxt * 64 + (k - 64) : nrows);
    };
    uint32_t x[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) x[u] = load_rel(seq_row((uint32_t)u));
    uint2 cw = cur < nch ? coefs64(cur * 64) : make_uint2(0, 0);
    for (; cur < nch;) {
      const uint32_t rb = cur * 64;
      const uint2 cwn = nxt < nch ? coefs64(nxt * 64) : make_uint2(0, 0);  // next chunk's words, in flight
      const uint32_t nb = nrows - rb < 64 ? nrows - rb : 64;
      for (uint32_t j0 = 0; j0 < nb; j0 += 16) {
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          const uint32_t j = j0 + 8 * g;
          // ---- the wave's table of the 8 rows' coefficient combinations
#pragma unroll
          for (int d = 0; d < WD; ++d) {
            uint32_t w[8];
#pragma unroll
            for (int r = 0; r < 8; ++r)
              w[r] = (uint32_t)__builtin_amdgcn_readlane((int)(d ? cw.y : cw.x), (int)(j + r));
            uint32_t e = 0;
#pragma unroll
            for (int r = 0; r < 6; ++r) e = __builtin_amdgcn_bitop3_b32(e, w[r], lm[r], 0x78);
            const uint32_t e6 = e ^ w[6], e7 = e ^ w[7];
            tw[lane * WD + d] = e;
            tw[(lane + 64) * WD + d] = e6;
            tw[(lane + 128) * WD + d] = e7;
            tw[(lane + 192) * WD + d] = e6 ^ w[7];
          }
          __builtin_amdgcn_wave_barrier();  // the wave's own table: LDS keeps its order
          // ---- bit j of the 8 rows -> index byte; one lookup per bit position
          uint32_t (&R)[8] = *reinterpret_cast<uint32_t(*)[8]>(&x[8 * g]);  // in place
          transpose8x32(R);
          uint32_t id[32];
#pragma unroll
          for (int jj = 0; jj < 32; ++jj) id[jj] = (R[jj & 7] >> (8 * (jj >> 3))) & 0xffu;
          // 4 chunks of 8 lookups, software-pipelined: chunk c + 1's reads are issued before
          // chunk c's XORs (16 reads in flight; left alone the scheduler waits on each read)
          using Ent = typename std::conditional<WD == 2, uint2, uint32_t>::type;
          const Ent* te = reinterpret_cast<const Ent*>(tw);
          Ent ta[8], tb[8];
          auto issue = [&](Ent (&t)[8], int ch) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < 8; ++q) t[q] = te[id[8 * ch + q]];
            __builtin_amdgcn_sched_barrier(0);
          };
          auto fold = [&](const Ent (&t)[8], int ch) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              if constexpr (WD == 2) {
                Zt[8 * ch + q][0] ^= t[q].x;
                Zt[8 * ch + q][1] ^= t[q].y;
              } else {
                Zt[8 * ch + q][0] ^= t[q];
              }
            }
            __builtin_amdgcn_sched_barrier(0);
          };
          issue(ta, 0);
          issue(tb, 1);
          fold(ta, 0);
          issue(ta, 2);
          fold(tb, 1);
          issue(tb, 3);
          fold(ta, 2);
          fold(tb, 3);
          __builtin_amdgcn_wave_barrier();  // reads done before the next group's table
#pragma unroll
          for (int r = 0; r < 8; ++r) x[8 * g + r] = load_rel(seq_row(j + 16 + r));
          __builtin_amdgcn_sched_barrier(0);  // one group at a time (register pressure)
        }
      }
      cw = cwn;
      cur = nxt;
      nxt = dyn ? (cur < nch ? claim() : nch) : cur + 1;
    }
  }
  __syncthreads();  // red[] zeroed
  if (active) {
#pragma unroll
    for (int d = 0; d < WD; ++d) {
      if (4 * d >= NQ) continue;
      uint32_t Y[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) Y[j] = Zt[j][d];
      transpose32(Y);  // Y[q]: plane 32 d + q = (round 4 d + q / 8, bit q % 8)
#pragma unroll
      for (int a4 = 0; a4 < 4; ++a4) {
        const int a = 4 * d + a4;
        if (a >= NQ) continue;
        uint32_t acc = Y[8 * a4 + 7];
#pragma unroll
        for (int b = 6; b >= 0; --b) acc = gf_xtime4_t(acc) ^ Y[8 * a4 + b];
        if (acc) atomicXor(&red[a * GW + lane], acc);
      }
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

// $PIR_SCAN_T: 0 = never, 2 = every 4-8 round shape it can take (diagnostics), else the default
static int scan_t_mode() {  // read per plan (tests switch it within one process)
  const char* v = getenv("PIR_SCAN_T");
  return v ? atoi(v) : 1;
}
bool scan_t_enabled() { return scan_t_mode() != 0; }

// 6-8 rounds (64 and 48 planes: 3.9 TB/s against 2.2 for the GPR-index fold at configs[2]'s
// 8); 4-5 rounds only for records narrower than a VEC = 2 wave row (the 768-thread GPR-index
// k_scan_uni at two dwords per lane is faster there: Hollanti 5 rounds at 1 KiB 4.53 against
// 4.91 ms, profiles/r03_bench_ch5_*.json)
bool scan_t_shape(int nq, int nrp, uint32_t pitch) {
  if (!scan_t_enabled() || nq < 4 || nq > 8 || nq > nrp || (nrp != 4 && nrp != 8)) return false;
  if (pitch % 4 != 0 || pitch / 4 < (uint32_t)kColGroupLanes) return false;
  return nq >= 6 || pitch / 8 < (uint32_t)kColGroupLanes || scan_t_mode() == 2;
}

template <int NQ, int NRP>
static hipError_t scan_t_launch(const ScanShape& sh, const uint8_t* d_shard, uint64_t nrec,
                                const uint8_t* d_c, uint8_t* d_slabs, int acc, hipStream_t s) {
  if (sh.ckey != 0 && (sh.ckey > 4 || NRP % sh.ckey != 0)) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_scan_t<NQ, NRP>), sh.grid, dim3(kScanTThreads), 0, s, d_shard, nrec,
                     sh.pitch, sh.cpr, d_c, d_slabs, acc, sh.ckey, sh.ckoff);
  return hipGetLastError();
}

hipError_t launch_scan_t(const ScanShape& sh, const uint8_t* d_shard, uint64_t nrec,
                         const uint8_t* d_c, uint8_t* d_slabs, int acc, hipStream_t s) {
  if (sh.threads != kScanTThreads || sh.vec != 1 || !sh.uniform) return hipErrorInvalidValue;
#define PIR_ST(NQ, NRP) \
  if (sh.nq == NQ && sh.nrp == NRP) return scan_t_launch<NQ, NRP>(sh, d_shard, nrec, d_c, d_slabs, acc, s)
  PIR_ST(4, 4); PIR_ST(4, 8); PIR_ST(5, 8); PIR_ST(6, 8); PIR_ST(7, 8); PIR_ST(8, 8);
#undef PIR_ST
  return hipErrorInvalidValue;
}

}  // namespace pir
