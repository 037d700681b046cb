// pir_aes.h -- AES-128 for CDNA4.  The PRG G of the reference (src/c/utils.cpp:37-51) is
// AES-128-CTR keyed by each tree node's seed, so there is no fixed key schedule to amortise:
// every node runs the key schedule on the fly next to its rounds.
//
// T-box form with TWO LDS tables, Te0[x] = {2S,S,S,3S} and Te2 = rotl16(Te0) = {S,3S,2S,S}
// (S = the FIPS-197 S-box, computed on the host from the field definition), each replicated
// 32x per entry (row e = 32 copies of Te0[e], then 32 of Te2[e]): every lane of a 32-lane
// ds_read_b32 group reads its own bank, conflict-free for any index pattern, and a lookup
// address costs one v_perm_b32.  With Te1 = rotl8(Te0) and Te3 = rotl8(Te2) a column is
//     Te0[a] ^ Te2[c] ^ rotl8(Te0[b] ^ Te2[d] ^ rotr8(k))
// -- one v_alignbit and two v_bitop3 (3-input XOR) per column.  The last round and the key
// schedule read S from byte 1/2 of Te0 and byte 0/3 of Te2.
//
// Two execution shapes:
//   * row shape (1 lane = 1 key): aes3_ctr() runs the 3 CTR blocks of an internal node
//     (G(seed, blen<=48)) on one shared key schedule -- throughput levels;
//   * column shape (4 lanes = 1 block, lane q holds column q; DPP quad permutes for ShiftRows
//     and the key schedule's prefix XOR): aes_col() -- 4x lower latency for narrow levels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pir {

// Te0[x] = {2 S(x), S(x), S(x), 3 S(x)} (bytes 0-3), S = the AES S-box: affine(x^-1) over
// GF(2^8)/0x11b (FIPS-197 5.1.1), computed at compile time.  Each translation unit that includes
// this header owns its own statically initialised copy (nothing to upload at engine creation).
struct Te0Table {
  uint32_t v[256];
};
constexpr uint8_t aes_xtime_c(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }
constexpr uint8_t aes_mul_c(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = aes_xtime_c(a);
    b >>= 1;
  }
  return r;
}
constexpr Te0Table make_te0() {
  Te0Table t{};
  for (int x = 0; x < 256; ++x) {
    uint8_t inv = 0;
    if (x) {
      uint8_t r = 1, b = (uint8_t)x;
      for (int e = 254; e; e >>= 1) {
        if (e & 1) r = aes_mul_c(r, b);
        b = aes_mul_c(b, b);
      }
      inv = r;
    }
    uint8_t sb = inv;
    for (int k = 1; k <= 4; ++k) sb ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
    sb ^= 0x63;
    t.v[x] = (uint32_t)aes_mul_c(sb, 2) | ((uint32_t)sb << 8) | ((uint32_t)sb << 16) |
             ((uint32_t)aes_mul_c(sb, 3) << 24);
  }
  return t;
}
static_assert(make_te0().v[0] == 0xa56363c6u && make_te0().v[1] == 0x847c7cf8u, "AES Te0");
static __constant__ Te0Table c_te0 = make_te0();

constexpr uint32_t kTeBytes = 256 * 32 * 4;  // one replicated table: 32 KiB
constexpr uint32_t kTablesBytes = 2 * kTeBytes;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }
__device__ __forceinline__ uint32_t rotr8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 8); }

// LDS layout: 256 rows of 256 B, row e = [Te0[e] x 32 lanes | Te2[e] x 32 lanes].  The byte
// address of a lookup is (index << 8) | (table << 7) | (lane & 31) << 2: index byte k of w lands in
// address byte 1 and the per-lane constant in byte 0, so ONE v_perm_b32 forms the address.
template <int K>
__device__ __forceinline__ uint32_t tab_addr(uint32_t w, uint32_t lane_part) {
  // bytes of {w, lane_part}: 0-3 = lane_part, 4-7 = w; 0x0c = zero
  return __builtin_amdgcn_perm(w, lane_part, 0x0c0c0000u | ((4u + K) << 8));
}

struct Tab {
  const char* base;  // LDS: the interleaved table (64 KiB)
  uint32_t l0, l2;   // (lane & 31) * 4, and the same + 128 (the Te2 half of a row)
  __device__ __forceinline__ explicit Tab(const void* lds)
      : base(reinterpret_cast<const char*>(lds)), l0((threadIdx.x & 31u) * 4u), l2(l0 | 128u) {}
  template <int K>
  __device__ __forceinline__ uint32_t t0(uint32_t w) const {  // Te0[byte K of w]
    return *reinterpret_cast<const uint32_t*>(base + tab_addr<K>(w, l0));
  }
  template <int K>
  __device__ __forceinline__ uint32_t t2(uint32_t w) const {  // Te2[byte K of w]
    return *reinterpret_cast<const uint32_t*>(base + tab_addr<K>(w, l2));
  }
};

// fill the interleaved table (all threads of the block)
__device__ __forceinline__ void load_tables(uint32_t* lds) {
  for (int i = threadIdx.x; i < 256 * 64; i += blockDim.x) {
    const uint32_t v = c_te0.v[i >> 6];
    lds[i] = (i & 32) ? __builtin_amdgcn_alignbit(v, v, 16) : v;
  }
}
// the same for a block of exactly NT threads: every load is issued before the first store,
// and entry (i >> 6) is wave-uniform, so the loads are scalar
template <int NT>
__device__ __forceinline__ void load_tables_n(uint32_t* lds) {
  constexpr int K = (256 * 64 + NT - 1) / NT;  // NT a multiple of 64 (768 leaves a partial pass)
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t e = wv + k * (NT / 64);
    v[k] = e < 256 ? c_te0.v[e] : 0u;
  }
  const bool hi = threadIdx.x & 32;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if ((256 * 64) % NT == 0 || wv + k * (NT / 64) < 256)
      lds[threadIdx.x + k * NT] = hi ? __builtin_amdgcn_alignbit(v[k], v[k], 16) : v[k];
}

// SubWord(RotWord(k3)) ^ rcon, then the word chain (FIPS-197 5.2)
__device__ __forceinline__ void key_next(const Tab& T, uint32_t& k0, uint32_t& k1, uint32_t& k2,
                                         uint32_t& k3, uint32_t rcon) {
  const uint32_t t = (T.t2<1>(k3) & 0xffu) | (T.t0<2>(k3) & 0xff00u) |
                     (T.t0<3>(k3) & 0xff0000u) | (T.t2<0>(k3) & 0xff000000u);
  k0 = xor3(k0, t, rcon);
  k1 ^= k0;
  k2 ^= k1;
  k3 ^= k2;
}

// one full round on a row-shape state; kr = rotr8 of the round key words
__device__ __forceinline__ void round_row(const Tab& T, uint32_t& w0, uint32_t& w1, uint32_t& w2,
                                          uint32_t& w3, uint32_t kr0, uint32_t kr1, uint32_t kr2,
                                          uint32_t kr3) {
  const uint32_t n0 = xor3(T.t0<0>(w0), T.t2<2>(w2), rotl8(xor3(T.t0<1>(w1), T.t2<3>(w3), kr0)));
  const uint32_t n1 = xor3(T.t0<0>(w1), T.t2<2>(w3), rotl8(xor3(T.t0<1>(w2), T.t2<3>(w0), kr1)));
  const uint32_t n2 = xor3(T.t0<0>(w2), T.t2<2>(w0), rotl8(xor3(T.t0<1>(w3), T.t2<3>(w1), kr2)));
  const uint32_t n3 = xor3(T.t0<0>(w3), T.t2<2>(w1), rotl8(xor3(T.t0<1>(w0), T.t2<3>(w2), kr3)));
  w0 = n0; w1 = n1; w2 = n2; w3 = n3;
}

// last-round column from (w_c, w_c+1, w_c+2, w_c+3): SubBytes + ShiftRows + AddRoundKey
__device__ __forceinline__ uint32_t last_col(const Tab& T, uint32_t a, uint32_t b, uint32_t c,
                                             uint32_t d, uint32_t k) {
  uint32_t x = (T.t2<0>(a) & 0xffu) | (T.t0<1>(b) & 0xff00u);
  x |= (T.t0<2>(c) & 0xff0000u) | (T.t2<3>(d) & 0xff000000u);
  return x ^ k;
}

// the first NB (1-3) bytes of a last-round column, AddRoundKey included (the others: don't care)
template <int NB>
__device__ __forceinline__ uint32_t last_col_b(const Tab& T, uint32_t a, uint32_t b, uint32_t c,
                                               uint32_t k) {
  uint32_t x = T.t2<0>(a);  // byte 0 = S[a.b0]
  if constexpr (NB >= 2) x = (x & 0xffu) | (T.t0<1>(b) & 0xff00u);
  if constexpr (NB >= 3) x |= T.t0<2>(c) & 0xff0000u;
  return x ^ k;
}

constexpr uint32_t kRcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};

// Row shape, one key, NB CTR blocks with counters c0..c0+NB-1 (c0 a multiple of NB, NB <= 256,
// passed as ctr_be = the byte-swapped c0, i.e. BE128(c0)'s last word); block NB-1 only needs its
// first LASTW output words (the control-bit bytes); out[b] = AES_key(BE128(c0 + b)).  The
// counters differ in byte 15 only.  LASTB in 1-3 (one block): only the first LASTB output
// bytes are valid (a leaf's 1-2 share bytes): LASTB last-round lookups, the last key word's
// bytes alone, and the ninth round's columns nothing reads are dropped by the compiler.
template <int NB, int LASTW, int LASTB = 0>
__device__ __forceinline__ void aes_ctr_row(const Tab& T, uint4 key, uint4 (&out)[NB],
                                            uint32_t ctr_be = 0) {
  static_assert(LASTB == 0 || (NB == 1 && LASTB < 4), "byte-trimmed: one block, 1-3 bytes");
  uint32_t k0 = key.x, k1 = key.y, k2 = key.z, k3 = key.w;
  uint32_t w[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    w[b][0] = k0; w[b][1] = k1; w[b][2] = k2; w[b][3] = k3 ^ ctr_be ^ ((uint32_t)b << 24);
  }
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    key_next(T, k0, k1, k2, k3, kRcon[r]);
    const uint32_t r0 = rotr8(k0), r1 = rotr8(k1), r2 = rotr8(k2), r3 = rotr8(k3);
    if (r == 0) {
      // first round: the blocks differ only in byte 15 (the counter), which only output column
      // 0 reads (T.t2<3>(w3) in round_row), so columns 1-3 are block 0's for every block
      // (NB = 1 costs the same as round_row in this and the next round)
#pragma unroll
      for (int b = 1; b < NB; ++b)
        w[b][0] = xor3(T.t0<0>(w[b][0]), T.t2<2>(w[b][2]),
                       rotl8(xor3(T.t0<1>(w[b][1]), T.t2<3>(w[b][3]), r0)));
      round_row(T, w[0][0], w[0][1], w[0][2], w[0][3], r0, r1, r2, r3);
#pragma unroll
      for (int b = 1; b < NB; ++b) {
        w[b][1] = w[0][1]; w[b][2] = w[0][2]; w[b][3] = w[0][3];
      }
      continue;
    }
    if (r == 1) {
      // second round: the blocks still share columns 1-3, so each output column is three
      // lookups of the shared columns (once) plus one of the block's own column 0 (rotl8 is
      // linear over XOR, so the column-0 term can leave round_row's rotl8)
      const uint32_t a1 = w[0][1], a2 = w[0][2], a3 = w[0][3];
      const uint32_t s0 = T.t2<2>(a2) ^ rotl8(xor3(T.t0<1>(a1), T.t2<3>(a3), r0));
      const uint32_t s1 = xor3(T.t0<0>(a1), T.t2<2>(a3), rotl8(T.t0<1>(a2) ^ r1));
      const uint32_t s2 = T.t0<0>(a2) ^ rotl8(xor3(T.t0<1>(a3), T.t2<3>(a1), r2));
      const uint32_t s3 = xor3(T.t0<0>(a3), T.t2<2>(a1), rotl8(T.t2<3>(a2) ^ r3));
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const uint32_t x = w[b][0];
        w[b][0] = T.t0<0>(x) ^ s0;
        w[b][1] = s1 ^ rotl8(T.t2<3>(x));
        w[b][2] = s2 ^ T.t2<2>(x);
        w[b][3] = s3 ^ rotl8(T.t0<1>(x));
      }
      continue;
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) round_row(T, w[b][0], w[b][1], w[b][2], w[b][3], r0, r1, r2, r3);
  }
  if constexpr (LASTB > 0) {
    // k0 of the last round key, bytes < LASTB: k0 ^ SubWord(RotWord(k3)) ^ rcon
    uint32_t t = T.t2<1>(k3);  // byte 0 = S[k3.b1]
    if constexpr (LASTB >= 2) t = (t & 0xffu) | (T.t0<2>(k3) & 0xff00u);
    if constexpr (LASTB >= 3) t |= T.t0<3>(k3) & 0xff0000u;
    out[0] = make_uint4(last_col_b<LASTB>(T, w[0][0], w[0][1], w[0][2], k0 ^ t ^ kRcon[9]), 0, 0, 0);
    return;
  }
  key_next(T, k0, k1, k2, k3, kRcon[9]);
  const uint32_t kk[4] = {k0, k1, k2, k3};
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    uint32_t o[4] = {0, 0, 0, 0};
    const int nw = (b == NB - 1) ? LASTW : 4;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < nw) o[c] = last_col(T, w[b][c], w[b][(c + 1) & 3], w[b][(c + 2) & 3], w[b][(c + 3) & 3], kk[c]);
    out[b] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// NK independent keys in lockstep, row shape, NB CTR blocks each (counters 0..NB-1): every
// round of the NK instances is issued together, so a lane keeps NK dependent AES chains in
// flight.  For levels that are bound by AES latency rather than by LDS lookups (the tree waves
// of k_query beside the scan: 8 waves, so one chain per lane leaves the LDS mostly idle).
// Same outputs as NK calls of aes_ctr_row<NB, LASTW, LASTB>(T, key[k], out[k]).
template <int NK, int NB, int LASTW, int LASTB = 0>
__device__ __forceinline__ void aes_ctr_rowk(const Tab& T, const uint4 (&key)[NK],
                                             uint4 (&out)[NK][NB]) {
  static_assert(LASTB == 0 || (NB == 1 && LASTB < 4), "byte-trimmed: one block, 1-3 bytes");
  uint32_t k0[NK], k1[NK], k2[NK], k3[NK];
  uint32_t w[NK][NB][4];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    k0[k] = key[k].x; k1[k] = key[k].y; k2[k] = key[k].z; k3[k] = key[k].w;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      w[k][b][0] = k0[k]; w[k][b][1] = k1[k]; w[k][b][2] = k2[k];
      w[k][b][3] = k3[k] ^ ((uint32_t)b << 24);
    }
  }
#pragma unroll
  for (int r = 0; r < 9; ++r) {
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      key_next(T, k0[k], k1[k], k2[k], k3[k], kRcon[r]);
      const uint32_t r0 = rotr8(k0[k]), r1 = rotr8(k1[k]), r2 = rotr8(k2[k]), r3 = rotr8(k3[k]);
      auto& wk = w[k];
      if (r == 0) {  // as aes_ctr_row: the blocks share columns 1-3 after the first round
#pragma unroll
        for (int b = 1; b < NB; ++b)
          wk[b][0] = xor3(T.t0<0>(wk[b][0]), T.t2<2>(wk[b][2]),
                          rotl8(xor3(T.t0<1>(wk[b][1]), T.t2<3>(wk[b][3]), r0)));
        round_row(T, wk[0][0], wk[0][1], wk[0][2], wk[0][3], r0, r1, r2, r3);
#pragma unroll
        for (int b = 1; b < NB; ++b) {
          wk[b][1] = wk[0][1]; wk[b][2] = wk[0][2]; wk[b][3] = wk[0][3];
        }
      } else if (r == 1) {
        const uint32_t a1 = wk[0][1], a2 = wk[0][2], a3 = wk[0][3];
        const uint32_t s0 = T.t2<2>(a2) ^ rotl8(xor3(T.t0<1>(a1), T.t2<3>(a3), r0));
        const uint32_t s1 = xor3(T.t0<0>(a1), T.t2<2>(a3), rotl8(T.t0<1>(a2) ^ r1));
        const uint32_t s2 = T.t0<0>(a2) ^ rotl8(xor3(T.t0<1>(a3), T.t2<3>(a1), r2));
        const uint32_t s3 = xor3(T.t0<0>(a3), T.t2<2>(a1), rotl8(T.t2<3>(a2) ^ r3));
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const uint32_t x = wk[b][0];
          wk[b][0] = T.t0<0>(x) ^ s0;
          wk[b][1] = s1 ^ rotl8(T.t2<3>(x));
          wk[b][2] = s2 ^ T.t2<2>(x);
          wk[b][3] = s3 ^ rotl8(T.t0<1>(x));
        }
      } else {
#pragma unroll
        for (int b = 0; b < NB; ++b)
          round_row(T, wk[b][0], wk[b][1], wk[b][2], wk[b][3], r0, r1, r2, r3);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    if constexpr (LASTB > 0) {
      uint32_t t = T.t2<1>(k3[k]);
      if constexpr (LASTB >= 2) t = (t & 0xffu) | (T.t0<2>(k3[k]) & 0xff00u);
      if constexpr (LASTB >= 3) t |= T.t0<3>(k3[k]) & 0xff0000u;
      out[k][0] = make_uint4(
          last_col_b<LASTB>(T, w[k][0][0], w[k][0][1], w[k][0][2], k0[k] ^ t ^ kRcon[9]), 0, 0, 0);
    } else {
      key_next(T, k0[k], k1[k], k2[k], k3[k], kRcon[9]);
      const uint32_t kk[4] = {k0[k], k1[k], k2[k], k3[k]};
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        uint32_t o[4] = {0, 0, 0, 0};
        const int nw = (b == NB - 1) ? LASTW : 4;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (c < nw)
            o[c] = last_col(T, w[k][b][c], w[k][b][(c + 1) & 3], w[k][b][(c + 2) & 3],
                            w[k][b][(c + 3) & 3], kk[c]);
        out[k][b] = make_uint4(o[0], o[1], o[2], o[3]);
      }
    }
  }
}

// 20 LDS lookups as one group (the row-shape round: the key schedule's 4 + the state's 16), as
// lds_read8 below for the column shape.  `a` are LDS byte addresses.
__device__ __forceinline__ void lds_read20(uint32_t (&v)[20], const uint32_t (&a)[20]) {
  asm volatile(
      "ds_read_b32 %0, %20\n\t" "ds_read_b32 %1, %21\n\t" "ds_read_b32 %2, %22\n\t"
      "ds_read_b32 %3, %23\n\t" "ds_read_b32 %4, %24\n\t" "ds_read_b32 %5, %25\n\t"
      "ds_read_b32 %6, %26\n\t" "ds_read_b32 %7, %27\n\t" "ds_read_b32 %8, %28\n\t"
      "ds_read_b32 %9, %29\n\t" "ds_read_b32 %10, %30\n\t" "ds_read_b32 %11, %31\n\t"
      "ds_read_b32 %12, %32\n\t" "ds_read_b32 %13, %33\n\t" "ds_read_b32 %14, %34\n\t"
      "ds_read_b32 %15, %35\n\t" "ds_read_b32 %16, %36\n\t" "ds_read_b32 %17, %37\n\t"
      "ds_read_b32 %18, %38\n\t" "ds_read_b32 %19, %39\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]),
        "=&v"(v[6]), "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]),
        "=&v"(v[12]), "=&v"(v[13]), "=&v"(v[14]), "=&v"(v[15]), "=&v"(v[16]), "=&v"(v[17]),
        "=&v"(v[18]), "=&v"(v[19])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
        "v"(a[8]), "v"(a[9]), "v"(a[10]), "v"(a[11]), "v"(a[12]), "v"(a[13]), "v"(a[14]),
        "v"(a[15]), "v"(a[16]), "v"(a[17]), "v"(a[18]), "v"(a[19])
      : "memory");
}

// Row shape, one block with counter `ctr` (k_query's 3-lanes-per-node levels, key generation).
// Per round the key schedule's 4 S-box lookups (from the previous round key) and the state's
// 16 T-box lookups (from the previous state) go out as one group (lds_read20): one LDS round
// trip per round where the compiler, at k_query's register limit, issued a few at a time.
__device__ __forceinline__ uint4 aes_ctr_block(const Tab& T, uint4 key, uint32_t ctr) {
  const uint32_t lb = (uint32_t)(uintptr_t)T.base;  // LDS byte address (see aes_col)
  uint32_t k0 = key.x, k1 = key.y, k2 = key.z, k3 = key.w;
  uint32_t w[4] = {k0, k1, k2, k3 ^ (ctr << 24)};
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t p1 = k0 ^ k1, p2 = p1 ^ k2, p3 = p2 ^ k3;  // the word chain, old key
    uint32_t ad[20], v[20];
    ad[0] = lb + tab_addr<1>(k3, T.l2);  // SubWord(RotWord(k3)): S in byte 0..3
    ad[1] = lb + tab_addr<2>(k3, T.l0);
    ad[2] = lb + tab_addr<3>(k3, T.l0);
    ad[3] = lb + tab_addr<0>(k3, T.l2);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t a0 = w[c], a1 = w[(c + 1) & 3], a2 = w[(c + 2) & 3], a3 = w[(c + 3) & 3];
      if (r < 9) {  // round_row's column c
        ad[4 + 4 * c] = lb + tab_addr<0>(a0, T.l0);
        ad[5 + 4 * c] = lb + tab_addr<2>(a2, T.l2);
        ad[6 + 4 * c] = lb + tab_addr<1>(a1, T.l0);
        ad[7 + 4 * c] = lb + tab_addr<3>(a3, T.l2);
      } else {  // last_col's S-box bytes
        ad[4 + 4 * c] = lb + tab_addr<0>(a0, T.l2);
        ad[5 + 4 * c] = lb + tab_addr<1>(a1, T.l0);
        ad[6 + 4 * c] = lb + tab_addr<2>(a2, T.l0);
        ad[7 + 4 * c] = lb + tab_addr<3>(a3, T.l2);
      }
    }
    lds_read20(v, ad);
    const uint32_t t = ((v[0] & 0xffu) | (v[1] & 0xff00u) | (v[2] & 0xff0000u) |
                        (v[3] & 0xff000000u)) ^ kRcon[r];
    k0 ^= t; k1 = p1 ^ t; k2 = p2 ^ t; k3 = p3 ^ t;
    const uint32_t kk[4] = {k0, k1, k2, k3};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (r < 9)
        w[c] = xor3(v[4 + 4 * c], v[5 + 4 * c], rotl8(xor3(v[6 + 4 * c], v[7 + 4 * c], rotr8(kk[c]))));
      else
        w[c] = ((v[4 + 4 * c] & 0xffu) | (v[5 + 4 * c] & 0xff00u) | (v[6 + 4 * c] & 0xff0000u) |
                (v[7 + 4 * c] & 0xff000000u)) ^ kk[c];
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// ---- column shape: 4 lanes (a DPP quad) per block, lane q = column q ----------------------
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
constexpr int kQ1230 = 0x39;  // lane q reads q+1
constexpr int kQ2301 = 0x4E;  // q+2
constexpr int kQ3012 = 0x93;  // q+3
constexpr int kQ3333 = 0xFF;  // lane 3
constexpr int kQ0012 = 0x90;  // q-1 (lane 0 reads itself)
constexpr int kQ0101 = 0x44;  // q-2 (lanes 0,1 read themselves)

// The 8 LDS lookups of a column-shape round as ONE group (one LDS round trip): left to itself,
// the scheduler of a kernel at its register limit (k_query: 128 VGPRs) issued them as three
// dependent batches -- the state's 4, then the key schedule's 2 + 2 -- so a tile-root descent
// level took ≈3 600 cycles against ≈2 000 for the same code in a register-rich kernel
// (tools/micro/aes_col_latency.hip; the k_query disassembly).  `a` are LDS byte addresses.
__device__ __forceinline__ void lds_read8(uint32_t (&v)[8], const uint32_t (&a)[8]) {
  asm volatile(
      "ds_read_b32 %0, %8\n\t"
      "ds_read_b32 %1, %9\n\t"
      "ds_read_b32 %2, %10\n\t"
      "ds_read_b32 %3, %11\n\t"
      "ds_read_b32 %4, %12\n\t"
      "ds_read_b32 %5, %13\n\t"
      "ds_read_b32 %6, %14\n\t"
      "ds_read_b32 %7, %15\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]),
        "=&v"(v[6]), "=&v"(v[7])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7])
      : "memory");
}

// AES-128_k(pt) where lane q holds key word k_q and plaintext word pt_q; returns ciphertext
// word q.  All 4 lanes of the quad must be active.  mq1/mq2: all-ones when q >= 1 / q >= 2.
// Per round the key schedule's 4 S-box lookups (from the previous round key) and the state's 4
// T-box lookups (from the previous state) go out together (lds_read8); the schedule's prefix XOR
// (two DPP steps on the previous key) runs while they are in flight.
__device__ __forceinline__ uint32_t aes_col(const Tab& T, uint32_t kq, uint32_t ptq, uint32_t mq1,
                                            uint32_t mq2) {
  // LDS byte address of the table: the low 32 bits of the generic address (the shared
  // aperture's base has zero low bits)
  const uint32_t lb = (uint32_t)(uintptr_t)T.base;
  uint32_t w = kq ^ ptq;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // key schedule: k'_q = SubWordRot(k3) ^ rcon ^ (k_0 ^ ... ^ k_q)
    const uint32_t k3 = qperm<kQ3333>(kq);
    uint32_t pre = kq ^ (qperm<kQ0012>(kq) & mq1);
    pre ^= qperm<kQ0101>(pre) & mq2;
    const uint32_t b = qperm<kQ1230>(w), c = qperm<kQ2301>(w), d = qperm<kQ3012>(w);
    uint32_t ad[8], v[8];
    ad[0] = lb + tab_addr<1>(k3, T.l2);  // Te2[byte 1]: S in byte 0
    ad[1] = lb + tab_addr<2>(k3, T.l0);                // Te0[byte 2]: S in byte 1
    ad[2] = lb + tab_addr<3>(k3, T.l0);                // Te0[byte 3]: S in byte 2
    ad[3] = lb + tab_addr<0>(k3, T.l2);                // Te2[byte 0]: S in byte 3
    if (r < 9) {
      ad[4] = lb + tab_addr<0>(w, T.l0);
      ad[5] = lb + tab_addr<2>(c, T.l2);
      ad[6] = lb + tab_addr<1>(b, T.l0);
      ad[7] = lb + tab_addr<3>(d, T.l2);
    } else {  // last round (last_col): S-box bytes only
      ad[4] = lb + tab_addr<0>(w, T.l2);
      ad[5] = lb + tab_addr<1>(b, T.l0);
      ad[6] = lb + tab_addr<2>(c, T.l0);
      ad[7] = lb + tab_addr<3>(d, T.l2);
    }
    lds_read8(v, ad);
    const uint32_t t = (v[0] & 0xffu) | (v[1] & 0xff00u) | (v[2] & 0xff0000u) | (v[3] & 0xff000000u);
    kq = xor3(pre, t, kRcon[r]);
    if (r < 9)
      w = xor3(v[4], v[5], rotl8(xor3(v[6], v[7], rotr8(kq))));
    else
      w = ((v[4] & 0xffu) | (v[5] & 0xff00u) | (v[6] & 0xff0000u) | (v[7] & 0xff000000u)) ^ kq;
  }
  return w;
}

__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}
__device__ __forceinline__ uint4 and4(uint4 a, uint32_t m) {
  return make_uint4(a.x & m, a.y & m, a.z & m, a.w & m);
}

}  // namespace pir
