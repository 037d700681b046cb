// pir_aes4.h -- the 4-table T-box AES-128 of the depth-first leaf stage (pir_leaves.hip).
//
// pir_aes.h keeps two tables (Te0, Te2 = rotl16 Te0; 64 KiB replicated) and rotates the other
// two into place: a round column costs 4 address v_perm + 1 v_alignbit + 2 v_bitop3, and each
// round key word one more v_alignbit.  A kernel that holds nothing else in LDS can afford all
// four tables (128 KiB at 32x replication, one 1024-thread workgroup per CU), and a column is
//     Te0[a] ^ Te1[b] ^ Te2[c] ^ Te3[d] ^ k   -- 4 v_perm + 2 v_bitop3, no rotation at all.
// Te1 = rotl8 Te0, Te3 = rotl8 Te2 (FIPS-197 5.2.1's T-box identities).
//
// LDS layout: region A = bytes [0, 64 KiB): row e (256 B) = 32 copies of Te0[e], 32 of Te2[e]
// (the pir_aes.h layout); region B = [64 KiB, 128 KiB): the same rows of Te1 and Te3.  A
// lookup address is ONE v_perm: index byte -> address byte 1, the per-lane constant
// (lane & 31) * 4 (+128 for the second table of a row, +64 KiB for region B) -> bytes 0 and 2.
// Every lane of a 32-lane ds_read_b32 group reads its own bank for any index pattern.
//
// Byte-trimmed outputs: the control-bit block of an internal node needs 1-4 bytes (2(p-1)
// bits) and a leaf block nq bytes; only those last-round S-box lookups are issued, and the
// compiler drops the ninth-round columns nothing reads (LASTB < 4: columns >= LASTB).
#pragma once
#include "pir_aes.h"

namespace pir {

constexpr uint32_t kTab4Bytes = 4 * kTeBytes;  // 128 KiB

struct Tab4 {
  const char* base;
  uint32_t l0, l2, l1, l3;  // lane parts of Te0, Te2 (region A) and Te1, Te3 (region B)
  __device__ __forceinline__ explicit Tab4(const void* lds)
      : base(reinterpret_cast<const char*>(lds)),
        l0((threadIdx.x & 31u) * 4u),
        l2(l0 | 128u),
        l1(l0 | 0x10000u),
        l3(l0 | 0x10080u) {}
  template <int K, bool B>
  __device__ __forceinline__ uint32_t look(uint32_t w, uint32_t lp) const {
    // byte 0 = lane part byte 0, byte 1 = byte K of w, byte 2 = lane part byte 2 (region B)
    constexpr uint32_t sel = (B ? 0x0c020000u : 0x0c0c0000u) | ((4u + K) << 8);
    return *reinterpret_cast<const uint32_t*>(base + __builtin_amdgcn_perm(w, lp, sel));
  }
  template <int K> __device__ __forceinline__ uint32_t t0(uint32_t w) const { return look<K, false>(w, l0); }
  template <int K> __device__ __forceinline__ uint32_t t2(uint32_t w) const { return look<K, false>(w, l2); }
  template <int K> __device__ __forceinline__ uint32_t t1(uint32_t w) const { return look<K, true>(w, l1); }
  template <int K> __device__ __forceinline__ uint32_t t3(uint32_t w) const { return look<K, true>(w, l3); }
};

// fill all four tables; a block of exactly NT threads (NT a multiple of 64 dividing 16384)
template <int NT>
__device__ __forceinline__ void load_tables4_n(uint32_t* lds) {
  constexpr int K = 256 * 64 / NT;
  static_assert(256 * 64 % NT == 0, "block size");
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = c_te0.v[wv + k * (NT / 64)];  // row e = wave-uniform
  const bool hi = threadIdx.x & 32;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t x = v[k];
    lds[threadIdx.x + k * NT] = hi ? __builtin_amdgcn_alignbit(x, x, 16) : x;            // Te2 : Te0
    lds[16384 + threadIdx.x + k * NT] =
        hi ? __builtin_amdgcn_alignbit(x, x, 8) : __builtin_amdgcn_alignbit(x, x, 24);   // Te3 : Te1
  }
}

// one state column: Te0[a.b0] ^ Te1[b.b1] ^ Te2[c.b2] ^ Te3[d.b3] ^ k
__device__ __forceinline__ uint32_t col4(const Tab4& T, uint32_t a, uint32_t b, uint32_t c,
                                         uint32_t d, uint32_t k) {
  return xor3(xor3(T.t0<0>(a), T.t1<1>(b), T.t2<2>(c)), T.t3<3>(d), k);
}

// the S-box bytes of a last-round column (SubBytes + ShiftRows) before AddRoundKey; S sits in
// byte 0 of Te2, bytes 1-2 of Te0, byte 3 of Te2; two byte merges by v_perm.  NB bytes (1-4).
template <int NB>
__device__ __forceinline__ uint32_t sub_col4(const Tab4& T, uint32_t a, uint32_t b, uint32_t c,
                                             uint32_t d) {
  if constexpr (NB == 1) return T.t2<0>(a);  // bytes 1-3: don't care
  const uint32_t lo = __builtin_amdgcn_perm(T.t0<1>(b), T.t2<0>(a), 0x0c0c0500u);
  if constexpr (NB == 2) return lo;
  if constexpr (NB == 3) return lo ^ (T.t0<2>(c) & 0x00ff0000u);
  const uint32_t hi = __builtin_amdgcn_perm(T.t2<3>(d), T.t0<2>(c), 0x07020c0cu);
  return lo ^ hi;  // disjoint bytes: the caller's ^ k makes one v_bitop3
}

// the next round key (FIPS-197 5.2): k0 ^= SubWord(RotWord(k3)) ^ rcon, then the word chain
__device__ __forceinline__ void key_next4(const Tab4& T, uint32_t& k0, uint32_t& k1, uint32_t& k2,
                                          uint32_t& k3, uint32_t rcon) {
  // SubWord(RotWord(k3)) = [S(k3.b1), S(k3.b2), S(k3.b3), S(k3.b0)] = sub_col4 of (k3 >> 8 ...)
  const uint32_t lo = __builtin_amdgcn_perm(T.t0<2>(k3), T.t2<1>(k3), 0x0c0c0500u);
  const uint32_t hi = __builtin_amdgcn_perm(T.t2<0>(k3), T.t0<3>(k3), 0x07020c0cu);
  k0 = xor3(k0, lo ^ rcon, hi);
  k1 ^= k0;
  k2 ^= k1;
  k3 ^= k2;
}
// the last round key's word 0, NB bytes (the rest: don't care)
template <int NB>
__device__ __forceinline__ uint32_t key_last0(const Tab4& T, uint32_t k0, uint32_t k3,
                                              uint32_t rcon) {
  if constexpr (NB == 1) return k0 ^ T.t2<1>(k3) ^ rcon;
  const uint32_t lo = __builtin_amdgcn_perm(T.t0<2>(k3), T.t2<1>(k3), 0x0c0c0500u);
  if constexpr (NB == 2) return k0 ^ lo ^ rcon;
  const uint32_t hi = __builtin_amdgcn_perm(T.t2<0>(k3), T.t0<3>(k3), 0x07020c0cu);
  return xor3(k0, lo ^ rcon, hi);
}

__device__ __forceinline__ void round4(const Tab4& T, uint32_t (&w)[4], uint32_t k0, uint32_t k1,
                                       uint32_t k2, uint32_t k3) {
  const uint32_t n0 = col4(T, w[0], w[1], w[2], w[3], k0);
  const uint32_t n1 = col4(T, w[1], w[2], w[3], w[0], k1);
  const uint32_t n2 = col4(T, w[2], w[3], w[0], w[1], k2);
  const uint32_t n3 = col4(T, w[3], w[0], w[1], w[2], k3);
  w[0] = n0; w[1] = n1; w[2] = n2; w[3] = n3;
}

// Row shape, one key, NB CTR blocks with counters 0..NB-1 (BE128: byte 15); out[b] =
// AES_key(BE128(b)); of block NB-1 only the first LASTB bytes are valid (LASTB >= 16: all).
// Same results as pir_aes.h's aes_ctr_row<NB, *> on the valid bytes.
template <int NB, int LASTB>
__device__ __forceinline__ void aes_ctr_row4(const Tab4& T, uint4 key, uint4 (&out)[NB]) {
  static_assert(NB >= 1 && NB <= 4 && LASTB >= 1, "shape");
  uint32_t k0 = key.x, k1 = key.y, k2 = key.z, k3 = key.w;
  uint32_t w[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    w[b][0] = k0; w[b][1] = k1; w[b][2] = k2; w[b][3] = k3 ^ ((uint32_t)b << 24);
  }
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    key_next4(T, k0, k1, k2, k3, kRcon[r]);
    if (r == 0 && NB > 1) {
      // the blocks differ only in byte 15 (the counter), which only output column 0 reads
#pragma unroll
      for (int b = 1; b < NB; ++b) w[b][0] = col4(T, w[b][0], w[b][1], w[b][2], w[b][3], k0);
      round4(T, w[0], k0, k1, k2, k3);
#pragma unroll
      for (int b = 1; b < NB; ++b) {
        w[b][1] = w[0][1]; w[b][2] = w[0][2]; w[b][3] = w[0][3];
      }
      continue;
    }
    if (r == 1 && NB > 1) {
      // the blocks still share columns 1-3 (a1..a3): 3 lookups per output column are shared,
      // the fourth reads the block's own column 0 (x)
      const uint32_t a1 = w[0][1], a2 = w[0][2], a3 = w[0][3];
      const uint32_t s0 = xor3(T.t1<1>(a1), T.t2<2>(a2), T.t3<3>(a3) ^ k0);
      const uint32_t s1 = xor3(T.t0<0>(a1), T.t1<1>(a2), T.t2<2>(a3) ^ k1);
      const uint32_t s2 = xor3(T.t0<0>(a2), T.t1<1>(a3), T.t3<3>(a1) ^ k2);
      const uint32_t s3 = xor3(T.t0<0>(a3), T.t2<2>(a1), T.t3<3>(a2) ^ k3);
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const uint32_t x = w[b][0];
        w[b][0] = s0 ^ T.t0<0>(x);
        w[b][1] = s1 ^ T.t3<3>(x);
        w[b][2] = s2 ^ T.t2<2>(x);
        w[b][3] = s3 ^ T.t1<1>(x);
      }
      continue;
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) round4(T, w[b], k0, k1, k2, k3);
  }
  if constexpr (NB == 1 && LASTB < 4) {  // one word of one block: trimmed last key word
    const uint32_t kl = key_last0<LASTB>(T, k0, k3, kRcon[9]);
    out[0] = make_uint4(sub_col4<LASTB>(T, w[0][0], w[0][1], w[0][2], w[0][3]) ^ kl, 0, 0, 0);
    return;
  }
  key_next4(T, k0, k1, k2, k3, kRcon[9]);
  const uint32_t kk[4] = {k0, k1, k2, k3};
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    uint32_t o[4] = {0, 0, 0, 0};
    const int nbytes = (b == NB - 1) ? (LASTB < 16 ? LASTB : 16) : 16;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t a = w[b][c], bb = w[b][(c + 1) & 3], cc = w[b][(c + 2) & 3], d = w[b][(c + 3) & 3];
      if (4 * c + 4 <= nbytes) o[c] = sub_col4<4>(T, a, bb, cc, d) ^ kk[c];
      else if (4 * c + 3 == nbytes) o[c] = sub_col4<3>(T, a, bb, cc, d) ^ kk[c];
      else if (4 * c + 2 == nbytes) o[c] = sub_col4<2>(T, a, bb, cc, d) ^ kk[c];
      else if (4 * c + 1 == nbytes) o[c] = sub_col4<1>(T, a, bb, cc, d) ^ kk[c];
    }
    out[b] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

}  // namespace pir
