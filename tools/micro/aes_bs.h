// aes_bs.h -- the table-free, bitsliced AES-128-CTR of the micro-benchmarks (not part of the
// product): aes_bitsliced.hip measures it alone and against the T-table AES, aes_hybrid.hip
// beside the T-table AES on the same CU.  Layout ("DPP quad"): a quad of 4
// lanes holds 32 nodes; lane q holds COLUMN q of each node's state and round key as 32
// bit-planes (plane 8r + i = bit i of row r; bit j of a plane = node j).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

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
