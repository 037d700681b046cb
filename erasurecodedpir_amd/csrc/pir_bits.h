// pir_bits.h -- bit-matrix transposes of the transposed four-Russians scan (pir_scan_t.hip).
// Plain integer code, host and device (tools/test_bits.cpp checks it on the CPU).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PIR_HD __host__ __device__ __forceinline__
#else
#define PIR_HD inline
#endif

namespace pir {

// swap the off-diagonal S x S blocks of rows a (block row 0) and b (block row 1): positions p
// with (p & S) == 0 are selected by m
template <int S>
PIR_HD void bit_swap(uint32_t& a, uint32_t& b, uint32_t m) {
  const uint32_t t = ((a >> S) ^ b) & m;
  b ^= t;
  a ^= t << S;
}

// 8 rows x 32 bits -> 32 bytes: afterwards byte i of x[k] holds bit (8i + k) of the original
// rows, row r in bit r (four independent 8 x 8 transposes, one per byte column)
PIR_HD void transpose8x32(uint32_t (&x)[8]) {
  bit_swap<4>(x[0], x[4], 0x0F0F0F0Fu); bit_swap<4>(x[1], x[5], 0x0F0F0F0Fu);
  bit_swap<4>(x[2], x[6], 0x0F0F0F0Fu); bit_swap<4>(x[3], x[7], 0x0F0F0F0Fu);
  bit_swap<2>(x[0], x[2], 0x33333333u); bit_swap<2>(x[1], x[3], 0x33333333u);
  bit_swap<2>(x[4], x[6], 0x33333333u); bit_swap<2>(x[5], x[7], 0x33333333u);
  bit_swap<1>(x[0], x[1], 0x55555555u); bit_swap<1>(x[2], x[3], 0x55555555u);
  bit_swap<1>(x[4], x[5], 0x55555555u); bit_swap<1>(x[6], x[7], 0x55555555u);
}

// 32 x 32 bits in place: afterwards bit j of a[p] = bit p of the original a[j]
PIR_HD void transpose32(uint32_t (&a)[32]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) bit_swap<16>(a[k], a[k + 16], 0x0000FFFFu);
#pragma unroll
  for (int k = 0; k < 32; ++k)
    if (!(k & 8)) bit_swap<8>(a[k], a[k + 8], 0x00FF00FFu);
#pragma unroll
  for (int k = 0; k < 32; ++k)
    if (!(k & 4)) bit_swap<4>(a[k], a[k + 4], 0x0F0F0F0Fu);
#pragma unroll
  for (int k = 0; k < 32; ++k)
    if (!(k & 2)) bit_swap<2>(a[k], a[k + 2], 0x33333333u);
#pragma unroll
  for (int k = 0; k < 32; ++k)
    if (!(k & 1)) bit_swap<1>(a[k], a[k + 1], 0x55555555u);
}

}  // namespace pir
