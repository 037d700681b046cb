// pir_coefs.hip -- the coefficient layout step of explicit-coefficient answers (pir_coefs.h).
// Round-major vectors (what the client sends: key[k][i], server.cpp:337) become record-major
// share bytes (what k_scan reads per record).  Reads are coalesced along i for each round; each
// lane writes its record's nrp bytes (one 1/2/4/8/16-byte store).  HBM-bound: nq + nrp bytes
// per record, against the record_bytes of shard the scan then reads.
#include "pir_coefs.h"

#include <algorithm>

namespace pir {

template <int NRP>
__global__ __launch_bounds__(256) void k_interleave_coefs(const uint8_t* __restrict__ src,
                                                          uint64_t pitch, uint64_t nrows, int nq,
                                                          uint8_t* __restrict__ dst) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrows;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t b[NRP];
#pragma unroll
    for (int a = 0; a < NRP; ++a) b[a] = a < nq ? src[(uint64_t)a * pitch + i] : 0;
    if constexpr (NRP == 1) {
      dst[i] = b[0];
    } else if constexpr (NRP == 2) {
      reinterpret_cast<uint16_t*>(dst)[i] = (uint16_t)(b[0] | (b[1] << 8));
    } else {
      uint32_t w[NRP / 4];
#pragma unroll
      for (int k = 0; k < NRP / 4; ++k)
        w[k] = b[4 * k] | (b[4 * k + 1] << 8) | (b[4 * k + 2] << 16) | ((uint32_t)b[4 * k + 3] << 24);
      if constexpr (NRP == 4) reinterpret_cast<uint32_t*>(dst)[i] = w[0];
      else if constexpr (NRP == 8) reinterpret_cast<uint2*>(dst)[i] = make_uint2(w[0], w[1]);
      else reinterpret_cast<uint4*>(dst)[i] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

hipError_t launch_interleave_coefs(const uint8_t* src, uint64_t src_pitch, uint64_t nrows, int nq,
                                   int nrp, uint8_t* d_c, hipStream_t s) {
  if (nrows == 0) return hipSuccess;
  const dim3 grid((unsigned)std::min<uint64_t>((nrows + 255) / 256, 1u << 16));
#define PIR_IL(N) hipLaunchKernelGGL(k_interleave_coefs<N>, grid, dim3(256), 0, s, src, src_pitch, nrows, nq, d_c)
  switch (nrp) {
    case 1: PIR_IL(1); break;
    case 2: PIR_IL(2); break;
    case 4: PIR_IL(4); break;
    case 8: PIR_IL(8); break;
    case 16: PIR_IL(16); break;
    default: return hipErrorInvalidValue;
  }
#undef PIR_IL
  return hipGetLastError();
}

// ---- k_encode_within: the Hollanti-mode shard on the GPU ------------------------------------
// One lane per 16-byte chunk of an encoded row; the k coefficients gf_pow(party, j) are
// wave-uniform (scalar branches over their bits, x * alpha^b by xtime, poly 0x11d).
struct WithinCoefs {
  uint8_t c[16];
};

__device__ __forceinline__ uint32_t xtime4_w(uint32_t x) {
  return ((x & 0x7f7f7f7fu) << 1) ^ (((x >> 7) & 0x01010101u) * 0x1du);
}

__device__ __forceinline__ uint4 gf_mul_const4_w(uint4 x, uint32_t c) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int b = 0; b < 8; ++b) {
    if (c & (1u << b)) acc = make_uint4(acc.x ^ x.x, acc.y ^ x.y, acc.z ^ x.z, acc.w ^ x.w);
    x = make_uint4(xtime4_w(x.x), xtime4_w(x.y), xtime4_w(x.z), xtime4_w(x.w));
  }
  return acc;
}

// bytes [off, off + 4) of file v, zero at or past fbytes (synthetic database, client.cpp:16-33)
__device__ __forceinline__ uint32_t synth_word_w(uint64_t v, uint32_t off, uint32_t fbytes) {
  uint32_t w = 0;
  for (uint32_t t = 0; t < 4; ++t)
    if (off + t < fbytes) w |= (v == 1 ? ((off + t) & 0xffu) : (uint32_t)(v & 0xffu)) << (8 * t);
  return w;
}

__global__ __launch_bounds__(256) void k_encode_within(
    const uint8_t* __restrict__ files, uint64_t fpitch, uint64_t nfiles, uint32_t fbytes, int k,
    WithinCoefs co, uint8_t* __restrict__ shard, uint64_t rows, uint64_t row0, uint32_t pitch,
    uint32_t efs) {
  const uint32_t cpr = pitch / 16;
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < rows * cpr;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = idx / cpr;
    const uint32_t ch = (uint32_t)(idx - r * cpr);
    const uint64_t gr = row0 + r;  // file gr
    uint4 acc = make_uint4(0, 0, 0, 0);
    if (gr < nfiles && ch * 16u < efs) {
      for (int j = 0; j < k; ++j) {
        const uint32_t off = (uint32_t)j * efs + ch * 16u;  // byte offset in the file
        if (off >= fbytes) break;
        uint32_t w[4];
        for (int t = 0; t < 4; ++t) {
          const uint32_t o = off + 4u * t;
          if (files) {
            uint32_t v = 0;
            const uint8_t* f = files + gr * fpitch;
            for (uint32_t u = 0; u < 4; ++u)
              if (o + u < fbytes && ch * 16u + 4u * t + u < efs) v |= (uint32_t)f[o + u] << (8 * u);
            w[t] = v;
          } else {
            w[t] = synth_word_w(gr, o, fbytes);
          }
        }
        const uint4 m = gf_mul_const4_w(make_uint4(w[0], w[1], w[2], w[3]), co.c[j]);
        acc = make_uint4(acc.x ^ m.x, acc.y ^ m.y, acc.z ^ m.z, acc.w ^ m.w);
      }
    }
    uint32_t o[4] = {acc.x, acc.y, acc.z, acc.w};
    for (int t = 0; t < 16; ++t)  // bytes of a part past efs (the row's pad): zero
      if (ch * 16u + t >= efs) o[t >> 2] &= ~(0xffu << (8 * (t & 3)));
    *reinterpret_cast<uint4*>(shard + r * pitch + ch * 16u) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

hipError_t launch_encode_within(const uint8_t* d_files, uint64_t file_pitch, uint64_t num_files,
                                uint32_t file_bytes, int k, int party, uint8_t* d_shard,
                                uint64_t rows, uint64_t row0, uint32_t pitch, uint32_t efs,
                                hipStream_t s) {
  if (k < 1 || k > 16 || pitch % 16 != 0 || efs > pitch) return hipErrorInvalidValue;
  WithinCoefs co{};
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
  const uint64_t total = rows * (pitch / 16);
  const dim3 grid((unsigned)std::min<uint64_t>((total + 255) / 256, 1u << 16));
  hipLaunchKernelGGL(k_encode_within, grid, dim3(256), 0, s, d_files, file_pitch, num_files,
                     file_bytes, k, co, d_shard, rows, row0, pitch, efs);
  return hipGetLastError();
}

}  // namespace pir
