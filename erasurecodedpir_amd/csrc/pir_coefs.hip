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

}  // namespace pir
