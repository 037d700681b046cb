// pir_coefs.h -- internal: explicit-coefficient answers (the Hollanti/Goldberg polynomial-PIR
// server scan, src/c/server.cpp:321-382).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pir {

// d_c[i * nrp + a] = a < nq ? src[a * src_pitch + i] : 0 for i < nrows: the client's per-round
// coefficient vectors (one row of N bytes per round) interleaved into the record-major share
// layout the GF(2^8) scan kernels read (coefficient bytes of record i at d_c + i * nrp)
hipError_t launch_interleave_coefs(const uint8_t* src, uint64_t src_pitch, uint64_t nrows, int nq,
                                   int nrp, uint8_t* d_c, hipStream_t s);

}  // namespace pir
