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

// The Hollanti-mode shard, encoded within files on the GPU (client.cpp:43-56, 99-103; the
// shim's encode_within_files_server): row r (file r, r < num_files; rows past are zero) =
// XOR_{j<k} gf_pow(party, j) * part j of file r, part j = bytes [j*efs, (j+1)*efs) of the
// file zero-padded past file_bytes.  d_files: num_files rows file_pitch apart, or nullptr for
// the reference's synthetic database (client.cpp:16-33: file v = the byte v & 0xff, file 1 =
// 0, 1, 2, ...).  Rows [row0, row0 + rows) of the global encoded database.
hipError_t launch_encode_within(const uint8_t* d_files, uint64_t file_pitch, uint64_t num_files,
                                uint32_t file_bytes, int k, int party, uint8_t* d_shard,
                                uint64_t rows, uint64_t row0, uint32_t pitch, uint32_t efs,
                                hipStream_t s);

}  // namespace pir
