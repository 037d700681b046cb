// pir_aes.h -- AES-128 for CDNA4: the PRG G of the reference (src/c/utils.cpp:37-51) is
// AES-128-CTR keyed by each tree node's seed, so there is no fixed key schedule to amortise:
// every block runs the key schedule on the fly next to its rounds.
//
// T-table form: one 1 KiB table Te0 (Te0[x] = {2S, S, S, 3S}, S = the FIPS-197 S-box, computed
// on the host from the field definition) replicated 32x in LDS as [entry][lane & 31], so each
// lane of a 32-lane ds_read_b32 group reads its own bank (conflict-free for any index pattern).
// Te1..Te3 are byte rotations of Te0 (v_alignbit); the last round and the key schedule read
// S = byte 1 of Te0.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pir {

// Each translation unit that includes this header owns its own copy of the table.
static __constant__ uint32_t c_te0[256];

// ------------------------------------------------------------------------------------------
// AES-128 encryption of one CTR block with an on-the-fly key schedule
// ------------------------------------------------------------------------------------------
struct Te {
  const char* base;  // LDS table (byte address)
  uint32_t lane4;    // (lane & 31) * 4
  __device__ __forceinline__ uint32_t at(uint32_t off) const {
    return *reinterpret_cast<const uint32_t*>(base + (off | lane4));
  }
  // byte k of w -> offset of its Te0 row (entry stride 128 B)
  __device__ __forceinline__ uint32_t b0(uint32_t w) const { return at((w << 7) & 0x7f80u); }
  __device__ __forceinline__ uint32_t b1(uint32_t w) const { return at((w >> 1) & 0x7f80u); }
  __device__ __forceinline__ uint32_t b2(uint32_t w) const { return at((w >> 9) & 0x7f80u); }
  __device__ __forceinline__ uint32_t b3(uint32_t w) const { return at((w >> 17) & 0x7f80u); }
};

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) {
  return __builtin_amdgcn_alignbit(x, x, 32 - s);
}

// Te0[x] = {2S, S, S, 3S} (bytes 0..3); S[x] sits in byte 1.
__device__ __forceinline__ uint32_t s_at0(uint32_t te) { return (te >> 8) & 0xffu; }
__device__ __forceinline__ uint32_t s_at1(uint32_t te) { return te & 0xff00u; }
__device__ __forceinline__ uint32_t s_at2(uint32_t te) { return (te << 8) & 0xff0000u; }
__device__ __forceinline__ uint32_t s_at3(uint32_t te) { return (te << 16) & 0xff000000u; }

__device__ __forceinline__ void key_step(const Te& T, uint32_t& k0, uint32_t& k1, uint32_t& k2,
                                         uint32_t& k3, uint32_t rcon) {
  // SubWord(RotWord(k3)) ^ rcon
  uint32_t t = s_at0(T.b1(k3)) | s_at1(T.b2(k3)) | s_at2(T.b3(k3)) | s_at3(T.b0(k3));
  k0 ^= t ^ rcon;
  k1 ^= k0;
  k2 ^= k1;
  k3 ^= k2;
}

__device__ __forceinline__ void aes_round(const Te& T, uint32_t& w0, uint32_t& w1, uint32_t& w2,
                                          uint32_t& w3, uint32_t k0, uint32_t k1, uint32_t k2,
                                          uint32_t k3) {
  uint32_t n0 = T.b0(w0) ^ rotl(T.b1(w1), 8) ^ rotl(T.b2(w2), 16) ^ rotl(T.b3(w3), 24) ^ k0;
  uint32_t n1 = T.b0(w1) ^ rotl(T.b1(w2), 8) ^ rotl(T.b2(w3), 16) ^ rotl(T.b3(w0), 24) ^ k1;
  uint32_t n2 = T.b0(w2) ^ rotl(T.b1(w3), 8) ^ rotl(T.b2(w0), 16) ^ rotl(T.b3(w1), 24) ^ k2;
  uint32_t n3 = T.b0(w3) ^ rotl(T.b1(w0), 8) ^ rotl(T.b2(w1), 16) ^ rotl(T.b3(w2), 24) ^ k3;
  w0 = n0; w1 = n1; w2 = n2; w3 = n3;
}

__device__ __forceinline__ void aes_last(const Te& T, uint32_t& w0, uint32_t& w1, uint32_t& w2,
                                         uint32_t& w3, uint32_t k0, uint32_t k1, uint32_t k2,
                                         uint32_t k3) {
  uint32_t n0 = (s_at0(T.b0(w0)) | s_at1(T.b1(w1)) | s_at2(T.b2(w2)) | s_at3(T.b3(w3))) ^ k0;
  uint32_t n1 = (s_at0(T.b0(w1)) | s_at1(T.b1(w2)) | s_at2(T.b2(w3)) | s_at3(T.b3(w0))) ^ k1;
  uint32_t n2 = (s_at0(T.b0(w2)) | s_at1(T.b1(w3)) | s_at2(T.b2(w0)) | s_at3(T.b3(w1))) ^ k2;
  uint32_t n3 = (s_at0(T.b0(w3)) | s_at1(T.b1(w0)) | s_at2(T.b2(w1)) | s_at3(T.b3(w2))) ^ k3;
  w0 = n0; w1 = n1; w2 = n2; w3 = n3;
}

// AES-128_key(BE128(ctr)), ctr < 256: the ctr-th 16-byte block of G(key, .) (utils.cpp:37-51)
__device__ __forceinline__ uint4 aes_ctr_block(const Te& T, uint4 key, uint32_t ctr) {
  uint32_t k0 = key.x, k1 = key.y, k2 = key.z, k3 = key.w;
  uint32_t w0 = k0, w1 = k1, w2 = k2, w3 = k3 ^ (ctr << 24);
  constexpr uint32_t rc[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    key_step(T, k0, k1, k2, k3, rc[r]);
    aes_round(T, w0, w1, w2, w3, k0, k1, k2, k3);
  }
  key_step(T, k0, k1, k2, k3, rc[9]);
  aes_last(T, w0, w1, w2, w3, k0, k1, k2, k3);
  return make_uint4(w0, w1, w2, w3);
}

__device__ __forceinline__ void load_te_lds(uint32_t* lds_te) {
  for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x) lds_te[i] = c_te0[i >> 5];
}

__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}
__device__ __forceinline__ uint4 and4(uint4 a, uint32_t m) {
  return make_uint4(a.x & m, a.y & m, a.z & m, a.w & m);
}

// ------------------------------------------------------------------------------------------
// host: Te0 generation + upload into this translation unit's __constant__ copy
// ------------------------------------------------------------------------------------------
static inline uint8_t aes_xtime_h(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }
static inline uint8_t aes_mul_h(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = aes_xtime_h(a);
    b >>= 1;
  }
  return r;
}

static inline void upload_te0(hipStream_t s) {
  uint32_t te0[256];
  for (int x = 0; x < 256; ++x) {  // S-box = affine(x^-1) over GF(2^8)/0x11b (FIPS-197 5.1.1)
    uint8_t inv = 0;
    if (x) {
      uint8_t r = 1, b = (uint8_t)x;
      for (int e = 254; e; e >>= 1) {
        if (e & 1) r = aes_mul_h(r, b);
        b = aes_mul_h(b, b);
      }
      inv = r;
    }
    uint8_t sb = inv;
    for (int k = 1; k <= 4; ++k) sb ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
    sb ^= 0x63;
    te0[x] = (uint32_t)aes_mul_h(sb, 2) | ((uint32_t)sb << 8) | ((uint32_t)sb << 16) |
             ((uint32_t)aes_mul_h(sb, 3) << 24);
  }
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(c_te0), te0, sizeof(te0), 0, hipMemcpyHostToDevice, s);
  (void)hipStreamSynchronize(s);
}

}  // namespace pir
