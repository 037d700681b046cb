// pir_client.hip -- client side: DPF key generation on the GPU (include/pir_client.h).
//
// genOptimizedDPF (dpf_tree.cpp:142-274) walks the p parties' seeds down the path of `index`:
// at each level every party's node is expanded (3 AES-CTR blocks = 3 lanes), the correction
// words are formed from the LOSE children, and each party keeps its KEEP child corrected by
// the CWs its control bits select.  One 64-lane workgroup: 3p <= 51 lanes expand, lane 0
// forms the CWs, every lane writes key bytes.
#include <stdio.h>
#include <string.h>

#include "../../include/pir_client.h"
#include "../../include/pir_engine.h"
#include "pir_aes.h"

namespace pir {
namespace {

struct KeygenSmem {
  uint32_t tab[2 * 256 * 32];
  uint4 s[PIR_MAX_PARTIES];
  uint32_t t[PIR_MAX_PARTIES];
  uint4 out[PIR_MAX_PARTIES][3];
  uint4 scw[PIR_MAX_PARTIES];
  uint32_t tcw[PIR_MAX_PARTIES];
};

__device__ inline uint4 load_seed(const uint8_t* b) {
  uint32_t w[4];
  for (int i = 0; i < 4; ++i)
    w[i] = b[4 * i] | (b[4 * i + 1] << 8) | (b[4 * i + 2] << 16) | ((uint32_t)b[4 * i + 3] << 24);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ inline uint8_t byte_of(const uint4& v, int i) {
  const uint32_t w = i < 4 ? v.x : (i < 8 ? v.y : (i < 12 ? v.z : v.w));
  return (uint8_t)(w >> (8 * (i & 3)));
}

__global__ __launch_bounds__(64) void k_keygen(int n, uint64_t index, const uint8_t* __restrict__ fcw,
                                               int p, int nq, const uint8_t* __restrict__ seeds,
                                               uint8_t* __restrict__ keys, int kl) {
  __shared__ KeygenSmem sm;
  load_tables(sm.tab);
  const Tab T(sm.tab);
  const int tid = threadIdx.x, pm1 = p - 1, CWk = 16 + 2 * p - 2, CW = pm1 * CWk;
  const uint32_t tbits = 2 * pm1;
  const uint32_t tb_mask = tbits >= 32 ? 0xffffffffu : ((1u << tbits) - 1u);
  const uint32_t tmask = (1u << pm1) - 1u;
  if (tid < p) {
    sm.s[tid] = load_seed(seeds + 16 * tid);
    sm.t[tid] = tid >= 1 ? (1u << (tid - 1)) : 0u;  // dpf_tree.cpp:154-163
  }
  for (int i = tid; i < p * 16; i += blockDim.x) keys[(size_t)(i >> 4) * kl + (i & 15)] = seeds[i];
  __syncthreads();
  for (int L = 1; L <= n; ++L) {
    if (tid < 3 * p) {  // G(s[j]) for every party (dpf_tree.cpp:172-179)
      const int j = tid / 3, r = tid - 3 * j;
      sm.out[j][r] = aes_ctr_block(T, sm.s[j], (uint32_t)r);
    }
    __syncthreads();
    if (tid == 0) {
      const uint32_t bit = (uint32_t)((index >> (n - L)) & 1u);  // getbit(index, n, L)
      const int KEEP = (int)bit, LOSE = 1 - (int)bit;
      const uint32_t t0 = sm.out[0][2].x & tb_mask;
      for (int j = 0; j < pm1; ++j) {  // dpf_tree.cpp:189-204
        sm.scw[j] = xor4(sm.out[0][LOSE], sm.out[j + 1][LOSE]);
        const uint32_t tj = sm.out[j + 1][2].x & tb_mask;
        uint32_t m = (t0 ^ tj) & tb_mask;
        m ^= ((bit ^ 1u) << j) | (bit << (pm1 + j));
        sm.tcw[j] = m;
      }
      for (int b = 0; b < p; ++b) {  // dpf_tree.cpp:215-235
        uint4 ns = sm.out[b][KEEP];
        uint32_t nt = ((sm.out[b][2].x & tb_mask) >> (KEEP * pm1)) & tmask;
        for (int k = 0; k < pm1; ++k)
          if ((sm.t[b] >> k) & 1u) {
            ns = xor4(ns, sm.scw[k]);
            nt ^= (sm.tcw[k] >> (KEEP * pm1)) & tmask;
          }
        sm.s[b] = ns;
        sm.t[b] = nt;
      }
    }
    __syncthreads();
    // key bytes of this level for every party (dpf_tree.cpp:204-212, :254-262)
    for (int i = tid; i < p * CW; i += blockDim.x) {
      const int q = i / CW, o = i - q * CW, j = o / CWk, b = o - j * CWk;
      const uint8_t v = b < 16 ? byte_of(sm.scw[j], b) : (uint8_t)((sm.tcw[j] >> (b - 16)) & 1u);
      keys[(size_t)q * kl + 16 + (size_t)(L - 1) * CW + o] = v;
    }
    __syncthreads();
  }
  if (tid < p) sm.out[tid][0] = aes_ctr_block(T, sm.s[tid], 0u);  // convert (dpf_tree.cpp:238-244)
  __syncthreads();
  for (int i = tid; i < p * nq * pm1; i += blockDim.x) {  // lastCW (dpf_tree.cpp:246-251)
    const int q = i / (nq * pm1), o = i - q * (nq * pm1), a = o / pm1, j = o - a * pm1 + 1;
    const uint8_t v = fcw[a * pm1 + j - 1] ^ byte_of(sm.out[0][0], a) ^ byte_of(sm.out[j][0], a);
    keys[(size_t)q * kl + 16 + (size_t)n * CW + o] = v;
  }
}

uint8_t gf_mul_h(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1d : 0));
    b >>= 1;
  }
  return r;
}

}  // namespace
}  // namespace pir

extern "C" {

void pir_final_cw(int p, int nq, int rho, uint8_t* out) {
  for (int a = 1; a <= nq; ++a)
    for (int j = 2; j <= p; ++j) {
      uint8_t r = 1;  // gf_pow(j, rho*a) with the exponent taken mod 256 as uint8_t (coding.cpp:46)
      const int e = (rho * a) & 0xff;
      for (int k = 0; k < e; ++k) r = pir::gf_mul_h(r, (uint8_t)j);
      out[(a - 1) * (p - 1) + (j - 2)] = (uint8_t)(r ^ 1);
    }
}

int pir_gen_keys(int device, int n, uint64_t index, const uint8_t* fcw, int p, int nq,
                 const uint8_t* root_seeds, uint8_t* keys_out) {
  if (!fcw || !root_seeds || !keys_out || p < 2 || p > PIR_MAX_PARTIES || nq < 1 ||
      nq > PIR_MAX_ROUNDS || n < 0 || n > PIR_MAX_LOG_RECORDS || (n < 64 && (index >> n) != 0))
    return PIR_EINVAL;
  const int kl = pir_engine_key_len(p, n, nq);
  if (hipSetDevice(device) != hipSuccess) return PIR_EHIP;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return PIR_EHIP;
  uint8_t *d_fcw = nullptr, *d_seeds = nullptr, *d_keys = nullptr;
  int rc = PIR_OK;
  if (hipMalloc(&d_fcw, (size_t)nq * (p - 1)) != hipSuccess ||
      hipMalloc(&d_seeds, (size_t)p * 16) != hipSuccess ||
      hipMalloc(&d_keys, (size_t)p * kl) != hipSuccess) {
    rc = PIR_ENOMEM;
  } else if (hipMemcpyAsync(d_fcw, fcw, (size_t)nq * (p - 1), hipMemcpyHostToDevice, s) != hipSuccess ||
             hipMemcpyAsync(d_seeds, root_seeds, (size_t)p * 16, hipMemcpyHostToDevice, s) != hipSuccess) {
    rc = PIR_EHIP;
  } else {
    hipLaunchKernelGGL(pir::k_keygen, dim3(1), dim3(64), 0, s, n, index, d_fcw, p, nq, d_seeds,
                       d_keys, kl);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(keys_out, d_keys, (size_t)p * kl, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      rc = PIR_EHIP;
  }
  if (d_fcw) (void)hipFree(d_fcw);
  if (d_seeds) (void)hipFree(d_seeds);
  if (d_keys) (void)hipFree(d_keys);
  (void)hipStreamDestroy(s);
  return rc;
}

}  // extern "C"
