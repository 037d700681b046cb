// Micro-benchmark (not part of the product): how long ONE dependent AES SubWord (the S-box on
// the 4 bytes of a dword) takes for a single wave, through the LDS table k_query uses against
// register-resident (table-free) forms -- the question of VERDICT r05 item 3: can a register
// S-box shorten the tile-root descent's per-level chain (10 dependent AES rounds, each waiting on
// its S-box lookups; pir_aes.h aes_col)?
//   lds   : 4 ds_read_b32 of the replicated Te0 table (one v_perm address each), S bytes merged
//           -- the lookup k_query's column round does (its 8 lookups go out as one group)
//   reg1  : the S-box as 64 dwords in VGPRs of every lane: 32 v_perm (8-entry byte lookups on
//           register pairs, selector = low 3 bits) and a 5-level per-byte mux on bits 3-7
//   reg4  : the same split over a DPP quad: lane j holds S-box quarter j (16 dwords), 8 v_perm,
//           a 3-level mux, a quarter mask, then an XOR all-reduce of the quad (2 DPP)
// Each variant is checked against the S-box on the host for every byte value.  Output: shader
// cycles (s_memtime) per dependent SubWord, one wave per CU, the other waves idle.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o aes_sbox_latency aes_sbox_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <algorithm>

static uint8_t xt(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }
static uint8_t mul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = xt(a);
    b >>= 1;
  }
  return r;
}
static void make_sbox(uint8_t* s) {
  for (int x = 0; x < 256; ++x) {
    uint8_t inv = 0;
    if (x) {
      uint8_t r = 1, b = (uint8_t)x;
      for (int e = 254; e; e >>= 1) {
        if (e & 1) r = mul(r, b);
        b = mul(b, b);
      }
      inv = r;
    }
    uint8_t sb = inv;
    for (int k = 1; k <= 4; ++k) sb ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
    s[x] = sb ^ 0x63;
  }
}

// per-byte 0x00 / 0xff mask from bit k of each byte of x
template <int K>
__device__ __forceinline__ uint32_t bytemask(uint32_t x) {
  const uint32_t t = (x << (7 - K)) & 0x80808080u;
  return t | (t - (t >> 7));
}
__device__ __forceinline__ uint32_t sel(uint32_t m, uint32_t a, uint32_t b) {  // m ? a : b per bit
  return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);  // TTBL index = S0*4 + S1*2 + S2
}

// 8-entry byte lookups of the 4 bytes of x (selector = low 3 bits) in each of P register pairs
template <int P>
__device__ __forceinline__ void perm8(const uint32_t* t, uint32_t s3, uint32_t* o) {
#pragma unroll
  for (int p = 0; p < P; ++p) o[p] = __builtin_amdgcn_perm(t[2 * p + 1], t[2 * p], s3);
}

__device__ __forceinline__ uint32_t sub_reg1(const uint32_t (&t)[64], uint32_t x) {
  uint32_t o[32];
  perm8<32>(t, x & 0x07070707u, o);
  const uint32_t m3 = bytemask<3>(x), m4 = bytemask<4>(x), m5 = bytemask<5>(x),
                 m6 = bytemask<6>(x), m7 = bytemask<7>(x);
#pragma unroll
  for (int i = 0; i < 16; ++i) o[i] = sel(m3, o[2 * i + 1], o[2 * i]);
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = sel(m4, o[2 * i + 1], o[2 * i]);
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = sel(m5, o[2 * i + 1], o[2 * i]);
#pragma unroll
  for (int i = 0; i < 2; ++i) o[i] = sel(m6, o[2 * i + 1], o[2 * i]);
  return sel(m7, o[1], o[0]);
}

template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}

// lane j of a quad holds S-box entries [64 j, 64 j + 64) as 16 dwords
__device__ __forceinline__ uint32_t sub_reg4(const uint32_t (&t)[16], uint32_t x, uint32_t jbits) {
  uint32_t o[8];
  perm8<8>(t, x & 0x07070707u, o);
  const uint32_t m3 = bytemask<3>(x), m4 = bytemask<4>(x), m5 = bytemask<5>(x);
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = sel(m3, o[2 * i + 1], o[2 * i]);
#pragma unroll
  for (int i = 0; i < 2; ++i) o[i] = sel(m4, o[2 * i + 1], o[2 * i]);
  uint32_t r = sel(m5, o[1], o[0]);
  // keep the bytes whose bits 6-7 name this lane's quarter (jbits = j << 6 in every byte)
  const uint32_t d = (x & 0xc0c0c0c0u) ^ jbits;          // 0 in bits 6-7 where it matches
  const uint32_t hit = (d | (d << 1)) & 0x80808080u;      // bit 7 set where it does not
  const uint32_t mk = hit | (hit - (hit >> 7));           // 0xff where it does not
  r &= ~mk;
  r ^= qperm<0xB1>(r);  // [1,0,3,2]
  r ^= qperm<0x4E>(r);  // [2,3,0,1]
  return r;
}

// the LDS form: Te0 replicated 32x ([e][lane & 31]), S(x) = byte 1 of Te0[x]
__device__ __forceinline__ uint32_t sub_lds(uint32_t lb, uint32_t lane_part, uint32_t x) {
  uint32_t a[4], v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)  // address = (byte k of x) << 7 | lane_part (32 lanes x 4 B)
    a[k] = lb + ((((x >> (8 * k)) & 0xffu) << 7) | lane_part);
  asm volatile(
      "ds_read_b32 %0, %4\n\t"
      "ds_read_b32 %1, %5\n\t"
      "ds_read_b32 %2, %6\n\t"
      "ds_read_b32 %3, %7\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3])
      : "memory");
  return __builtin_amdgcn_perm(__builtin_amdgcn_perm(v[3], v[2], 0x05010000u),
                               __builtin_amdgcn_perm(v[1], v[0], 0x05010000u), 0x07060302u);
}

struct Out {
  unsigned long long cyc[3];
  uint32_t sb[3][256];  // per variant: S(x) for x = 0..255 (one byte per entry)
};

__global__ __launch_bounds__(256) void k_sbox(int iters, const uint8_t* sbox, Out* out) {
  __shared__ uint32_t te[256 * 32];
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t i = threadIdx.x; i < 256 * 32; i += blockDim.x) te[i] = (uint32_t)sbox[i >> 5] << 8;
  __syncthreads();
  if (threadIdx.x >= 64) return;
  uint32_t t64[64], t16[16];
#pragma unroll
  for (int i = 0; i < 64; ++i)
    t64[i] = sbox[4 * i] | (uint32_t)sbox[4 * i + 1] << 8 | (uint32_t)sbox[4 * i + 2] << 16 |
             (uint32_t)sbox[4 * i + 3] << 24;
  const uint32_t j = lane & 3u;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int e = 64 * (int)j + 4 * i;
    t16[i] = sbox[e] | (uint32_t)sbox[e + 1] << 8 | (uint32_t)sbox[e + 2] << 16 | (uint32_t)sbox[e + 3] << 24;
  }
  const uint32_t jbits = (j << 6) * 0x01010101u;
  const uint32_t lb = (uint32_t)(uintptr_t)te, lp = (lane & 31u) << 2;
  // correctness: lanes 0..63 map x = 4 lane + {0..3}
  const uint32_t xin = (4 * lane) | (4 * lane + 1) << 8 | (4 * lane + 2) << 16 | (4 * lane + 3) << 24;
  const uint32_t ys[3] = {sub_lds(lb, lp, xin), sub_reg1(t64, xin), 0u};
  // reg4: every lane of a quad must hold the same x: quad l of 16 takes x = 4 (16 g + l) + {0..3}
  for (int g = 0; g < 4; ++g) {
    const uint32_t l = 16 * (uint32_t)g + (lane >> 2);
    const uint32_t xg = (4 * l) | (4 * l + 1) << 8 | (4 * l + 2) << 16 | (4 * l + 3) << 24;
    const uint32_t r = sub_reg4(t16, xg, jbits);
    if (j == 0)
#pragma unroll
      for (int b = 0; b < 4; ++b) out->sb[2][4 * l + b] = (r >> (8 * b)) & 0xffu;
  }
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int b = 0; b < 4; ++b) out->sb[v][4 * lane + b] = (ys[v] >> (8 * b)) & 0xffu;
  // latency: dependent chains (x' = S(x) ^ iteration constant, so the chain does not cycle)
  uint32_t x = xin;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) x = sub_lds(lb, lp, x) ^ (uint32_t)i;
  long long t1 = clock64();
  uint32_t keep = x;
  if (lane == 0) out->cyc[0] = (unsigned long long)(t1 - t0);
  x = xin;
  t0 = clock64();
  for (int i = 0; i < iters; ++i) x = sub_reg1(t64, x) ^ (uint32_t)i;
  t1 = clock64();
  keep ^= x;
  if (lane == 0) out->cyc[1] = (unsigned long long)(t1 - t0);
  x = qperm<0x00>(xin);  // a quad-uniform x
  t0 = clock64();
  for (int i = 0; i < iters; ++i) x = sub_reg4(t16, x, jbits) ^ (uint32_t)i;
  t1 = clock64();
  keep ^= x;
  if (lane == 0) out->cyc[2] = (unsigned long long)(t1 - t0);
  if (keep == 0x12345678u) out->sb[0][0] = 0xEE;  // keep the chains
}

int main() {
  uint8_t sb[256];
  make_sbox(sb);
  uint8_t* d_sb;
  Out* d_out;
  if (hipMalloc(&d_sb, 256) != hipSuccess || hipMalloc(&d_out, sizeof(Out)) != hipSuccess) return 1;
  (void)hipMemcpy(d_sb, sb, 256, hipMemcpyHostToDevice);
  const int iters = 4000;
  Out best{};
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_sbox, dim3(1), dim3(256), 0, 0, iters, d_sb, d_out);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    Out o;
    (void)hipMemcpy(&o, d_out, sizeof o, hipMemcpyDeviceToHost);
    for (int v = 0; v < 3; ++v)
      if (rep == 0 || o.cyc[v] < best.cyc[v]) best.cyc[v] = o.cyc[v];
    if (rep == 0) std::copy(&o.sb[0][0], &o.sb[0][0] + 3 * 256, &best.sb[0][0]);
  }
  const char* names[3] = {"lds", "reg1", "reg4"};
  int bad_total = 0;
  for (int v = 0; v < 3; ++v) {
    int bad = 0;
    for (int x = 0; x < 256; ++x) bad += best.sb[v][x] != sb[x];
    bad_total += bad;
    printf("%-5s %7.1f shader cycles per dependent SubWord   S-box %s (%d of 256 wrong)\n", names[v],
           (double)best.cyc[v] / iters, bad ? "WRONG" : "right", bad);
  }
  return bad_total ? 2 : 0;
}
