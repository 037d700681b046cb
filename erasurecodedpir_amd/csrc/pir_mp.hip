// pir_mp.hip -- multiparty sqrt(N) DPF evaluation on CDNA4 (pir_mp.h).
//
// One lane = one item of W = min(16 R, mu) consecutive records of one row i (R = 4 CTR blocks
// when mu >= 64).  For every seed j of the row whose toggle byte is set for any share, the lane
// runs ONE AES key schedule and R counter blocks of G(s[i][j]) (the T-table row shape of
// pir_aes.h, counters c0..c0+R-1 sharing the first two rounds' columns), XORs in cw[j] and folds
// the block into the toggled shares' accumulators.  It then writes the items' share bytes in the
// record-major layout the GF(2^8) scan reads (nrp bytes per record: 16 R nrp contiguous bytes
// per lane).  AES work per query = N / 16 x p2 blocks (p2 = 4 for p = 3, t = 1): an eighth of
// the tree DPF's, so the answer stays bound by the shard scan's HBM stream.
#include "pir_aes.h"
#include "pir_mp.h"

#include <math.h>

#include <algorithm>

namespace pir {


int mp_choose(int n, int k) { return k == 0 ? 1 : (n * mp_choose(n - 1, k - 1)) / k; }

bool mp_layout(int p, int n, int t, MpLayout* L) {
  *L = MpLayout{};
  if (p < 2 || t < 1 || t >= p || n < 0 || n > 40) return false;
  const int q = mp_choose(p, t);
  if (q < 1 || q > 31) return false;
  L->n = n; L->p = p; L->t = t;
  L->nrk = q * (p - t) / p;
  L->p2 = 1u << (q - 1);
  // the reference evaluates the sizes in double precision; so does this
  L->mu_pow = (int)ceil(log2(ceil(pow(2.0, n / 2.0) * pow(2.0, (p - 1) / 2.0))));
  L->mu = 1ull << L->mu_pow;
  L->nu = L->mu_pow > n ? 0 : 1ull << (n - L->mu_pow);
  L->tog_off = L->nu * 16ull * L->p2;
  L->cw_off = L->tog_off + (uint64_t)L->nrk * L->nu * L->p2;
  L->eval_bytes = L->cw_off + (uint64_t)L->p2 * L->mu;
  return L->nrk >= 1;
}

bool cd_layout(int n, int q_needed, int num_cd_keys, MpLayout* L) {
  *L = MpLayout{};
  if (n < 0 || n > 40 || q_needed < 1 || q_needed > 31 || num_cd_keys < 1 || num_cd_keys > 16)
    return false;
  L->n = n;
  L->nrk = num_cd_keys;
  L->p2 = 1u << (q_needed - 1);
  L->mu_pow = n / 2 + 3;  // ceil((double)(n/2)) + 3: integer n / 2
  L->mu = 1ull << L->mu_pow;
  L->nu = L->mu_pow > n ? 0 : 1ull << (n - L->mu_pow);
  L->tog_off = L->nu * 16ull * L->p2;
  L->cw_off = L->tog_off + (uint64_t)L->nrk * L->nu * L->p2;
  L->eval_bytes = L->cw_off + (uint64_t)L->p2 * L->mu;
  return true;
}

namespace {

__device__ __forceinline__ uint32_t byte_of(uint4 v, int k) {
  const uint32_t w = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
  return (w >> (8 * (k & 3))) & 0xffu;
}
__device__ __forceinline__ uint32_t word_of(uint4 v, int q) {
  return q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
}

// 16 bytes of cw at byte offset `off` of the key: one 16-byte load when the section is aligned
__device__ __forceinline__ uint4 load_cw(const uint8_t* key, uint64_t off, bool aligned, int nbytes) {
  if (aligned && nbytes == 16) return *reinterpret_cast<const uint4*>(key + off);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int k = 0; k < nbytes; ++k) w[k >> 2] |= (uint32_t)key[off + k] << (8 * (k & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// 1024-thread workgroups (16 waves per CU: the 64 KiB of tables allow one such workgroup per
// CU, and R <= 4 counter blocks with NRP accumulators fit 128 VGPRs: R = 4 / 2 / 1 for
// NRP = 1 / 2-4 / 8-16).  Round 4: at 256 threads, R = 4 and 180 VGPRs (NRP = 4) the LDS and
// the registers held a CU to 8 waves, too few to hide the per-seed AES chains.
constexpr int kMpThreads = 1024;

template <int NRP, int R>
__global__ __launch_bounds__(kMpThreads) void k_mp_shares(const uint8_t* __restrict__ key,
                                                          MpLayout L, uint64_t rec_lo,
                                                          uint64_t rec_hi,
                                                          uint8_t* __restrict__ d_c) {
  __shared__ uint32_t lds_tab[kTablesBytes / 4];
  load_tables_n<kMpThreads>(lds_tab);
  __syncthreads();
  const Tab T(lds_tab);
  const uint64_t W = L.mu < 16ull * R ? L.mu : 16ull * R;  // records per item
  const int wb = (int)(W < 16 ? W : 16);                    // bytes used per CTR block
  const uint64_t it0 = rec_lo / W, it1 = (rec_hi + W - 1) / W;
  const bool cw_al = (L.cw_off & 15) == 0 && (L.mu & 15) == 0;
  const uint64_t row_tog = (uint64_t)L.nu * L.p2;
  for (uint64_t it = it0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; it < it1;
       it += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t g0 = it * W, i = g0 / L.mu, x0 = g0 - i * L.mu;
    const uint32_t b0 = (uint32_t)(x0 >> 4);
    uint4 acc[NRP][R];
#pragma unroll
    for (int a = 0; a < NRP; ++a)
#pragma unroll
      for (int r = 0; r < R; ++r) acc[a][r] = make_uint4(0, 0, 0, 0);
    for (uint32_t j = 0; j < L.p2; ++j) {
      uint32_t m[NRP];
      uint32_t any = 0;
#pragma unroll
      for (int a = 0; a < NRP; ++a) {
        m[a] = (a < L.nrk && key[L.tog_off + a * row_tog + i * L.p2 + j]) ? ~0u : 0u;
        any |= m[a];
      }
      if (!any) continue;
      const uint4 seed = *reinterpret_cast<const uint4*>(key + i * 16ull * L.p2 + 16ull * j);
      uint4 ks[R];
      aes_ctr_row<R, 4>(T, seed, ks, __builtin_bswap32(b0));
      const uint64_t cwb = L.cw_off + (uint64_t)j * L.mu + 16ull * b0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint4 v = xor4(ks[r], load_cw(key, cwb + 16ull * r, cw_al, wb));
#pragma unroll
        for (int a = 0; a < NRP; ++a) acc[a][r] = xor4(acc[a][r], and4(v, m[a]));
      }
    }
    // records g0 + 16 r + k  ->  d_c[(record - rec_lo) * NRP + a]
    const bool full = wb == 16 && g0 >= rec_lo && g0 + W <= rec_hi && ((g0 - rec_lo) & 15) == 0;
    if (full) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        uint4* dst = reinterpret_cast<uint4*>(d_c + (g0 + 16ull * r - rec_lo) * NRP);
        if constexpr (NRP == 1) {
          dst[0] = acc[0][r];
        } else if constexpr (NRP == 2) {
          uint32_t o[8];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t x = word_of(acc[0][r], q), y = word_of(acc[1][r], q);
            o[2 * q] = __builtin_amdgcn_perm(y, x, 0x05010400u);
            o[2 * q + 1] = __builtin_amdgcn_perm(y, x, 0x07030602u);
          }
          dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
          dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
        } else if constexpr (NRP == 4) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // 4x4 byte transpose of word q of the four shares
            const uint32_t a0 = word_of(acc[0][r], q), a1 = word_of(acc[1][r], q);
            const uint32_t a2 = word_of(acc[2][r], q), a3 = word_of(acc[3][r], q);
            const uint32_t l01 = __builtin_amdgcn_perm(a1, a0, 0x05010400u);
            const uint32_t h01 = __builtin_amdgcn_perm(a1, a0, 0x07030602u);
            const uint32_t l23 = __builtin_amdgcn_perm(a3, a2, 0x05010400u);
            const uint32_t h23 = __builtin_amdgcn_perm(a3, a2, 0x07030602u);
            dst[q] = make_uint4(__builtin_amdgcn_perm(l23, l01, 0x05040100u),
                                __builtin_amdgcn_perm(l23, l01, 0x07060302u),
                                __builtin_amdgcn_perm(h23, h01, 0x05040100u),
                                __builtin_amdgcn_perm(h23, h01, 0x07060302u));
          }
        } else {  // 8 or 16 shares: record k = NRP / 4 words, bytes gathered share by share
          uint32_t* dst32 = reinterpret_cast<uint32_t*>(dst);
#pragma unroll
          for (int k = 0; k < 16; ++k)
#pragma unroll
            for (int g = 0; g < NRP / 4; ++g)
              dst32[k * (NRP / 4) + g] =
                  byte_of(acc[4 * g][r], k) | (byte_of(acc[4 * g + 1][r], k) << 8) |
                  (byte_of(acc[4 * g + 2][r], k) << 16) | (byte_of(acc[4 * g + 3][r], k) << 24);
        }
      }
    } else {  // range edges, rows shorter than 16 records: byte stores
#pragma unroll
      for (int r = 0; r < R; ++r)
        for (int k = 0; k < wb; ++k) {
          const uint64_t rec = g0 + 16ull * r + k;
          if (rec < rec_lo || rec >= rec_hi) continue;
#pragma unroll
          for (int a = 0; a < NRP; ++a)
            d_c[(rec - rec_lo) * NRP + a] = (uint8_t)byte_of(acc[a][r], k);
        }
    }
  }
}

template <int NRP>
hipError_t launch_nrp(const MpLayout& L, const uint8_t* d_key, uint64_t lo, uint64_t hi,
                      uint8_t* d_c, int num_cus, hipStream_t s) {
  constexpr int RW = NRP <= 1 ? 4 : (NRP <= 4 ? 2 : 1);  // counter blocks per lane, wide rows
  const bool wide = L.mu >= 16ull * RW;
  const uint64_t W = wide ? 16ull * RW : std::min<uint64_t>(L.mu, 16);
  const uint64_t items = (hi + W - 1) / W - lo / W;
  const unsigned grid = (unsigned)std::max<uint64_t>(
      1, std::min<uint64_t>((items + kMpThreads - 1) / kMpThreads, (uint64_t)num_cus * 2));
  if (wide)
    hipLaunchKernelGGL((k_mp_shares<NRP, RW>), dim3(grid), dim3(kMpThreads), 0, s, d_key, L, lo,
                       hi, d_c);
  else
    hipLaunchKernelGGL((k_mp_shares<NRP, 1>), dim3(grid), dim3(kMpThreads), 0, s, d_key, L, lo,
                       hi, d_c);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_mp_shares(const MpLayout& L, const uint8_t* d_key, uint64_t rec_lo,
                            uint64_t rec_hi, int nrp, uint8_t* d_c, int num_cus, hipStream_t s) {
  if (rec_hi <= rec_lo || L.nu == 0) return hipSuccess;
  if (nrp < L.nrk || rec_hi > L.nu * L.mu) return hipErrorInvalidValue;
  switch (nrp) {
    case 1: return launch_nrp<1>(L, d_key, rec_lo, rec_hi, d_c, num_cus, s);
    case 2: return launch_nrp<2>(L, d_key, rec_lo, rec_hi, d_c, num_cus, s);
    case 4: return launch_nrp<4>(L, d_key, rec_lo, rec_hi, d_c, num_cus, s);
    case 8: return launch_nrp<8>(L, d_key, rec_lo, rec_hi, d_c, num_cus, s);
    case 16: return launch_nrp<16>(L, d_key, rec_lo, rec_hi, d_c, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pir
