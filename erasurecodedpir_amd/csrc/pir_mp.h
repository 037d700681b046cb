// pir_mp.h -- internal: the multiparty sqrt(N) DPF's full-domain evaluation
// (evalAllOptMultiPartyDPF, src/c/multiparty_dpf.cpp:467-539), feeding the GF(2^8) shard scan of
// runOptimizedMultiPartyDPFQuery[Thread] (src/c/server.cpp:136-176, :384-430).  Not part of the
// C ABI.
//
// The domain of 2^n records is nu rows of mu records.  A key holds, per row i and seed j < p2,
// a 16-byte seed s[i][j]; per output share a < nrk, a toggle byte per (i, j); and p2 correction
// words cw[j] of mu bytes:
//     share[a][i*mu + x] = XOR_{j : toggle[a][i][j] != 0} ( G(s[i][j], mu)[x] ^ cw[j][x] )
// with G the AES-128-CTR stream of utils.cpp:37-51.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pir {

struct MpLayout {
  int n = 0, p = 0, t = 0;
  int nrk = 0;          // NUM_RSS_KEYS = choose(p,t) * (p - t) / p   (params.cpp:618)
  uint32_t p2 = 0;      // 2^(choose(p,t) - 1) seeds per row
  int mu_pow = 0;       // ceil(log2(ceil(2^(n/2) * 2^((p-1)/2))))     (multiparty_dpf.cpp:473)
  uint64_t mu = 0;      // records per row
  uint64_t nu = 0;      // rows (0 when mu_pow > n: the reference's (uint64_t)pow(2, negative))
  uint64_t tog_off = 0; // nu * 16 * p2
  uint64_t cw_off = 0;  // tog_off + nrk * nu * p2
  uint64_t eval_bytes = 0;  // cw_off + p2 * mu: the key bytes the evaluation reads
};

// choose() of utils.cpp:168-174 (the same recursion order, so the same integer)
int mp_choose(int n, int k);
// false when the parameters give no usable layout (t < 1, t >= p, too many seeds/shares)
bool mp_layout(int p, int n, int t, MpLayout* out);
// the covering-design layout of evalAllCDThread (multiparty_dpf.cpp:617-690): nrk = NUM_CD_KEYS
// shares, p2 = 2^(NUM_CD_KEYS_NEEDED - 1) seeds per row, mu = 2^(n/2 + 3) (integer n / 2), the
// same key sections (p, t unused: 0)
bool cd_layout(int n, int q_needed, int num_cd_keys, MpLayout* out);

// d_c[(r - rec_lo) * nrp + a] = share[a][r] (0 for a >= nrk) for records r in [rec_lo, rec_hi)
// (row-aligned or 16-aligned bounds not required); d_key: the raw key, eval_bytes long
hipError_t launch_mp_shares(const MpLayout& L, const uint8_t* d_key, uint64_t rec_lo,
                            uint64_t rec_hi, int nrp, uint8_t* d_c, int num_cus, hipStream_t s);
// this translation unit's copy of the AES table (once per device, before the first launch)

}  // namespace pir
