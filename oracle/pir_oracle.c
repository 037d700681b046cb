/* pir_oracle.c -- TEST INFRASTRUCTURE ONLY (see pir_oracle.h).
 *
 * A deliberately plain, byte-at-a-time restatement of the reference algorithm.  It is the
 * checker, never the product: the HIP engine under erasurecodedpir_amd/ does not link or
 * call anything here.  Reference line numbers are relative to /root/reference/src/c.
 */
#include "pir_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* AES-128 (FIPS-197).  Tables are computed at load time from the field definition.     */
/* ------------------------------------------------------------------------------------ */
static uint8_t SBOX[256];

static uint8_t aes_xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }
static uint8_t aes_mul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = aes_xtime(a);
        b >>= 1;
    }
    return r;
}

/* GF(2^8) for the PIR code: polynomial 0x11d, generator 2 (coding.cpp / ec_base.h). */
static uint8_t GF_EXP[512];
static uint8_t GF_LOG[256];

__attribute__((constructor)) static void orc_tables_init(void) {
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        if (x) { /* x^254 */
            uint8_t r = 1, b = (uint8_t)x;
            for (int e = 254; e; e >>= 1) {
                if (e & 1) r = aes_mul(r, b);
                b = aes_mul(b, b);
            }
            inv = r;
        }
        uint8_t s = inv;
        for (int k = 1; k <= 4; k++) s ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
        SBOX[x] = (uint8_t)(s ^ 0x63);
    }
    unsigned v = 1;
    for (int i = 0; i < 255; i++) {
        GF_EXP[i] = (uint8_t)v;
        GF_LOG[v] = (uint8_t)i;
        v <<= 1;
        if (v & 0x100) v ^= 0x11d;
    }
    for (int i = 255; i < 512; i++) GF_EXP[i] = GF_EXP[i - 255];
    GF_LOG[0] = 0; /* isa-l's gflog_base[0]; only gf_pow ever reads it (see orc_gf_pow) */
}

static void aes_expand(const uint8_t key[16], uint8_t rk[176]) {
    memcpy(rk, key, 16);
    uint8_t rcon = 1;
    for (int i = 4; i < 44; i++) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 4 == 0) {
            uint8_t t0 = t[0];
            t[0] = (uint8_t)(SBOX[t[1]] ^ rcon);
            t[1] = SBOX[t[2]];
            t[2] = SBOX[t[3]];
            t[3] = SBOX[t0];
            rcon = aes_xtime(rcon);
        }
        for (int b = 0; b < 4; b++) rk[4 * i + b] = (uint8_t)(rk[4 * (i - 4) + b] ^ t[b]);
    }
}

static void aes_encrypt_rk(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; i++) s[i] = (uint8_t)(in[i] ^ rk[i]);
    for (int round = 1; round <= 10; round++) {
        /* SubBytes + ShiftRows: state byte (row r, col c) lives at s[r + 4c] */
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++) t[r + 4 * c] = SBOX[s[r + 4 * ((c + r) & 3)]];
        if (round != 10) { /* MixColumns */
            for (int c = 0; c < 4; c++) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                s[4 * c + 0] = (uint8_t)(aes_mul(a0, 2) ^ aes_mul(a1, 3) ^ a2 ^ a3);
                s[4 * c + 1] = (uint8_t)(a0 ^ aes_mul(a1, 2) ^ aes_mul(a2, 3) ^ a3);
                s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ aes_mul(a2, 2) ^ aes_mul(a3, 3));
                s[4 * c + 3] = (uint8_t)(aes_mul(a0, 3) ^ a1 ^ a2 ^ aes_mul(a3, 2));
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; i++) s[i] ^= rk[16 * round + i];
    }
    memcpy(out, s, 16);
}

void orc_aes128(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
    uint8_t rk[176];
    aes_expand(key, rk);
    aes_encrypt_rk(rk, in, out);
}

/* utils.cpp:37-51: EVP aes_128_ctr, key = seed, zero IV, plaintext = plen zero bytes.
 * Keystream block j = AES_seed(BE128(j)); the counter restarts at 0 on every call. */
void orc_G(const uint8_t seed[16], uint32_t plen, uint8_t *out) {
    uint8_t rk[176], ctr[16], blk[16];
    aes_expand(seed, rk);
    for (uint32_t off = 0, j = 0; off < plen; off += 16, j++) {
        memset(ctr, 0, 16);
        ctr[15] = (uint8_t)j;
        ctr[14] = (uint8_t)(j >> 8);
        ctr[13] = (uint8_t)(j >> 16);
        ctr[12] = (uint8_t)(j >> 24);
        aes_encrypt_rk(rk, ctr, blk);
        uint32_t m = plen - off < 16 ? plen - off : 16;
        memcpy(out + off, blk, m);
    }
}

uint32_t orc_blen(uint32_t p) { return 32 + (2 * (p - 1) + 7) / 8; }                  /* :53-55 */
int orc_key_len(int p, int n, int nq) { return 16 + n * (p - 1) * (16 + 2 * p - 2) + nq * (p - 1); }

/* ------------------------------------------------------------------------------------ */
/* GF(2^8) -- coding.cpp:9-60                                                           */
/* ------------------------------------------------------------------------------------ */
uint8_t orc_gf_mul(uint8_t a, uint8_t b) {
    if (!a || !b) return 0;
    return GF_EXP[GF_LOG[a] + GF_LOG[b]];
}
uint8_t orc_gf_inv(uint8_t a) { return a ? GF_EXP[255 - GF_LOG[a]] : 0; }
/* coding.cpp:46-60 square-and-multiply through the log tables WITHOUT a zero test:
 * with log[0] = 0 (isa-l) this makes gf_pow(0, e) = 1 -- reproduced on purpose. */
uint8_t orc_gf_pow(uint8_t base, uint8_t exp) {
    uint8_t out = 1;
    while (exp > 0) {
        if (exp & 1) out = GF_EXP[GF_LOG[out] + GF_LOG[base]];
        base = GF_EXP[(2 * GF_LOG[base]) % 255];
        exp >>= 1;
    }
    return out;
}

/* ------------------------------------------------------------------------------------ */
/* Tree DPF                                                                             */
/* ------------------------------------------------------------------------------------ */
void orc_final_cw(int p, int nq, int rho, uint8_t *out) {                 /* client.cpp:144 */
    for (int i = 1; i <= nq; i++)
        for (int j = 2; j <= p; j++)
            out[(i - 1) * (p - 1) + (j - 2)] = (uint8_t)(orc_gf_pow((uint8_t)j, (uint8_t)(rho * i)) ^ 1);
}

/* parse_prg_output (utils.cpp:57-70): t bit j = (out[32 + j/8] >> (j%8)) & 1, j < 2(p-1) */
static uint32_t prg_tbits(const uint8_t *out, int p) {
    uint32_t t = 0;
    for (int j = 0; j < 2 * (p - 1); j++) t |= (uint32_t)((out[32 + j / 8] >> (j % 8)) & 1) << j;
    return t;
}

/* dpf_tree.cpp:142-274 */
void orc_gen_opt_dpf(int n, uint64_t index, const uint8_t *fcw, int p, int nq,
                     const uint8_t *root_seeds, uint8_t *keys_out) {
    const int CWk = 16 + 2 * p - 2, CW = (p - 1) * CWk, kl = orc_key_len(p, n, nq);
    const uint32_t bl = orc_blen(p);
    uint8_t *s = malloc((size_t)p * 16);      /* current seeds per party      */
    uint32_t *t = calloc(p, sizeof(uint32_t)); /* current control bits (p-1)   */
    uint8_t *sL = malloc((size_t)p * 32), prg[64];
    uint32_t *tt = malloc(p * sizeof(uint32_t));
    uint8_t *sCW = malloc((size_t)(p - 1) * 16);
    uint32_t *tCW = malloc((p - 1) * sizeof(uint32_t));
    memcpy(s, root_seeds, (size_t)p * 16);
    for (int i = 0; i < p; i++) t[i] = (i >= 1) ? (1u << (i - 1)) : 0; /* :154-163 */
    for (int j = 0; j < p; j++) memcpy(keys_out + (size_t)j * kl, root_seeds + 16 * j, 16);
    for (int L = 1; L <= n; L++) {
        for (int j = 0; j < p; j++) {
            orc_G(s + 16 * j, bl, prg);
            memcpy(sL + 32 * j, prg, 32);
            tt[j] = prg_tbits(prg, p);
        }
        int bit = (int)((index >> (n - L)) & 1); /* getbit(index, n, L), utils.cpp:155 */
        int KEEP = bit, LOSE = 1 - bit;
        for (int j = 0; j < p - 1; j++) {
            for (int b = 0; b < 16; b++)
                sCW[16 * j + b] = sL[16 * LOSE + b] ^ sL[32 * (j + 1) + 16 * LOSE + b];
            uint32_t m = 0;
            for (int q = 0; q < p - 1; q++) {
                uint32_t lo = ((tt[0] >> q) ^ (tt[j + 1] >> q)) & 1;
                uint32_t hi = ((tt[0] >> (p - 1 + q)) ^ (tt[j + 1] >> (p - 1 + q))) & 1;
                if (j == q) { lo ^= (uint32_t)bit ^ 1; hi ^= (uint32_t)bit; }
                m |= lo << q;
                m |= hi << (p - 1 + q);
            }
            tCW[j] = m;
            uint8_t *dst = keys_out + 16 + (size_t)(L - 1) * CW + (size_t)j * CWk; /* :254-262 */
            memcpy(dst, sCW + 16 * j, 16);
            for (int k = 0; k < 2 * p - 2; k++) dst[16 + k] = (uint8_t)((m >> k) & 1);
        }
        for (int b = 0; b < p; b++) {
            uint8_t ns[16];
            uint32_t nt = (tt[b] >> (KEEP * (p - 1))) & ((1u << (p - 1)) - 1);
            memcpy(ns, sL + 32 * b + 16 * KEEP, 16);
            for (int k = 0; k < p - 1; k++)
                if ((t[b] >> k) & 1) {
                    for (int x = 0; x < 16; x++) ns[x] ^= sCW[16 * k + x];
                    nt ^= (tCW[k] >> (KEEP * (p - 1))) & ((1u << (p - 1)) - 1);
                }
            memcpy(s + 16 * b, ns, 16);
            t[b] = nt;
        }
    }
    /* :238-262 final correction words */
    uint8_t conv0[16], convj[16];
    orc_G(s, 16, conv0);
    for (int j = 1; j < p; j++) {
        orc_G(s + 16 * j, 16, convj);
        for (int a = 0; a < nq; a++) {
            uint8_t v = (uint8_t)(fcw[a * (p - 1) + j - 1] ^ conv0[a] ^ convj[a]);
            for (int q = 0; q < p; q++)
                keys_out[(size_t)q * kl + 16 + (size_t)n * CW + a * (p - 1) + (j - 1)] = v;
        }
    }
    /* the CW blocks are identical in every party's key */
    for (int q = 1; q < p; q++)
        memcpy(keys_out + (size_t)q * kl + 16, keys_out + 16, (size_t)n * CW);
    free(s); free(t); free(sL); free(tt); free(sCW); free(tCW);
}

/* dpf_tree.cpp:473-598, level by level (BFS order: children of level-index u are 2u, 2u+1). */
void orc_eval_all_opt(int p, int party0, int n, const uint8_t *key, int nq, uint8_t *out) {
    const int CWk = 16 + 2 * p - 2, CW = (p - 1) * CWk;
    const uint32_t bl = orc_blen(p), tmask = (1u << (p - 1)) - 1;
    const size_t N = (size_t)1 << n;
    uint8_t *seeds = malloc(N * 16), *next = malloc(N * 16), prg[64];
    uint32_t *t = malloc(N * sizeof(uint32_t)), *tn = malloc(N * sizeof(uint32_t));
    memcpy(seeds, key, 16);
    t[0] = (party0 >= 1) ? (1u << (party0 - 1)) : 0; /* :496-502 */
    for (int L = 0; L < n; L++) {
        const size_t W = (size_t)1 << L;
        for (size_t u = 0; u < W; u++) {
            orc_G(seeds + 16 * u, bl, prg);
            uint32_t tb = prg_tbits(prg, p);
            for (int j = 0; j < p - 1; j++) {
                if (!((t[u] >> j) & 1)) continue; /* :533-541 */
                const uint8_t *cw = key + 16 + (size_t)L * CW + (size_t)j * CWk;
                for (int x = 0; x < 16; x++) { prg[x] ^= cw[x]; prg[16 + x] ^= cw[x]; }
                for (int k = 0; k < 2 * p - 2; k++) tb ^= (uint32_t)(cw[16 + k] & 1) << k;
            }
            memcpy(next + 32 * u, prg, 32);
            tn[2 * u] = tb & tmask;
            tn[2 * u + 1] = (tb >> (p - 1)) & tmask;
        }
        uint8_t *sw = seeds; seeds = next; next = sw;
        uint32_t *tw = t; t = tn; tn = tw;
    }
    const uint8_t *last = key + 16 + (size_t)n * CW; /* lastCWs[i][a] = last[a*(p-1) + i] */
    uint8_t blk[16];
    for (size_t j = 0; j < N; j++) { /* :567-580 */
        orc_G(seeds + 16 * j, 16, blk);
        for (int a = 0; a < nq; a++) {
            uint8_t v = blk[a];
            for (int i = 0; i < p - 1; i++)
                if ((t[j] >> i) & 1) v ^= last[a * (p - 1) + i];
            out[(size_t)a * N + j] = v;
        }
    }
    free(seeds); free(next); free(t); free(tn);
}

void orc_scan(int n, int efs, int nq, const uint8_t *c, const uint8_t *shard, uint64_t lo,
              uint64_t hi, uint8_t *result) {
    const size_t N = (size_t)1 << n;
    memset(result, 0, (size_t)nq * efs);
    for (uint64_t i = lo; i < hi; i++) /* server.cpp:121-127 */
        for (int b = 0; b < efs; b++)
            for (int a = 0; a < nq; a++)
                result[(size_t)a * efs + b] ^= orc_gf_mul(c[a * N + i], shard[i * efs + b]);
}

void orc_answer(int p, int party1, int n, int efs, int nq, const uint8_t *key,
                const uint8_t *shard, uint8_t *result) {
    orc_answer_slice(p, party1, n, efs, nq, key, shard, 0, 1, result);
}

void orc_answer_slice(int p, int party1, int n, int efs, int nq, const uint8_t *key,
                      const uint8_t *shard, int thread_num, int num_threads, uint8_t *result) {
    const size_t N = (size_t)1 << n, slice = N / (size_t)num_threads;
    uint8_t *c = malloc((size_t)nq * N);
    orc_eval_all_opt(p, party1 - 1, n, key, nq, c);
    orc_scan(n, efs, nq, c, shard, thread_num * slice, (thread_num + 1) * slice, result);
    free(c);
}

void orc_assemble(int num_threads, int nq, int efs, const uint8_t *in, uint8_t *out) {
    memset(out, 0, (size_t)nq * efs);
    for (int t = 0; t < num_threads; t++)
        for (size_t i = 0; i < (size_t)nq * efs; i++) out[i] ^= in[(size_t)t * nq * efs + i];
}

void orc_xorshift_fill(uint64_t seed, uint8_t *buf, size_t len) {
    uint64_t x = seed ? seed : 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < len; i++) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        buf[i] = (uint8_t)x;
    }
}

static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_splitmix_fill(uint64_t seed, uint64_t row0, uint64_t rows, uint32_t efs, uint8_t *buf) {
    for (uint64_t r = 0; r < rows; r++) {
        const uint64_t gr = row0 + r;
        uint8_t *row = buf + r * efs;
        for (uint32_t b = 0; b < efs; b += 8) {
            uint64_t z = splitmix64(seed ^ ((gr << 20) | (b >> 3)));
            for (uint32_t k = 0; k < 8 && b + k < efs; k++) row[b + k] = (uint8_t)(z >> (8 * k));
        }
    }
}

/* ------------------------------------------------------------------------------------ */
/* Client side: sizing, synthetic DB, encode-across, erasure decode                     */
/* ------------------------------------------------------------------------------------ */
static int ceil_log2(long v) { int l = 0; while ((1L << l) < v) l++; return l; }

void orc_tree_sizes(int L, int f, int k, int r, int rho, int *out5) {
    int p = k + r + 1 + (rho - 1);                        /* params.cpp:416 (T=1, B=0) */
    long nfiles = 1L << L;
    int n = ceil_log2((nfiles + k - 1) / k);              /* params.cpp:486            */
    int nq = (k == 1) ? 1 : k / rho;                      /* params.cpp:508-512        */
    out5[0] = p; out5[1] = n; out5[2] = f; out5[3] = nq; out5[4] = orc_key_len(p, n, nq);
}

void orc_synthetic_db(int L, int f, uint8_t *files) {     /* client.cpp:16-33 */
    long nfiles = 1L << L;
    for (long i = 0; i < nfiles; i++)
        for (int j = 0; j < f; j++) files[i * f + j] = (uint8_t)(i == 1 ? j : i);
}

void orc_encode_across(int L, int f, int k, int p, int party1, const uint8_t *files,
                       uint8_t *shard) {                  /* client.cpp:64-97 */
    long nfiles = 1L << L;
    long encdb = (nfiles + k - 1) / k;
    int n = ceil_log2(encdb);
    long N = 1L << n;
    for (long fi = 0; fi < N; fi++) {
        uint8_t *row = shard + fi * f;
        memset(row, 0, f);
        for (int j = 0; j < k; j++) {
            long src = encdb * j + fi;
            if (src >= nfiles) continue;
            uint8_t e = orc_gf_pow((uint8_t)party1, (uint8_t)j); /* encodeMat[j*p + party-1] */
            for (int b = 0; b < f; b++) row[b] ^= orc_gf_mul(files[src * f + b], e);
        }
    }
    (void)p;
}

int orc_gf_invert_matrix(uint8_t *in, uint8_t *out, int n) {  /* coding.cpp:73-126 */
    memset(out, 0, (size_t)n * n);
    for (int i = 0; i < n; i++) out[i * n + i] = 1;
    for (int i = 0; i < n; i++) {
        if (in[i * n + i] == 0) {
            int j;
            for (j = i + 1; j < n; j++) if (in[j * n + i]) break;
            if (j == n) return -1;
            for (int k = 0; k < n; k++) {
                uint8_t x = in[i * n + k]; in[i * n + k] = in[j * n + k]; in[j * n + k] = x;
                x = out[i * n + k]; out[i * n + k] = out[j * n + k]; out[j * n + k] = x;
            }
        }
        uint8_t piv = orc_gf_inv(in[i * n + i]);
        for (int j = 0; j < n; j++) {
            in[i * n + j] = orc_gf_mul(in[i * n + j], piv);
            out[i * n + j] = orc_gf_mul(out[i * n + j], piv);
        }
        for (int j = 0; j < n; j++) {
            if (j == i) continue;
            uint8_t x = in[j * n + i];
            for (int k = 0; k < n; k++) {
                out[j * n + k] ^= orc_gf_mul(x, out[i * n + k]);
                in[j * n + k] ^= orc_gf_mul(x, in[i * n + k]);
            }
        }
    }
    return 0;
}

/* interpolation.cpp:176-196: solve the (deg+1) Vandermonde system on the first deg+1 points */
static void lagrange_semihonest(const uint8_t *pts, const uint8_t *evals, int deg, uint8_t *out) {
    int m = deg + 1;
    uint8_t *gen = malloc((size_t)m * m), *inv = malloc((size_t)m * m);
    for (int i = 0; i < m; i++)
        for (int c = 0; c < m; c++) gen[i * m + c] = orc_gf_pow(pts[i], (uint8_t)c);
    orc_gf_invert_matrix(gen, inv, m);
    for (int i = 0; i < m; i++) {
        uint8_t v = 0;
        for (int j = 0; j < m; j++) v ^= orc_gf_mul(evals[j], inv[i * m + j]);
        out[i] = v;
    }
    free(gen); free(inv);
}

void orc_decode(int p, int k, int r, int rho, int nq, int efs, const uint8_t *erasure,
                const uint8_t *responses, uint8_t *out) {        /* client.cpp:211-268 */
    const int nr = p - r, deg = k + rho - 1;
    uint8_t *acc = calloc((size_t)k * efs, 1);
    uint8_t *pts = malloc(nr), *sh = malloc((size_t)efs * nr), *tmp = malloc(k + rho);
    for (int i = 0; i < nq; i++) {
        int cur = 1;
        for (int j = 0; j < nr; j++) {
            while (erasure[cur - 1] == 0) cur++;
            pts[j] = (uint8_t)cur;
            for (int a = 0; a < efs; a++) {
                uint8_t v = responses[((size_t)j * nq + i) * efs + a];
                for (int b = 0; b < i; b++)
                    v ^= orc_gf_mul(acc[(size_t)(k - 1 - b) * efs + a],
                                    orc_gf_pow((uint8_t)cur, (uint8_t)(k + i - b)));
                sh[(size_t)a * nr + j] = v;
            }
            cur++;
        }
        for (int a = 0; a < efs; a++) {
            lagrange_semihonest(pts, sh + (size_t)a * nr, deg, tmp);
            for (int q = 0; q < rho; q++) acc[(size_t)(k - 1 - i - q) * efs + a] = tmp[k + rho - 1 - q];
        }
    }
    memcpy(out, acc, efs); /* FILE_SIZE_BYTES (no MAC) == efs in tree mode */
    free(acc); free(pts); free(sh); free(tmp);
}

/* ---- multiparty sqrt(N) DPF ---------------------------------------------------------------- */
int orc_choose(int n, int k) { return k == 0 ? 1 : (n * orc_choose(n - 1, k - 1)) / k; } /* utils.cpp:168 */

void orc_mp_sizes(int p, int n, int t, uint64_t *o) {
    int q = orc_choose(p, t);
    uint64_t nrk = (uint64_t)(q * (p - t) / p), p2 = 1ull << (q - 1);        /* params.cpp:618 */
    int mu_pow = (int)ceil(log2(ceil(pow(2, n / 2.0) * pow(2, (p - 1) / 2.0)))); /* :473 */
    uint64_t mu = 1ull << mu_pow, nu = mu_pow > n ? 0 : 1ull << (n - mu_pow);
    o[0] = nrk; o[1] = p2; o[2] = mu; o[3] = nu;
    o[4] = 16 * p2 * nu + nrk * nu * p2 + p2 * mu;       /* seeds | toggle bytes | cw (:485-511) */
    uint64_t kmu = 1ull << (n / 2), knu = 1ull << (n - n / 2);               /* utils.cpp:111-113 */
    o[5] = (uint64_t)(int)(16 * p2 * knu + nrk * knu * p2 + p2 * kmu);
}

/* share[a][i*mu + x] over rows [thread_num*slice, (thread_num+1)*slice) of a layout
   {nrk, p2, mu, nu}: the loop both evalAllOptMultiPartyDPFThread (multiparty_dpf.cpp:590-601)
   and evalAllCDThread (:665-675) run */
static void layout_eval(const uint64_t *z, int n, const uint8_t *key, int thread_num,
                        int num_threads, uint8_t *out) {
    const uint64_t nrk = z[0], p2 = z[1], mu = z[2], nu = z[3], N = 1ull << n;
    const uint64_t tog = nu * 16 * p2, cw = tog + nrk * nu * p2, slice = nu / num_threads;
    uint8_t *g = malloc(mu);
    memset(out, 0, nrk * N);
    for (uint64_t i = thread_num * slice; i < (thread_num + 1) * slice; i++)
        for (uint64_t j = 0; j < p2; j++) {
            orc_G(key + i * 16 * p2 + 16 * j, (uint32_t)mu, g);
            for (uint64_t a = 0; a < nrk; a++) {
                if (!key[tog + a * nu * p2 + i * p2 + j]) continue;
                uint8_t *o = out + a * N + i * mu;
                for (uint64_t x = 0; x < mu; x++) o[x] ^= g[x] ^ key[cw + j * mu + x];
            }
        }
    free(g);
}

/* the scan of runOptimizedMultiPartyDPFQueryThread (server.cpp:416-422) and runCDQueryThread
   (:477-484) over the thread's slice of rows */
static void layout_answer(const uint64_t *z, int n, int efs, const uint8_t *key,
                          const uint8_t *shard, int thread_num, int num_threads, uint8_t *result) {
    const uint64_t nrk = z[0], mu = z[2], nu = z[3], N = 1ull << n, slice = nu / num_threads;
    uint8_t *c = malloc(nrk * N);
    layout_eval(z, n, key, thread_num, num_threads, c);
    memset(result, 0, nrk * efs);
    for (uint64_t i = thread_num * slice * mu; i < (thread_num + 1) * slice * mu; i++)
        for (int b = 0; b < efs; b++)
            for (uint64_t a = 0; a < nrk; a++)
                result[a * efs + b] ^= orc_gf_mul(c[a * N + i], shard[i * (uint64_t)efs + b]);
    free(c);
}

void orc_mp_eval(int p, int n, int t, const uint8_t *key, int thread_num, int num_threads,
                 uint8_t *out) {
    uint64_t z[6];
    orc_mp_sizes(p, n, t, z);
    layout_eval(z, n, key, thread_num, num_threads, out);
}

void orc_mp_answer(int p, int t, int n, int efs, const uint8_t *key, const uint8_t *shard,
                   int thread_num, int num_threads, uint8_t *result) {
    uint64_t z[6];
    orc_mp_sizes(p, n, t, z);
    layout_answer(z, n, efs, key, shard, thread_num, num_threads, result);
}

/* ---- covering-design (CD) sqrt(N) DPF ------------------------------------------------------ */
void orc_cd_sizes(int n, int q_needed, int num_cd_keys, uint64_t *o) {
    /* evalAllCDThread (multiparty_dpf.cpp:620-625): p2 = 2^(q-1), mu_pow = n/2 + 3 (integer
       n/2: ceil((double)(n/2))), nu = 2^(n - mu_pow) (0 below 1: (uint64_t)pow(2, negative)) */
    const int mu_pow = n / 2 + 3;
    const uint64_t p2 = 1ull << (q_needed - 1), mu = 1ull << mu_pow;
    const uint64_t nu = mu_pow > n ? 0 : 1ull << (n - mu_pow), nrk = (uint64_t)num_cd_keys;
    o[0] = nrk; o[1] = p2; o[2] = mu; o[3] = nu;
    o[4] = 16 * p2 * nu + nrk * nu * p2 + p2 * mu;            /* calcCDDPFKeyLength, utils.cpp:118 */
    o[5] = (uint64_t)(int)o[4];
}

void orc_cd_eval(int n, int q_needed, int num_cd_keys, const uint8_t *key, int thread_num,
                 int num_threads, uint8_t *out) {
    uint64_t z[6];
    orc_cd_sizes(n, q_needed, num_cd_keys, z);
    layout_eval(z, n, key, thread_num, num_threads, out);
}

void orc_cd_answer(int n, int q_needed, int num_cd_keys, int efs, const uint8_t *key,
                   const uint8_t *shard, int thread_num, int num_threads, uint8_t *result) {
    uint64_t z[6];
    orc_cd_sizes(n, q_needed, num_cd_keys, z);
    layout_answer(z, n, efs, key, shard, thread_num, num_threads, result);
}
