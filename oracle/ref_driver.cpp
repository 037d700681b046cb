// ref_driver.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
//
// A thin extern "C" harness around the reference's own C++ sources
// (/root/reference/src/c/*.cpp, compiled where they lie by oracle/Makefile into
// oracle/_ref/libref.so).  It exists for two purposes:
//   1. generating the golden fixtures under tests/golden/ (tests/golden/make_golden.py);
//   2. the "reference" CPU baseline leg of bench.py (runOptimizedDPFTreeQuery timed on the
//      GPU box's host cores).
// Nothing here re-implements the reference: every entry point calls the reference symbol
// named in its comment.  No reference source is copied into this repository.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <time.h>
#include <thread>
#include <vector>

#include "utils.h"
#include "coding.h"
#include "params.h"
#include "dpf_tree.h"
#include "multiparty_dpf.h"
#include "server.h"
#include "client.h"

extern "C" {

// utils.cpp:37-51
void ref_G(const uint8_t* seed, uint32_t plen, uint8_t* out) {
    EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
    uint8_t s[16];
    memcpy(s, seed, 16);
    G(ctx, s, plen, out);
    EVP_CIPHER_CTX_free(ctx);
}

// coding.cpp:9-60
uint8_t ref_gf_mul(uint8_t a, uint8_t b) { return gf_mul(a, b); }
uint8_t ref_gf_inv(uint8_t a) { return gf_inv(a); }
uint8_t ref_gf_pow(uint8_t a, uint8_t e) { return gf_pow(a, e); }

// utils.cpp:85-90
int ref_key_len(int p, int n, int nq) { return calcOptimizedDPFTreeKeyLength(p, n, nq); }
// utils.cpp:53-55
uint32_t ref_blen(uint32_t p) { return blen(p); }

// dpf_tree.cpp:142-274 (root seeds from RAND_bytes: the output keys ARE the fixture)
void ref_gen_opt_dpf(int n, uint64_t index, const uint8_t* finalCW, int p, int nq,
                     uint8_t* keys_out) {
    EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
    int kl = calcOptimizedDPFTreeKeyLength(p, n, nq);
    std::vector<uint8_t> fcw(finalCW, finalCW + nq * (p - 1));
    uint8_t** keys = (uint8_t**)malloc(p * sizeof(uint8_t*));
    for (int j = 0; j < p; j++) keys[j] = (uint8_t*)malloc(kl);
    genOptimizedDPF(ctx, n, (uint128_t)index, 1, fcw, p, nq, &keys);
    for (int j = 0; j < p; j++) {
        memcpy(keys_out + (size_t)j * kl, keys[j], kl);
        free(keys[j]);
    }
    free(keys);
    EVP_CIPHER_CTX_free(ctx);
}

// dpf_tree.cpp:473-598; out is nq x 2^n (a-major, like dataShare[a][j])
void ref_eval_all_opt(int p, int party0, int n, const uint8_t* key, int nq, uint8_t* out) {
    EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
    size_t N = (size_t)1 << n;
    uint8_t** ds = (uint8_t**)malloc(nq * sizeof(uint8_t*));
    for (int a = 0; a < nq; a++) ds[a] = out + a * N;
    evalAllOptimizedDPF(ctx, p, party0, n, (uint8_t*)key, 1, nq, ds);
    free(ds);
    EVP_CIPHER_CTX_free(ctx);
}

// dpf_tree.cpp:600-765 -- the DEFECTIVE threaded eval (negative fixture only)
void ref_eval_all_opt_thread(int p, int party0, int n, const uint8_t* key, int nq,
                             int threadNum, int numThreads, uint8_t* out) {
    EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
    size_t N = (size_t)1 << n;
    uint8_t** ds = (uint8_t**)malloc(nq * sizeof(uint8_t*));
    for (int a = 0; a < nq; a++) ds[a] = out + a * N;
    evalAllOptimizedDPFThread(ctx, p, party0, n, (uint8_t*)key, 1, nq, ds, threadNum, numThreads);
    free(ds);
    EVP_CIPHER_CTX_free(ctx);
}

static void set_tree_globals(int p, int n, int efs, int nq) {
    NUM_PARTIES = p;
    LOG_NUM_ENCODED_FILES = n;
    NUM_ENCODED_FILES = 1 << n;
    ENCODED_FILE_SIZE_BYTES = efs;
    NUM_ROUNDS = nq;
    IS_HERMITE = 0;
}

// A resident reference server (server.cpp:17-42) holding a contiguous N x efs shard.
struct ref_srv {
    server s;
    int p, n, efs, nq;
};

void* ref_server_new(int p, int party1, int n, int efs, int nq, const uint8_t* shard,
                     int isByzantine, int numThreads) {
    set_tree_globals(p, n, efs, nq);
    ref_srv* h = new ref_srv;
    h->p = p; h->n = n; h->efs = efs; h->nq = nq;
    initializeServer(&h->s, party1, n, efs, isByzantine, numThreads);
    size_t N = (size_t)1 << n;
    for (size_t i = 0; i < N; i++) memcpy(h->s.indexList[i], shard + i * efs, efs);
    return h;
}

// A reference server whose indexList rows point into a caller-owned contiguous N x efs shard
// (e.g. a shared read-only file mapping: the all-cores CPU leg runs one process per core over
// ONE copy of a 16 GiB shard).  The fields are those initializeServer sets (server.cpp:17-42);
// only the row storage differs (the reference mallocs each row; the answer path reads rows
// through indexList either way).  Free with ref_server_view_free.
void* ref_server_view(int p, int party1, int n, int efs, int nq, const uint8_t* shard) {
    set_tree_globals(p, n, efs, nq);
    ref_srv* h = new ref_srv;
    h->p = p; h->n = n; h->efs = efs; h->nq = nq;
    size_t N = (size_t)1 << n;
    h->s.ctx = EVP_CIPHER_CTX_new();
    h->s.ctxThreads = (EVP_CIPHER_CTX**)malloc(sizeof(EVP_CIPHER_CTX*));
    h->s.ctxThreads[0] = EVP_CIPHER_CTX_new();
    h->s.partyIndex = party1;
    h->s.indexList = (uint8_t**)malloc(N * sizeof(uint8_t*));
    for (size_t i = 0; i < N; i++) h->s.indexList[i] = (uint8_t*)shard + i * efs;
    h->s.isByzantine = 0;
    h->s.numThreads = 1;
    return h;
}

void ref_server_view_free(void* hv) {
    ref_srv* h = (ref_srv*)hv;
    EVP_CIPHER_CTX_free(h->s.ctx);
    EVP_CIPHER_CTX_free(h->s.ctxThreads[0]);
    free(h->s.ctxThreads);
    free(h->s.indexList);
    delete h;
}

// server.cpp:96-134; result is nq x efs
void ref_server_answer(void* hv, const uint8_t* key, uint8_t* result) {
    ref_srv* h = (ref_srv*)hv;
    set_tree_globals(h->p, h->n, h->efs, h->nq);
    uint8_t** res = (uint8_t**)malloc(h->nq * sizeof(uint8_t*));
    for (int a = 0; a < h->nq; a++) res[a] = result + (size_t)a * h->efs;
    runOptimizedDPFTreeQuery(&h->s, (uint8_t*)key, h->nq, res);
    free(res);
}

// server.cpp:505-549 + :553-562 (defective thread path; negative fixture only)
void ref_server_answer_threads(void* hv, const uint8_t* key, int numThreads, uint8_t* result) {
    ref_srv* h = (ref_srv*)hv;
    set_tree_globals(h->p, h->n, h->efs, h->nq);
    uint8_t*** in = (uint8_t***)malloc(numThreads * sizeof(uint8_t**));
    for (int t = 0; t < numThreads; t++) {
        in[t] = (uint8_t**)malloc(h->nq * sizeof(uint8_t*));
        for (int a = 0; a < h->nq; a++) in[t][a] = (uint8_t*)malloc(h->efs);
        runOptimizedDPFTreeQueryThread(&h->s, (uint8_t*)key, t, numThreads, in[t]);
    }
    uint8_t** res = (uint8_t**)malloc(h->nq * sizeof(uint8_t*));
    for (int a = 0; a < h->nq; a++) res[a] = result + (size_t)a * h->efs;
    assemblDPFTreeQueryThreadResults(&h->s, in, numThreads, res);
    for (int t = 0; t < numThreads; t++) {
        for (int a = 0; a < h->nq; a++) free(in[t][a]);
        free(in[t]);
    }
    free(in);
    free(res);
}

void ref_server_free(void* hv) {
    ref_srv* h = (ref_srv*)hv;
    set_tree_globals(h->p, h->n, h->efs, h->nq);
    freeServer(&h->s);
    delete h;
}

// Wall-clock seconds of `reps` runOptimizedDPFTreeQuery calls (CPU-baseline leg).
double ref_server_time(void* hv, const uint8_t* key, uint8_t* result, int reps) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; r++) ref_server_answer(hv, key, result);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}

// All-cores aggregate: `nthreads` independent runOptimizedDPFTreeQuery
// calls at once, one per thread.  Each thread gets a shallow copy of the server whose only
// private member is its EVP context (the reference's ctx is not shareable); the shard rows
// are shared read-only.  Returns the wall-clock seconds until the last query finishes.
double ref_server_time_parallel(void* hv, const uint8_t* key, uint8_t* result, int nthreads) {
    ref_srv* h = (ref_srv*)hv;
    set_tree_globals(h->p, h->n, h->efs, h->nq);
    std::vector<server> views(nthreads, h->s);
    std::vector<std::vector<uint8_t>> outs(nthreads, std::vector<uint8_t>((size_t)h->nq * h->efs));
    for (auto& v : views) v.ctx = EVP_CIPHER_CTX_new();
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    std::vector<std::thread> th;
    for (int i = 0; i < nthreads; i++)
        th.emplace_back([&, i] {
            std::vector<uint8_t*> res(h->nq);
            for (int a = 0; a < h->nq; a++) res[a] = outs[i].data() + (size_t)a * h->efs;
            runOptimizedDPFTreeQuery(&views[i], (uint8_t*)key, h->nq, res.data());
        });
    for (auto& t : th) t.join();
    clock_gettime(CLOCK_MONOTONIC, &t1);
    for (auto& v : views) EVP_CIPHER_CTX_free(v.ctx);
    memcpy(result, outs[0].data(), outs[0].size());
    int same = 1;
    for (int i = 1; i < nthreads; i++) same &= outs[i] == outs[0];
    double dt = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    return same ? dt : -dt;
}

// `count` independent runOptimizedDPFTreeQuery calls (server.cpp:96-134) at once, one thread
// each: call i answers keys[i*kl ..] as party party1[i] into results[i*nq*efs ..].  Each thread
// gets a shallow copy of the server with its own EVP context and partyIndex (the fields the
// answer reads); the shard rows are shared read-only.  Used for the full-size goldens.
void ref_server_answer_many(void* hv, const uint8_t* keys, int kl, const int* party1, int count,
                            uint8_t* results) {
    ref_srv* h = (ref_srv*)hv;
    set_tree_globals(h->p, h->n, h->efs, h->nq);
    std::vector<server> views(count, h->s);
    for (int i = 0; i < count; i++) {
        views[i].ctx = EVP_CIPHER_CTX_new();
        views[i].partyIndex = party1[i];
        views[i].isByzantine = 0;
    }
    std::vector<std::thread> th;
    for (int i = 0; i < count; i++)
        th.emplace_back([&, i] {
            std::vector<uint8_t*> res(h->nq);
            for (int a = 0; a < h->nq; a++)
                res[a] = results + ((size_t)i * h->nq + a) * h->efs;
            runOptimizedDPFTreeQuery(&views[i], (uint8_t*)keys + (size_t)i * kl, h->nq, res.data());
        });
    for (auto& t : th) t.join();
    for (auto& v : views) EVP_CIPHER_CTX_free(v.ctx);
}

// params.cpp:467-642 sizing for tree mode: setSystemParams(L,f,t=1,k,r,b=0,rho,mac,mode=0)
void ref_e2e_sizes(int L, int f, int k, int r, int rho, int* out5) {
    setSystemParams(L, f, 1, k, r, 0, rho, 0, 0);
    out5[0] = NUM_PARTIES;
    out5[1] = LOG_NUM_ENCODED_FILES;
    out5[2] = ENCODED_FILE_SIZE_BYTES;
    out5[3] = NUM_ROUNDS;
    out5[4] = calcOptimizedDPFTreeKeyLength(NUM_PARTIES, LOG_NUM_ENCODED_FILES, NUM_ROUNDS);
}

// The in-process cluster of correctness_tests.cpp:230-372 with the Go server's
// encode-across setup (server.go:299-331): synthetic DB (client.cpp:16-33), p servers
// encoded across files (client.cpp:70-97), keys (client.cpp:144-153), every party's
// runOptimizedDPFTreeQuery answer, first r parties erased, decode (client.cpp:211-268).
// Buffers: files[2^L*f], shards[p*N*efs], keys[p*kl], answers[p*nq*efs], decoded[f].
// Returns 1 when decoded == file[idx].
int ref_e2e(int L, int f, int k, int r, int rho, int idx, uint8_t* files, uint8_t* shards,
            uint8_t* keys_out, uint8_t* answers, uint8_t* decoded) {
    setSystemParams(L, f, 1, k, r, 0, rho, 0, 0);
    int p = NUM_PARTIES, nq = NUM_ROUNDS, efs = ENCODED_FILE_SIZE_BYTES;
    size_t N = NUM_ENCODED_FILES;
    int kl = calcOptimizedDPFTreeKeyLength(p, LOG_NUM_ENCODED_FILES, nq);
    client c;
    initialize_client(&c, L, FILE_SIZE_BYTES);
    for (int i = 0; i < NUM_FILES; i++) memcpy(files + (size_t)i * f, c.unencoded_files[i], f);
    std::vector<server> servers(p);
    for (int i = 0; i < p; i++) {
        initializeServer(&servers[i], i + 1, LOG_NUM_ENCODED_FILES, efs, 0, 1);
        encode_across_files_server(&c, &servers[i]);
        for (size_t j = 0; j < N; j++)
            memcpy(shards + ((size_t)i * N + j) * efs, servers[i].indexList[j], efs);
    }
    uint8_t** keys = (uint8_t**)malloc(p * sizeof(uint8_t*));
    for (int j = 0; j < p; j++) keys[j] = (uint8_t*)malloc(kl);
    generate_opt_DPF_tree_query(&c, idx, &keys);
    std::vector<std::vector<uint8_t*>> resp(p, std::vector<uint8_t*>(nq));
    for (int i = 0; i < p; i++) {
        memcpy(keys_out + (size_t)i * kl, keys[i], kl);
        for (int a = 0; a < nq; a++) resp[i][a] = answers + ((size_t)i * nq + a) * efs;
        runOptimizedDPFTreeQuery(&servers[i], keys[i], nq, resp[i].data());
    }
    std::vector<uint8_t> erasure(p);
    for (int i = 0; i < p; i++) erasure[i] = (i < r) ? 0 : 1;
    int numResponses = p - r;
    uint8_t*** test = (uint8_t***)malloc(numResponses * sizeof(uint8_t**));
    for (int i = 0, cur = 0; i < p; i++) {
        if (!erasure[i]) continue;
        test[cur++] = resp[i].data();
    }
    std::vector<uint8_t> out(FILE_SIZE_BYTES);
    assembleDPFTreeQueryResponses(&c, erasure.data(), test, out.data());
    memcpy(decoded, out.data(), f);
    int ok = memcmp(out.data(), c.unencoded_files[idx], f) == 0;
    free(test);
    for (int j = 0; j < p; j++) free(keys[j]);
    free(keys);
    for (int i = 0; i < p; i++) freeServer(&servers[i]);
    return ok;
}

// Polynomial (Hollanti) PIR end to end, the harness of correctness_tests.cpp:924-1020 with the
// Go server's setup (server.go:299-319, ENCODE_ACROSS == 0): setSystemParams(mode 3), the
// synthetic DB, p servers encoded within files (client.cpp:99-103), generateHollantiQuery
// (client.cpp:201-203 -> shamir_dpf.cpp:190-237), every party's runHollantiQuery answer, the
// same answer from T runHollantiQueryThread slices + assembleHollantiQueryThreadResults
// (server.cpp:345-382), the first r parties erased, assembleHollantiResponses (client.cpp:499).
// Buffers: shards[p*N*efs], keys[p*nq*N], answers[p*nq*efs], thread_answers[p*nq*efs],
// decoded[f].  Returns 1 when decoded == file[idx].
int ref_hollanti_e2e(int L, int f, int t, int k, int r, int rho, int idx, int nthreads,
                     uint8_t* shards, uint8_t* keys_out, uint8_t* answers,
                     uint8_t* thread_answers, uint8_t* decoded) {
    setSystemParams(L, f, t, k, r, 0, rho, 0, 3);
    int p = NUM_PARTIES, nq = NUM_ROUNDS, efs = ENCODED_FILE_SIZE_BYTES;
    size_t N = NUM_ENCODED_FILES;
    client c;
    initialize_client(&c, L, FILE_SIZE_BYTES);
    std::vector<server> servers(p);
    for (int i = 0; i < p; i++) {
        initializeServer(&servers[i], i + 1, LOG_NUM_ENCODED_FILES, efs, 0, nthreads);
        encode_within_files_server(&c, &servers[i]);
        for (size_t j = 0; j < N; j++)
            memcpy(shards + ((size_t)i * N + j) * efs, servers[i].indexList[j], efs);
    }
    uint8_t*** keys = (uint8_t***)malloc(p * sizeof(uint8_t**));
    for (int i = 0; i < p; i++) {
        keys[i] = (uint8_t**)malloc(nq * sizeof(uint8_t*));
        for (int j = 0; j < nq; j++) keys[i][j] = (uint8_t*)malloc(NUM_FILES);
    }
    generateHollantiQuery(&c, idx, keys);
    std::vector<std::vector<uint8_t*>> resp(p, std::vector<uint8_t*>(nq));
    int slice = (int)N / nthreads;
    for (int i = 0; i < p; i++) {
        for (int j = 0; j < nq; j++) {
            memcpy(keys_out + ((size_t)i * nq + j) * N, keys[i][j], N);
            resp[i][j] = answers + ((size_t)i * nq + j) * efs;
        }
        runHollantiQuery(&servers[i], keys[i], resp[i].data());
        uint8_t*** in = (uint8_t***)malloc(nthreads * sizeof(uint8_t**));
        for (int th = 0; th < nthreads; th++) {
            in[th] = (uint8_t**)malloc(nq * sizeof(uint8_t*));
            for (int j = 0; j < nq; j++) in[th][j] = (uint8_t*)malloc(efs);
            runHollantiQueryThread(&servers[i], keys[i], th, th * slice, (th + 1) * slice, in[th]);
        }
        std::vector<uint8_t*> out(nq);
        for (int j = 0; j < nq; j++) out[j] = thread_answers + ((size_t)i * nq + j) * efs;
        assembleHollantiQueryThreadResults(&servers[i], in, nthreads, out.data());
        for (int th = 0; th < nthreads; th++) {
            for (int j = 0; j < nq; j++) free(in[th][j]);
            free(in[th]);
        }
        free(in);
    }
    std::vector<uint8_t> erasure(p);
    for (int i = 0; i < p; i++) erasure[i] = (i < r) ? 0 : 1;
    int numResponses = p - r;
    uint8_t*** test = (uint8_t***)malloc(numResponses * sizeof(uint8_t**));
    for (int i = 0, cur = 0; i < p; i++)
        if (erasure[i]) test[cur++] = resp[i].data();
    std::vector<uint8_t> out(FILE_SIZE_BYTES);
    assembleHollantiResponses(&c, erasure.data(), test, out.data());
    memcpy(decoded, out.data(), f);
    int ok = memcmp(out.data(), c.unencoded_files[idx], f) == 0;
    free(test);
    for (int i = 0; i < p; i++) {
        for (int j = 0; j < nq; j++) free(keys[i][j]);
        free(keys[i]);
    }
    free(keys);
    for (int i = 0; i < p; i++) freeServer(&servers[i]);
    return ok;
}

// setSystemParams(L,f,t,k,r,0,rho,0,3) sizing: p, efs, nq
void ref_hollanti_sizes(int L, int f, int t, int k, int r, int rho, int* out3) {
    setSystemParams(L, f, t, k, r, 0, rho, 0, 3);
    out3[0] = NUM_PARTIES;
    out3[1] = ENCODED_FILE_SIZE_BYTES;
    out3[2] = NUM_ROUNDS;
}

int ref_shamir_key_len(int n) { return calcShamirDPFKeyLength(n); }

// client-side names of package c (src/client, src/benchmark): utils.cpp:32-34, 118-129, 145-174
void ref_mac(uint8_t* key, uint8_t* input, int inputLen, uint8_t* out32) {
    mac(key, input, inputLen, out32, 32);
}
int ref_cd_key_len(int p, int n, int t, int needed, int keys) {
    return calcCDDPFKeyLength(p, n, t, needed, keys);
}
int ref_woodruff_key_len(int p, int r, int t, int n, int f) {
    return calcWoodruffKeyLength(p, r, t, n, f);
}
int ref_choose(int n, int k) { return choose(n, k); }

// ---- multiparty sqrt(N) DPF (mode 1) --------------------------------------------------------
// utils.cpp:105-116
int ref_mp_key_len(int p, int n, int t) { return calcMultiPartyOptDPFKeyLength(p, n, t); }

// setSystemParams(L,f,t,k,r,b,rho,0,mode=1) sizing: p, n, efs, NUM_RSS_KEYS, key length
void ref_mp_sizes(int L, int f, int t, int k, int r, int b, int rho, int* out5) {
    setSystemParams(L, f, t, k, r, b, rho, 0, 1);
    out5[0] = NUM_PARTIES;
    out5[1] = LOG_NUM_ENCODED_FILES;
    out5[2] = ENCODED_FILE_SIZE_BYTES;
    out5[3] = NUM_RSS_KEYS;
    out5[4] = calcMultiPartyOptDPFKeyLength(NUM_PARTIES, LOG_NUM_ENCODED_FILES, T);
}

// multiparty_dpf.cpp:467-539 (num_threads == 0) or the Thread form :541-615 for one thread;
// out is nrk x 2^n (dataShare[a][r])
void ref_mp_eval(int p, int n, int t, int nrk, const uint8_t* key, int thread_num,
                 int num_threads, uint8_t* out) {
    NUM_RSS_KEYS = nrk;
    EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
    size_t N = (size_t)1 << n;
    std::vector<uint8_t*> ds(nrk);
    for (int a = 0; a < nrk; a++) ds[a] = out + a * N;
    if (num_threads == 0)
        evalAllOptMultiPartyDPF(ctx, p, n, (uint8_t*)key, t, ds.data());
    else
        evalAllOptMultiPartyDPFThread(ctx, p, n, (uint8_t*)key, t, ds.data(), thread_num,
                                      num_threads);
    EVP_CIPHER_CTX_free(ctx);
}

// server.cpp:136-176 (num_threads == 0) or num_threads runOptimizedMultiPartyDPFQueryThread
// calls + assembleMultipartyDPFQueryThreadResults (server.cpp:384-441) on a resident server
// (ref_server_new with nq = nrk); result is nrk x efs
void ref_mp_server_answer(void* hv, int p, int t, int nrk, const uint8_t* key, int num_threads,
                          uint8_t* result) {
    ref_srv* h = (ref_srv*)hv;
    set_tree_globals(h->p, h->n, h->efs, h->nq);
    NUM_PARTIES = p;
    T = t;
    NUM_RSS_KEYS = nrk;
    std::vector<uint8_t*> res(nrk);
    for (int a = 0; a < nrk; a++) res[a] = result + (size_t)a * h->efs;
    if (num_threads == 0) {
        runOptimizedMultiPartyDPFQuery(&h->s, (uint8_t*)key, res.data());
        return;
    }
    if (num_threads > h->s.numThreads) {  // one EVP context per thread (server.cpp:393)
        fprintf(stderr, "ref_mp_server_answer: server built with %d threads\n", h->s.numThreads);
        abort();
    }
    std::vector<std::vector<std::vector<uint8_t>>> buf(
        num_threads, std::vector<std::vector<uint8_t>>(nrk, std::vector<uint8_t>(h->efs)));
    std::vector<std::vector<uint8_t*>> rows(num_threads, std::vector<uint8_t*>(nrk));
    std::vector<uint8_t**> in(num_threads);
    for (int th = 0; th < num_threads; th++) {
        for (int a = 0; a < nrk; a++) rows[th][a] = buf[th][a].data();
        in[th] = rows[th].data();
        runOptimizedMultiPartyDPFQueryThread(&h->s, (uint8_t*)key, th, num_threads, in[th]);
    }
    assembleMultipartyDPFQueryThreadResults(&h->s, in.data(), num_threads, res.data());
}

// ---- covering-design (CD) sqrt(N) DPF (mode 4) -----------------------------------------------
// params.cpp:12 `int M = 4`: setModeParams(CD) sets it to 2 for K = 2, B = 1 and nothing resets
// it, so every setup below starts from the default (a fresh process would)
extern int M;

// setSystemParams(L,f,t,k,r,b,rho,0,mode=4) sizing: p, n, efs, NUM_CD_KEYS, NUM_CD_KEYS_NEEDED,
// calcCDDPFKeyLength (utils.cpp:118-129)
void ref_cd_sizes(int L, int f, int t, int k, int r, int b, int rho, int* out6) {
    M = 4;
    setSystemParams(L, f, t, k, r, b, rho, 0, 4);
    out6[0] = NUM_PARTIES;
    out6[1] = LOG_NUM_ENCODED_FILES;
    out6[2] = ENCODED_FILE_SIZE_BYTES;
    out6[3] = NUM_CD_KEYS;
    out6[4] = NUM_CD_KEYS_NEEDED;
    out6[5] = calcCDDPFKeyLength(NUM_PARTIES, LOG_NUM_ENCODED_FILES, T, NUM_CD_KEYS_NEEDED,
                                 NUM_CD_KEYS);
}

// The CD harness of correctness_tests.cpp:568-715 (the reference's one active test, main :1236)
// with the Go server's encode-across setup: setSystemParams(mode 4), the synthetic DB
// (client.cpp:16-33), p servers encoded across files (client.cpp:70-97; the last b of them
// Byzantine, as the harness marks them -- runCDQueryThread answers honestly either way,
// server.cpp:464-485), generateCDQuery (client.cpp:159-161 -> genCDDPF,
// multiparty_dpf.cpp:275-408), every party's answer from nthreads runCDQueryThread slices +
// assembleCDQueryThreadResults (server.cpp:443-503), the first r parties erased,
// assembleCDResponses (client.cpp:562-615) when `decode`.  Buffers: shards[p*N*efs],
// keys[p*kl], answers[p*nck*efs], decoded[f].  Returns 1 when decoded == file[idx] (-1: no decode).
int ref_cd_e2e(int L, int f, int t, int k, int r, int b, int rho, int idx, int nthreads,
               int decode, uint8_t* shards, uint8_t* keys_out, uint8_t* answers,
               uint8_t* decoded) {
    M = 4;
    setSystemParams(L, f, t, k, r, b, rho, 0, 4);
    int p = NUM_PARTIES, nck = NUM_CD_KEYS, efs = ENCODED_FILE_SIZE_BYTES;
    size_t N = NUM_ENCODED_FILES;
    int kl = calcCDDPFKeyLength(p, LOG_NUM_ENCODED_FILES, T, NUM_CD_KEYS_NEEDED, NUM_CD_KEYS);
    client c;
    initialize_client(&c, L, FILE_SIZE_BYTES);
    std::vector<server> servers(p);
    for (int i = p - 1, byz = 0; i >= 0; i--) {
        const int isByz = byz < b ? 1 : 0;
        byz += isByz;
        initializeServer(&servers[i], i + 1, LOG_NUM_ENCODED_FILES, efs, isByz, nthreads);
        encode_across_files_server(&c, &servers[i]);
        for (size_t j = 0; j < N; j++)
            memcpy(shards + ((size_t)i * N + j) * efs, servers[i].indexList[j], efs);
    }
    uint8_t** keys = (uint8_t**)malloc(p * sizeof(uint8_t*));
    for (int j = 0; j < p; j++) keys[j] = (uint8_t*)malloc(kl);
    generateCDQuery(&c, idx, &keys);
    std::vector<std::vector<uint8_t*>> resp(p, std::vector<uint8_t*>(nck));
    for (int i = 0; i < p; i++) {
        memcpy(keys_out + (size_t)i * kl, keys[i], kl);
        for (int a = 0; a < nck; a++) resp[i][a] = answers + ((size_t)i * nck + a) * efs;
        std::vector<std::vector<std::vector<uint8_t>>> buf(
            nthreads, std::vector<std::vector<uint8_t>>(nck, std::vector<uint8_t>(efs)));
        std::vector<std::vector<uint8_t*>> rows(nthreads, std::vector<uint8_t*>(nck));
        std::vector<uint8_t**> in(nthreads);
        for (int th = 0; th < nthreads; th++) {
            for (int a = 0; a < nck; a++) rows[th][a] = buf[th][a].data();
            in[th] = rows[th].data();
            runCDQueryThread(&servers[i], keys[i], th, nthreads, in[th]);
        }
        assembleCDQueryThreadResults(&servers[i], in.data(), nthreads, resp[i].data());
    }
    int ok = -1;
    if (decode) {
    std::vector<uint8_t> erasure(p);
    for (int i = 0; i < p; i++) erasure[i] = (i < r) ? 0 : 1;
    uint8_t*** test = (uint8_t***)malloc((p - r) * sizeof(uint8_t**));
    for (int i = 0, cur = 0; i < p; i++)
        if (erasure[i]) test[cur++] = resp[i].data();
    std::vector<uint8_t> out(FILE_SIZE_BYTES);
    assembleCDResponses(&c, erasure.data(), test, out.data());
    memcpy(decoded, out.data(), f);
    ok = memcmp(out.data(), c.unencoded_files[idx], f) == 0;
    free(test);
    }
    for (int j = 0; j < p; j++) free(keys[j]);
    free(keys);
    for (int i = 0; i < p; i++) freeServer(&servers[i]);
    return ok;
}

}  // extern "C"
