/* pir_engine.h -- C ABI of the MI355X tree-DPF PIR answer engine (libpir_engine.so).
 *
 * Plain pointers and sizes only.  One engine = one PIR server's shard (or one partition of
 * it) resident in the HBM of one GPU.  Every entry point returns 0 on success and a
 * negative PIR_E* code on failure (message: pir_engine_last_error()); the server.h-compatible
 * shim (pir_server.h) turns failures into abort(), like the reference's handleErrors()
 * (src/c/utils.cpp:11-15).
 *
 * Reference interfaces replaced (paths relative to /root/reference/src/c):
 *   pir_engine_create / _destroy     initializeServer / freeServer          server.cpp:17-52
 *   pir_engine_set_shard[_rows]      the indexList rows written by encode_across_files_server
 *                                                                           client.cpp:93-97
 *   pir_engine_answer                runOptimizedDPFTreeQuery               server.cpp:96-134
 *   pir_engine_answer_slice          runOptimizedDPFTreeQueryThread (intended semantics)
 *                                                                           server.cpp:505-549
 *   pir_engine_answer_slices[_dev]   the T concurrent ...Thread calls of one query
 *                                    (src/server_util/tree.go:60-76)        server.cpp:505-549
 *   pir_engine_eval_all              evalAllOptimizedDPF                    dpf_tree.cpp:473-598
 *   pir_engine_answer_coefs[_dev]    runHollantiQuery / ...Thread           server.cpp:321-371
 *   pir_engine_answer_mp[_dev]       runOptimizedMultiPartyDPFQuery[Thread] server.cpp:136-176,
 *                                    (evalAllOptMultiPartyDPF[Thread])      :384-430,
 *                                                                 multiparty_dpf.cpp:467-615
 *   pir_engine_mp_key_len            calcMultiPartyOptDPFKeyLength          utils.cpp:105-116
 *   pir_engine_mp_num_keys           NUM_RSS_KEYS                           params.cpp:618
 *   pir_engine_answer_cd[_dev]       runCDQueryThread (evalAllCDThread)     server.cpp:443-492,
 *                                                                 multiparty_dpf.cpp:617-690
 *   pir_engine_cd_key_len            calcCDDPFKeyLength                     utils.cpp:118-129
 *   pir_engine_key_len               calcOptimizedDPFTreeKeyLength          utils.cpp:85-90
 *   pir_comm_* + partitions          (new) split-shard across GPUs, XOR all-reduce over RCCL
 */
#ifndef PIR_ENGINE_H
#define PIR_ENGINE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PIR_OK 0
#define PIR_EINVAL (-1)  /* bad argument / unsupported shape          */
#define PIR_EHIP (-2)    /* a HIP runtime call failed                  */
#define PIR_ENOMEM (-3)  /* device or host allocation failed           */
#define PIR_ECOMM (-4)   /* RCCL failure                               */
#define PIR_ESTATE (-5)  /* call not valid in the engine's state       */

#define PIR_MAX_PARTIES 17 /* p - 1 <= 16 control bits                   */
#define PIR_MAX_ROUNDS 16  /* NUM_ROUNDS bytes come from one AES block   */
#define PIR_MAX_LOG_RECORDS 40

typedef struct pir_engine pir_engine_t;

typedef struct {
    int device;             /* HIP device ordinal                                     */
    int num_parties;        /* p = NUM_PARTIES (2..17)                                */
    int party_index;        /* 1-based, as server.partyIndex                          */
    int log_num_records;    /* n = LOG_NUM_ENCODED_FILES: depth of the DPF tree       */
    uint32_t record_bytes;  /* ENCODED_FILE_SIZE_BYTES                                */
    int num_rounds;         /* NUM_ROUNDS (1..16): output bytes per leaf              */
    int log_num_partitions; /* G: the logical shard is split into 2^G row partitions  */
    int partition_index;    /* which partition this engine holds (0 when G == 0)      */
    int is_byzantine;       /* answers are random bytes (server.cpp:116-119)          */
} pir_engine_config;

const char *pir_engine_last_error(void);
int pir_engine_create(const pir_engine_config *cfg, pir_engine_t **out);
void pir_engine_destroy(pir_engine_t *e);
int pir_engine_key_len(int num_parties, int log_num_records, int num_rounds);
/* records (rows) held by this engine = 2^(n - G) */
uint64_t pir_engine_num_rows(const pir_engine_t *e);
/* answer later queries as party `party_index` (1-based) over the same shard: the reference's
 * server.partyIndex (server.h:16), which only selects the root control bits of the DPF
 * evaluation (dpf_tree.cpp:496-502).  Lets one resident shard serve every party's key in
 * tests and benchmarks without a second copy of it. */
int pir_engine_set_party_index(pir_engine_t *e, int party_index);

/* ---- shard (device-resident; rows are this engine's partition, row 0 = its first) ---- */
/* rows [row0, row0+nrows) from a host buffer with src_pitch bytes between rows */
int pir_engine_set_shard(pir_engine_t *e, const uint8_t *host, uint64_t row0, uint64_t nrows,
                         uint64_t src_pitch);
/* rows [row0, row0+nrows) from an array of row pointers (server.indexList): host threads
 * ($PIR_GATHER_THREADS, default min(8, cores)) gather ~64 MiB chunks into two pinned buffers,
 * chunk c + 1 while the DMA of chunk c runs */
int pir_engine_set_shard_rows(pir_engine_t *e, const uint8_t *const *rows, uint64_t row0,
                              uint64_t nrows);
/* the reverse: rows [row0, row0+nrows) of the device shard into row pointers (record_bytes
 * each), DMA into two pinned buffers, host threads scattering one while the other fills */
int pir_engine_get_shard_rows(pir_engine_t *e, uint8_t *const *rows, uint64_t row0,
                              uint64_t nrows);
/* synthetic shard generated on the device (bench): byte b of GLOBAL row i is a function of
 * (seed, i, b), so every partition of a logical shard agrees with the whole */
int pir_engine_fill_shard_random(pir_engine_t *e, uint64_t seed);
/* the server's erasure-coded shard, computed on the GPU (client.cpp:70-97, the server setup of
 * src/server/server.go:299-331): global row r = XOR_{j<k, src = encdb*j + r < num_files}
 * gf_pow(party_index, j) * file[src], encdb = ceil(num_files / k), for this engine's rows.
 * d_files: num_files device rows file_pitch bytes apart (record_bytes used), or NULL for the
 * reference's synthetic database (client.cpp:16-33). */
int pir_engine_encode_across_dev(pir_engine_t *e, const uint8_t *d_files, uint64_t file_pitch,
                                 uint64_t num_files, int k);
/* pir_engine_encode_across_dev from the client's HOST file rows (client.unencoded_files:
 * num_files row pointers, record_bytes read from each): the server setup of server.go:299-331
 * with the encode on the GPU.  Per ~64 MiB chunk of this engine's rows, host threads gather the
 * k source files of each row into pinned staging (chunk c + 1 while chunk c's DMA and encode
 * kernel run); the shard is left resident in HBM. */
int pir_engine_encode_across_rows(pir_engine_t *e, const uint8_t *const *files,
                                  uint64_t num_files, int k);
/* the same for pir_engine_encode_within_dev: num_files host rows of file_bytes each */
int pir_engine_encode_within_rows(pir_engine_t *e, const uint8_t *const *files,
                                  uint64_t num_files, uint32_t file_bytes, int k, int party);
/* the Hollanti-mode shard (MODE 3: encoded within files), computed on the GPU (client.cpp:43-56,
 * 99-103; replaces the host encode_within_files_server of the server setup): row r of this
 * engine's rows = XOR_{j<k} gf_pow(party, j) * part j of file r, part j = bytes
 * [j*record_bytes, (j+1)*record_bytes) of the file, zero past file_bytes; rows >= num_files are
 * zero.  d_files: num_files device rows file_pitch >= file_bytes bytes apart, or NULL for the
 * reference's synthetic database (client.cpp:16-33).  party: the server's party index (1..),
 * or 0 for the engine's party_index (a Hollanti engine is created with 2 parties: they only
 * size tree-DPF keys). */
int pir_engine_encode_within_dev(pir_engine_t *e, const uint8_t *d_files, uint64_t file_pitch,
                                 uint64_t num_files, uint32_t file_bytes, int k, int party);
int pir_engine_get_shard_row(pir_engine_t *e, uint64_t row, uint8_t *out);
/* rows [row0, row0+nrows) back to the host, record_bytes per row, packed */
int pir_engine_get_shard(pir_engine_t *e, uint64_t row0, uint64_t nrows, uint8_t *out);

/* ---- answers, host buffers (synchronous; key_len bytes of key) ---- */
/* result: num_rounds * record_bytes bytes, round a at result + a*record_bytes.  With a
 * communicator attached (pir_comm_attach) every rank receives the XOR over partitions. */
int pir_engine_answer(pir_engine_t *e, const uint8_t *key, uint8_t *result);
/* partial answer over the engine rows [t*R/T, (t+1)*R/T), R = rows held, T a power of 2 */
int pir_engine_answer_slice(pir_engine_t *e, const uint8_t *key, int thread_num,
                            int num_threads, uint8_t *result);
/* every slice of one query at once: results[t] (t < num_threads, num_rounds * record_bytes
 * each, back to back) = pir_engine_answer_slice(e, key, t, num_threads, .) -- the T calls of
 * one query that src/server_util/tree.go:60-76 issues concurrently with the same key
 * (runOptimizedDPFTreeQueryThread, server.cpp:505-549), computed by ONE tree and ONE pass over
 * the shard where the shape allows (the pir_server.h shim serves its Thread calls from it) */
int pir_engine_answer_slices(pir_engine_t *e, const uint8_t *key, int num_threads,
                             uint8_t *results);
int pir_engine_answer_slices_dev(pir_engine_t *e, const uint8_t *d_key, int num_threads,
                                 uint8_t *d_results, void *stream);
/* ---- explicit-coefficient answers: the Hollanti/Goldberg polynomial-PIR server scan
 *      (runHollantiQuery / runHollantiQueryThread, server.cpp:321-371) -- no DPF, the client
 *      sends one coefficient vector per round ----
 * result[a] = XOR_{r in [row0, row0+nrows)} coefs[a][r] * shard row r over GF(2^8)/0x11d, for
 * a < num_rounds; coefs[a] is indexed by engine row (num_rounds host pointers).  Always the
 * honest answer: the reference's Thread variant ignores isByzantine (server.cpp:353-369). */
int pir_engine_answer_coefs(pir_engine_t *e, const uint8_t *const *coefs, uint64_t row0,
                            uint64_t nrows, uint8_t *result);
/* device form: round a's coefficient of engine row r at d_coefs[a * coef_pitch + r] */
int pir_engine_answer_coefs_dev(pir_engine_t *e, const uint8_t *d_coefs, uint64_t coef_pitch,
                                uint64_t row0, uint64_t nrows, uint8_t *d_result, void *stream);
/* Multiparty sqrt(N) DPF answer of party index 1..p with threshold t (the engine must have
 * num_rounds == pir_engine_mp_num_keys(p, t), one output share per round):
 *   result[a] = XOR_{r in rows} share[a][r] * shard row r,   a < NUM_RSS_KEYS,
 *   share[a][i*mu + x] = XOR_{j: toggle[a][i][j] != 0} G(seed[i][j], mu)[x] ^ cw[j][x]
 * over the key layout of multiparty_dpf.cpp:133-273 / :467-539 (seeds, toggle bytes, correction
 * words; mu = 2^ceil(log2(ceil(2^(n/2) * 2^((p-1)/2)))) records per row, nu = 2^n / mu rows).
 * rows: the thread slice [thread_num*S*mu, (thread_num+1)*S*mu), S = nu / num_threads, of
 * runOptimizedMultiPartyDPFQueryThread (num_threads = 1: the whole domain), within this engine's
 * partition.  key_bytes >= pir_engine_mp_eval_bytes(p, n, t) (the bytes the evaluation reads;
 * calcMultiPartyOptDPFKeyLength sizes the buffer the Go client sends).  Always the honest
 * answer (the Byzantine branch of server.cpp:157-160 is the caller's). */
int pir_engine_answer_mp(pir_engine_t *e, const uint8_t *key, uint64_t key_bytes, int p, int t,
                         int thread_num, int num_threads, uint8_t *result);
int pir_engine_answer_mp_dev(pir_engine_t *e, const uint8_t *d_key, int p, int t, int thread_num,
                             int num_threads, uint8_t *d_result, void *stream);
int pir_engine_mp_num_keys(int p, int t);
int pir_engine_mp_key_len(int p, int n, int t);
long long pir_engine_mp_eval_bytes(int p, int n, int t); /* -1: no layout for (p, n, t) */
/* Covering-design sqrt(N) DPF answer (runCDQueryThread, server.cpp:443-492): the multiparty
 * evaluation and scan above on the layout of evalAllCDThread (multiparty_dpf.cpp:617-690):
 * NUM_CD_KEYS output shares (the engine must have num_rounds == num_cd_keys), 2^(q-1) seeds per
 * row (q = NUM_CD_KEYS_NEEDED), mu = 2^(n/2 + 3) records per row (integer n / 2), nu = 2^n / mu
 * rows (0 when mu > 2^n: the answer is zero), the same thread slices.  key_bytes >=
 * pir_engine_cd_key_len(...) (= the bytes the evaluation reads).  Always the honest answer:
 * both branches of runCDQueryThread compute it (server.cpp:466-485). */
int pir_engine_answer_cd(pir_engine_t *e, const uint8_t *key, uint64_t key_bytes,
                         int num_cd_keys_needed, int num_cd_keys, int thread_num, int num_threads,
                         uint8_t *result);
int pir_engine_answer_cd_dev(pir_engine_t *e, const uint8_t *d_key, int num_cd_keys_needed,
                             int num_cd_keys, int thread_num, int num_threads, uint8_t *d_result,
                             void *stream);
/* calcCDDPFKeyLength(p, n, t, q, c) (p and t unused there too); 0 for no layout */
int pir_engine_cd_key_len(int p, int n, int t, int num_cd_keys_needed, int num_cd_keys);
/* DPF shares of this engine's rows: out[a*R + i] (dataShare[a][i]) */
int pir_engine_eval_all(pir_engine_t *e, const uint8_t *key, uint8_t *out);

/* ---- answers, device-resident (asynchronous on `stream`, a hipStream_t or NULL for the
 *      engine's own stream).  Answers share the engine's work buffers: one enqueued on a
 *      different stream than the previous answer waits on the device for that answer (an
 *      event recorded on the previous stream; answers that stay on one stream record none, so
 *      back-to-back launches there carry no event-record dispatch gap). ---- */
int pir_engine_answer_dev(pir_engine_t *e, const uint8_t *d_key, uint8_t *d_result,
                          void *stream);
/* `num_keys` keys of key_len bytes back to back; results num_keys x num_rounds x record_bytes.
 * Keys are answered in groups of pir_engine_batch_group() keys per pass over the shard (the
 * shard is read once per group, each key's tree is evaluated separately). */
int pir_engine_answer_batch_dev(pir_engine_t *e, const uint8_t *d_keys, int num_keys,
                                uint8_t *d_result, void *stream);
/* host-buffer form of the above (synchronous) */
int pir_engine_answer_batch(pir_engine_t *e, const uint8_t *keys, int num_keys,
                            uint8_t *results);
/* a queue of `num_keys` independent queries (keys of key_len bytes back to back; results
 * num_keys x num_rounds x record_bytes), each answered exactly as pir_engine_answer_dev would
 * -- its own DPF tree and its own full pass over the shard -- back to back in one launch where
 * the shape allows, so that the tree of query k+1 is built while query k's rows stream. */
int pir_engine_answer_stream_dev(pir_engine_t *e, const uint8_t *d_keys, int num_keys,
                                 uint8_t *d_result, void *stream);
/* pre-size the device work buffers of pir_engine_answer_stream_dev for queues of up to
 * `num_keys` queries (a server sizes its queue at setup), so that no answer call allocates:
 * the reference has no counterpart (its buffers are host mallocs per call, server.cpp:108-114). */
int pir_engine_reserve_queue(pir_engine_t *e, int num_keys);
/* keys per shard pass: 0 = automatic (8 / nrp), else a power of two <= 16 / nrp, where nrp =
 * num_rounds rounded up to a power of two.  Default from $PIR_BATCH_G. */
int pir_engine_set_batch_group(pir_engine_t *e, int keys_per_pass);
int pir_engine_batch_group(const pir_engine_t *e);
void *pir_engine_stream(pir_engine_t *e);
int pir_engine_sync(pir_engine_t *e);
/* device scratch the caller may use for keys/results (freed with the engine) */
int pir_engine_alloc_dev(pir_engine_t *e, size_t bytes, void **d_ptr);
/* release a pir_engine_alloc_dev buffer before the engine is destroyed (waits for the device) */
int pir_engine_free_dev(pir_engine_t *e, void *d_ptr);
int pir_engine_memcpy_h2d(pir_engine_t *e, void *d_dst, const void *h_src, size_t bytes);
int pir_engine_memcpy_d2h(pir_engine_t *e, void *h_dst, const void *d_src, size_t bytes);

/* ---- per-phase device time of answers (HIP events on the answering stream) ---- */
/* phases: key_prep, tree_frontier, tree_leaves, scan, reduce, comm_fold.  `slots` event sets
 * are kept in a ring (0 = off); last_timings averages the answers recorded since the previous
 * read (at most `slots`), fills up to `max` {name, ms} pairs and returns the count. */
typedef struct {
    char name[32];
    float ms;
} pir_kernel_time;
int pir_engine_set_profiling(pir_engine_t *e, int slots);
int pir_engine_last_timings(pir_engine_t *e, pir_kernel_time *out, int max);
/* diagnostics: each phase run alone `iters` times back to back (no pipelining); out_ms[5] =
 * mean ms of key_prep, tree_frontier, tree_stages (all expand stages), scan (one launch over
 * all rows), reduce.  d_key: device pointer to one raw key. */
int pir_engine_profile_phases(pir_engine_t *e, const uint8_t *d_key, int iters, float *out_ms);
/* diagnostics: one single-launch answer (k_query) of a queue of num_keys keys with
 * per-workgroup phase stamps.  out holds max_wgs x 256 uint64 wall-clock ticks (100 MHz)
 * relative to the earliest start (0 = not reached): [0..6] start, key parsed, first tile root,
 * tile 0 shares ready, last tile of query 0 ready, query 0 scanned, query 0 slab written;
 * [8+d] descent level d of the first tile root (d < 32); [40+l] expansion level l of tile 0
 * (l < 16); [56], [57] shader clock (s_memtime) at start and at the first tile root; with
 * end-of-query work stealing (a lone query): [58] the tree waves' last chunk folded, [59] chunks
 * of other workgroups folded by this one's tree waves, [60] own chunks folded by the tree
 * waves, [61] own chunks folded by the scan waves (counts, not ticks); [64+g]
 * queue tile g ready, [96+g] queue tile g consumed by scan wave 0, [128+g] shader clock at
 * [64+g] (g < 32); [160+l] expansion level l of queue tile 1 (built by the tree waves beside
 * the scan), [176] its root ready; [192+8w+k] (diagnostic builds with -DPIR_FOLD_STAMPS=1
 * only) shader cycles of fold phase k of four-Russians scan wave w.  Returns the number
 * of workgroups (>= 0), or an error code; PIR_EINVAL when the shape does not use k_query. */
int pir_engine_trace_query(pir_engine_t *e, const uint8_t *d_key, int num_keys, uint64_t *out,
                           int max_wgs);

/* ---- split shard across GPUs: XOR all-reduce of partition answers over RCCL ---- */
#define PIR_COMM_ID_BYTES 128
int pir_comm_unique_id(uint8_t id[PIR_COMM_ID_BYTES]);
/* rank r of nranks; nranks must equal 2^G of the engine's config and r its partition.  Every
 * answer then ends with ONE ncclAllGather of the partition partials (all queued queries'
 * nq x efs answers, query-major) + the XOR fold below.  An exchange that fails or does not
 * enqueue within $PIR_COMM_TIMEOUT seconds (default 60) aborts the communicator; the engine
 * then refuses every later answer with PIR_ECOMM. */
int pir_comm_attach(pir_engine_t *e, const uint8_t id[PIR_COMM_ID_BYTES], int nranks, int rank);
/* drop the communicator (aborted, never waited on) and answer this partition alone again; also
 * clears the refusal state after a failed exchange.  For callers that fall back to exchanging
 * partition answers themselves when a communicator could not be set up on every rank.  Call it
 * with no answer in flight: it waits for the engine's own stream only, and an exchange enqueued
 * on a caller's stream would be cut off by the abort. */
int pir_comm_detach(pir_engine_t *e);
/* what RCCL and HIP report for this engine (a multi-GPU run's self-check): attached = 1 when a
 * communicator is attached; count, user_rank and device = ncclCommCount, ncclCommUserRank and
 * ncclCommCuDevice of that communicator (-1 when none); engine_device = the engine's HIP device;
 * pci_bus_id = hipDeviceGetPCIBusId of it (so N ranks can be checked to sit on N distinct GPUs). */
typedef struct pir_comm_info {
  int attached;
  int count;
  int user_rank;
  int device;
  int engine_device;
  char pci_bus_id[64];
} pir_comm_info_t;
int pir_comm_info(pir_engine_t *e, pir_comm_info_t *out);
/* the combine step after the all-gather, on its own: d_gathered = nranks blocks of
 * bytes_per_rank (rank r's partial answers at r * bytes_per_rank: ncclAllGather's output
 * layout); d_result[i] = XOR over r of d_gathered[r * bytes_per_rank + i] (the XOR assembly of
 * server.cpp:553-562 across partitions).  Exposed so that one GPU can check a multi-rank
 * combine against the whole-shard answer before any multi-GPU run. */
int pir_engine_fold_gathered_dev(pir_engine_t *e, const uint8_t *d_gathered, int nranks,
                                 uint64_t bytes_per_rank, uint8_t *d_result, void *stream);

#ifdef __cplusplus
}
#endif
#endif
