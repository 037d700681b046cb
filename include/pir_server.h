/* pir_server.h -- drop-in for the tree-mode subset of the reference's src/c headers that the
 * Go server binds through SWIG/cgo (src/c/c.swigcxx:15-24).  Same names, argument meaning and
 * error behaviour (abort() on unrecoverable errors, like utils.cpp:11-15 handleErrors), backed
 * by the MI355X engine (pir_engine.h).  Exported with C linkage from libpir_engine.so.
 *
 * Replaces (paths relative to /root/reference/src/c):
 *   server struct                      server.h:13-25
 *   initializeServer / freeServer      server.h:27-28,  server.cpp:17-52
 *   runOptimizedDPFTreeQuery           server.h:33,     server.cpp:96-134
 *   runOptimizedDPFTreeQueryThread     server.h:48,     server.cpp:505-549 (intended semantics:
 *                                      partial answer over rows [t*N/T,(t+1)*N/T); the reference
 *                                      body is defective)
 *   assemblDPFTreeQueryThreadResults   server.h:53,     server.cpp:553-562
 *   setSystemParams / freeParams       params.h:63-64,  params.cpp:467-642 (tree, multiparty,
 *                                      Hollanti and covering-design modes; the others abort)
 *   runOptimizedMultiPartyDPFQuery[Thread], assembleMultipartyDPFQueryThreadResults
 *                                      server.h:37,46,52, server.cpp:136-176, :384-441
 *   calcMultiPartyOptDPFKeyLength      utils.h,         utils.cpp:105-116
 *   runCDQueryThread, assembleCDQueryThreadResults, calcCDDPFKeyLength
 *                                      server.h:49,53,  server.cpp:443-503, utils.cpp:118-129
 *   runHollantiQuery[Thread], assemble*QueryThreadResults, the other modes' entry points (abort)
 *                                      server.h:39-53,  server.cpp:304-665
 *   encode_within_files_server         client.h:29,     client.cpp:93-110
 *   the sizing globals                 params.h:9-33
 *   client / initialize_client / free_client / encode_across_files_server
 *                                      client.h:15-28,  client.cpp:16-41, :70-97 (server setup
 *                                      path of src/server/server.go:299-331)
 *   assembleDPFTreeQueryResponses      client.h:33,     client.cpp:211-268 (client decode)
 *   lagrangeInterpolationSemihonest    interpolation.h:10, interpolation.cpp:176-196
 *   calcOptimizedDPFTreeKeyLength      utils.h:26,      utils.cpp:85-90
 *
 * Deliberate differences (each a reference defect):
 *   - ctx / ctxThreads hold the engine handle instead of OpenSSL contexts (no Go code reads them);
 *   - NUM_RESPONSES is computed after NUM_PARTIES (params.cpp:473 reads it before);
 *   - every setSystemParams starts from the covering designs' M = 4 and isRss = 1
 *     (params.cpp:12, :372): the reference keeps the M = 2 of a K = 2, B = 1 CD setup
 *     (params.cpp:440) and a cleared isRss (:520-599) for all later calls;
 *   - no Woodruff MAPPING_INDEX tables (params.cpp:621-640; out of scope, and overflowing).
 *
 * Setup (src/server/server.go:299-331: setSystemParams, initialize_client, initializeServer,
 * encode_*_files_server): the encode runs on the GPU from the client's host files and leaves the
 * shard resident in HBM, so the first query after a setup answers from device memory.  indexList
 * is then materialised lazily: the shim itself syncs it back before anything reads or writes the
 * host rows (an engine re-creation, pirServerSetRows, a second encode); a C caller that reads or
 * writes indexList directly after a setup calls pirServerSyncRows first ($PIR_SHIM_HOST_SETUP=1:
 * the reference's host encode into indexList, uploaded lazily on the first query).
 *
 * Setup also stays on the host when indexList already holds data: rows written through
 * pirServerSetRows / pirServerShardChanged, or written (or read) directly -- any resident page of
 * the row block (mincore) -- so the encode is XORed into them as client.cpp:88 does.
 *
 * Cost model of runOptimizedDPFTreeQueryThread (N rows, T threads, one full pass = one shard
 * read): the first of a query's calls (same key, same T) waits for a second one -- up to
 * $PIR_SLICE_JOIN_US (default 200 us), or up to 5 ms when a fan-out is expected (the call comes
 * from pirRunTreeQueryThreads' pool, the server's last decided query met a partner, or an earlier
 * call of the same query already answered alone); it is woken by the first partner, so a fan-out
 * whose calls are on time pays nothing for the wait.
 *   - A partner arrives (the T goroutines of tree.go:60-76 start microseconds apart): the first
 *     call answers all T slices in ONE full pass (pir_engine_answer_slices); the others copy
 *     their slice out of it.  T calls cost one pass (+ the copies).
 *   - No partner: the call answers its own slice alone (pir_engine_answer_slice: a descent to
 *     node t and the scan of N/T rows), i.e. the wait + ~1/T of a pass + a lone query's head.
 *     A caller that asks for slices one at a time, or spreads them over processes, pays that
 *     per slice -- T slices then cost about one pass plus T heads and waits (the first lone
 *     call after a fan-out, and a repeat of a key answered alone, wait the 5 ms).
 * At most 8 queries' slice groups (and 256 MiB of their parts) are kept; the oldest is dropped
 * first.
 *
 * freeServer returns once no call can reach the server any more; the engine teardown (device
 * memory) and the row block's unmap run on a background thread ~20 ms later
 * ($PIR_REAPER_DEFER_MS); an engine created meanwhile (a setup or first query of any server) whose
 * device allocation does not fit beside it waits for the teardown and tries again.
 * tree.go:90-100 frees the server BEFORE sending each answer, so this keeps the teardown off the
 * response path.
 */
#ifndef PIR_SERVER_H
#define PIR_SERVER_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    void *ctx;          /* the shim's engine state (engine created at setup or first query) */
    void **ctxThreads;  /* unused, kept for field-name compatibility        */
    int partyIndex;
    uint8_t **indexList;
    int isByzantine;
    int numThreads;
} server;

typedef struct {
    void *ctx;
    const void *macCtx;
    uint8_t **unencoded_files;
    uint8_t *macKey;
} client;

extern int NUM_PARTIES;
extern int NUM_FILES;
extern uint32_t LOG_NUM_FILES;
extern uint32_t FILE_SIZE_BYTES;
extern uint32_t PAYLOAD_SIZE_BYTES;
extern int NUM_ENCODED_FILES;
extern int LOG_NUM_ENCODED_FILES;
extern int ENCODED_PAYLOAD_SIZE_BYTES;
extern int ENCODED_FILE_SIZE_BYTES;
extern int ENCODE_ACROSS;
extern int NUM_ROUNDS;
extern int RHO;
extern int K;
extern int T;
extern int R;
extern int B;
extern int NUM_RESPONSES;
extern int MODE;
extern int IS_HERMITE;
extern int D;
extern int MAC_SIZE_BYTES;
extern int CHECK_MAC;
/* globals of the other PIR modes (params.h:39-54), read by the Go mode handlers
 * (src/server_util/{multiparty,cd732,woodruff}.go); NUM_RSS_KEYS = the multiparty answer's
 * share count (params.cpp:603-619), NUM_CD_KEYS the covering-design answer's (params.cpp:519-599);
 * the Shamir and Woodruff modes are not served (see below) */
extern int NUM_RSS_KEYS;
extern int NUM_CD_KEYS;
extern int WOODRUFF_M;
extern int WOODRUFF_D;
extern int WOODRUFF_DERIVATIVE;

void setSystemParams(int logNumFiles, int fileSizeBytes, int t, int k, int r, int b, int rho,
                     int checkMac, int mode);
void freeParams(void);
int calcOptimizedDPFTreeKeyLength(int p, int log_domainSize, int numQueries);

void initializeServer(server *s, int partyIndex, uint32_t logNumFiles, uint32_t fileSizeBytes,
                      int isByzantine, int numThreads);
void freeServer(server *s);
void runOptimizedDPFTreeQuery(server *s, uint8_t *key, int numQueries, uint8_t **result);
void runOptimizedDPFTreeQueryThread(server *s, uint8_t *key, int threadNum, int numThreads,
                                    uint8_t **result);
void assemblDPFTreeQueryThreadResults(server *s, uint8_t ***in, int numThreads, uint8_t **out);

/* ---- polynomial (Hollanti/Goldberg, mode 3) PIR: the explicit-coefficient scan on the engine
 *      (server.h:39,44,51; server.cpp:321-382).  key[k] = the NUM_ROUNDS coefficient vectors of
 *      NUM_ENCODED_FILES bytes; result[k] = ENCODED_FILE_SIZE_BYTES. ---- */
void runHollantiQuery(server *s, uint8_t **key, uint8_t **result);
void runHollantiQueryThread(server *s, uint8_t **keys, int threadNum, int startIndex, int endIndex,
                            uint8_t **result);
void assembleHollantiQueryThreadResults(server *s, uint8_t ***in, int numThreads, uint8_t **out);

/* ---- multiparty sqrt(N) DPF PIR (mode 1): evalAllOptMultiPartyDPF[Thread]
 *      (multiparty_dpf.cpp:467-615) + the GF(2^8) scan, on the engine (pir_engine_answer_mp).
 *      key = calcMultiPartyOptDPFKeyLength(NUM_PARTIES, LOG_NUM_ENCODED_FILES, T) bytes (the
 *      evaluation reads the layout of multiparty_dpf.cpp:133-273, which fits inside it);
 *      result[a], a < NUM_RSS_KEYS, = ENCODED_FILE_SIZE_BYTES.  The Thread form answers rows
 *      [threadNum*S*mu, (threadNum+1)*S*mu), S = nu / numThreads (server.cpp:401-423); its
 *      Byzantine branch is the honest answer in the reference too. ---- */
int calcMultiPartyOptDPFKeyLength(int p, int log_domainSize, int t);
void runOptimizedMultiPartyDPFQuery(server *s, uint8_t *key, uint8_t **result);
void runOptimizedMultiPartyDPFQueryThread(server *s, uint8_t *key, int threadNum, int numThreads,
                                          uint8_t **result);
void assembleMultipartyDPFQueryThreadResults(server *s, uint8_t ***in, int numThreads,
                                             uint8_t **out);

/* ---- covering-design sqrt(N) DPF PIR (mode 4, src/server_util/cd732.go:64):
 *      evalAllCDThread (multiparty_dpf.cpp:617-690) + the GF(2^8) scan on the engine
 *      (pir_engine_answer_cd).  key = calcCDDPFKeyLength(NUM_PARTIES, LOG_NUM_ENCODED_FILES, T,
 *      NUM_CD_KEYS_NEEDED, NUM_CD_KEYS) bytes (genCDDPF's layout, multiparty_dpf.cpp:275-408);
 *      result[a], a < NUM_CD_KEYS, = ENCODED_FILE_SIZE_BYTES over rows
 *      [threadNum*S*mu, (threadNum+1)*S*mu), S = nu / numThreads (server.cpp:461-485; both
 *      of its branches are the honest answer). ---- */
void runCDQueryThread(server *s, uint8_t *key, int threadNum, int numThreads, uint8_t **result);
void assembleCDQueryThreadResults(server *s, uint8_t ***in, int numThreads, uint8_t **out);

/* ---- the other PIR modes' server entry points, bound by src/server_util/ (shamir.go:52,
 *      woodruff.go:69).  Their modes are outside this engine's scope: setSystemParams refuses
 *      modes 2, 5, 6, and these abort with a message if reached anyway.  The assemble functions
 *      are the reference's XOR folds (server.cpp:304-319, 647-665). ---- */
void runOptShamirDPFQueryThread(server *s, uint8_t **keys, int threadNum, int startIndex,
                                int endIndex, uint8_t **result);
void runWoodruffQueryThread(server *s, uint8_t *key, int threadNum, int startIndex, int endIndex,
                            uint8_t **result);
void assembleShamirQueryThreadResults(server *s, uint8_t ***in, int numThreads, uint8_t **out);
void assembleWoodruffQueryThreadResults(server *s, uint8_t ***in, int numThreads, uint8_t **out);
/* utils.h:29-30 */
int calcShamirDPFKeyLength(int log_domainSize);
int calcShamirResponseLength(int log_domainSize, int fileSizeBytes);

void initialize_client(client *c, uint8_t log_num_files, uint32_t file_size_bytes);
void free_client(client *c);
void encode_across_files_server(client *c, server *s);
/* client.cpp:93-110 (ENCODE_ACROSS == 0 modes, i.e. Hollanti): row i of party q =
 * XOR_{j<K} gf_pow(q, j) * file_i[j*EFS .. (j+1)*EFS) (gen_encode_matrix, coding.cpp:64-70) */
void encode_within_files_server(client *c, server *s);
/* client-side erasure decode of one tree-mode query (client.h:33, client.cpp:211-268,
 * semi-honest: B == 0): responses[j][round][byte] from the NUM_PARTIES - R servers q with
 * erasureIndexList[q-1] == 1, in increasing q; output = the FILE_SIZE_BYTES record. */
void assembleDPFTreeQueryResponses(client *c, uint8_t *erasureIndexList, uint8_t ***responses,
                                   uint8_t *output);
/* client-side decode of one polynomial (Hollanti) query (client.h:46, client.cpp:499-552,
 * semi-honest): responses[j][round][byte] from the NUM_PARTIES - R servers not erased */
void assembleHollantiResponses(client *c, uint8_t *erasureIndexList, uint8_t ***responses,
                               uint8_t *output);
/* interpolation.h:10, interpolation.cpp:176-196 */
void lagrangeInterpolationSemihonest(uint8_t *evalPoints, uint8_t numPoints, uint8_t *evals,
                                     uint8_t funcDegree, uint8_t *output);

/* ---- client-side names of package c: the Go files of src/client and src/benchmark bind
 *      the same SWIG package as the server (client.h:26-46, utils.h:22-48, shamir_dpf.h:4-6,
 *      woodruff.h:9-11), so the drop-in declares them too. ---- */
#ifndef SWIG
typedef unsigned __int128 uint128_t; /* utils.h:13-15 */
#endif
extern int NUM_CD_KEYS_NEEDED;       /* params.h:55 */
/* client.cpp:144-153 (tree.go:55): finalCW gf_pow(j, RHO*i) ^ 1 and genOptimizedDPF
 * (dpf_tree.cpp:142-274) on the GPU (pir_gen_keys), root seeds from the OS CSPRNG (the
 * reference: RAND_bytes); (*keys)[j] = party j's calcOptimizedDPFTreeKeyLength-byte key. */
void generate_opt_DPF_tree_query(client *c, int index, uint8_t ***keys);
/* client.cpp:201-203 -> genHollantiDPF (shamir_dpf.cpp:190-237) (hollanti.go:37):
 * keys[q][round][record] = value at q+1 of a random polynomial whose coefficient
 * T + (round+1)*RHO - 1 is [record == index] (host side; see pir_server.cpp for the
 * reference's one-byte over-read that is not inherited). */
void generateHollantiQuery(client *c, int index, uint8_t ***keys);
/* utils.cpp:32-34 (benchmark.go:198): HMAC-SHA256 under a 16-byte key; writes 32 bytes. */
void mac(uint8_t *key, uint8_t *input, int inputLen, unsigned char *output, int outputLen);
int choose(int n, int k);               /* utils.cpp:168-174 */
uint128_t convertInt(int x);            /* utils.cpp:221-223 */
int calcCDDPFKeyLength(int p, int log_domainSize, int t, int num_cd_keys_needed,
                       int num_cd_keys); /* utils.cpp:118-129 */
int calcWoodruffKeyLength(int p, int r, int t, int logDomainSize,
                          int fileSizeBytes); /* utils.cpp:145-153 */
/* The other modes' client halves (multiparty key generation and decode, CD key generation and
 * decode, Shamir, Woodruff): outside the server path this engine replaces; these abort with a
 * message. */
void generateMultiPartyDPFQuery(client *c, int index, uint8_t ***keys);
void assembleMultiPartyResponses(client *c, uint8_t *erasureIndexList, uint8_t ***responses,
                                 uint8_t *output);
void generateCDQuery(client *c, int index, uint8_t ***keys);
void assembleCDResponses(client *c, uint8_t *erasureIndexList, uint8_t ***responses,
                         uint8_t *output);
void genShamirCoeffs(int n, int t, int numRounds, uint128_t index, uint8_t ***coeffs_x,
                     uint8_t ***coeffs_y);
void genOptShamirDPF(int log_domainSize, uint128_t index, int t, int p, int numRounds,
                     uint8_t ***key_output, uint8_t ***coeffs_x, uint8_t ***coeffs_y);
void assembleShamirResponses(client *c, uint8_t *erasureIndexList, uint8_t ***responses,
                             uint8_t *output, uint8_t ***coeffs_x, uint8_t ***coeffs_y);
void genWoodruffVs(int t, int m, uint8_t **v);
void genWoodruffQuery(uint128_t index, int t, int p, int m, uint8_t **v, uint8_t **key_output);
void assembleWoodruffResponses(client *c, uint8_t *erasureIndexList, uint8_t ***responses,
                               uint8_t *output, uint8_t **v);

/* Harness helper (the fan-out of src/server_util/tree.go:60-80 for callers without Go):
 * numThreads threads of a persistent pool call runOptimizedDPFTreeQueryThread(s, key, t,
 * numThreads, .) concurrently, then assemblDPFTreeQueryThreadResults XORs the partials into
 * result[round] (ENCODED_FILE_SIZE_BYTES each). */
void pirRunTreeQueryThreads(server *s, uint8_t *key, int numThreads, uint8_t **result);

/* Engine device used by servers created after this call (default: $PIR_DEVICE or 0). */
void pirSetDevice(int device);
/* indexList rows were written by something other than encode_across_files_server: the next
 * query re-uploads the shard to HBM (encode_across_files_server does this implicitly).  After a
 * GPU setup, call pirServerSyncRows BEFORE writing the rows directly. */
void pirServerShardChanged(server *s);
/* After a setup that encoded on the GPU: copy the device shard into indexList (no-op if the
 * host rows are current).  For C callers that read or write indexList directly. */
void pirServerSyncRows(server *s);
/* Harness helper (no reference counterpart): copy `nrows` packed rows of `rowBytes` bytes
 * (rowBytes <= the server's fileSizeBytes) into indexList[row0 ..] and mark the shard changed
 * -- what a test or benchmark would otherwise do row by row through indexList. */
void pirServerSetRows(server *s, const uint8_t *rows, uint64_t row0, uint64_t nrows,
                      uint32_t rowBytes);
/* Harness helper (no reference counterpart): block until every freeServer's background
 * teardown has finished (device memory and host rows released). */
void pirServerWaitFreed(void);

#ifdef __cplusplus
}
#endif
#endif
