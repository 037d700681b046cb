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
 *   setSystemParams / freeParams       params.h:63-64,  params.cpp:467-642 (tree mode only)
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
 *   - no Woodruff MAPPING_INDEX tables (params.cpp:621-640; out of scope, and overflowing).
 */
#ifndef PIR_SERVER_H
#define PIR_SERVER_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    void *ctx;          /* pir_engine_t* (created lazily on the first query) */
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

void initialize_client(client *c, uint8_t log_num_files, uint32_t file_size_bytes);
void free_client(client *c);
void encode_across_files_server(client *c, server *s);
/* client-side erasure decode of one tree-mode query (client.h:33, client.cpp:211-268,
 * semi-honest: B == 0): responses[j][round][byte] from the NUM_PARTIES - R servers q with
 * erasureIndexList[q-1] == 1, in increasing q; output = the FILE_SIZE_BYTES record. */
void assembleDPFTreeQueryResponses(client *c, uint8_t *erasureIndexList, uint8_t ***responses,
                                   uint8_t *output);
/* interpolation.h:10, interpolation.cpp:176-196 */
void lagrangeInterpolationSemihonest(uint8_t *evalPoints, uint8_t numPoints, uint8_t *evals,
                                     uint8_t funcDegree, uint8_t *output);

/* Engine device used by servers created after this call (default: $PIR_DEVICE or 0). */
void pirSetDevice(int device);
/* indexList rows were written by something other than encode_across_files_server: the next
 * query re-uploads the shard to HBM (encode_across_files_server does this implicitly). */
void pirServerShardChanged(server *s);

#ifdef __cplusplus
}
#endif
#endif
