/* pir_client.h -- client-side helpers of the tree-DPF PIR protocol, on the GPU.
 *
 * Key generation (the client's half of the hot path's input) runs the same device AES as the
 * engine.  Replaces (paths relative to /root/reference/src/c):
 *   pir_gen_keys       genOptimizedDPF          dpf_tree.cpp:142-274 (root seeds supplied by the
 *                                               caller; the reference draws them with RAND_bytes)
 *   pir_final_cw       generate_opt_DPF_tree_query's finalCW values   client.cpp:144-153
 */
#ifndef PIR_CLIENT_H
#define PIR_CLIENT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* keys_out: p keys of pir_engine_key_len(p, n, nq) bytes, party j at keys_out + j*key_len.
 * fcw: nq*(p-1) bytes, fcw[a*(p-1) + j-1] = finalCW of party j (1 <= j < p) for round a.
 * root_seeds: p*16 bytes.  Synchronous; returns 0 or a negative PIR_E* code. */
int pir_gen_keys(int device, int n, uint64_t index, const uint8_t *fcw, int p, int nq,
                 const uint8_t *root_seeds, uint8_t *keys_out);
/* out[a*(p-1) + j-2] = gf_pow(j, rho*(a+1)) ^ 1 for j = 2..p, a < nq (GF(2^8)/0x11d) */
void pir_final_cw(int p, int nq, int rho, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif
