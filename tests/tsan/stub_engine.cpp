// TEST INFRASTRUCTURE ONLY: a host stand-in for libpir_engine's device side, linked with the
// shim (erasurecodedpir_amd/csrc/pir_server.cpp) into a ThreadSanitizer build on the CPU
// (tests/tsan/Makefile, tests/test_tsan_shim.py).  The shard lives in host memory and every
// answer comes from the plain-C oracle (oracle/pir_oracle.c), so the shim's concurrency -- slice
// groups, the engine-lifetime lock, the fan-out pool, the lazy host rows after a GPU setup --
// runs unchanged and its answers can be checked.  Only the entry points pir_server.cpp calls are
// here; the modes the TSan scenarios do not reach refuse.
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/pir_client.h"
#include "../../include/pir_engine.h"
extern "C" {
#include "../../oracle/pir_oracle.h"
}

struct pir_engine {
  pir_engine_config cfg;
  uint64_t rows;
  std::vector<uint8_t> shard;  // rows x record_bytes
  std::mutex mu;               // the real engine serialises its host API the same way
};

extern "C" {

const char* pir_engine_last_error(void) { return "stub engine"; }

int pir_engine_create(const pir_engine_config* c, pir_engine_t** out) {
  if (!c || !out || c->log_num_records > 24) return PIR_EINVAL;
  auto* e = new pir_engine;
  e->cfg = *c;
  e->rows = 1ull << (c->log_num_records - c->log_num_partitions);
  e->shard.assign((size_t)e->rows * c->record_bytes, 0);
  *out = e;
  return PIR_OK;
}

// the real teardown frees device memory for hundreds of ms: slow enough here that freeServer's
// reaper thread is still at it when the scenarios set the next server up
void pir_engine_destroy(pir_engine_t* e) {
  {
    std::lock_guard<std::mutex> lk(e->mu);
    usleep(20000);
  }
  delete e;
}

uint64_t pir_engine_num_rows(const pir_engine_t* e) { return e ? e->rows : 0; }

int pir_engine_key_len(int p, int n, int nq) { return orc_key_len(p, n, nq); }

int pir_engine_mp_num_keys(int p, int t) {
  return t < 1 || t > p ? 0 : orc_choose(p, t) * (p - t) / p;
}

int pir_engine_mp_key_len(int p, int n, int t) {
  uint64_t s[6];
  orc_mp_sizes(p, n, t, s);
  return (int)s[5];
}

int pir_engine_set_shard_rows(pir_engine_t* e, const uint8_t* const* rows, uint64_t row0,
                              uint64_t nrows) {
  std::lock_guard<std::mutex> lk(e->mu);
  if (row0 + nrows > e->rows) return PIR_EINVAL;
  const uint32_t efs = e->cfg.record_bytes;
  for (uint64_t i = 0; i < nrows; ++i) memcpy(&e->shard[(row0 + i) * efs], rows[i], efs);
  return PIR_OK;
}

int pir_engine_get_shard_rows(pir_engine_t* e, uint8_t* const* rows, uint64_t row0,
                              uint64_t nrows) {
  std::lock_guard<std::mutex> lk(e->mu);
  if (row0 + nrows > e->rows) return PIR_EINVAL;
  const uint32_t efs = e->cfg.record_bytes;
  for (uint64_t i = 0; i < nrows; ++i) memcpy(rows[i], &e->shard[(row0 + i) * efs], efs);
  return PIR_OK;
}

// client.cpp:70-97 on the host (the real engine runs k_encode_across)
int pir_engine_encode_across_rows(pir_engine_t* e, const uint8_t* const* files,
                                  uint64_t num_files, int k) {
  std::lock_guard<std::mutex> lk(e->mu);
  const uint32_t efs = e->cfg.record_bytes;
  const uint64_t encdb = (num_files + (uint64_t)k - 1) / (uint64_t)k;
  std::fill(e->shard.begin(), e->shard.end(), 0);
  for (uint64_t r = 0; r < e->rows; ++r)
    for (int j = 0; j < k; ++j) {
      const uint64_t src = encdb * (uint64_t)j + r;
      if (src >= num_files) continue;
      const uint8_t c = orc_gf_pow((uint8_t)e->cfg.party_index, (uint8_t)j);
      for (uint32_t b = 0; b < efs; ++b) e->shard[r * efs + b] ^= orc_gf_mul(files[src][b], c);
    }
  return PIR_OK;
}

int pir_engine_encode_within_rows(pir_engine_t*, const uint8_t* const*, uint64_t, uint32_t, int,
                                  int) {
  return PIR_EINVAL;  // not reached by the scenarios (tree mode)
}

int pir_engine_answer(pir_engine_t* e, const uint8_t* key, uint8_t* result) {
  std::lock_guard<std::mutex> lk(e->mu);
  const auto& c = e->cfg;
  orc_answer(c.num_parties, c.party_index, c.log_num_records, (int)c.record_bytes, c.num_rounds,
             key, e->shard.data(), result);
  return PIR_OK;
}

int pir_engine_answer_slices(pir_engine_t* e, const uint8_t* key, int num_threads,
                             uint8_t* results) {
  std::lock_guard<std::mutex> lk(e->mu);
  const auto& c = e->cfg;
  const size_t ans = (size_t)c.num_rounds * c.record_bytes;
  for (int t = 0; t < num_threads; ++t)
    orc_answer_slice(c.num_parties, c.party_index, c.log_num_records, (int)c.record_bytes,
                     c.num_rounds, key, e->shard.data(), t, num_threads, results + t * ans);
  return PIR_OK;
}

int pir_engine_answer_slice(pir_engine_t* e, const uint8_t* key, int thread_num, int num_threads,
                            uint8_t* result) {
  std::lock_guard<std::mutex> lk(e->mu);
  const auto& c = e->cfg;
  orc_answer_slice(c.num_parties, c.party_index, c.log_num_records, (int)c.record_bytes,
                   c.num_rounds, key, e->shard.data(), thread_num, num_threads, result);
  return PIR_OK;
}

int pir_engine_answer_coefs(pir_engine_t*, const uint8_t* const*, uint64_t, uint64_t, uint8_t*) {
  return PIR_EINVAL;
}
int pir_engine_answer_mp(pir_engine_t*, const uint8_t*, uint64_t, int, int, int, int, uint8_t*) {
  return PIR_EINVAL;
}
int pir_engine_answer_cd(pir_engine_t*, const uint8_t*, uint64_t, int, int, int, int, uint8_t*) {
  return PIR_EINVAL;
}

int pir_gen_keys(int, int n, uint64_t index, const uint8_t* fcw, int p, int nq,
                 const uint8_t* root_seeds, uint8_t* keys_out) {
  orc_gen_opt_dpf(n, index, fcw, p, nq, root_seeds, keys_out);
  return PIR_OK;
}

void pir_final_cw(int p, int nq, int rho, uint8_t* out) { orc_final_cw(p, nq, rho, out); }

}  // extern "C"
