// pir_engine.cpp -- host side of the C ABI in include/pir_engine.h.
//
// One engine = one GPU holding one shard (or one 2^-G partition of a logical shard) in HBM,
// laid out as rows of `pitch` = round_up(record_bytes, 16) bytes (zero padding), so every
// lane of the scan reads aligned 16-byte chunks.  An answer is four kernels on one stream:
//   key prep -> tree (frontier + leaves) -> GF(2^8) scan -> slab reduce
// plus, for a split shard, an RCCL all-gather of the per-partition answers and an XOR fold
// (RCCL has no XOR reduction op).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/pir_engine.h"
#include "pir_coefs.h"
#include "pir_kernels.h"
#include "pir_mp.h"

#ifndef PIR_TRACE_TREE_TILES
#define PIR_TRACE_TREE_TILES 0  // diagnostics build only (pir_kernels.hip)
#endif

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return fail(PIR_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                  __LINE__);                                                                \
  } while (0)

#define RCCL_TRY(expr)                                                                        \
  do {                                                                                        \
    ncclResult_t _r = (expr);                                                                 \
    if (_r != ncclSuccess) return fail(PIR_ECOMM, "%s failed: %s", #expr, ncclGetErrorString(_r)); \
  } while (0)

// The engine's communicators are non-blocking (ncclConfig_t.blocking = 0), so that a refused or
// stuck rank cannot hang the others inside ncclCommInitRank: a call may return ncclInProgress,
// settled here by polling ncclCommGetAsyncError, bounded by timeout_s.
ncclResult_t rccl_settle(ncclComm_t comm, ncclResult_t r, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  while (r == ncclInProgress) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      return ncclInProgress;
    std::this_thread::yield();
    if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) return ncclSystemError;
  }
  return r;
}


int ilog2_exact(uint64_t v) {
  if (v == 0 || (v & (v - 1))) return -1;
  int l = 0;
  while ((1ull << l) < v) ++l;
  return l;
}

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

}  // namespace

// Event layout of one profiled answer.  Leaves and scans run as kMaxChunks-way pipelined
// chunks on two streams (tree leaves of chunk j+1 overlap the shard scan of chunk j).
constexpr int kMaxChunks = 8;
constexpr int kFrontBatch = 256;  // batched answers: keys whose upper tree levels run together
constexpr uint64_t kBatchNodeBytes = 4ull << 30;  // ... within this much node memory
enum {
  EV_START = 0, EV_KEY = 1, EV_FRONT = 2,
  EV_LEAF_B = 3, EV_LEAF_E = EV_LEAF_B + kMaxChunks,
  EV_SCAN_B = EV_LEAF_E + kMaxChunks, EV_SCAN_E = EV_SCAN_B + kMaxChunks,
  EV_PRERED = EV_SCAN_E + kMaxChunks, EV_RED, EV_END, kNumEv
};

struct pir_engine {
  pir_engine_config cfg{};
  int nrp = 1;
  uint32_t pitch = 0;
  uint64_t rows = 0;  // rows held = 2^(n - G)
  int key_len = 0;
  int num_cus = 256;
  hipStream_t stream = nullptr;
  hipStream_t aux = nullptr;              // scan stream of the leaves/scan pipeline
  hipEvent_t ev_leaf[kMaxChunks] = {};    // leaves of chunk j written
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_cb_ready[2] = {}, ev_cb_free[2] = {};  // batched answers: share buffers
  int last_chunks = 1;
  int last_fused = 0;
  bool allow_fused = true;  // $PIR_FUSED=0 forces the 2-kernel path (A/B diagnostics)
  bool allow_query = true;  // $PIR_QUERY=0: frontier + k_fused instead of k_query
  uint8_t* d_shard = nullptr;
  uint8_t* d_key_raw = nullptr;  // max_batch keys
  pir::DevKey* d_keys = nullptr; // max_batch parsed keys
  int max_batch = 0;
  pir::NodeBufs nodes{};  // tree levels between kernels (ping-pong)
  uint8_t* d_c = nullptr;
  uint8_t* d_slabs = nullptr;
  size_t slab_cap = 0;
  uint8_t* d_part = nullptr;    // nq*efs partition answer
  uint8_t* d_gather = nullptr;  // nranks*nq*efs
  // batched answers: interleaved shares of a key group, group answer, batch partition answer
  uint8_t* d_cb = nullptr;
  size_t cb_cap = 0;
  pir::NodeBufs bnodes{};       // upper tree levels of a batch's super-group (FB x max_nodes)
  uint64_t bnodes_cap = 0;
  uint8_t* d_gtmp = nullptr;    // 16*efs
  uint8_t* d_bpart = nullptr;   // batch partition answers (split shard)
  uint8_t* d_bgather = nullptr; // nranks x batch answers
  size_t bpart_cap = 0, bgather_cap = 0;
  int batch_group = 0;          // keys per shard pass (0: automatic; $PIR_BATCH_G)
  int last_batch_group = 0;
  int batch_scan_bpc = 2;       // scan workgroups per CU in batched answers ($PIR_BATCH_SCAN_BPC)
  int batch_k_last = -1;        // levels of the batched leaf stage (-1: make_plan's; $PIR_BATCH_KLAST)
  uint8_t* d_result = nullptr;  // nq*efs (host-API staging)
  uint8_t* d_qscratch = nullptr;  // k_query super-tile tile inputs
  size_t qscratch_cap = 0;
  uint32_t* d_qcnt = nullptr;     // k_query fused reduce: per-query slab counters (kept zero)
  int qcnt_cap = 0;
  // k_query's end-of-query work stealing for a lone whole answer (StealArgs, pir_kernels.h):
  // per-workgroup chunk counters + publication flags + last-tile shares, zeroed once; steal_gen
  // numbers the launches that use it ($PIR_QUERY_STEAL=0 turns it off)
  uint32_t* d_steal = nullptr;
  size_t steal_cap = 0;
  uint32_t steal_gen = 0;
  int steal = PIR_QUERY_STEAL ? 3 : 0;
  // k_query's in-kernel reduce (no k_reduce launch), $PIR_FUSED_REDUCE: 0 = off (k_reduce);
  // 1 = the last workgroup XORs the slabs (measured slower for a lone 2^20 x 1 KiB query: kernel
  // 0.250 vs 0.218 ms, one workgroup's 256 KiB of cross-XCD sc1 loads outlast a k_reduce
  // launch); 2 = every workgroup adds its partial to the answer with memory-side atomics
  // (answers of efs % 4 == 0 bytes at 4-byte aligned addresses; else k_reduce)
  int fused_reduce = 0;
  uint8_t* d_coef_stage = nullptr;  // explicit-coefficient answers: host vectors staged here
  size_t coef_stage_cap = 0;
  uint8_t* d_mpkey = nullptr;       // multiparty DPF keys: host keys / unaligned device keys
  size_t mpkey_cap = 0;
  uint8_t* h_key = nullptr;     // pinned
  uint8_t* h_res = nullptr;     // pinned
  uint8_t* d_slices = nullptr;  // pir_engine_answer_slices: T x nq x efs partials
  size_t slices_cap = 0;
  uint8_t* h_slices = nullptr;  // pinned
  size_t h_slices_cap = 0;
  std::vector<DevBuf> user;     // pir_engine_alloc_dev
  std::mutex mu;
  uint64_t byz_counter = 0;
  // profiling: a ring of event sets, one per answer, read back after a sync
  struct ProfSlot {
    hipEvent_t ev[kNumEv];
  };
  std::vector<ProfSlot> prof;
  int prof_next = 0, prof_count = 0;
  hipEvent_t* ev = nullptr;  // the current answer's slot (nullptr: profiling off)
  // the engine's work buffers (slabs, tree nodes, share buffers, staged keys) are shared by
  // every answer: an answer enqueued on a stream other than the previous answer's waits for
  // that answer's last use of them (ev_ws: recorded after an answer on a caller's stream, and
  // for the engine's own stream when the next answer comes on another one)
  hipEvent_t ev_ws = nullptr;
  hipStream_t ws_stream = nullptr;
  // RCCL
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  bool comm_failed = false;   // an exchange failed: the communicator was aborted, answers refuse
  double comm_timeout_s = 60; // $PIR_COMM_TIMEOUT: bound on one exchange's enqueue
};

namespace {

int ensure_batch(pir_engine* e, int nk) {
  if (nk <= e->max_batch) return PIR_OK;
  if (e->d_key_raw) (void)hipFree(e->d_key_raw);
  if (e->d_keys) (void)hipFree(e->d_keys);
  e->d_key_raw = nullptr;
  e->d_keys = nullptr;
  HIP_TRY(hipMalloc(&e->d_key_raw, (size_t)nk * e->key_len));
  HIP_TRY(hipMalloc(&e->d_keys, (size_t)nk * sizeof(pir::DevKey)));
  e->max_batch = nk;
  return PIR_OK;
}

int ensure_buf(uint8_t** p, size_t* cap, size_t bytes) {
  if (bytes <= *cap) return PIR_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  HIP_TRY(hipMalloc(p, bytes));
  *cap = bytes;
  return PIR_OK;
}

// nb.s/t[0..nbuf) with room for `nodes` nodes each
int ensure_nodes(pir::NodeBufs* nb, uint64_t* cap, uint64_t nodes, int nbuf) {
  if (nodes <= *cap) return PIR_OK;
  for (int i = 0; i < 2; ++i) {
    if (nb->s[i]) (void)hipFree(nb->s[i]);
    if (nb->t[i]) (void)hipFree(nb->t[i]);
    nb->s[i] = nullptr;
    nb->t[i] = nullptr;
  }
  *cap = 0;
  for (int i = 0; i < nbuf; ++i) {
    HIP_TRY(hipMalloc(&nb->s[i], nodes * sizeof(uint4)));
    HIP_TRY(hipMalloc(&nb->t[i], nodes * sizeof(uint32_t)));
  }
  *cap = nodes;
  return PIR_OK;
}

int ensure_host(uint8_t** p, size_t* cap, size_t bytes) {  // pinned host staging
  if (bytes <= *cap) return PIR_OK;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *cap = 0;
  HIP_TRY(hipHostMalloc(p, bytes));
  *cap = bytes;
  return PIR_OK;
}

int ensure_slabs(pir_engine* e, size_t bytes) {
  if (bytes <= e->slab_cap) return PIR_OK;
  if (e->d_slabs) (void)hipFree(e->d_slabs);
  e->d_slabs = nullptr;
  HIP_TRY(hipMalloc(&e->d_slabs, bytes));
  e->slab_cap = bytes;
  return PIR_OK;
}

int pick_chunks(const pir::TreePlan& pl, int num_cus) {
  // pipeline the leaf stage only while each chunk's launch still covers every CU
  const int blocks = pir::final_stage_blocks(pl);
  int c = 1;
  while (2 * c <= kMaxChunks && blocks % (2 * c) == 0 && blocks / (2 * c) >= num_cus) c *= 2;
  return c;
}

// Answer one partition slice: rows [row0, row0 + 2^(n - log_parts_total)) of this engine
// with the tree rooted at `prefix` (depth log_parts_total).  d_key points at ONE parsed key.
//   s  : key prep, frontier, leaves(0..C-1), [join], reduce
//   aux: scan(j) after leaves(j)  -- so leaves(j+1) overlaps scan(j)
pir::KeySrc key_src(pir_engine* e, const uint8_t* d_raw) {
  const auto& c = e->cfg;
  return pir::KeySrc{d_raw, c.num_parties, c.log_num_records, c.num_rounds, c.party_index - 1,
                     e->d_keys};
}

int answer_fused(pir_engine* e, const uint8_t* d_raw, int log_parts_total, uint64_t prefix,
                 uint64_t row0, uint8_t* d_out, hipStream_t s, int tile) {
  const pir::DevKey* d_key = e->d_keys;
  const auto& c = e->cfg;
  const pir::TreePlan pl =
      pir::make_plan(c.log_num_records, log_parts_total, prefix, pir::fused_k(tile), c.num_parties);
  const pir::ScanShape sh =
      pir::make_fused_shape(pl.nleaves, e->pitch, c.num_rounds, e->num_cus, tile);
  int rc = ensure_slabs(e, (size_t)sh.grid.x * sh.grid.y * sh.slab_bytes);
  if (rc) return rc;
  e->last_chunks = 1;
  e->last_fused = 1;
  hipEvent_t* ev = e->ev;
  if (ev) HIP_TRY(hipEventRecord(ev[EV_KEY], s));
  HIP_TRY(pir::launch_frontier(pl, key_src(e, d_raw), e->nodes, s));
  HIP_TRY(pir::launch_stages(pl, d_key, e->nodes, 0, 1, e->d_c, e->nrp, s, 0, pl.nstages - 1));
  if (ev) {
    HIP_TRY(hipEventRecord(ev[EV_FRONT], s));
    HIP_TRY(hipEventRecord(ev[EV_LEAF_B], s));
    HIP_TRY(hipEventRecord(ev[EV_LEAF_E], s));
    HIP_TRY(hipEventRecord(ev[EV_SCAN_B], s));
  }
  HIP_TRY(pir::launch_fused(pl, d_key, e->nodes, e->d_shard + row0 * e->pitch, sh, e->d_slabs,
                            tile, s));
  if (ev) {
    HIP_TRY(hipEventRecord(ev[EV_SCAN_E], s));
    HIP_TRY(hipEventRecord(ev[EV_PRERED], s));
  }
  HIP_TRY(pir::launch_reduce(sh, e->d_slabs, c.record_bytes, d_out, s));
  if (ev) HIP_TRY(hipEventRecord(ev[EV_RED], s));
  return PIR_OK;
}

// nk zeroed slab counters for k_query's fused reduce (the kernel leaves them zero)
int ensure_qcnt(pir_engine* e, int nk, hipStream_t s) {
  if (nk <= e->qcnt_cap) return PIR_OK;
  if (e->d_qcnt) {
    HIP_TRY(hipStreamSynchronize(s));
    (void)hipFree(e->d_qcnt);
  }
  e->d_qcnt = nullptr;
  e->qcnt_cap = 0;
  HIP_TRY(hipMalloc(&e->d_qcnt, (size_t)nk * sizeof(uint32_t)));
  HIP_TRY(hipMemsetAsync(e->d_qcnt, 0, (size_t)nk * sizeof(uint32_t), s));
  e->qcnt_cap = nk;
  return PIR_OK;
}

// the work-stealing arguments of a k_query launch (empty = static tiles): a lone query (nk == 1)
// answered whole (nslices == 1: a stolen chunk is folded into the thief's region slab) with one
// column group, on at most one workgroup per CU (every workgroup resident, so the bounded wait
// for unpublished last tiles never outlasts a late one's dispatch)
int steal_args(pir_engine* e, const pir::QueryPlan& qp, int nk, int nslices, hipStream_t s,
               pir::StealArgs* out) {
  *out = pir::StealArgs{};
  if (!PIR_QUERY_STEAL || !e->steal || nk != 1 || nslices != 1 || qp.shape.nq > 2 || !qp.shape.uniform ||
      qp.shape.grid.y != 1 || (int)qp.shape.grid.x > e->num_cus || qp.m4r)
    return PIR_OK;
  // a captured launch would replay one generation: flags left equal to it by the previous
  // replay would read as published shares
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIP_TRY(hipStreamIsCapturing(s, &cap));
  if (cap != hipStreamCaptureStatusNone) return PIR_OK;
  const size_t bytes = pir::query_steal_bytes(qp);
  if (bytes > e->steal_cap) {
    if (e->d_steal) {  // a launch still in flight may read the old buffer (as ensure_qcnt)
      HIP_TRY(hipStreamSynchronize(s));
      (void)hipFree(e->d_steal);
    }
    e->d_steal = nullptr;
    e->steal_cap = 0;
    HIP_TRY(hipMalloc(&e->d_steal, bytes));
    HIP_TRY(hipMemsetAsync(e->d_steal, 0, bytes, s));  // no flag equals a generation (>= 1)
    e->steal_cap = bytes;
  }
  if (++e->steal_gen == 0) e->steal_gen = 1;
  out->buf = e->d_steal;
  out->gen = e->steal_gen;
  out->mode = (uint32_t)e->steal;
  return PIR_OK;
}

// one launch: key parse, tree and scan of nk queued keys (key_len apart) in k_query; then the
// slab reduce of all nk answers (d_out: nk x nq x efs)
// nslices > 1 (a power of two <= 2^qp.lr, nk == 1): d_out gets the nslices partial answers
// over equal consecutive row ranges instead of the whole answer (runOptimizedDPFTreeQueryThread
// for every thread of a query at once: the slices are runs of k_query's region slabs)
int answer_query(pir_engine* e, const pir::QueryPlan& qp, const uint8_t* d_raw, int nk,
                 int log_parts_total, uint64_t prefix, uint64_t row0, uint8_t* d_out,
                 hipStream_t s, int nslices = 1) {
  const auto& c = e->cfg;
  const pir::ScanShape& sh = qp.shape;
  int rc = ensure_slabs(e, (size_t)nk * pir::query_slab_bytes(qp));
  if (!rc) rc = ensure_buf(&e->d_qscratch, &e->qscratch_cap, pir::query_scratch_bytes(qp));
  // modes 2 and 3 need whole answer words at aligned addresses, mode 3 at least 8 slabs;
  // otherwise k_reduce (always for slices)
  int fred = e->fused_reduce;
  if (fred >= 2 && (c.record_bytes % 4 != 0 || reinterpret_cast<uintptr_t>(d_out) % 4 != 0)) fred = 0;
  if (fred == 3 && qp.lr < 3) fred = 1;
  if (nslices > 1) fred = 0;
  if (!rc && fred) rc = ensure_qcnt(e, nk * (fred == 3 ? 8 : 1), s);
  pir::StealArgs steal;
  if (!rc) rc = steal_args(e, qp, nk, nslices, s, &steal);
  if (rc) return rc;
  if (fred >= 2)  // the workgroups (mode 2) or slab groups (mode 3) XOR into zeroed answers
    HIP_TRY(hipMemsetAsync(d_out, 0, (size_t)nk * c.num_rounds * c.record_bytes, s));
  e->last_chunks = 1;
  e->last_fused = 2;
  // profiling: k_query has no separate key / tree / scan kernels, so only its own bounds and
  // the reduce are stamped (each event record between two launches costs the next one a few us
  // of dispatch: fewer stamps keep the profiled answer close to the unprofiled one)
  hipEvent_t* ev = e->ev;
  if (ev) HIP_TRY(hipEventRecord(ev[EV_SCAN_B], s));
  HIP_TRY(pir::launch_query(qp, d_raw, (uint32_t)e->key_len, nk, c.num_parties,
                            c.log_num_records, c.party_index - 1, log_parts_total, prefix,
                            e->d_shard + row0 * e->pitch, e->d_slabs, e->d_qscratch, s, nullptr,
                            fred ? d_out : nullptr, e->d_qcnt, c.record_bytes, (uint32_t)fred,
                            steal));
  if (ev) HIP_TRY(hipEventRecord(ev[EV_SCAN_E], s));
  if (!fred) HIP_TRY(pir::launch_reduce(sh, e->d_slabs, c.record_bytes, d_out, s, nk, nslices));
  if (ev) HIP_TRY(hipEventRecord(ev[EV_RED], s));
  return PIR_OK;
}

int answer_core(pir_engine* e, const uint8_t* d_raw, int log_parts_total, uint64_t prefix,
                uint64_t row0, uint8_t* d_out, hipStream_t s) {
  const auto& c = e->cfg;
  const pir::DevKey* d_key = e->d_keys;
  const uint64_t nleaves = 1ull << (c.log_num_records - log_parts_total);
  if (e->allow_query && e->allow_fused) {
    const pir::QueryPlan qp = pir::make_query_plan(c.log_num_records, log_parts_total,
                                                   c.num_parties, c.num_rounds, e->pitch, e->num_cus);
    if (qp.tile) return answer_query(e, qp, d_raw, 1, log_parts_total, prefix, row0, d_out, s);
  }
  const int tile = e->allow_fused ? pir::fused_tile(c.num_rounds, e->pitch, nleaves, e->num_cus) : 0;
  if (tile) return answer_fused(e, d_raw, log_parts_total, prefix, row0, d_out, s, tile);
  e->last_fused = 0;
  const pir::TreePlan pl = pir::make_plan(c.log_num_records, log_parts_total, prefix, -1, c.num_parties);
  const int C = pick_chunks(pl, e->num_cus);
  e->last_chunks = C;
  const uint64_t nrec = pl.nleaves / C;
  const pir::ScanShape sh = pir::make_scan_shape(nrec, e->pitch, c.num_rounds, e->num_cus);
  int rc = ensure_slabs(e, (size_t)sh.grid.x * sh.grid.y * sh.slab_bytes);
  if (rc) return rc;
  hipEvent_t* ev = e->ev;
  if (ev) HIP_TRY(hipEventRecord(ev[EV_KEY], s));
  HIP_TRY(pir::launch_frontier(pl, key_src(e, d_raw), e->nodes, s));
  HIP_TRY(pir::launch_stages(pl, d_key, e->nodes, 0, 1, e->d_c, e->nrp, s, 0, pl.nstages - 1));
  if (ev) HIP_TRY(hipEventRecord(ev[EV_FRONT], s));
  for (int j = 0; j < C; ++j) {
    if (ev) HIP_TRY(hipEventRecord(ev[EV_LEAF_B + j], s));
    HIP_TRY(pir::launch_stages(pl, d_key, e->nodes, j, C, e->d_c, e->nrp, s, pl.nstages - 1));
    if (ev) HIP_TRY(hipEventRecord(ev[EV_LEAF_E + j], s));
    HIP_TRY(hipEventRecord(e->ev_leaf[j], s));
    HIP_TRY(hipStreamWaitEvent(e->aux, e->ev_leaf[j], 0));
    if (ev) HIP_TRY(hipEventRecord(ev[EV_SCAN_B + j], e->aux));
    HIP_TRY(pir::launch_scan(sh, e->d_shard + (row0 + j * nrec) * e->pitch, nrec,
                             e->d_c + j * nrec * e->nrp, e->d_slabs, j > 0, e->aux));
    if (ev) HIP_TRY(hipEventRecord(ev[EV_SCAN_E + j], e->aux));
  }
  HIP_TRY(hipEventRecord(e->ev_join, e->aux));
  HIP_TRY(hipStreamWaitEvent(s, e->ev_join, 0));
  if (ev) HIP_TRY(hipEventRecord(ev[EV_PRERED], s));
  HIP_TRY(pir::launch_reduce(sh, e->d_slabs, c.record_bytes, d_out, s));
  if (ev) HIP_TRY(hipEventRecord(ev[EV_RED], s));
  return PIR_OK;
}

// keys answered per shard pass: G keys x nrp share bytes per record (a power of two <= 16)
int batch_group(const pir_engine* e) {
  const int maxg = 16 / e->nrp;
  int g = e->batch_group > 0 ? e->batch_group : 8 / std::min(e->nrp, 8);
  g = std::max(1, std::min(g, maxg));
  while (g & (g - 1)) g &= g - 1;  // power of two
  return g;
}

// nk keys (raw, key_len apart) against one partition slice, one shard pass per group of G
// keys: each key's tree writes its shares into slot g of the interleaved coefficient rows
// cb[i][G*nrp]; one multi-round scan of G*nrp rounds answers the group (round g*nrp + a =
// key g, round a).  d_out: nk x nq x efs.
//   s  : per super-group of FB keys: frontier + all but the last tree stage of the FB keys
//        (one launch per stage, keys along grid y); then per group of G keys the last
//        (leaf) stage into share buffer j%2 (after scan j-2 has read it)
//   aux: scan + reduce of group j (after its leaf stage)
// so the leaf stage of group j+1 runs beside the scan of group j.  (Node-writing stages beside
// a scan are starved of the CU's memory pipeline, hence the up-front upper stages.)
int answer_batch_core(pir_engine* e, const uint8_t* d_raw, int nk, int log_parts_total,
                      uint64_t prefix, uint64_t row0, uint8_t* d_out, hipStream_t s) {
  const auto& c = e->cfg;
  const int G = batch_group(e);
  const int W = G * e->nrp;
  e->last_batch_group = G;
  e->last_fused = 0;
  e->last_chunks = 1;
  const pir::TreePlan pl = pir::make_plan(c.log_num_records, log_parts_total, prefix, e->batch_k_last, c.num_parties, 8);
  pir::ScanShape sh =
      pir::make_scan_shape(pl.nleaves, e->pitch, W, e->num_cus, e->batch_scan_bpc);
  const size_t cb_bytes = (size_t)pl.nleaves * W;
  // k_scan_t reads the group's shares key-major (key g's nrp bytes of leaf i at g * nleaves *
  // nrp + i * nrp), so each tree's leaf stage writes its shares contiguously (packed 16-byte
  // stores); the other scans read them interleaved per record (cb[i][W], key g at g * nrp)
  const bool kmaj = sh.tfold && !(getenv("PIR_BATCH_KMAJOR") && atoi(getenv("PIR_BATCH_KMAJOR")) == 0);
  if (kmaj) {
    sh.ckey = (uint32_t)e->nrp;
    sh.ckoff = (uint64_t)pl.nleaves * e->nrp;
  }
  // super-group: as many keys as kBatchNodeBytes of upper-level nodes hold (a multiple of G)
  const uint64_t per_key = 2 * pl.max_nodes * (sizeof(uint4) + sizeof(uint32_t));
  int FB = (int)std::min<uint64_t>(kFrontBatch, std::max<uint64_t>(1, kBatchNodeBytes / per_key));
  FB = std::max(G, FB / G * G);
  const int nsg = std::min(nk, FB);
  int rc = ensure_slabs(e, (size_t)sh.grid.x * sh.grid.y * sh.slab_bytes);
  if (!rc) rc = ensure_buf(&e->d_cb, &e->cb_cap, 2 * cb_bytes);
  if (!rc) rc = ensure_batch(e, nk);
  if (!rc) rc = ensure_nodes(&e->bnodes, &e->bnodes_cap, (uint64_t)nsg * pl.max_nodes, 2);
  if (rc) return rc;
  if (!e->d_gtmp) HIP_TRY(hipMalloc(&e->d_gtmp, (size_t)16 * c.record_bytes));
  const size_t out_bytes = (size_t)c.num_rounds * c.record_bytes;
  const int last = pl.nstages - 1;
  HIP_TRY(hipEventRecord(e->ev_fork, s));
  HIP_TRY(hipStreamWaitEvent(e->aux, e->ev_fork, 0));
  for (int q0 = 0, j = 0; q0 < nk; q0 += G, ++j) {
    const int ng = std::min(G, nk - q0), b = j & 1, r0 = q0 % FB;
    if (r0 == 0) {  // frontier + upper stages of the next FB keys
      const int nf = std::min(FB, nk - q0);
      const pir::KeySrc ks{d_raw + (size_t)q0 * e->key_len, c.num_parties, c.log_num_records,
                           c.num_rounds, c.party_index - 1, e->d_keys + q0};
      HIP_TRY(pir::launch_frontier(pl, ks, e->bnodes, s, nf, (size_t)e->key_len, pl.max_nodes));
      if (last > 0) {
        const pir::StageBatch up{nf, pl.max_nodes, 0, nullptr, nullptr, 0};
        HIP_TRY(pir::launch_stages(pl, e->d_keys + q0, e->bnodes, 0, 1, nullptr, e->nrp, s, 0,
                                   last, 0, &up));
      }
    }
    uint8_t* cb = e->d_cb + b * cb_bytes;
    if (j >= 2) HIP_TRY(hipStreamWaitEvent(s, e->ev_cb_free[b], 0));
    // the leaf stage of the ng trees of the group side by side: grid row y = key q0 + y
    const uint64_t off = (uint64_t)r0 * pl.max_nodes;
    const pir::NodeBufs nbg{{e->bnodes.s[0] + off, e->bnodes.s[1] + off},
                            {e->bnodes.t[0] + off, e->bnodes.t[1] + off}};
    const pir::StageBatch sb{ng, pl.max_nodes, kmaj ? (uint32_t)sh.ckoff : (uint32_t)e->nrp,
                             nullptr, nullptr, 0};
    HIP_TRY(pir::launch_stages(pl, e->d_keys + q0, nbg, 0, 1, cb, e->nrp, s, last, last + 1,
                               kmaj ? e->nrp : W, &sb));
    HIP_TRY(hipEventRecord(e->ev_cb_ready[b], s));
    HIP_TRY(hipStreamWaitEvent(e->aux, e->ev_cb_ready[b], 0));
    // slots g >= ng hold stale shares: their rounds are computed and dropped
    HIP_TRY(pir::launch_scan(sh, e->d_shard + row0 * e->pitch, pl.nleaves, cb, e->d_slabs, false,
                             e->aux));
    HIP_TRY(hipEventRecord(e->ev_cb_free[b], e->aux));
    uint8_t* dst = d_out + (size_t)q0 * out_bytes;
    if (e->nrp == c.num_rounds && ng == G) {
      HIP_TRY(pir::launch_reduce(sh, e->d_slabs, c.record_bytes, dst, e->aux));
    } else {
      HIP_TRY(pir::launch_reduce(sh, e->d_slabs, c.record_bytes, e->d_gtmp, e->aux));
      HIP_TRY(hipMemcpy2DAsync(dst, out_bytes, e->d_gtmp, (size_t)e->nrp * c.record_bytes,
                               out_bytes, ng, hipMemcpyDeviceToDevice, e->aux));
    }
  }
  HIP_TRY(hipEventRecord(e->ev_join, e->aux));
  HIP_TRY(hipStreamWaitEvent(s, e->ev_join, 0));
  return PIR_OK;
}

int check_key_ptr(const void* p) { return p ? PIR_OK : fail(PIR_EINVAL, "null key"); }

// The split-shard combine after the all-gather: d_gather holds nranks blocks of `bytes`
// (rank r's partial answers at r * bytes -- ncclAllGather's layout), d_result[i] = XOR_r of
// them (the XOR assembly of server.cpp:553-562 across partitions; RCCL has no XOR op).
int fold_gathered(pir_engine* e, const uint8_t* d_gather, int nranks, size_t bytes,
                  uint8_t* d_result, hipStream_t s) {
  (void)e;
  HIP_TRY(pir::launch_xor_fold(d_gather, nranks, bytes, d_result, s));
  return PIR_OK;
}

// Every rank's `bytes` of partial answers (d_part) -> every rank's XOR over ranks (d_result):
// ONE ncclAllGather into d_gather (nranks x bytes) + fold_gathered, on stream s.  A failed or
// timed-out exchange aborts the communicator (an operation may still be in flight on it) and
// marks the engine failed, so that later answers refuse instead of returning partition-only
// partials.
int exchange(pir_engine* e, const uint8_t* d_part, size_t bytes, uint8_t* d_gather,
             uint8_t* d_result, hipStream_t s) {
  const ncclResult_t r = rccl_settle(
      e->comm, ncclAllGather(d_part, d_gather, bytes, ncclUint8, e->comm, s), e->comm_timeout_s);
  if (r != ncclSuccess) {
    (void)ncclCommAbort(e->comm);
    e->comm = nullptr;
    e->comm_failed = true;
    return fail(PIR_ECOMM, "ncclAllGather of %zu bytes failed: %s (communicator aborted)", bytes,
                r == ncclInProgress ? "timed out" : ncclGetErrorString(r));
  }
  return fold_gathered(e, d_gather, e->nranks, bytes, d_result, s);
}

int check_comm(const pir_engine* e) {
  return e->comm_failed ? fail(PIR_ECOMM, "the engine's communicator was aborted after a failed "
                                          "exchange (%s)", "re-create the engine")
                        : PIR_OK;
}

// before an answer on stream s: order it after the previous answer's use of the workspace.
// The engine's own stream records that answer's event only now, when another stream needs it
// (everything enqueued on it so far, the previous answer included): an event record between
// two launches on one stream delays the second by ~5.6 us of dispatch (the lone-query gap of
// profiles/r05/r5af_lone_gaps_depth4_depth16.txt; tools/micro/dispatch_gap.hip, mode 7).  A
// caller's stream records at release, while it is known to exist.
int ws_acquire(pir_engine* e, hipStream_t s) {
  if (int rc = check_comm(e)) return rc;
  if (e->ws_stream && e->ws_stream != s) {
    if (e->ws_stream == e->stream) HIP_TRY(hipEventRecord(e->ev_ws, e->stream));
    HIP_TRY(hipStreamWaitEvent(s, e->ev_ws, 0));
  }
  return PIR_OK;
}
// after it: the next answer, on whatever stream, waits for this one
int ws_release(pir_engine* e, hipStream_t s, int rc) {
  if (rc) return rc;
  if (s != e->stream) HIP_TRY(hipEventRecord(e->ev_ws, s));
  e->ws_stream = s;
  return PIR_OK;
}

const char* const kPhaseNames[] = {"key_prep", "tree_frontier", "tree_leaves", "scan",
                                   "reduce", "comm_fold", "total", "chunks", "fused"};
constexpr int kNumPhases = 9;
// the k_query path (fused == 2: key, tree and scan are one kernel): "launch" = answer start ->
// k_query start (key upload, workspace ordering, dispatch), "scan" = the k_query launch,
// "reduce" = k_reduce (0 with an in-kernel reduce), "comm_fold" = the split-shard exchange and
// whatever follows; they add up to "total"
const char* const kQueryPhaseNames[] = {"launch", "scan", "reduce", "comm_fold", "total", "fused"};
constexpr int kNumQueryPhases = 6;

// Mean per-phase device times over the answers recorded since the last read.  tree_leaves and
// scan are the summed kernel durations of the C pipelined chunks (they overlap each other).
int read_timings(pir_engine* e, pir_kernel_time* out, int max) {
  const int n = std::min(max, kNumPhases);
  if (e->prof.empty() || e->prof_count == 0) return 0;
  const int cnt = e->prof_count, sz = (int)e->prof.size(), C = e->last_chunks;
  HIP_TRY(hipEventSynchronize(e->prof[(e->prof_next + sz - 1) % sz].ev[EV_END]));
  double acc[kNumPhases] = {};
  auto el = [](hipEvent_t a, hipEvent_t b, double& sum) -> hipError_t {
    float ms = 0;
    hipError_t r = hipEventElapsedTime(&ms, a, b);
    sum += ms;
    return r;
  };
  if (e->last_fused == 2) {
    const int nq = std::min(max, kNumQueryPhases);
    for (int k = 0; k < cnt; ++k) {
      const hipEvent_t* v = e->prof[(e->prof_next + sz - cnt + k) % sz].ev;
      HIP_TRY(el(v[EV_START], v[EV_SCAN_B], acc[0]));
      HIP_TRY(el(v[EV_SCAN_B], v[EV_SCAN_E], acc[1]));
      HIP_TRY(el(v[EV_SCAN_E], v[EV_RED], acc[2]));
      HIP_TRY(el(v[EV_RED], v[EV_END], acc[3]));
      HIP_TRY(el(v[EV_START], v[EV_END], acc[4]));
    }
    acc[5] = 2.0 * cnt;
    for (int i = 0; i < nq; ++i) {
      snprintf(out[i].name, sizeof out[i].name, "%s", kQueryPhaseNames[i]);
      out[i].ms = (float)(acc[i] / cnt);
    }
    e->prof_count = 0;
    return nq;
  }
  for (int k = 0; k < cnt; ++k) {
    const hipEvent_t* v = e->prof[(e->prof_next + sz - cnt + k) % sz].ev;
    HIP_TRY(el(v[EV_START], v[EV_KEY], acc[0]));
    HIP_TRY(el(v[EV_KEY], v[EV_FRONT], acc[1]));
    for (int j = 0; j < C; ++j) {
      HIP_TRY(el(v[EV_LEAF_B + j], v[EV_LEAF_E + j], acc[2]));
      HIP_TRY(el(v[EV_SCAN_B + j], v[EV_SCAN_E + j], acc[3]));
    }
    HIP_TRY(el(v[EV_PRERED], v[EV_RED], acc[4]));
    HIP_TRY(el(v[EV_RED], v[EV_END], acc[5]));
    HIP_TRY(el(v[EV_START], v[EV_END], acc[6]));
  }
  acc[7] = C * cnt;
  acc[8] = e->last_fused * cnt;
  for (int i = 0; i < n; ++i) {
    snprintf(out[i].name, sizeof out[i].name, "%s", kPhaseNames[i]);
    out[i].ms = (float)(acc[i] / cnt);
  }
  e->prof_count = 0;
  return n;
}

int answer_dev_locked(pir_engine* e, const uint8_t* d_key, uint8_t* d_result, hipStream_t s) {
  const auto& c = e->cfg;
  const size_t out_bytes = (size_t)c.num_rounds * c.record_bytes;
  e->ev = nullptr;
  if (!e->prof.empty()) {
    e->ev = e->prof[e->prof_next].ev;
    e->prof_next = (e->prof_next + 1) % (int)e->prof.size();
    e->prof_count = std::min(e->prof_count + 1, (int)e->prof.size());
  }
  hipEvent_t* ev = e->ev;
  if (ev) HIP_TRY(hipEventRecord(ev[EV_START], s));
  if (c.is_byzantine) {  // server.cpp:116-119: random answer bytes
    HIP_TRY(pir::launch_fill_random(d_result, out_bytes, 0xB42u + (++e->byz_counter), s));
    if (ev)
      for (int i = 1; i < kNumEv; ++i) HIP_TRY(hipEventRecord(ev[i], s));
    e->last_chunks = 1;
    e->ev = nullptr;
    return PIR_OK;
  }
  uint8_t* part_out = e->comm ? e->d_part : d_result;
  // the key is parsed inside the frontier kernel (k_key_prep only when the tree is very deep)
  int rc = answer_core(e, d_key, c.log_num_partitions, (uint64_t)c.partition_index, 0,
                       part_out, s);
  if (rc) return rc;
  if (e->comm) {
    if (int rc = exchange(e, e->d_part, out_bytes, e->d_gather, d_result, s)) return rc;
  }
  if (ev) HIP_TRY(hipEventRecord(ev[EV_END], s));
  e->ev = nullptr;
  return PIR_OK;
}

int answer_batch_locked(pir_engine* e, const uint8_t* d_keys, int nk, uint8_t* d_result,
                        hipStream_t s) {
  const auto& c = e->cfg;
  const size_t out_bytes = (size_t)c.num_rounds * c.record_bytes;
  e->ev = nullptr;
  if (nk == 0) return PIR_OK;
  if (c.is_byzantine) {
    HIP_TRY(pir::launch_fill_random(d_result, out_bytes * nk, 0xB42u + (++e->byz_counter), s));
    return PIR_OK;
  }
  if (nk == 1 || batch_group(e) == 1) {  // one key per shard pass: the single-query path
    for (int q = 0; q < nk; ++q) {
      int rc = answer_dev_locked(e, d_keys + (size_t)q * e->key_len, d_result + q * out_bytes, s);
      if (rc) return rc;
    }
    return PIR_OK;
  }
  const size_t total = out_bytes * nk;
  uint8_t* part_out = d_result;
  if (e->comm) {
    int rc = ensure_buf(&e->d_bpart, &e->bpart_cap, total);
    if (!rc) rc = ensure_buf(&e->d_bgather, &e->bgather_cap, total * e->nranks);
    if (rc) return rc;
    part_out = e->d_bpart;
  }
  int rc = answer_batch_core(e, d_keys, nk, c.log_num_partitions, (uint64_t)c.partition_index, 0,
                             part_out, s);
  if (rc) return rc;
  if (e->comm) {
    if (int rc = exchange(e, e->d_bpart, total, e->d_bgather, d_result, s)) return rc;
  }
  return PIR_OK;
}

// nk independent queries, each its own tree and full shard pass, answered back to back: one
// k_query launch when the shape allows (the tree of query k+1 overlaps the scan of query k),
// else one answer after another.  d_result: nk x nq x efs.
int answer_stream_locked(pir_engine* e, const uint8_t* d_keys, int nk, uint8_t* d_result,
                         hipStream_t s) {
  const auto& c = e->cfg;
  const size_t out_bytes = (size_t)c.num_rounds * c.record_bytes;
  e->ev = nullptr;
  if (nk == 0) return PIR_OK;
  const pir::QueryPlan qp = pir::make_query_plan(c.log_num_records, c.log_num_partitions,
                                                 c.num_parties, c.num_rounds, e->pitch, e->num_cus,
                                                 nk);
  if (c.is_byzantine || !qp.tile || !e->allow_query || !e->allow_fused) {
    for (int k = 0; k < nk; ++k) {
      int rc = answer_dev_locked(e, d_keys + (size_t)k * e->key_len, d_result + k * out_bytes, s);
      if (rc) return rc;
    }
    return PIR_OK;
  }
  const size_t total = out_bytes * nk;
  uint8_t* part_out = d_result;
  if (e->comm) {
    int rc = ensure_buf(&e->d_bpart, &e->bpart_cap, total);
    if (!rc) rc = ensure_buf(&e->d_bgather, &e->bgather_cap, total * e->nranks);
    if (rc) return rc;
    part_out = e->d_bpart;
  }
  if (!e->prof.empty()) {  // one event set for the whole queue (phases of the one launch)
    e->ev = e->prof[e->prof_next].ev;
    e->prof_next = (e->prof_next + 1) % (int)e->prof.size();
    e->prof_count = std::min(e->prof_count + 1, (int)e->prof.size());
    HIP_TRY(hipEventRecord(e->ev[EV_START], s));
  }
  int rc = answer_query(e, qp, d_keys, nk, c.log_num_partitions, (uint64_t)c.partition_index, 0,
                        part_out, s);
  if (rc) return rc;
  if (e->comm) {
    if (int rc = exchange(e, e->d_bpart, total, e->d_bgather, d_result, s)) return rc;
  }
  if (e->ev) HIP_TRY(hipEventRecord(e->ev[EV_END], s));
  e->ev = nullptr;
  return PIR_OK;
}

// Every slice of one query: d_result[t] (t < 2^lt, num_rounds x record_bytes each) = the
// partial answer over this engine's rows [t*R/2^lt, (t+1)*R/2^lt) -- what the T calls
// runOptimizedDPFTreeQueryThread(t, T) of one query return (server.cpp:505-549, intended
// semantics; tree.go:60-76 issues them concurrently with the same key).  One k_query launch over
// the whole shard when its 2^lr regions split evenly into the slices (one tree, one pass, a
// slab reduce per run of regions); else one answer per slice.  Partials stay per engine: no
// all-gather (the Thread form has none either).
int answer_slices_locked(pir_engine* e, const uint8_t* d_key, int lt, uint8_t* d_result,
                         hipStream_t s) {
  const auto& c = e->cfg;
  const size_t out_bytes = (size_t)c.num_rounds * c.record_bytes;
  const int T = 1 << lt;
  e->ev = nullptr;
  const pir::QueryPlan qp = pir::make_query_plan(c.log_num_records, c.log_num_partitions,
                                                 c.num_parties, c.num_rounds, e->pitch, e->num_cus);
  if (qp.tile && lt <= qp.lr && e->allow_query && e->allow_fused)
    return answer_query(e, qp, d_key, 1, c.log_num_partitions, (uint64_t)c.partition_index, 0,
                        d_result, s, T);
  for (int t = 0; t < T; ++t) {
    const uint64_t prefix = ((uint64_t)c.partition_index << lt) | (uint64_t)t;
    const uint64_t row0 = (uint64_t)t * (e->rows >> lt);
    int rc = answer_core(e, d_key, c.log_num_partitions + lt, prefix, row0,
                         d_result + (size_t)t * out_bytes, s);
    if (rc) return rc;
  }
  return PIR_OK;
}

int check_slices(const pir_engine* e, int num_threads, int* lt) {
  *lt = ilog2_exact((uint64_t)(num_threads > 0 ? num_threads : 0));
  if (*lt < 0 || e->cfg.log_num_partitions + *lt > e->cfg.log_num_records)
    return fail(PIR_EINVAL, "num_threads %d must be a power of two <= 2^%d", num_threads,
                e->cfg.log_num_records - e->cfg.log_num_partitions);
  return PIR_OK;
}

// Explicit-coefficient answer (server.cpp:321-382): out[a] = XOR_{i < nrows} src[a*pitch + i] *
// shard[row0 + i].  The vectors are interleaved into the record-major share buffer, then the
// same GF(2^8) scan + slab reduce as the 2-kernel DPF path; with a communicator, the partition
// partials are combined like answers (all-gather + XOR fold).
int answer_coefs_locked(pir_engine* e, const uint8_t* src, uint64_t pitch, uint64_t row0,
                        uint64_t nrows, uint8_t* d_result, hipStream_t s) {
  const auto& c = e->cfg;
  const size_t out_bytes = (size_t)c.num_rounds * c.record_bytes;
  uint8_t* out = e->comm ? e->d_part : d_result;
  e->ev = nullptr;
  if (nrows == 0) {
    HIP_TRY(hipMemsetAsync(out, 0, out_bytes, s));
  } else {
    const pir::ScanShape sh = pir::make_scan_shape(nrows, e->pitch, c.num_rounds, e->num_cus);
    int rc = ensure_slabs(e, (size_t)sh.grid.x * sh.grid.y * sh.slab_bytes);
    if (rc) return rc;
    HIP_TRY(pir::launch_interleave_coefs(src, pitch, nrows, c.num_rounds, e->nrp, e->d_c, s));
    HIP_TRY(pir::launch_scan(sh, e->d_shard + row0 * e->pitch, nrows, e->d_c, e->d_slabs, false, s));
    HIP_TRY(pir::launch_reduce(sh, e->d_slabs, c.record_bytes, out, s));
  }
  if (e->comm) {
    if (int rc = exchange(e, e->d_part, out_bytes, e->d_gather, d_result, s)) return rc;
  }
  return PIR_OK;
}

// Multiparty sqrt(N) DPF answer (server.cpp:384-430): the thread's rows of the domain
// [thr * slice * mu, (thr + 1) * slice * mu), slice = nu / num_threads (the reference drops the
// nu % num_threads remainder rows; so does this), intersected with this engine's partition:
// shares (k_mp_shares) -> GF(2^8) scan -> slab reduce [-> all-gather + XOR fold].
int answer_mp_locked(pir_engine* e, const pir::MpLayout& L, const uint8_t* d_key, int thread_num,
                     int num_threads, uint8_t* d_result, hipStream_t s) {
  const auto& c = e->cfg;
  const size_t out_bytes = (size_t)c.num_rounds * c.record_bytes;
  uint8_t* out = e->comm ? e->d_part : d_result;
  e->ev = nullptr;
  // the whole domain of a layout k_query tiles (the plan's tile divides mu; few seeds per row):
  // ONE launch, its tree waves building each tile's shares from the key while the scan waves
  // stream the shard.  $PIR_MP_FUSED: 0 = never (k_mp_shares, then the scan), 2 = always (an
  // answer k_query cannot take fails: tests), default: where it applies with >= 3 shares, or
  // with 1-2 shares and <= 8 seeds a row (4 share waves + 12 scan waves, query_nq_mp).
  // Measured on 2^24 x 1 KiB (profiles/r04/r4o_ab.jsonl, r4q_ab.jsonl, r4ae_ab.jsonl): CD842 (3
  // shares) 3.19 -> 2.79 ms, CD732 (4) 4.19 -> 3.67 ms, multiparty p = 3 (2 shares, 4 seeds)
  // 2.70 -> 2.52 ms (with 8 share waves it was 2.77: r4p_ab.jsonl)
  const char* fv = getenv("PIR_MP_FUSED");
  const int fmode = fv ? atoi(fv) : 1;
  if (fmode != 0) {
    const pir::QueryPlan qp = pir::make_query_plan(c.log_num_records, c.log_num_partitions, 2,
                                                   c.num_rounds, e->pitch, e->num_cus);
    // more than 32 seeds per row (CD732: 64): the 4 share waves beside the scan fall behind and
    // the separate share kernel + scan is faster (3.77 -> 3.56 ms; CD842's 32 seeds and the
    // multiparty shapes stay fused: 2.82 / 2.51 / 2.64 against 3.15 / 2.66 / 2.81,
    // profiles/r06/r7i_ccd7_fused_ab.*, r7j_mp_fused_ab.*); $PIR_MP_FUSED=2 forces up to 64
    const bool takes = thread_num == 0 && num_threads == 1 && L.nu && L.p2 <= (fmode == 2 ? 64u : 32u) &&
                       e->allow_query && qp.tile && qp.shape.uniform &&
                       L.mu % (uint64_t)qp.tile == 0 &&
                       (fmode == 2 || L.nrk >= 3 || L.p2 <= 8);
    if (!takes && fmode == 2)
      return fail(PIR_EINVAL, "k_query's sqrt(N) mode does not take this answer ($PIR_MP_FUSED=2)");
    if (takes) {
      if (int rc = ensure_slabs(e, pir::query_slab_bytes(qp))) return rc;
      HIP_TRY(pir::launch_query_mp(qp, d_key, 0, 1, L, c.log_num_records, c.log_num_partitions,
                                   (uint64_t)c.partition_index, e->d_shard, e->d_slabs, s));
      HIP_TRY(pir::launch_reduce(qp.shape, e->d_slabs, c.record_bytes, out, s));
      e->last_fused = 3;
      if (e->comm) {
        if (int rc = exchange(e, e->d_part, out_bytes, e->d_gather, d_result, s)) return rc;
      }
      return PIR_OK;
    }
  }
  const uint64_t slice = L.nu / (uint64_t)num_threads;
  const uint64_t p0 = (uint64_t)c.partition_index * e->rows;
  const uint64_t lo = std::max<uint64_t>((uint64_t)thread_num * slice * L.mu, p0);
  const uint64_t hi = std::min<uint64_t>((uint64_t)(thread_num + 1) * slice * L.mu, p0 + e->rows);
  if (hi <= lo) {
    HIP_TRY(hipMemsetAsync(out, 0, out_bytes, s));
  } else {
    const uint64_t nrows = hi - lo;
    const pir::ScanShape sh = pir::make_scan_shape(nrows, e->pitch, c.num_rounds, e->num_cus);
    int rc = ensure_slabs(e, (size_t)sh.grid.x * sh.grid.y * sh.slab_bytes);
    if (rc) return rc;
    HIP_TRY(pir::launch_mp_shares(L, d_key, lo, hi, e->nrp, e->d_c, e->num_cus, s));
    HIP_TRY(pir::launch_scan(sh, e->d_shard + (lo - p0) * e->pitch, nrows, e->d_c, e->d_slabs,
                             false, s));
    HIP_TRY(pir::launch_reduce(sh, e->d_slabs, c.record_bytes, out, s));
  }
  if (e->comm) {
    if (int rc = exchange(e, e->d_part, out_bytes, e->d_gather, d_result, s)) return rc;
  }
  return PIR_OK;
}

// the layout's share count against the engine's rounds, the thread slot
int check_layout(const pir_engine* e, const pir::MpLayout& L, int thread_num, int num_threads,
                 const char* what) {
  if (L.nrk != e->cfg.num_rounds)
    return fail(PIR_EINVAL, "the %s layout gives %d shares but the engine has %d rounds", what,
                L.nrk, e->cfg.num_rounds);
  if (num_threads < 1 || thread_num < 0 || thread_num >= num_threads)
    return fail(PIR_EINVAL, "thread_num %d of %d", thread_num, num_threads);
  return PIR_OK;
}

int check_mp(const pir_engine* e, int p, int t, int thread_num, int num_threads,
             pir::MpLayout* L) {
  if (!pir::mp_layout(p, e->cfg.log_num_records, t, L))
    return fail(PIR_EINVAL, "no multiparty DPF layout for p=%d t=%d n=%d", p, t,
                e->cfg.log_num_records);
  return check_layout(e, *L, thread_num, num_threads, "multiparty (NUM_RSS_KEYS)");
}

int check_cd(const pir_engine* e, int q_needed, int num_cd_keys, int thread_num,
             int num_threads, pir::MpLayout* L) {
  if (!pir::cd_layout(e->cfg.log_num_records, q_needed, num_cd_keys, L))
    return fail(PIR_EINVAL, "no covering-design DPF layout for NUM_CD_KEYS_NEEDED=%d "
                "NUM_CD_KEYS=%d n=%d", q_needed, num_cd_keys, e->cfg.log_num_records);
  return check_layout(e, *L, thread_num, num_threads, "covering-design (NUM_CD_KEYS)");
}

// a validated sqrt(N) layout's answer from a device key (any alignment)
int answer_layout_dev(pir_engine* e, const pir::MpLayout& L, const uint8_t* d_key, int thread_num,
                      int num_threads, uint8_t* d_result, void* stream) {
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  if (int rc = ws_acquire(e, s)) return rc;
  if (((uintptr_t)d_key & 15) && L.eval_bytes) {  // the seeds are read as 16-byte words
    if (int rc = ensure_buf(&e->d_mpkey, &e->mpkey_cap, L.eval_bytes)) return rc;
    HIP_TRY(hipMemcpyAsync(e->d_mpkey, d_key, L.eval_bytes, hipMemcpyDeviceToDevice, s));
    d_key = e->d_mpkey;
  }
  return ws_release(e, s, answer_mp_locked(e, L, d_key, thread_num, num_threads, d_result, s));
}

// ... and from a host key of key_bytes bytes, answer copied back to host memory
int answer_layout_host(pir_engine* e, const pir::MpLayout& L, const uint8_t* key,
                       uint64_t key_bytes, int thread_num, int num_threads, uint8_t* result,
                       const char* what) {
  if (key_bytes < L.eval_bytes)
    return fail(PIR_EINVAL, "%s key of %llu bytes; the evaluation reads %llu", what,
                (unsigned long long)key_bytes, (unsigned long long)L.eval_bytes);
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const size_t out_bytes = (size_t)e->cfg.num_rounds * e->cfg.record_bytes;
  if (int rc = ws_acquire(e, e->stream)) return rc;
  if (int rc = ensure_buf(&e->d_mpkey, &e->mpkey_cap, std::max<uint64_t>(16, L.eval_bytes))) return rc;
  if (L.eval_bytes)
    HIP_TRY(hipMemcpyAsync(e->d_mpkey, key, L.eval_bytes, hipMemcpyHostToDevice, e->stream));
  int rc = ws_release(e, e->stream, answer_mp_locked(e, L, e->d_mpkey, thread_num, num_threads,
                                                     e->d_result, e->stream));
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(e->h_res, e->d_result, out_bytes, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  memcpy(result, e->h_res, out_bytes);
  return PIR_OK;
}

int check_rows(const pir_engine* e, uint64_t row0, uint64_t nrows) {
  if (row0 > e->rows || nrows > e->rows - row0)
    return fail(PIR_EINVAL, "rows [%llu,%llu) beyond the %llu held", (unsigned long long)row0,
                (unsigned long long)(row0 + nrows), (unsigned long long)e->rows);
  return PIR_OK;
}

}  // namespace

extern "C" {

const char* pir_engine_last_error(void) { return g_err.c_str(); }

int pir_engine_key_len(int p, int n, int nq) {  // utils.cpp:85-90
  return 16 + n * (p - 1) * (16 + 2 * p - 2) + nq * (p - 1);
}

int pir_engine_create(const pir_engine_config* cfg, pir_engine_t** out) {
  if (!cfg || !out) return fail(PIR_EINVAL, "null argument");
  const auto& c = *cfg;
  if (c.num_parties < 2 || c.num_parties > PIR_MAX_PARTIES)
    return fail(PIR_EINVAL, "num_parties %d outside [2,%d]", c.num_parties, PIR_MAX_PARTIES);
  if (c.party_index < 1 || c.party_index > c.num_parties)
    return fail(PIR_EINVAL, "party_index %d outside [1,%d]", c.party_index, c.num_parties);
  if (c.num_rounds < 1 || c.num_rounds > PIR_MAX_ROUNDS)
    return fail(PIR_EINVAL, "num_rounds %d outside [1,%d]", c.num_rounds, PIR_MAX_ROUNDS);
  if (c.log_num_records < 0 || c.log_num_records > PIR_MAX_LOG_RECORDS)
    return fail(PIR_EINVAL, "log_num_records %d", c.log_num_records);
  if (c.record_bytes < 1) return fail(PIR_EINVAL, "record_bytes must be >= 1");
  if (c.log_num_partitions < 0 || c.log_num_partitions > c.log_num_records ||
      c.partition_index < 0 || (uint64_t)c.partition_index >= (1ull << c.log_num_partitions))
    return fail(PIR_EINVAL, "bad partition %d of 2^%d", c.partition_index, c.log_num_partitions);
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (c.device < 0 || c.device >= ndev) return fail(PIR_EINVAL, "device %d of %d", c.device, ndev);
  HIP_TRY(hipSetDevice(c.device));

  auto* e = new pir_engine;
  e->cfg = c;
  e->nrp = c.num_rounds == 1 ? 1 : (c.num_rounds == 2 ? 2 : (c.num_rounds <= 4 ? 4 : (c.num_rounds <= 8 ? 8 : 16)));
  e->pitch = (c.record_bytes + 15u) & ~15u;
  e->rows = 1ull << (c.log_num_records - c.log_num_partitions);
  e->key_len = pir_engine_key_len(c.num_parties, c.log_num_records, c.num_rounds);
  auto cleanup = [&](int rc) { pir_engine_destroy(e); return rc; };
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c.device) == hipSuccess) e->num_cus = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&e->aux, hipStreamNonBlocking) != hipSuccess)
    return cleanup(fail(PIR_EHIP, "hipStreamCreate failed"));
  for (auto& ev : e->ev_leaf)
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
      return cleanup(fail(PIR_EHIP, "hipEventCreate failed"));
  if (hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_ws, hipEventDisableTiming) != hipSuccess)
    return cleanup(fail(PIR_EHIP, "hipEventCreate failed"));
  for (int i = 0; i < 2; ++i)
    if (hipEventCreateWithFlags(&e->ev_cb_ready[i], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_cb_free[i], hipEventDisableTiming) != hipSuccess)
      return cleanup(fail(PIR_EHIP, "hipEventCreate failed"));
  const size_t shard_bytes = (size_t)e->rows * e->pitch;
  if (hipMalloc(&e->d_shard, shard_bytes) != hipSuccess)
    return cleanup(fail(PIR_ENOMEM, "hipMalloc shard %zu bytes", shard_bytes));
  if (hipMemsetAsync(e->d_shard, 0, shard_bytes, e->stream) != hipSuccess)
    return cleanup(fail(PIR_EHIP, "hipMemset shard"));
  pir::TreePlan pl = pir::make_plan(c.log_num_records, c.log_num_partitions, 0, -1, c.num_parties);
  {
    const char* f = getenv("PIR_FUSED");
    e->allow_fused = !(f && f[0] == '0');
    const char* qy = getenv("PIR_QUERY");
    e->allow_query = !(qy && qy[0] == '0');
    const char* fr = getenv("PIR_FUSED_REDUCE");
    if (fr) e->fused_reduce = std::max(0, std::min(3, atoi(fr)));
    // $PIR_QUERY_STEAL: 0 = off; else the kernel's StealArgs::mode (default 3)
    const char* st = getenv("PIR_QUERY_STEAL");
    if (st) e->steal = std::max(0, std::min(3, atoi(st)));
    const char* bg = getenv("PIR_BATCH_G");
    if (bg) e->batch_group = atoi(bg);
    const char* bb = getenv("PIR_BATCH_SCAN_BPC");
    if (bb) e->batch_scan_bpc = std::max(1, atoi(bb));
    const char* bk = getenv("PIR_BATCH_KLAST");
    if (bk) e->batch_k_last = std::max(1, std::min(12, atoi(bk)));
    const int tile = pir::fused_tile(c.num_rounds, e->pitch, e->rows, e->num_cus);
    if (tile) {
      const pir::TreePlan pf =
          pir::make_plan(c.log_num_records, c.log_num_partitions, 0, pir::fused_k(tile), c.num_parties);
      if (pf.max_nodes > pl.max_nodes) pl = pf;
    }
  }
  const size_t out_bytes = (size_t)c.num_rounds * c.record_bytes;
  if (hipMalloc(&e->nodes.s[0], pl.max_nodes * sizeof(uint4)) != hipSuccess ||
      hipMalloc(&e->nodes.s[1], pl.max_nodes * sizeof(uint4)) != hipSuccess ||
      hipMalloc(&e->nodes.t[0], pl.max_nodes * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&e->nodes.t[1], pl.max_nodes * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&e->d_c, (size_t)e->rows * e->nrp) != hipSuccess ||
      hipMalloc(&e->d_part, out_bytes) != hipSuccess ||
      hipMalloc(&e->d_result, out_bytes) != hipSuccess ||
      hipHostMalloc(&e->h_key, e->key_len) != hipSuccess ||
      hipHostMalloc(&e->h_res, out_bytes) != hipSuccess)
    return cleanup(fail(PIR_ENOMEM, "workspace allocation failed"));
  int rc = ensure_batch(e, 1);
  if (rc) return cleanup(rc);
  if (hipStreamSynchronize(e->stream) != hipSuccess) return cleanup(fail(PIR_EHIP, "sync"));
  *out = e;
  return PIR_OK;
}

void pir_engine_destroy(pir_engine_t* e) {
  if (!e) return;
  (void)hipSetDevice(e->cfg.device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->aux) (void)hipStreamSynchronize(e->aux);
  if (e->comm) (void)ncclCommDestroy(e->comm);
  for (auto* p : {(void*)e->d_shard, (void*)e->d_key_raw, (void*)e->d_keys,
                  (void*)e->nodes.s[0], (void*)e->nodes.s[1], (void*)e->nodes.t[0],
                  (void*)e->nodes.t[1], (void*)e->d_c, (void*)e->d_slabs, (void*)e->d_part,
                  (void*)e->d_gather, (void*)e->d_result, (void*)e->d_cb, (void*)e->d_gtmp,
                  (void*)e->d_bpart, (void*)e->d_bgather, (void*)e->d_qscratch, (void*)e->d_coef_stage,
                  (void*)e->d_qcnt, (void*)e->d_steal, (void*)e->d_mpkey,
                  (void*)e->bnodes.s[0],
                  (void*)e->bnodes.s[1], (void*)e->bnodes.t[0], (void*)e->bnodes.t[1]})
    if (p) (void)hipFree(p);
  for (auto& b : e->user) (void)hipFree(b.p);
  if (e->h_key) (void)hipHostFree(e->h_key);
  if (e->h_res) (void)hipHostFree(e->h_res);
  if (e->h_slices) (void)hipHostFree(e->h_slices);
  if (e->d_slices) (void)hipFree(e->d_slices);
  for (auto& sl : e->prof)
    for (auto& ev : sl.ev) (void)hipEventDestroy(ev);
  for (auto& ev : e->ev_leaf)
    if (ev) (void)hipEventDestroy(ev);
  for (int i = 0; i < 2; ++i) {
    if (e->ev_cb_ready[i]) (void)hipEventDestroy(e->ev_cb_ready[i]);
    if (e->ev_cb_free[i]) (void)hipEventDestroy(e->ev_cb_free[i]);
  }
  if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
  if (e->ev_join) (void)hipEventDestroy(e->ev_join);
  if (e->ev_ws) (void)hipEventDestroy(e->ev_ws);
  if (e->aux) (void)hipStreamDestroy(e->aux);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

uint64_t pir_engine_num_rows(const pir_engine_t* e) { return e ? e->rows : 0; }

int pir_engine_set_shard(pir_engine_t* e, const uint8_t* host, uint64_t row0, uint64_t nrows,
                         uint64_t src_pitch) {
  if (!e || (!host && nrows)) return fail(PIR_EINVAL, "null argument");
  if (row0 + nrows > e->rows) return fail(PIR_EINVAL, "rows [%llu,%llu) beyond %llu",
                                          (unsigned long long)row0,
                                          (unsigned long long)(row0 + nrows),
                                          (unsigned long long)e->rows);
  if (src_pitch < e->cfg.record_bytes) return fail(PIR_EINVAL, "src_pitch < record_bytes");
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  // 2-D copy writes record_bytes per row; the pad bytes stay zero from the create memset
  HIP_TRY(hipMemcpy2DAsync(e->d_shard + row0 * e->pitch, e->pitch, host, src_pitch,
                           e->cfg.record_bytes, nrows, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return PIR_OK;
}

extern "C++" {
namespace {

// Host threads for the staged row copies below ($PIR_GATHER_THREADS; the GPU box grants 16
// CPUs per GPU, OMP_NUM_THREADS says how many)
int gather_threads() {
  if (const char* v = getenv("PIR_GATHER_THREADS")) return std::max(1, atoi(v));
  int n = (int)std::thread::hardware_concurrency();
  if (const char* v = getenv("OMP_NUM_THREADS")) n = std::min(n, std::max(1, atoi(v)));
  return std::max(1, std::min(8, n));
}

// T - 1 host threads kept for the length of one staged copy (a 64 GiB setup is ~1000 chunks:
// spawning a thread team per chunk cost more than some chunks' copies); run(fn) calls fn(t, T)
// on every thread, the caller's as t = 0, and returns when all have.
class Crew {
 public:
  explicit Crew(int T) : T_(T) {
    for (int t = 1; t < T_; ++t) th_.emplace_back([this, t] { loop(t); });
  }
  ~Crew() {
    {
      std::lock_guard<std::mutex> lk(m_);
      quit_ = true;
    }
    go_.notify_all();
    for (auto& x : th_) x.join();
  }
  void run(const std::function<void(int, int)>& fn) {
    {
      std::lock_guard<std::mutex> lk(m_);
      job_ = &fn;
      pending_ = T_ - 1;
      ++gen_;
    }
    go_.notify_all();
    fn(0, T_);
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int, int)>* job;
      {
        std::unique_lock<std::mutex> lk(m_);
        go_.wait(lk, [&] { return quit_ || gen_ != seen; });
        if (quit_) return;
        seen = gen_;
        job = job_;
      }
      (*job)(t, T_);
      std::lock_guard<std::mutex> lk(m_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  const int T_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable go_, done_;
  const std::function<void(int, int)>* job_ = nullptr;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool quit_ = false;
};

// [a, b) of n items split into T contiguous slices: slice t
inline void slice_of(uint64_t n, int t, int T, uint64_t& a, uint64_t& b) {
  a = n * (uint64_t)t / (uint64_t)T;
  b = n * (uint64_t)(t + 1) / (uint64_t)T;
}

// dst + i * efs <- rows[i] for i in [a, b), each run of rows that lie back to back in host
// memory (the shim's client files and indexList rows are one block) as one memcpy
inline void gather_rows(uint8_t* dst, const uint8_t* const* rows, uint64_t a, uint64_t b,
                        uint32_t efs) {
  for (uint64_t i = a; i < b;) {
    const uint8_t* s0 = rows[i];
    uint64_t j = i + 1;
    while (j < b && rows[j] == s0 + (j - i) * efs) ++j;
    memcpy(dst + i * efs, s0, (size_t)(j - i) * efs);
    i = j;
  }
}
// the reverse: rows[i] <- src + i * efs
inline void scatter_rows(uint8_t* const* rows, const uint8_t* src, uint64_t a, uint64_t b,
                         uint32_t efs) {
  for (uint64_t i = a; i < b;) {
    uint8_t* d0 = rows[i];
    uint64_t j = i + 1;
    while (j < b && rows[j] == d0 + (j - i) * efs) ++j;
    memcpy(d0, src + i * efs, (size_t)(j - i) * efs);
    i = j;
  }
}

// Host rows -> device through two pinned staging buffers of `chunk_bytes`: chunk c is gathered
// by T host threads (fill(c, pinned, t, T)) while the DMA and kernel of chunk c - 1 run
// (issue(c, pinned, stream): its H2D copy and whatever consumes it, enqueued on the engine
// stream); a pinned buffer is refilled only after the copy that read it has completed.  The
// pageable single-threaded gather this replaces moved a 16 GiB shard at a few GB/s.
template <class Fill, class Issue>
int staged_h2d(pir_engine* e, uint64_t nchunks, size_t chunk_bytes, const Fill& fill,
               const Issue& issue) {
  if (!nchunks) return PIR_OK;
  uint8_t* h[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  Crew crew(gather_threads());
  int rc = PIR_OK;
  for (int i = 0; i < 2 && !rc; ++i) {
    if (hipHostMalloc(&h[i], chunk_bytes) != hipSuccess ||
        hipEventCreateWithFlags(&done[i], hipEventDisableTiming) != hipSuccess)
      rc = fail(PIR_ENOMEM, "pinned staging of %zu bytes", chunk_bytes);
  }
  for (uint64_t c = 0; c < nchunks && !rc; ++c) {
    const int b = (int)(c & 1);
    if (c >= 2 && hipEventSynchronize(done[b]) != hipSuccess) {
      rc = fail(PIR_EHIP, "staged upload: chunk %llu", (unsigned long long)(c - 2));
      break;
    }
    const std::function<void(int, int)> job = [&](int t, int nt) { fill(c, h[b], t, nt); };
    crew.run(job);
    hipError_t err = issue(c, h[b], e->stream);
    if (err == hipSuccess) err = hipEventRecord(done[b], e->stream);
    if (err != hipSuccess) rc = fail(PIR_EHIP, "staged upload: %s", hipGetErrorString(err));
  }
  if (hipStreamSynchronize(e->stream) != hipSuccess && !rc) rc = fail(PIR_EHIP, "staged upload sync");
  for (int i = 0; i < 2; ++i) {
    if (h[i]) (void)hipHostFree(h[i]);
    if (done[i]) (void)hipEventDestroy(done[i]);
  }
  return rc;
}

// rows per staging chunk: ~64 MiB of `bytes_per_row` ($PIR_STAGE_CHUNK_BYTES: tests use small
// chunks so a small shard crosses several, with a ragged last one)
uint64_t chunk_rows_for(uint64_t bytes_per_row) {
  uint64_t chunk = 64ull << 20;
  if (const char* v = getenv("PIR_STAGE_CHUNK_BYTES")) chunk = std::max<uint64_t>(1, strtoull(v, nullptr, 10));
  return std::max<uint64_t>(1, chunk / std::max<uint64_t>(1, bytes_per_row));
}

}  // namespace
}  // extern "C++"

int pir_engine_set_shard_rows(pir_engine_t* e, const uint8_t* const* rows, uint64_t row0,
                              uint64_t nrows) {
  if (!e || (!rows && nrows)) return fail(PIR_EINVAL, "null argument");
  if (row0 + nrows > e->rows) return fail(PIR_EINVAL, "rows beyond shard");
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const uint32_t efs = e->cfg.record_bytes;
  const uint64_t m = chunk_rows_for(efs);
  return staged_h2d(
      e, (nrows + m - 1) / m, (size_t)m * efs,
      [&](uint64_t c, uint8_t* dst, int t, int nt) {
        const uint64_t r0 = c * m, n = std::min(m, nrows - r0);
        uint64_t a, b;
        slice_of(n, t, nt, a, b);
        gather_rows(dst, rows + r0, a, b, efs);
      },
      [&](uint64_t c, const uint8_t* src, hipStream_t s) {
        const uint64_t r0 = c * m, n = std::min(m, nrows - r0);
        // record_bytes per row; the pad bytes stay zero from the create memset
        return hipMemcpy2DAsync(e->d_shard + (row0 + r0) * e->pitch, e->pitch, src, efs, efs, n,
                                hipMemcpyHostToDevice, s);
      });
}

int pir_engine_get_shard_rows(pir_engine_t* e, uint8_t* const* rows, uint64_t row0,
                              uint64_t nrows) {
  if (!e || (!rows && nrows)) return fail(PIR_EINVAL, "null argument");
  if (row0 + nrows > e->rows) return fail(PIR_EINVAL, "rows beyond shard");
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const uint32_t efs = e->cfg.record_bytes;
  const uint64_t m = chunk_rows_for(efs), nchunks = (nrows + m - 1) / m;
  // device -> two pinned buffers (DMA of chunk c + 1 while host threads scatter chunk c)
  uint8_t* h[2] = {nullptr, nullptr};
  hipEvent_t ready[2] = {nullptr, nullptr};
  int rc = PIR_OK;
  for (int i = 0; i < 2 && !rc; ++i)
    if (hipHostMalloc(&h[i], (size_t)m * efs) != hipSuccess ||
        hipEventCreateWithFlags(&ready[i], hipEventDisableTiming) != hipSuccess)
      rc = fail(PIR_ENOMEM, "pinned staging of %zu bytes", (size_t)m * efs);
  auto enqueue = [&](uint64_t c) {
    const uint64_t r0 = c * m, n = std::min(m, nrows - r0);
    hipError_t err = hipMemcpy2DAsync(h[c & 1], efs, e->d_shard + (row0 + r0) * e->pitch, e->pitch,
                                      efs, n, hipMemcpyDeviceToHost, e->stream);
    if (err == hipSuccess) err = hipEventRecord(ready[c & 1], e->stream);
    return err;
  };
  if (!rc && nchunks && enqueue(0) != hipSuccess) rc = fail(PIR_EHIP, "get_shard_rows: copy");
  Crew crew(gather_threads());
  for (uint64_t c = 0; c < nchunks && !rc; ++c) {
    if (hipEventSynchronize(ready[c & 1]) != hipSuccess) {
      rc = fail(PIR_EHIP, "get_shard_rows: chunk %llu", (unsigned long long)c);
      break;
    }
    if (c + 1 < nchunks && enqueue(c + 1) != hipSuccess) {
      rc = fail(PIR_EHIP, "get_shard_rows: copy");
      break;
    }
    const uint64_t r0 = c * m, n = std::min(m, nrows - r0);
    const uint8_t* src = h[c & 1];
    const std::function<void(int, int)> job = [&](int t, int nt) {
      uint64_t a, b;
      slice_of(n, t, nt, a, b);
      scatter_rows(rows + r0, src, a, b, efs);
    };
    crew.run(job);
  }
  (void)hipStreamSynchronize(e->stream);
  for (int i = 0; i < 2; ++i) {
    if (h[i]) (void)hipHostFree(h[i]);
    if (ready[i]) (void)hipEventDestroy(ready[i]);
  }
  return rc;
}

int pir_engine_fill_shard_random(pir_engine_t* e, uint64_t seed) {
  if (!e) return fail(PIR_EINVAL, "null engine");
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const uint64_t row0 = (uint64_t)e->cfg.partition_index * e->rows;
  HIP_TRY(pir::launch_fill_shard(e->d_shard, e->rows, e->pitch, e->cfg.record_bytes, row0, seed,
                                 e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return PIR_OK;
}

int pir_engine_encode_across_dev(pir_engine_t* e, const uint8_t* d_files, uint64_t file_pitch,
                                 uint64_t num_files, int k) {
  if (!e) return fail(PIR_EINVAL, "null engine");
  if (k < 1 || k > 16) return fail(PIR_EINVAL, "k = %d outside [1,16]", k);
  if (d_files && file_pitch < e->cfg.record_bytes) return fail(PIR_EINVAL, "file_pitch < record_bytes");
  const uint64_t encdb = (num_files + (uint64_t)k - 1) / (uint64_t)k;
  if (encdb > (1ull << e->cfg.log_num_records))
    return fail(PIR_EINVAL, "%llu files over k=%d need %llu rows > 2^%d", (unsigned long long)num_files,
                k, (unsigned long long)encdb, e->cfg.log_num_records);
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const uint64_t row0 = (uint64_t)e->cfg.partition_index * e->rows;
  HIP_TRY(pir::launch_encode_across(d_files, file_pitch, num_files, k, e->cfg.party_index,
                                    e->d_shard, e->rows, row0, e->pitch, e->cfg.record_bytes,
                                    e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return PIR_OK;
}

int pir_engine_encode_across_rows(pir_engine_t* e, const uint8_t* const* files, uint64_t num_files,
                                  int k) {
  if (!e || (!files && num_files)) return fail(PIR_EINVAL, "null argument");
  if (k < 1 || k > 16) return fail(PIR_EINVAL, "k = %d outside [1,16]", k);
  const uint64_t encdb = (num_files + (uint64_t)k - 1) / (uint64_t)k;
  if (encdb > (1ull << e->cfg.log_num_records))
    return fail(PIR_EINVAL, "%llu files over k=%d need %llu rows > 2^%d", (unsigned long long)num_files,
                k, (unsigned long long)encdb, e->cfg.log_num_records);
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const uint32_t efs = e->cfg.record_bytes;
  const uint64_t prow0 = (uint64_t)e->cfg.partition_index * e->rows;
  // chunk c = this engine's rows [c m, (c + 1) m): its k source files per row staged as k blocks
  // of m rows (block j row r = file encdb j + global row; zero past num_files), so the encode
  // kernel sees k m "files" of which row r takes m j + r -- the encdb of a k m-file database
  const uint64_t m = chunk_rows_for((uint64_t)k * efs), nchunks = (e->rows + m - 1) / m;
  uint8_t* d_stage[2] = {nullptr, nullptr};
  const size_t sbytes = (size_t)k * m * efs;
  int rc = PIR_OK;
  for (int i = 0; i < 2 && !rc; ++i)
    if (hipMalloc(&d_stage[i], sbytes) != hipSuccess) rc = fail(PIR_ENOMEM, "encode staging");
  if (!rc)
    rc = staged_h2d(
        e, nchunks, sbytes,
        [&](uint64_t c, uint8_t* dst, int t, int nt) {
          const uint64_t r0 = c * m, n = std::min(m, e->rows - r0), tot = (uint64_t)k * n;
          uint64_t a, b;
          slice_of(tot, t, nt, a, b);  // items i = j n + r: block j, row r
          while (a < b) {
            const uint64_t j = a / n, r = a - j * n, e_r = std::min(n, r + (b - a));  // rows [r, e_r) of block j
            const uint64_t f0 = encdb * j + prow0 + r0;  // the file of row 0 of block j
            uint8_t* d = dst + j * n * efs;
            const uint64_t live = f0 + e_r <= num_files ? e_r : (f0 >= num_files ? 0 : num_files - f0);
            if (live > r) gather_rows(d, files + f0, r, live, efs);
            const uint64_t z0 = std::max(r, live);
            if (e_r > z0) memset(d + z0 * efs, 0, (size_t)(e_r - z0) * efs);
            a += e_r - r;
          }
        },
        [&](uint64_t c, const uint8_t* src, hipStream_t s) {
          const uint64_t r0 = c * m, n = std::min(m, e->rows - r0);
          uint8_t* ds = d_stage[c & 1];
          hipError_t err = hipMemcpyAsync(ds, src, (size_t)k * n * efs, hipMemcpyHostToDevice, s);
          if (err == hipSuccess)
            err = pir::launch_encode_across(ds, efs, (uint64_t)k * n, k, e->cfg.party_index,
                                            e->d_shard + r0 * e->pitch, n, 0, e->pitch, efs, s);
          return err;
        });
  for (auto* d : d_stage)
    if (d) (void)hipFree(d);
  return rc;
}

int pir_engine_encode_within_rows(pir_engine_t* e, const uint8_t* const* files, uint64_t num_files,
                                  uint32_t file_bytes, int k, int party) {
  if (!e || (!files && num_files)) return fail(PIR_EINVAL, "null argument");
  if (k < 1 || k > 16) return fail(PIR_EINVAL, "k = %d outside [1,16]", k);
  if (party < 0 || party > 255) return fail(PIR_EINVAL, "party %d outside [0,255]", party);
  if ((uint64_t)file_bytes > (uint64_t)k * e->cfg.record_bytes)
    return fail(PIR_EINVAL, "file_bytes %u > k * record_bytes (%d * %u)", file_bytes, k,
                e->cfg.record_bytes);
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const uint64_t prow0 = (uint64_t)e->cfg.partition_index * e->rows;
  const uint32_t fb = std::max<uint32_t>(file_bytes, 1);
  // chunk c = this engine's rows [c m, (c + 1) m) = files prow0 + c m + r (one file per row)
  const uint64_t m = chunk_rows_for(fb), nchunks = (e->rows + m - 1) / m;
  uint8_t* d_stage[2] = {nullptr, nullptr};
  const size_t sbytes = (size_t)m * fb;
  int rc = PIR_OK;
  for (int i = 0; i < 2 && !rc; ++i)
    if (hipMalloc(&d_stage[i], sbytes) != hipSuccess) rc = fail(PIR_ENOMEM, "encode staging");
  auto nfiles_of = [&](uint64_t r0, uint64_t n) {
    const uint64_t g0 = prow0 + r0;
    return g0 >= num_files ? 0ull : std::min<uint64_t>(n, num_files - g0);
  };
  if (!rc)
    rc = staged_h2d(
        e, nchunks, sbytes,
        [&](uint64_t c, uint8_t* dst, int t, int nt) {
          const uint64_t r0 = c * m, n = std::min(m, e->rows - r0), nf = nfiles_of(r0, n);
          uint64_t a, b;
          slice_of(nf, t, nt, a, b);
          if (file_bytes == fb) {
            gather_rows(dst, files + prow0 + r0, a, b, fb);
          } else {
            for (uint64_t i = a; i < b; ++i) memcpy(dst + i * fb, files[prow0 + r0 + i], file_bytes);
          }
        },
        [&](uint64_t c, const uint8_t* src, hipStream_t s) {
          const uint64_t r0 = c * m, n = std::min(m, e->rows - r0), nf = nfiles_of(r0, n);
          uint8_t* ds = d_stage[c & 1];
          hipError_t err = nf ? hipMemcpyAsync(ds, src, (size_t)nf * fb, hipMemcpyHostToDevice, s)
                              : hipSuccess;
          if (err == hipSuccess)
            err = pir::launch_encode_within(ds, fb, nf, file_bytes, k,
                                            party ? party : e->cfg.party_index,
                                            e->d_shard + r0 * e->pitch, n, 0, e->pitch,
                                            e->cfg.record_bytes, s);
          return err;
        });
  for (auto* d : d_stage)
    if (d) (void)hipFree(d);
  return rc;
}

int pir_engine_encode_within_dev(pir_engine_t* e, const uint8_t* d_files, uint64_t file_pitch,
                                 uint64_t num_files, uint32_t file_bytes, int k, int party) {
  if (!e) return fail(PIR_EINVAL, "null engine");
  if (k < 1 || k > 16) return fail(PIR_EINVAL, "k = %d outside [1,16]", k);
  if (party < 0 || party > 255) return fail(PIR_EINVAL, "party %d outside [0,255]", party);
  if (d_files && file_pitch < file_bytes) return fail(PIR_EINVAL, "file_pitch < file_bytes");
  if ((uint64_t)file_bytes > (uint64_t)k * e->cfg.record_bytes)
    return fail(PIR_EINVAL, "file_bytes %u > k * record_bytes (%d * %u)", file_bytes, k,
                e->cfg.record_bytes);
  if (num_files > (1ull << e->cfg.log_num_records))
    return fail(PIR_EINVAL, "%llu files > 2^%d rows", (unsigned long long)num_files,
                e->cfg.log_num_records);
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const uint64_t row0 = (uint64_t)e->cfg.partition_index * e->rows;
  HIP_TRY(pir::launch_encode_within(d_files, file_pitch, num_files, file_bytes, k,
                                    party ? party : e->cfg.party_index, e->d_shard, e->rows,
                                    row0, e->pitch,
                                    e->cfg.record_bytes, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return PIR_OK;
}

int pir_engine_get_shard_row(pir_engine_t* e, uint64_t row, uint8_t* out) {
  if (!e || !out) return fail(PIR_EINVAL, "null argument");
  if (row >= e->rows) return fail(PIR_EINVAL, "row %llu beyond shard", (unsigned long long)row);
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipMemcpyAsync(out, e->d_shard + row * e->pitch, e->cfg.record_bytes,
                         hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return PIR_OK;
}

int pir_engine_answer_dev(pir_engine_t* e, const uint8_t* d_key, uint8_t* d_result,
                          void* stream) {
  if (!e || !d_result) return fail(PIR_EINVAL, "null argument");
  if (int rc = check_key_ptr(d_key)) return rc;
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  if (int rc = ws_acquire(e, s)) return rc;
  return ws_release(e, s, answer_dev_locked(e, d_key, d_result, s));
}

int pir_engine_answer_batch_dev(pir_engine_t* e, const uint8_t* d_keys, int num_keys,
                                uint8_t* d_result, void* stream) {
  if (!e || !d_result || num_keys < 0) return fail(PIR_EINVAL, "bad argument");
  if (int rc = check_key_ptr(d_keys)) return rc;
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  if (int rc = ws_acquire(e, s)) return rc;
  return ws_release(e, s, answer_batch_locked(e, d_keys, num_keys, d_result, s));
}

int pir_engine_answer_batch(pir_engine_t* e, const uint8_t* keys, int num_keys,
                            uint8_t* results) {
  if (!e || (num_keys > 0 && (!keys || !results)) || num_keys < 0)
    return fail(PIR_EINVAL, "bad argument");
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const size_t out_bytes = (size_t)e->cfg.num_rounds * e->cfg.record_bytes;
  const size_t kb = (size_t)num_keys * e->key_len, rb = (size_t)num_keys * out_bytes;
  if (num_keys == 0) return PIR_OK;
  uint8_t *d_k = nullptr, *d_r = nullptr;
  HIP_TRY(hipMalloc(&d_k, kb));
  if (hipMalloc(&d_r, rb) != hipSuccess) {
    (void)hipFree(d_k);
    return fail(PIR_ENOMEM, "batch result buffer %zu bytes", rb);
  }
  int rc = ws_acquire(e, e->stream);
  if (!rc && hipMemcpyAsync(d_k, keys, kb, hipMemcpyHostToDevice, e->stream) != hipSuccess)
    rc = fail(PIR_EHIP, "key upload");
  if (!rc) rc = ws_release(e, e->stream, answer_batch_locked(e, d_k, num_keys, d_r, e->stream));
  if (!rc && (hipMemcpyAsync(results, d_r, rb, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
              hipStreamSynchronize(e->stream) != hipSuccess))
    rc = fail(PIR_EHIP, "batch answer: %s", hipGetErrorString(hipGetLastError()));
  (void)hipStreamSynchronize(e->stream);
  (void)hipFree(d_k);
  (void)hipFree(d_r);
  return rc;
}

int pir_engine_answer_stream_dev(pir_engine_t* e, const uint8_t* d_keys, int num_keys,
                                 uint8_t* d_result, void* stream) {
  if (!e || !d_result || num_keys < 0) return fail(PIR_EINVAL, "bad argument");
  if (int rc = check_key_ptr(d_keys)) return rc;
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  if (int rc = ws_acquire(e, s)) return rc;
  return ws_release(e, s, answer_stream_locked(e, d_keys, num_keys, d_result, s));
}

int pir_engine_reserve_queue(pir_engine_t* e, int num_keys) {
  if (!e || num_keys < 1) return fail(PIR_EINVAL, "bad argument");
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const auto& c = e->cfg;
  const pir::QueryPlan qp = pir::make_query_plan(c.log_num_records, c.log_num_partitions,
                                                 c.num_parties, c.num_rounds, e->pitch, e->num_cus,
                                                 num_keys);
  if (!qp.tile) return PIR_OK;  // shapes k_query does not take allocate per answer
  int rc = ensure_slabs(e, (size_t)num_keys * pir::query_slab_bytes(qp));
  if (!rc) rc = ensure_buf(&e->d_qscratch, &e->qscratch_cap, pir::query_scratch_bytes(qp));
  if (!rc && e->fused_reduce) rc = ensure_qcnt(e, num_keys * 8, e->stream);
  if (!rc && num_keys == 1) {  // the stealing buffer (this advances the generation once: harmless)
    pir::StealArgs st;
    rc = steal_args(e, qp, 1, 1, e->stream, &st);
    // its zeroing ran on the engine stream: done before an answer on any other stream reads it
    if (!rc) HIP_TRY(hipStreamSynchronize(e->stream));
  }
  if (!rc && e->comm) {
    const size_t total = (size_t)num_keys * c.num_rounds * c.record_bytes;
    rc = ensure_buf(&e->d_bpart, &e->bpart_cap, total);
    if (!rc) rc = ensure_buf(&e->d_bgather, &e->bgather_cap, total * e->nranks);
  }
  return rc;
}

int pir_engine_set_batch_group(pir_engine_t* e, int keys_per_pass) {
  if (!e || keys_per_pass < 0 || keys_per_pass > 16) return fail(PIR_EINVAL, "bad argument");
  e->batch_group = keys_per_pass;
  return PIR_OK;
}

int pir_engine_batch_group(const pir_engine_t* e) { return e ? batch_group(e) : 0; }

int pir_engine_answer(pir_engine_t* e, const uint8_t* key, uint8_t* result) {
  if (!e || !result) return fail(PIR_EINVAL, "null argument");
  if (int rc = check_key_ptr(key)) return rc;
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const size_t out_bytes = (size_t)e->cfg.num_rounds * e->cfg.record_bytes;
  if (int rc = ws_acquire(e, e->stream)) return rc;
  memcpy(e->h_key, key, e->key_len);
  HIP_TRY(hipMemcpyAsync(e->d_key_raw, e->h_key, e->key_len, hipMemcpyHostToDevice, e->stream));
  int rc = ws_release(e, e->stream, answer_dev_locked(e, e->d_key_raw, e->d_result, e->stream));
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(e->h_res, e->d_result, out_bytes, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  memcpy(result, e->h_res, out_bytes);
  return PIR_OK;
}

int pir_engine_answer_coefs_dev(pir_engine_t* e, const uint8_t* d_coefs, uint64_t coef_pitch,
                                uint64_t row0, uint64_t nrows, uint8_t* d_result, void* stream) {
  if (!e || !d_result || (!d_coefs && nrows)) return fail(PIR_EINVAL, "null argument");
  if (int rc = check_rows(e, row0, nrows)) return rc;
  if (e->cfg.num_rounds > 1 && coef_pitch < row0 + nrows)
    return fail(PIR_EINVAL, "coef_pitch %llu < %llu rows", (unsigned long long)coef_pitch,
                (unsigned long long)(row0 + nrows));
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  if (int rc = ws_acquire(e, s)) return rc;
  return ws_release(e, s, answer_coefs_locked(e, d_coefs + row0, coef_pitch, row0, nrows,
                                              d_result, s));
}

int pir_engine_answer_coefs(pir_engine_t* e, const uint8_t* const* coefs, uint64_t row0,
                            uint64_t nrows, uint8_t* result) {
  if (!e || !result || (!coefs && nrows)) return fail(PIR_EINVAL, "null argument");
  if (int rc = check_rows(e, row0, nrows)) return rc;
  const auto& c = e->cfg;
  for (int a = 0; a < c.num_rounds && nrows; ++a)
    if (!coefs[a]) return fail(PIR_EINVAL, "null coefficient vector %d", a);
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(c.device));
  const size_t out_bytes = (size_t)c.num_rounds * c.record_bytes;
  if (int rc = ws_acquire(e, e->stream)) return rc;
  int rc = ensure_buf(&e->d_coef_stage, &e->coef_stage_cap,
                      std::max<size_t>(1, (size_t)c.num_rounds * nrows));
  if (rc) return rc;
  for (int a = 0; a < c.num_rounds && nrows; ++a)  // only the rows answered travel
    HIP_TRY(hipMemcpyAsync(e->d_coef_stage + (size_t)a * nrows, coefs[a] + row0, nrows,
                           hipMemcpyHostToDevice, e->stream));
  rc = ws_release(e, e->stream, answer_coefs_locked(e, e->d_coef_stage, nrows, row0, nrows,
                                                    e->d_result, e->stream));
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(e->h_res, e->d_result, out_bytes, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  memcpy(result, e->h_res, out_bytes);
  return PIR_OK;
}

int pir_engine_mp_num_keys(int p, int t) {  // params.cpp:618
  if (p < 1 || t < 0 || t > p) return 0;
  return pir::mp_choose(p, t) * (p - t) / p;
}

int pir_engine_mp_key_len(int p, int n, int t) {  // utils.cpp:105-116 (its own mu = 2^(n/2))
  if (p < 1 || t < 0 || t > p || n < 0 || n > 62) return 0;
  const int c = pir::mp_choose(p, t), q = (p - t) * c / p;
  if (c < 1 || c > 32) return 0;
  const uint64_t p2 = 1ull << (c - 1), mu = 1ull << (n / 2), nu = 1ull << (n - n / 2);
  return (int)(16 * p2 * nu + (uint64_t)q * nu * p2 + p2 * mu);
}

long long pir_engine_mp_eval_bytes(int p, int n, int t) {
  pir::MpLayout L;
  return pir::mp_layout(p, n, t, &L) ? (long long)L.eval_bytes : -1;
}

int pir_engine_answer_mp_dev(pir_engine_t* e, const uint8_t* d_key, int p, int t, int thread_num,
                             int num_threads, uint8_t* d_result, void* stream) {
  if (!e || !d_result) return fail(PIR_EINVAL, "null argument");
  if (int rc = check_key_ptr(d_key)) return rc;
  pir::MpLayout L;
  if (int rc = check_mp(e, p, t, thread_num, num_threads, &L)) return rc;
  return answer_layout_dev(e, L, d_key, thread_num, num_threads, d_result, stream);
}

int pir_engine_answer_mp(pir_engine_t* e, const uint8_t* key, uint64_t key_bytes, int p, int t,
                         int thread_num, int num_threads, uint8_t* result) {
  if (!e || !result) return fail(PIR_EINVAL, "null argument");
  if (int rc = check_key_ptr(key)) return rc;
  pir::MpLayout L;
  if (int rc = check_mp(e, p, t, thread_num, num_threads, &L)) return rc;
  return answer_layout_host(e, L, key, key_bytes, thread_num, num_threads, result, "multiparty");
}

int pir_engine_cd_key_len(int p, int n, int t, int num_cd_keys_needed, int num_cd_keys) {
  (void)p; (void)t;  // utils.cpp:118-129 takes them and does not use them
  pir::MpLayout L;
  return pir::cd_layout(n, num_cd_keys_needed, num_cd_keys, &L) ? (int)L.eval_bytes : 0;
}

int pir_engine_answer_cd_dev(pir_engine_t* e, const uint8_t* d_key, int num_cd_keys_needed,
                             int num_cd_keys, int thread_num, int num_threads, uint8_t* d_result,
                             void* stream) {
  if (!e || !d_result) return fail(PIR_EINVAL, "null argument");
  if (int rc = check_key_ptr(d_key)) return rc;
  pir::MpLayout L;
  if (int rc = check_cd(e, num_cd_keys_needed, num_cd_keys, thread_num, num_threads, &L)) return rc;
  return answer_layout_dev(e, L, d_key, thread_num, num_threads, d_result, stream);
}

int pir_engine_answer_cd(pir_engine_t* e, const uint8_t* key, uint64_t key_bytes,
                         int num_cd_keys_needed, int num_cd_keys, int thread_num, int num_threads,
                         uint8_t* result) {
  if (!e || !result) return fail(PIR_EINVAL, "null argument");
  if (int rc = check_key_ptr(key)) return rc;
  pir::MpLayout L;
  if (int rc = check_cd(e, num_cd_keys_needed, num_cd_keys, thread_num, num_threads, &L)) return rc;
  return answer_layout_host(e, L, key, key_bytes, thread_num, num_threads, result,
                            "covering-design");
}

int pir_engine_answer_slice(pir_engine_t* e, const uint8_t* key, int thread_num, int num_threads,
                            uint8_t* result) {
  if (!e || !result) return fail(PIR_EINVAL, "null argument");
  if (int rc = check_key_ptr(key)) return rc;
  const int lt = ilog2_exact((uint64_t)num_threads);
  const auto& c = e->cfg;
  if (lt < 0 || c.log_num_partitions + lt > c.log_num_records)
    return fail(PIR_EINVAL, "num_threads %d must be a power of two <= 2^%d", num_threads,
                c.log_num_records - c.log_num_partitions);
  if (thread_num < 0 || thread_num >= num_threads)
    return fail(PIR_EINVAL, "thread_num %d of %d", thread_num, num_threads);
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(c.device));
  const size_t out_bytes = (size_t)c.num_rounds * c.record_bytes;
  // NB: the reference's Thread variant computes the honest answer even when isByzantine is
  // set (both branches of server.cpp:526-541 are identical); mirrored here.
  if (int rc = ws_acquire(e, e->stream)) return rc;
  memcpy(e->h_key, key, e->key_len);
  HIP_TRY(hipMemcpyAsync(e->d_key_raw, e->h_key, e->key_len, hipMemcpyHostToDevice, e->stream));
  const uint64_t prefix = ((uint64_t)c.partition_index << lt) | (uint64_t)thread_num;
  const uint64_t row0 = (uint64_t)thread_num * (e->rows >> lt);
  int rc = ws_release(e, e->stream,
                      answer_core(e, e->d_key_raw, c.log_num_partitions + lt, prefix, row0,
                                  e->d_result, e->stream));
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(e->h_res, e->d_result, out_bytes, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  memcpy(result, e->h_res, out_bytes);
  return PIR_OK;
}

int pir_engine_answer_slices_dev(pir_engine_t* e, const uint8_t* d_key, int num_threads,
                                 uint8_t* d_results, void* stream) {
  if (!e || !d_results) return fail(PIR_EINVAL, "null argument");
  if (int rc = check_key_ptr(d_key)) return rc;
  int lt = 0;
  if (int rc = check_slices(e, num_threads, &lt)) return rc;
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  if (int rc = ws_acquire(e, s)) return rc;
  return ws_release(e, s, answer_slices_locked(e, d_key, lt, d_results, s));
}

int pir_engine_answer_slices(pir_engine_t* e, const uint8_t* key, int num_threads,
                             uint8_t* results) {
  if (!e || !results) return fail(PIR_EINVAL, "null argument");
  if (int rc = check_key_ptr(key)) return rc;
  int lt = 0;
  if (int rc = check_slices(e, num_threads, &lt)) return rc;
  const auto& c = e->cfg;
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(c.device));
  const size_t bytes = (size_t)num_threads * c.num_rounds * c.record_bytes;
  if (int rc = ws_acquire(e, e->stream)) return rc;
  if (int rc = ensure_buf(&e->d_slices, &e->slices_cap, bytes)) return rc;
  if (int rc = ensure_host(&e->h_slices, &e->h_slices_cap, bytes)) return rc;
  memcpy(e->h_key, key, e->key_len);
  HIP_TRY(hipMemcpyAsync(e->d_key_raw, e->h_key, e->key_len, hipMemcpyHostToDevice, e->stream));
  int rc = ws_release(e, e->stream, answer_slices_locked(e, e->d_key_raw, lt, e->d_slices,
                                                         e->stream));
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(e->h_slices, e->d_slices, bytes, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  memcpy(results, e->h_slices, bytes);
  return PIR_OK;
}

int pir_engine_eval_all(pir_engine_t* e, const uint8_t* key, uint8_t* out) {
  if (!e || !out) return fail(PIR_EINVAL, "null argument");
  if (int rc = check_key_ptr(key)) return rc;
  std::lock_guard<std::mutex> lk(e->mu);
  const auto& c = e->cfg;
  HIP_TRY(hipSetDevice(c.device));
  if (int rc = ws_acquire(e, e->stream)) return rc;
  memcpy(e->h_key, key, e->key_len);
  HIP_TRY(hipMemcpyAsync(e->d_key_raw, e->h_key, e->key_len, hipMemcpyHostToDevice, e->stream));
  const pir::TreePlan pl =
      pir::make_plan(c.log_num_records, c.log_num_partitions, (uint64_t)c.partition_index, -1, c.num_parties);
  HIP_TRY(pir::launch_frontier(pl, key_src(e, e->d_key_raw), e->nodes, e->stream));
  HIP_TRY(pir::launch_stages(pl, e->d_keys, e->nodes, 0, 1, e->d_c, e->nrp, e->stream));
  std::vector<uint8_t> ct((size_t)e->rows * e->nrp);
  HIP_TRY(hipMemcpyAsync(ct.data(), e->d_c, ct.size(), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->ws_stream = nullptr;  // synchronised: nothing left to order after
  for (uint64_t i = 0; i < e->rows; ++i)
    for (int a = 0; a < c.num_rounds; ++a) out[(size_t)a * e->rows + i] = ct[i * e->nrp + a];
  return PIR_OK;
}

void* pir_engine_stream(pir_engine_t* e) { return e ? (void*)e->stream : nullptr; }

int pir_engine_sync(pir_engine_t* e) {
  if (!e) return fail(PIR_EINVAL, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return PIR_OK;
}

int pir_engine_alloc_dev(pir_engine_t* e, size_t bytes, void** d_ptr) {
  if (!e || !d_ptr) return fail(PIR_EINVAL, "null argument");
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  void* p = nullptr;
  HIP_TRY(hipMalloc(&p, bytes ? bytes : 1));
  e->user.push_back({p, bytes});
  *d_ptr = p;
  return PIR_OK;
}

int pir_engine_free_dev(pir_engine_t* e, void* d_ptr) {
  if (!e) return fail(PIR_EINVAL, "null engine");
  if (!d_ptr) return PIR_OK;
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  for (size_t i = 0; i < e->user.size(); ++i)
    if (e->user[i].p == d_ptr) {
      // answers still queued on any stream may read it: hipFree waits for the device
      HIP_TRY(hipFree(d_ptr));
      e->user.erase(e->user.begin() + (long)i);
      return PIR_OK;
    }
  return fail(PIR_EINVAL, "%p was not allocated by pir_engine_alloc_dev", d_ptr);
}

int pir_engine_set_party_index(pir_engine_t* e, int party_index) {
  if (!e) return fail(PIR_EINVAL, "null engine");
  if (party_index < 1 || party_index > e->cfg.num_parties)
    return fail(PIR_EINVAL, "party_index %d outside [1,%d]", party_index, e->cfg.num_parties);
  std::lock_guard<std::mutex> lk(e->mu);
  e->cfg.party_index = party_index;  // read at enqueue time (a kernel argument), not by kernels
  return PIR_OK;                     // already queued
}

int pir_engine_memcpy_h2d(pir_engine_t* e, void* d_dst, const void* h_src, size_t bytes) {
  if (!e) return fail(PIR_EINVAL, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return PIR_OK;
}

int pir_engine_memcpy_d2h(pir_engine_t* e, void* h_dst, const void* d_src, size_t bytes) {
  if (!e) return fail(PIR_EINVAL, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return PIR_OK;
}

int pir_engine_set_profiling(pir_engine_t* e, int slots) {
  if (!e || slots < 0) return fail(PIR_EINVAL, "bad argument");
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (auto& sl : e->prof)
    for (auto& ev : sl.ev) (void)hipEventDestroy(ev);
  e->prof.assign((size_t)slots, {});
  e->prof_next = e->prof_count = 0;
  for (auto& sl : e->prof)
    // timing-only stamps: no system-scope fence (its cache write-back / invalidate at every
    // record slowed the bracketed k_query by ~2 % against the unprofiled answer)
    for (auto& ev : sl.ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableSystemFence));
  return PIR_OK;
}

int pir_engine_last_timings(pir_engine_t* e, pir_kernel_time* out, int max) {
  if (!e || !out) return fail(PIR_EINVAL, "null argument");
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  return read_timings(e, out, max);
}

int pir_engine_profile_phases(pir_engine_t* e, const uint8_t* d_key, int iters, float* out_ms) {
  if (!e || !d_key || !out_ms || iters < 1) return fail(PIR_EINVAL, "bad argument");
  std::lock_guard<std::mutex> lk(e->mu);
  const auto& c = e->cfg;
  HIP_TRY(hipSetDevice(c.device));
  hipStream_t s = e->stream;
  if (int rc = ws_acquire(e, s)) return rc;
  e->ws_stream = nullptr;  // synchronised below
  const pir::TreePlan pl =
      pir::make_plan(c.log_num_records, c.log_num_partitions, (uint64_t)c.partition_index, -1, c.num_parties);
  const pir::ScanShape sh = pir::make_scan_shape(pl.nleaves, e->pitch, c.num_rounds, e->num_cus);
  int rc = ensure_slabs(e, (size_t)sh.grid.x * sh.grid.y * sh.slab_bytes);
  if (rc) return rc;
  hipEvent_t ev[6];
  for (auto& x : ev) HIP_TRY(hipEventCreate(&x));
  HIP_TRY(hipEventRecord(ev[0], s));
  for (int i = 0; i < iters; ++i)
    HIP_TRY(pir::launch_key_prep(d_key, e->key_len, 1, c.num_parties, c.log_num_records,
                                 c.num_rounds, c.party_index - 1, e->d_keys, s));
  HIP_TRY(hipEventRecord(ev[1], s));
  for (int i = 0; i < iters; ++i)
    HIP_TRY(pir::launch_frontier(pl, key_src(e, nullptr), e->nodes, s));
  HIP_TRY(hipEventRecord(ev[2], s));
  for (int i = 0; i < iters; ++i)
    HIP_TRY(pir::launch_stages(pl, e->d_keys, e->nodes, 0, 1, e->d_c, e->nrp, s));
  HIP_TRY(hipEventRecord(ev[3], s));
  for (int i = 0; i < iters; ++i)
    HIP_TRY(pir::launch_scan(sh, e->d_shard, pl.nleaves, e->d_c, e->d_slabs, false, s));
  HIP_TRY(hipEventRecord(ev[4], s));
  for (int i = 0; i < iters; ++i) HIP_TRY(pir::launch_reduce(sh, e->d_slabs, c.record_bytes, e->d_result, s));
  HIP_TRY(hipEventRecord(ev[5], s));
  HIP_TRY(hipEventSynchronize(ev[5]));
  for (int i = 0; i < 5; ++i) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
    out_ms[i] = ms / iters;
  }
  for (auto& x : ev) (void)hipEventDestroy(x);
  return PIR_OK;
}

int pir_engine_trace_query(pir_engine_t* e, const uint8_t* d_key, int num_keys, uint64_t* out,
                           int max_wgs) {
  if (!e || !d_key || !out || max_wgs < 0 || num_keys < 1) return fail(PIR_EINVAL, "bad argument");
  std::lock_guard<std::mutex> lk(e->mu);
  const auto& c = e->cfg;
  HIP_TRY(hipSetDevice(c.device));
  const pir::QueryPlan qp = pir::make_query_plan(c.log_num_records, c.log_num_partitions,
                                                 c.num_parties, c.num_rounds, e->pitch, e->num_cus,
                                                 num_keys);
  if (!qp.tile) return fail(PIR_EINVAL, "shape does not use the single-launch query kernel");
  if (int rc = ws_acquire(e, e->stream)) return rc;
  e->ws_stream = nullptr;  // synchronised below
  const pir::ScanShape& sh = qp.shape;
  int rc = ensure_slabs(e, (size_t)num_keys * pir::query_slab_bytes(qp));
  if (!rc) rc = ensure_buf(&e->d_qscratch, &e->qscratch_cap, pir::query_scratch_bytes(qp));
  pir::StealArgs steal;
  if (!rc) rc = steal_args(e, qp, num_keys, 1, e->stream, &steal);
  if (rc) return rc;
  const int nwg = (int)sh.grid.x;
  const size_t bytes = (size_t)nwg * pir::kQueryTraceSlots * sizeof(uint64_t);
  uint64_t* d_tr = nullptr;
  HIP_TRY(hipMalloc(&d_tr, bytes + sizeof(uint64_t)));
  std::vector<uint64_t> h((size_t)nwg * pir::kQueryTraceSlots);
  hipError_t err = hipMemsetAsync(d_tr, 0, bytes, e->stream);
  const char* dbg = getenv("PIR_TRACE_NOSCAN");  // diagnostics: scan waves skip their rows
  uint64_t flags = (dbg && dbg[0] == '1') ? 1u : 0u;
#if PIR_TRACE_TREE_TILES
  if (const char* tv = getenv("PIR_TRACE_TILES")) {  // "a,b": two queue tiles' tree phases
    unsigned a = 0, b = 0;
    if (sscanf(tv, "%u,%u", &a, &b) >= 1) flags |= ((uint64_t)(a & 0xffu) << 8) | ((uint64_t)(b & 0xffu) << 16);
  }
#endif
  if (err == hipSuccess)
    err = hipMemcpyAsync(d_tr + (size_t)nwg * pir::kQueryTraceSlots, &flags, sizeof flags,
                         hipMemcpyHostToDevice, e->stream);
  if (err == hipSuccess)
    err = pir::launch_query(qp, d_key, (uint32_t)e->key_len, num_keys, c.num_parties, c.log_num_records,
                            c.party_index - 1, c.log_num_partitions, (uint64_t)c.partition_index,
                            e->d_shard, e->d_slabs, e->d_qscratch, e->stream, d_tr, nullptr,
                            nullptr, 0u, 0u, steal);
  if (err == hipSuccess) err = hipMemcpyAsync(h.data(), d_tr, bytes, hipMemcpyDeviceToHost, e->stream);
  if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
  (void)hipFree(d_tr);
  if (err != hipSuccess) return fail(PIR_EHIP, "trace_query: %s", hipGetErrorString(err));
  uint64_t t0 = ~0ull;
  for (int w = 0; w < nwg; ++w) t0 = std::min(t0, h[(size_t)w * pir::kQueryTraceSlots]);
  const int n = std::min(nwg, max_wgs);
  for (int w = 0; w < n; ++w)
    for (int k = 0; k < pir::kQueryTraceSlots; ++k) {
      const uint64_t v = h[(size_t)w * pir::kQueryTraceSlots + k];
      // shader-clock ticks and counts as they are
      const bool raw = k == 56 || k == 57 || k == 59 || k == 60 || k == 61 ||
                       (k >= 128 && k < 160) || (k >= 192 && !(PIR_TRACE_TREE_TILES && k >= 208));
      out[(size_t)w * pir::kQueryTraceSlots + k] = raw ? v : (v ? v - t0 : 0);
    }
  return nwg;
}

int pir_engine_get_shard(pir_engine_t* e, uint64_t row0, uint64_t nrows, uint8_t* out) {
  if (!e || (!out && nrows)) return fail(PIR_EINVAL, "null argument");
  if (row0 + nrows > e->rows) return fail(PIR_EINVAL, "rows beyond shard");
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipMemcpy2DAsync(out, e->cfg.record_bytes, e->d_shard + row0 * e->pitch, e->pitch,
                           e->cfg.record_bytes, nrows, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return PIR_OK;
}

int pir_engine_fold_gathered_dev(pir_engine_t* e, const uint8_t* d_gathered, int nranks,
                                 uint64_t bytes_per_rank, uint8_t* d_result, void* stream) {
  if (!e || !d_gathered || !d_result || nranks < 1) return fail(PIR_EINVAL, "bad argument");
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  return fold_gathered(e, d_gathered, nranks, (size_t)bytes_per_rank, d_result, s);
}

int pir_comm_unique_id(uint8_t id[PIR_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == PIR_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  RCCL_TRY(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof u);
  return PIR_OK;
}

int pir_comm_detach(pir_engine_t* e) {
  if (!e) return fail(PIR_EINVAL, "null argument");
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  // abort, not destroy: a peer that never joined (or already left) cannot block the caller
  if (e->comm) (void)ncclCommAbort(e->comm);
  e->comm = nullptr;
  e->comm_failed = false;
  e->nranks = 1;
  e->rank = 0;
  return PIR_OK;
}

int pir_comm_info(pir_engine_t* e, pir_comm_info_t* out) {
  if (!e || !out) return fail(PIR_EINVAL, "null argument");
  std::lock_guard<std::mutex> lk(e->mu);
  memset(out, 0, sizeof *out);
  out->attached = e->comm ? 1 : 0;
  out->count = out->user_rank = out->device = -1;
  out->engine_device = e->cfg.device;
  if (e->comm) {
    RCCL_TRY(ncclCommCount(e->comm, &out->count));
    RCCL_TRY(ncclCommUserRank(e->comm, &out->user_rank));
    RCCL_TRY(ncclCommCuDevice(e->comm, &out->device));
  }
  HIP_TRY(hipDeviceGetPCIBusId(out->pci_bus_id, (int)sizeof out->pci_bus_id, e->cfg.device));
  return PIR_OK;
}

int pir_comm_attach(pir_engine_t* e, const uint8_t id[PIR_COMM_ID_BYTES], int nranks, int rank) {
  if (!e || !id) return fail(PIR_EINVAL, "null argument");
  if (nranks != (1 << e->cfg.log_num_partitions) || rank != e->cfg.partition_index)
    return fail(PIR_EINVAL, "rank %d/%d does not match partition %d of 2^%d", rank, nranks,
                e->cfg.partition_index, e->cfg.log_num_partitions);
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->cfg.device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  // non-blocking init, bounded: a rank that cannot join (e.g. RCCL refuses the device) fails
  // here with PIR_ECOMM after at most $PIR_COMM_INIT_TIMEOUT seconds (default 120) instead of
  // leaving the other ranks blocked in ncclCommInitRank
  const char* ts = getenv("PIR_COMM_INIT_TIMEOUT");
  const double timeout_s = ts ? atof(ts) : 120.0;
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t comm = nullptr;
  ncclResult_t r = ncclCommInitRankConfig(&comm, nranks, u, rank, &cfg);
  if (comm) r = rccl_settle(comm, r, timeout_s);
  if (r != ncclSuccess) {
    if (comm) (void)ncclCommAbort(comm);
    return fail(PIR_ECOMM, "ncclCommInitRank(rank %d of %d) failed: %s", rank, nranks,
                r == ncclInProgress ? "timed out" : ncclGetErrorString(r));
  }
  e->comm = comm;
  e->nranks = nranks;
  e->rank = rank;
  e->comm_failed = false;
  const char* xt = getenv("PIR_COMM_TIMEOUT");  // seconds one exchange may take to enqueue
  if (xt && atof(xt) > 0) e->comm_timeout_s = atof(xt);
  if (e->d_gather) (void)hipFree(e->d_gather);  // a re-attach (after pir_comm_detach)
  e->d_gather = nullptr;
  HIP_TRY(hipMalloc(&e->d_gather, (size_t)nranks * e->cfg.num_rounds * e->cfg.record_bytes));
  return PIR_OK;
}

}  // extern "C"
