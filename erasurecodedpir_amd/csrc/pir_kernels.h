// pir_kernels.h -- internal interface between the HIP kernels (pir_kernels.hip) and the
// engine host code (pir_engine.cpp).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pir {

constexpr int kMaxLevels = 40;  // PIR_MAX_LOG_RECORDS
constexpr int kMaxCW = 16;      // p - 1 <= 16
constexpr int kScanThreads = 512;
constexpr int kScanBlocksPerCU = 2;
constexpr int kReduceThreads = 1024;
constexpr int kColGroupLanes = 64;  // one wave's lanes cover a column group of a record
constexpr int kBufRsrcWord3 = 0x00020000;  // gfx9 raw buffer: 32-bit data format, no swizzle

// One DPF key, parsed for the device (written by k_key_prep from the raw key bytes whose
// layout is genOptimizedDPF's: dpf_tree.cpp:254-269).
struct DevKey {
  uint4 root_seed;               // key[0:16]
  uint32_t root_t;               // party control bits: bit (party0-1) (dpf_tree.cpp:496-502)
  uint32_t p, n, nq;
  uint4 scw[kMaxLevels * kMaxCW];      // sCW[L][j]
  uint32_t tcw[kMaxLevels * kMaxCW];   // tCW[L][j] packed: bit k = key byte (16+k) of the CW
  uint4 lastcw[kMaxCW];                // lastCW[j][a] as byte a (a < nq; zero above)
};

// Key-independent shape of one answer pass (one partition of the logical tree):
//   k_frontier  : levels [0, log_parts + F) -> 2^F nodes (latency-bound, column-shape AES)
//   stages      : k_expand, <= 4 levels each; the last one converts the leaves
struct Stage {
  int L_in;      // absolute tree level of the stage's input nodes
  int k;         // levels expanded
  int tile;      // input nodes per workgroup
  uint64_t nin;  // input nodes (whole partition)
  bool final;
};
struct TreePlan {
  int n, log_parts;
  int p;  // parties (the control-bit bytes a node reads); 0: unknown (all 4 bytes)
  uint64_t prefix;
  int F, g, e;  // frontier: 2^g workgroups, each descends log_parts+g levels, expands e
  uint64_t nfront, nleaves, max_nodes;
  int nstages;
  Stage st[8];
};
struct NodeBufs {  // ping-pong node arrays in global memory (max_nodes entries each)
  uint4* s[2];
  uint32_t* t[2];
};

// k_last: levels of the leaf-converting last stage (-1: default 4 for k_expand<FINAL>)
// max_front: levels of the column-shape frontier (16; batched answers 8: their upper levels
// then run as depth-first node stages of 4 levels, F in [8, 11] so that they divide evenly)
TreePlan make_plan(int n, int log_parts, uint64_t prefix, int k_last = -1, int p = 0,
                   int max_front = 16);
int final_stage_blocks(const TreePlan& pl);  // workgroups of the leaf-converting stage


hipError_t launch_key_prep(const uint8_t* d_raw, size_t key_stride, int num_keys, int p, int n,
                           int nq, int party0, DevKey* d_keys, hipStream_t s);
// Where the frontier gets the key: raw bytes (parsed in-kernel; the DevKey for the later
// kernels is written to `key` by workgroup 0), or raw == nullptr: `key` already parsed.
struct KeySrc {
  const uint8_t* raw;
  int p, n, nq, party0;
  DevKey* key;
};
// A batch of keys expanded side by side (grid row y = key y): parsed keys d_key[y], node
// ranges node_stride nodes apart in both ping-pong buffers, shares at d_c + y * c_key_off; the
// first stage may read its input from a separate array (in0, in0_stride nodes per key).
struct StageBatch {
  int nkeys;
  uint64_t node_stride;
  uint32_t c_key_off;
  const uint4* in0_s;
  const uint32_t* in0_t;
  uint64_t in0_stride;
};
// nkeys > 1: a batch of keys (raw keys raw_stride bytes apart, parsed keys ks.key[y], node
// ranges node_stride nodes apart), one grid row per key
hipError_t launch_frontier(const TreePlan& pl, const KeySrc& ks, const NodeBufs& nb,
                           hipStream_t s, int nkeys = 1, size_t raw_stride = 0,
                           uint64_t node_stride = 0);
// expand stages [i0, i1) (i1 < 0: to the last) for chunk j of C of every stage's input range;
// the final stage writes leaf i's nrp share bytes at d_c + i * cstride (cstride <= 0: nrp)
hipError_t launch_stages(const TreePlan& pl, const DevKey* d_key, const NodeBufs& nb, int j, int C,
                         uint8_t* d_c, int nrp, hipStream_t s, int i0 = 0, int i1 = -1,
                         int cstride = 0, const StageBatch* batch = nullptr);
// k_leaves (pir_leaves.hip): the leaf-converting last stage of kd levels, depth first per lane
// (one input node per lane, its 2^kd leaves in registers; 4-table AES, pir_aes4.h); kd in
// [kLeavesMinK, kLeavesMaxK], p = parties (the control-bit bytes a node needs).
// Same arguments as a final k_expand stage: nkeys keys along grid y, input nodes in_stride
// apart per key, key y's shares at c + y * c_key_off, leaf i's nrp bytes at c + i * cstride.
constexpr int kLeavesMinK = 4;
constexpr int kLeavesMaxK = 5;
bool leaves_supported(int kd);
hipError_t launch_leaves(int p, int nrp, int kd, const DevKey* d_key, const uint4* is,
                         const uint32_t* it, int L0, uint64_t nin, int nkeys, uint64_t in_stride,
                         uint8_t* c, uint32_t cstride, uint32_t c_key_off, hipStream_t s);
// The node-writing stages of kd in [1, kNodesMaxK] levels the same way (one input node per
// lane, its 2^kd descendants of the stage's last level written to os/ot, out_stride per key).
constexpr int kNodesMaxK = 4;
bool nodes_dfs_supported(int kd);
hipError_t launch_nodes_dfs(int p, int kd, const DevKey* d_key, const uint4* is,
                            const uint32_t* it, int L0, uint64_t nin, int nkeys,
                            uint64_t in_stride, uint4* os, uint32_t* ot, uint64_t out_stride,
                            hipStream_t s);
// $PIR_LEAF_DFS=0: every stage on k_expand (breadth first in LDS) instead of k_subtree
bool leaf_dfs_enabled();
// scan rows [0, nrec) of `shard` (row pitch `pitch`) with coefficients cT[i*nrp + a]
struct ScanShape {
  int nq, nrp, vec;      // vec = dwords per lane chunk (4, 2, 1)
  bool uniform;          // a record spans >= one wave (one record per wave row)
  uint32_t pitch, cpr;   // bytes per row, chunks per row
  uint32_t slab_bytes;   // per-workgroup partial = nq * 64 * vec * 4
  dim3 grid;
  int threads;           // k_scan_uni workgroup: kScanThreads, or kScanM4rThreads (4-5 rounds)
  bool tfold;            // k_scan_t (pir_scan_t.hip): transposed four-Russians fold, VEC = 1
  // k_scan_t only: coefficients key-major (batched answers): ckey bytes per key and record, key
  // g's block at g * ckoff (record i's word = the NRP / ckey keys' ckey bytes, key g at byte
  // g * ckey); ckey == 0: record-major, record i's NRP bytes at i * NRP
  uint32_t ckey = 0;
  uint64_t ckoff = 0;
};
// k_scan_t takes 4-8 rounds of 4/8 coefficient bytes per record over records of >= 256 B
// ($PIR_SCAN_T=0: the k_scan_uni forms instead).  Workgroups of kScanTThreads, kScanTBlocksPerCU
// per CU, kScanTWavesPerEU waves per SIMD (its register budget: 512 / waves VGPRs)
#ifndef PIR_SCAN_T_THREADS
#define PIR_SCAN_T_THREADS 256
#endif
#ifndef PIR_SCAN_T_WPE
#define PIR_SCAN_T_WPE 4
#endif
constexpr int kScanTThreads = PIR_SCAN_T_THREADS;
constexpr int kScanTWavesPerEU = PIR_SCAN_T_WPE;
constexpr int kScanTBlocksPerCU = kScanTWavesPerEU * 4 * 64 / kScanTThreads;
bool scan_t_enabled();
bool scan_t_shape(int nq, int nrp, uint32_t pitch);
hipError_t launch_scan_t(const ScanShape& sh, const uint8_t* d_shard, uint64_t nrec,
                         const uint8_t* d_c, uint8_t* d_slabs, int acc, hipStream_t s);
// k_scan_uni for 4-5 rounds at two dwords per lane: four-Russians folds need 168 VGPRs, so one
// 768-thread workgroup per CU (only where the caller leaves the CU to the scan: blocks_per_cu 0)
constexpr int kScanM4rThreads = 768;
// blocks_per_cu <= 0: kScanBlocksPerCU.  One block per CU leaves room on every CU for a
// 1024-thread tree workgroup beside the scan (batched answers overlap the two).
ScanShape make_scan_shape(uint64_t nrec, uint32_t pitch, int nq, int num_cus, int blocks_per_cu = 0);
// accumulate: XOR into the slabs instead of overwriting them (chunked scans of one answer)
hipError_t launch_scan(const ScanShape& sh, const uint8_t* d_shard, uint64_t nrec,
                       const uint8_t* d_c, uint8_t* d_slabs, bool accumulate, hipStream_t s);
// Fused leaf stage + scan (one persistent workgroup per CU).  fused_tile() = leaves per tile
// (0: not supported for this shape -> 2-kernel path); plan with make_plan(.., fused_k(tile)).
int fused_tile(int nq, uint32_t pitch, uint64_t nleaves, int num_cus);
int fused_k(int tile);
ScanShape make_fused_shape(uint64_t nleaves, uint32_t pitch, int nq, int num_cus, int tile);
hipError_t launch_fused(const TreePlan& pl, const DevKey* d_key, const NodeBufs& nb,
                        const uint8_t* shard, const ScanShape& sh, uint8_t* slabs, int tile,
                        hipStream_t s);
// Single-launch queries (k_query): key parse + whole tree + scan in one persistent launch of
// 2^lr workgroups, each owning 2^lt tiles of `tile` leaves, for a queue of nk keys (raw keys
// key_stride bytes apart; query k's slabs at d_slabs + k * query_slab_bytes(qp)).
// tile == 0: shape not supported.
struct QueryPlan {
  int tile, lr, lt;
  int ls;           // 2^ls tiles per super-tile (their narrow top levels expanded once)
  int tw;           // tree waves per workgroup (the rest scan)
  int m4r;          // 3-5 rounds: the 768-thread four-Russians k_query (1: kM4rTW tree waves, 2: two)
  ScanShape shape;  // grid.x = 2^lr workgroups (slabs), grid.y = column groups
};
QueryPlan make_query_plan(int n, int log_parts, int p, int nq, uint32_t pitch, int num_cus,
                          int nk = 1);
inline size_t query_slab_bytes(const QueryPlan& qp) {
  return (size_t)qp.shape.grid.x * qp.shape.grid.y * qp.shape.slab_bytes;
}
constexpr int kQueryTraceSlots = 256;  // trace: per-workgroup phase stamps (wall clock, 100 MHz)
// device scratch for the super-tile tile inputs (0 when ls == 0)
size_t query_scratch_bytes(const QueryPlan& qp);
// out != nullptr: the answers are reduced in-kernel (no launch_reduce): query k's nq x efs bytes
// at out + k * nq * efs, by red_mode (k_query): 1 = the last workgroup reduces every slab (qcnt
// = nk zeroed counters, left zero); 2 = every workgroup adds its partial with memory-side
// atomics; 3 = the last workgroup of each of 8 slab groups adds the group's XOR (qcnt = 8 nk
// counters).  Modes 2-3: answers the host zeroed before the launch, efs % 4 == 0.
// End-of-query work stealing for a lone whole-shard answer (nk == 1, 1-2 rounds, one column
// group): the last tile's shares go to global memory and its rows past the scan waves' static
// prefix are handed out in chunks through a per-workgroup counter, to its own scan waves and then
// to any workgroup whose own work is done.  buf: 2 u32 per workgroup (chunk counter, published
// generation) then TILE * NRP bytes of shares per workgroup; zero-initialised once; gen: a new
// nonzero value per launch (0: off).  Per-slice answers (runs of slabs) must not use it.
// Compiled in only by the diagnostic build (make diag: -DPIR_QUERY_STEAL=1): measured no faster
// on configs[1] -- the last tiles' scan is HBM-bound, not imbalanced (profiles/r05/steal_*.txt)
// -- and its code costs the two-round k_query registers (spills 10 -> 69 VGPRs)
#ifndef PIR_QUERY_STEAL
#define PIR_QUERY_STEAL 0
#endif
struct StealArgs {
  uint32_t* buf = nullptr;
  uint32_t gen = 0;
  uint32_t mode = 3;  // bit 0: the tree waves fold chunks; bit 1: they help neighbours
};
size_t query_steal_bytes(const QueryPlan& qp);
hipError_t launch_query(const QueryPlan& qp, const uint8_t* d_raw, uint32_t key_stride, int nk,
                        int p, int n, int party0, int log_parts, uint64_t prefix,
                        const uint8_t* shard, uint8_t* slabs, uint8_t* scratch, hipStream_t s,
                        uint64_t* trace = nullptr, uint8_t* out = nullptr,
                        uint32_t* qcnt = nullptr, uint32_t efs = 0, uint32_t red_mode = 0,
                        StealArgs steal = StealArgs{});
// k_query for a sqrt(N) DPF key (multiparty / covering design, pir_mp.h's MpLayout): the tree
// waves build each tile's shares from the key's seeds, toggles and correction words (mp_tile)
// while the scan waves stream the shard; then launch_reduce as for launch_query.  nk keys
// key_stride bytes apart (16-aligned), L.nrk == the plan's rounds, the plan's tile divides L.mu.
struct MpLayout;
hipError_t launch_query_mp(const QueryPlan& qp, const uint8_t* d_key, uint32_t key_stride,
                           int nk, const MpLayout& L, int n, int log_parts, uint64_t prefix,
                           const uint8_t* shard, uint8_t* slabs, hipStream_t s);
// XOR the slabs, compact pitch -> record_bytes: d_out[a*efs + b]; nk queries (slabs of query k
// grid.x*grid.y*slab_bytes apart, answers nq*efs bytes apart).  nslices > 1 (dividing grid.x):
// per query, nslices answers over consecutive equal runs of the grid.x slabs, i.e. over equal
// consecutive row ranges when slab x covers rows [x*R, (x+1)*R) (k_query); answer (k, z) at
// d_out + (k*nslices + z)*nq*efs.
hipError_t launch_reduce(const ScanShape& sh, const uint8_t* d_slabs, uint32_t efs,
                         uint8_t* d_out, hipStream_t s, int nk = 1, int nslices = 1);
// d_out[i] = XOR_r d_in[r*len + i]
hipError_t launch_xor_fold(const uint8_t* d_in, int nranks, size_t len, uint8_t* d_out,
                           hipStream_t s);
hipError_t launch_fill_random(uint8_t* d, size_t bytes, uint64_t seed, hipStream_t s);
// the erasure-coded shard of server `party` (client.cpp:70-97): rows [row0, row0+rows) of the
// global encoded database from nfiles files (d_files rows file_pitch apart, or nullptr: the
// reference's synthetic database, client.cpp:16-33)
hipError_t launch_encode_across(const uint8_t* d_files, uint64_t file_pitch, uint64_t nfiles,
                               int k, int party, uint8_t* d_shard, uint64_t rows, uint64_t row0,
                               uint32_t pitch, uint32_t efs, hipStream_t s);
hipError_t launch_fill_shard(uint8_t* d_shard, uint64_t rows, uint32_t pitch, uint32_t efs,
                             uint64_t global_row0, uint64_t seed, hipStream_t s);

}  // namespace pir
