// pir_server.cpp -- the server.h / params.h / client.h-compatible shim (include/pir_server.h)
// over the MI355X engine.  Host glue only: every answer is computed by the HIP kernels behind
// pir_engine_answer / pir_engine_answer_slice.
#include "/root/repo/include/pir_server.h"

#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/random.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <random>
#include <utility>
#include <vector>

#include "/root/repo/include/pir_client.h"
#include "/root/repo/include/pir_engine.h"

extern "C" {
int NUM_PARTIES = 0;
int NUM_FILES = 0;
uint32_t LOG_NUM_FILES = 0;
uint32_t FILE_SIZE_BYTES = 0;
uint32_t PAYLOAD_SIZE_BYTES = 0;
int NUM_ENCODED_FILES = 0;
int LOG_NUM_ENCODED_FILES = 0;
int ENCODED_PAYLOAD_SIZE_BYTES = 0;
int ENCODED_FILE_SIZE_BYTES = 0;
int ENCODE_ACROSS = -1;
int NUM_ROUNDS = 0;
int RHO = 2;
int K = 0;
int T = 0;
int R = 0;
int B = 0;
int NUM_RESPONSES = 0;
int MODE = -1;
int IS_HERMITE = 0;
int D = 0;
int MAC_SIZE_BYTES = 32;
int CHECK_MAC = 0;
int NUM_RSS_KEYS = 0;  // params.cpp:39-46 defaults (Woodruff mode is not served)
int NUM_CD_KEYS = 2;   // params.cpp:368-369: the CD532 counts until a covering design is chosen
int NUM_CD_KEYS_NEEDED = 4;
int WOODRUFF_M = 0;
int WOODRUFF_D = 0;
int WOODRUFF_DERIVATIVE = 0;
}

namespace {

int g_device = -1;

int device_default() {
  if (g_device >= 0) return g_device;
  const char* s = getenv("PIR_DEVICE");
  return s ? atoi(s) : 0;
}

[[noreturn]] void die(const char* what) {
  fprintf(stderr, "pir engine failure in %s: %s\n", what, pir_engine_last_error());
  abort();  // the reference's handleErrors() (utils.cpp:11-15)
}

// The slices of one query, computed together for the T runOptimizedDPFTreeQueryThread calls
// that tree.go:60-76 issues with the same key: the first call to arrive answers every slice in
// one engine pass (pir_engine_answer_slices), the others copy theirs out.  An entry lives
// until each of its T slices has been taken once (or the shard / engine changes).
// The computing call publishes `state` (1 = parts ready, -1 = the engine failed); the other
// calls of the group wait for it WITHOUT the server lock -- polling with yields for a few ms (a
// query's pass), then sleeping on `cv` -- so the T - 1 waiters copy their slices concurrently
// instead of queueing for the server lock one by one.
struct SliceGroup {
  std::vector<uint8_t> key;
  int num_threads = 0;
  std::vector<uint8_t> parts;     // num_threads x NUM_ROUNDS x efs (immutable once published)
  std::vector<uint8_t> taken;     // per slice, under ShimState::mu
  std::atomic<int> left{0};       // slices not yet copied out
  std::atomic<int> joined{1};     // calls that found this group (the creator included)
  std::atomic<int> state{0};
  std::mutex m;
  std::condition_variable cv;
};
constexpr size_t kMaxSliceGroups = 8;  // queries whose slices are in flight at once
// and at most this many bytes of their parts (T x NUM_ROUNDS x EFS each); the oldest group goes
// first (its remaining callers, if any, still hold it and copy their slices out)
constexpr size_t kMaxSliceGroupBytes = 256ull << 20;

// Per-server engine state, hung off server.ctx.
struct ShimState {
  std::mutex mu;
  // held shared by a slice group's engine pass (which runs without mu); engine_for takes it
  // exclusively (under mu) before it replaces the engine or re-uploads the shard
  std::shared_mutex life;
  pir_engine_t* eng = nullptr;
  pir_engine_config cfg{};
  bool dirty = true;  // indexList changed since the last upload
  // the setup encoded the shard on the GPU (encode_*_files_server): the device copy is the only
  // one and indexList is materialised from it only when something reads or writes the host rows
  // (sync_rows_down: an engine remake, pirServerSetRows, pirServerSyncRows, a second encode)
  bool host_stale = false;
  bool rows_zero = true;  // indexList untouched since initializeServer (all zero)
  uint32_t rows_alloc = 0;
  uint32_t row_bytes = 0;          // bytes per indexList row (initializeServer's fileSizeBytes)
  uint8_t* row_block = nullptr;    // the rows' one allocation (indexList[i] = row_block + i * row_bytes)
  std::vector<std::shared_ptr<SliceGroup>> groups;  // oldest first
  size_t group_bytes = 0;          // parts held by `groups`
};

ShimState* state_of(server* s) {
  if (!s || !s->ctx) {
    fprintf(stderr, "pir shim: query on an uninitialised or freed server\n");
    abort();
  }
  return static_cast<ShimState*>(s->ctx);
}

[[noreturn]] void out_of_scope(const char* fn, const char* mode) {
  fprintf(stderr, "pir shim: %s (%s mode) is outside the tree-DPF engine's scope\n", fn, mode);
  abort();
}

// indexList <- the device shard, when the setup left the device copy as the only one (caller
// holds st->mu; no slice pass may be running: under the exclusive life lock, or before any)
void sync_rows_down(server* s, ShimState* st) {
  if (!st->host_stale || !st->eng) return;
  const uint64_t n = std::min<uint64_t>(pir_engine_num_rows(st->eng), st->rows_alloc);
  if (pir_engine_get_shard_rows(st->eng, s->indexList, 0, n) != PIR_OK) die("pirServerSyncRows");
  st->host_stale = false;
}

// Whether any page of the row block is resident: initializeServer's rows are an untouched
// anonymous mapping, so a resident page means something wrote (or read) indexList since.  A
// setup then keeps the reference's host XOR-encode into those rows (client.cpp:88).
bool rows_touched(const ShimState* st) {
  const size_t bytes = (size_t)st->rows_alloc * st->row_bytes;
  if (!st->row_block || !bytes) return false;
  const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
  std::vector<unsigned char> vec((bytes + pg - 1) / pg);
  if (mincore(st->row_block, bytes, vec.data()) != 0) return true;  // cannot tell: assume data
  for (unsigned char v : vec)
    if (v & 1) return true;
  return false;
}

void reaper_wait_idle();  // freeServer's deferred teardown (below): done before a new engine

// Make sure the engine matches the current globals / nq and holds the current indexList
// (upload = false: the caller is about to write the whole device shard itself).
// must = false: return nullptr instead of aborting when no engine can be created (a setup on a
// host without a usable GPU keeps the reference's host encode; every query still fails loudly).
pir_engine_t* engine_for(server* s, ShimState* st, int nq, bool upload = true, bool must = true) {
  pir_engine_config c{};
  c.device = device_default();
  // the party count only sizes DPF keys; polynomial-PIR setups may have p < 2 or > 17
  c.num_parties = NUM_PARTIES < 2 ? 2 : (NUM_PARTIES > PIR_MAX_PARTIES ? PIR_MAX_PARTIES : NUM_PARTIES);
  c.party_index = s->partyIndex;
  c.log_num_records = LOG_NUM_ENCODED_FILES;
  c.record_bytes = (uint32_t)ENCODED_FILE_SIZE_BYTES;
  c.num_rounds = nq;
  c.log_num_partitions = 0;
  c.partition_index = 0;
  c.is_byzantine = s->isByzantine;
  const bool remake = !st->eng || memcmp(&c, &st->cfg, sizeof c) != 0;
  std::unique_lock<std::shared_mutex> excl(st->life, std::defer_lock);
  if (remake || st->dirty) {  // no slice pass may be using the engine or the shard meanwhile
    excl.lock();
    st->groups.clear();
    st->group_bytes = 0;
  }
  if (remake) {
    if (upload) sync_rows_down(s, st);  // the old engine holds the only copy of the shard
    if (st->eng) pir_engine_destroy(st->eng);
    st->eng = nullptr;
    reaper_wait_idle();  // a freed server's device memory is released before this allocation
    if (pir_engine_create(&c, &st->eng) != PIR_OK) {
      if (must) die("pir_engine_create");
      st->eng = nullptr;
      return nullptr;
    }
    st->cfg = c;
    st->dirty = true;
    st->host_stale = false;
  }
  if (!upload) {
    st->dirty = false;
    return st->eng;
  }
  if (st->dirty) {
    const uint64_t n = 1ull << c.log_num_records;
    if (n > st->rows_alloc) {
      fprintf(stderr, "pir shim: %llu encoded rows but the server holds %u\n",
              (unsigned long long)n, st->rows_alloc);
      abort();
    }
    if (pir_engine_set_shard_rows(st->eng, s->indexList, 0, n) != PIR_OK)
      die("pir_engine_set_shard_rows");
    st->dirty = false;
  }
  return st->eng;
}

// Large zeroed host blocks (the client's files, the server's rows): anonymous mappings, so
// untouched pages cost nothing (a GPU setup never touches the server rows) and huge pages cut
// the faults of filling tens of GiB.  The sizes live here, keyed by address, for big_free.
std::mutex g_big_mu;
std::vector<std::pair<void*, size_t>> g_big;
uint8_t* big_alloc(size_t bytes) {
  bytes = std::max<size_t>(bytes, 1);
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return nullptr;
  (void)madvise(p, bytes, MADV_HUGEPAGE);
  std::lock_guard<std::mutex> lk(g_big_mu);
  g_big.emplace_back(p, bytes);
  return static_cast<uint8_t*>(p);
}
void big_free(void* p) {
  if (!p) return;
  size_t bytes = 0;
  {
    std::lock_guard<std::mutex> lk(g_big_mu);
    for (auto it = g_big.begin(); it != g_big.end(); ++it)
      if (it->first == p) {
        bytes = it->second;
        g_big.erase(it);
        break;
      }
  }
  if (bytes) (void)munmap(p, bytes);
}

// host threads for the shim's own bulk work (client files); the GPU box grants 16 CPUs per GPU
int shim_threads() {
  if (const char* v = getenv("PIR_GATHER_THREADS")) return std::max(1, atoi(v));
  int n = (int)std::thread::hardware_concurrency();
  if (const char* v = getenv("OMP_NUM_THREADS")) n = std::min(n, std::max(1, atoi(v)));
  return std::max(1, std::min(8, n));
}

// the host encode wrote indexList: the engine re-uploads it before the next query
void shard_written_on_host(server* s) {
  if (!s->ctx) return;
  ShimState* st = static_cast<ShimState*>(s->ctx);
  std::lock_guard<std::mutex> lk(st->mu);
  st->rows_zero = false;
  st->dirty = true;
}

// The worker threads of pirRunTreeQueryThreads: created once, T of them per fan-out.  A worker
// polls (with yields) for ~0.2 ms after each job and then sleeps on the condition variable, so
// back-to-back queries see goroutine-like wake-ups and an idle process burns no cores.
class FanoutPool {
 public:
  ~FanoutPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // job(t) for t < n on n pool threads, concurrently; returns when all are done
  void run(int n, const std::function<void(int)>& job) {
    std::lock_guard<std::mutex> one(run_mu_);  // one fan-out at a time
    {
      std::lock_guard<std::mutex> lk(mu_);
      while ((int)th_.size() < n) {
        const int i = (int)th_.size();
        th_.emplace_back([this, i] { worker(i); });
      }
      job_ = &job;
      n_ = n;
      remaining_.store(n, std::memory_order_relaxed);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    const auto t0 = std::chrono::steady_clock::now();
    while (remaining_.load(std::memory_order_acquire) != 0) {
      if (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200)) {
        std::this_thread::yield();
      } else {
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return remaining_.load(std::memory_order_acquire) == 0; });
      }
    }
  }

 private:
  void worker(int i) {
    uint64_t seen = 0;
    for (;;) {
      const auto t0 = std::chrono::steady_clock::now();
      while (gen_.load(std::memory_order_acquire) == seen &&
             std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200))
        std::this_thread::yield();
      const std::function<void(int)>* job;
      int n;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
        seen = gen_.load(std::memory_order_acquire);
        if (quit_) return;
        job = job_;
        n = n_;
      }
      if (i < n) {
        (*job)(i);
        if (remaining_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
          std::lock_guard<std::mutex> lk(mu_);
          done_cv_.notify_all();
        }
      }
    }
  }
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> th_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> remaining_{0};
  const std::function<void(int)>* job_ = nullptr;
  int n_ = 0;
  bool quit_ = false;
};

FanoutPool& fanout_pool() {
  static FanoutPool pool;
  return pool;
}

// freeServer's slow half off the caller's path.  The reference's RunTreeQuery calls FreeServer
// BEFORE it stamps SendTime and returns the response (src/server_util/tree.go:90-100), so every
// answer left behind the engine teardown (hipFree of the shard: 0.6-0.8 s at 16-64 GiB) and the
// row block's munmap.  freeServer now detaches them and one reaper thread releases them, a few
// ms later ($PIR_REAPER_DEFER_MS, default 20: unmapping tens of GiB holds the process's memory
// map lock, which the caller's own page faults -- the response being sent -- would wait on); a
// new engine (engine_for) waits until the reaper is idle (and has it start at once), so device
// memory is back before it is allocated again.  The destructor drains the queue at exit.
class Reaper {
 public:
  ~Reaper() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }
  void post(std::function<void()> job) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      jobs_.push_back({std::move(job), std::chrono::system_clock::now() + defer()});
      ++pending_;
      if (!th_.joinable()) th_ = std::thread([this] { loop(); });
    }
    cv_.notify_all();
  }
  // returns once every job posted before the call has run (they run now, not deferred)
  void wait_idle() {
    std::unique_lock<std::mutex> lk(mu_);
    ++waiters_;
    cv_.notify_all();
    idle_.wait(lk, [this] { return pending_ == 0; });
    --waiters_;
  }

 private:
  // (system_clock: libstdc++ waits on it with pthread_cond_timedwait, which ThreadSanitizer
  // intercepts; a steady_clock wait_until becomes pthread_cond_clockwait, which gcc 11's does not)
  struct Job {
    std::function<void()> fn;
    std::chrono::system_clock::time_point due;
  };
  static std::chrono::milliseconds defer() {
    static const long ms = [] {
      const char* v = getenv("PIR_REAPER_DEFER_MS");
      return v ? std::max(0L, atol(v)) : 20L;
    }();
    return std::chrono::milliseconds(ms);
  }
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [this] { return quit_ || !jobs_.empty(); });
      if (jobs_.empty()) return;  // quit_ with nothing left
      const auto due = jobs_.front().due;
      cv_.wait_until(lk, due, [this] { return quit_ || waiters_ > 0; });
      Job job = std::move(jobs_.front());
      jobs_.erase(jobs_.begin());
      lk.unlock();
      job.fn();
      lk.lock();
      if (--pending_ == 0) idle_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, idle_;
  std::vector<Job> jobs_;
  int pending_ = 0, waiters_ = 0;
  bool quit_ = false;
  std::thread th_;
};

Reaper& reaper() {
  static Reaper r;
  return r;
}

void reaper_wait_idle() { reaper().wait_idle(); }

int ceil_log2(long v) {
  int l = 0;
  while ((1L << l) < v) ++l;
  return l;
}

uint8_t gf_mul_h(uint8_t a, uint8_t b) {  // 0x11d field (coding.cpp:9-21), carry-less form
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1d : 0));
    b >>= 1;
  }
  return r;
}

uint8_t gf_pow_h(uint8_t base, int exp) {  // coding.cpp:46-60 (pow(0, e) == 1 there, too)
  if (base == 0) return 1;
  uint8_t r = 1;
  for (int i = 0; i < exp; ++i) r = gf_mul_h(r, base);
  return r;
}

uint8_t gf_inv_h(uint8_t a) {  // a^254 (coding.cpp:24-33: inv(0) == 0)
  if (!a) return 0;
  uint8_t r = 1, b = a;
  for (int e = 254; e; e >>= 1) {
    if (e & 1) r = gf_mul_h(r, b);
    b = gf_mul_h(b, b);
  }
  return r;
}

// Gauss-Jordan over GF(2^8) (coding.cpp:73-126): out = in^-1; false if singular; `in` destroyed
bool gf_invert_matrix_h(std::vector<uint8_t>& in, std::vector<uint8_t>& out, int n) {
  out.assign((size_t)n * n, 0);
  for (int i = 0; i < n; ++i) out[(size_t)i * n + i] = 1;
  for (int i = 0; i < n; ++i) {
    if (!in[(size_t)i * n + i]) {  // swap in a row with a non-zero pivot
      int j = i + 1;
      while (j < n && !in[(size_t)j * n + i]) ++j;
      if (j == n) return false;
      for (int k = 0; k < n; ++k) {
        std::swap(in[(size_t)i * n + k], in[(size_t)j * n + k]);
        std::swap(out[(size_t)i * n + k], out[(size_t)j * n + k]);
      }
    }
    const uint8_t piv = gf_inv_h(in[(size_t)i * n + i]);
    for (int k = 0; k < n; ++k) {
      in[(size_t)i * n + k] = gf_mul_h(in[(size_t)i * n + k], piv);
      out[(size_t)i * n + k] = gf_mul_h(out[(size_t)i * n + k], piv);
    }
    for (int j = 0; j < n; ++j) {
      if (j == i) continue;
      const uint8_t x = in[(size_t)j * n + i];
      if (!x) continue;
      for (int k = 0; k < n; ++k) {
        out[(size_t)j * n + k] ^= gf_mul_h(x, out[(size_t)i * n + k]);
        in[(size_t)j * n + k] ^= gf_mul_h(x, in[(size_t)i * n + k]);
      }
    }
  }
  return true;
}

// Inverse of the Vandermonde system of interpolation.cpp:176-196 on the first m = deg+1 points:
// gen[i][c] = pts[i]^c (calcFuncCoeffs, interpolation.cpp:50-54)
std::vector<uint8_t> vandermonde_inverse(const uint8_t* pts, int m) {
  std::vector<uint8_t> gen((size_t)m * m), inv;
  for (int i = 0; i < m; ++i)
    for (int c = 0; c < m; ++c) gen[(size_t)i * m + c] = gf_pow_h(pts[i], c);
  if (!gf_invert_matrix_h(gen, inv, m)) {
    fprintf(stderr, "pir shim: singular interpolation system (repeated evaluation points)\n");
    abort();
  }
  return inv;
}

// The OS CSPRNG (the reference draws key seeds and polynomial coefficients with RAND_bytes).
void os_random(uint8_t* buf, size_t len) {
  while (len) {
    const ssize_t got = getrandom(buf, len, 0);
    if (got < 0) {
      if (errno == EINTR) continue;
      perror("pir shim: getrandom");
      abort();
    }
    buf += got;
    len -= (size_t)got;
  }
}

// SHA-256 (FIPS 180-4) and HMAC (RFC 2104), for mac() -- the reference calls OpenSSL's HMAC.
struct Sha256 {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t blk[64];
  size_t fill = 0;
  uint64_t total = 0;
  static uint32_t ror(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }
  void compress(const uint8_t* p) {
    static const uint32_t k[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
        0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
        0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
        0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
        0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
        0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
        0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
        0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
        0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
      w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 |
             (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
      const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
      const uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) +
                          k[i] + w[i];
      const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void update(const uint8_t* p, size_t n) {
    total += n;
    while (n) {
      const size_t take = (64 - fill) < n ? (64 - fill) : n;
      memcpy(blk + fill, p, take);
      fill += take; p += take; n -= take;
      if (fill == 64) { compress(blk); fill = 0; }
    }
  }
  void final(uint8_t out[32]) {
    const uint64_t bits = total * 8;
    const uint8_t one = 0x80, zero = 0;
    update(&one, 1);
    while (fill != 56) update(&zero, 1);
    uint8_t len[8];
    for (int i = 0; i < 8; ++i) len[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(len, 8);
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(h[i] >> (24 - 8 * j));
  }
};

void hmac_sha256(const uint8_t* key, size_t klen, const uint8_t* msg, size_t mlen,
                 uint8_t out[32]) {
  uint8_t k0[64] = {0};
  if (klen > 64) {
    Sha256 s;
    s.update(key, klen);
    s.final(k0);
  } else {
    memcpy(k0, key, klen);
  }
  uint8_t ipad[64], opad[64], inner[32];
  for (int i = 0; i < 64; ++i) { ipad[i] = k0[i] ^ 0x36; opad[i] = k0[i] ^ 0x5c; }
  Sha256 si;
  si.update(ipad, 64);
  si.update(msg, mlen);
  si.final(inner);
  Sha256 so;
  so.update(opad, 64);
  so.update(inner, 32);
  so.final(out);
}

}  // namespace

extern "C" {

// interpolation.cpp:176-196: coefficients of the degree-funcDegree polynomial through the first
// funcDegree+1 (evalPoints[i], evals[i]); output[c] = coefficient of x^c
void lagrangeInterpolationSemihonest(uint8_t* evalPoints, uint8_t numPoints, uint8_t* evals,
                                     uint8_t funcDegree, uint8_t* output) {
  const int m = funcDegree + 1;
  if (numPoints < m) {  // the reference asserts (interpolation.cpp:179)
    fprintf(stderr, "pir shim: %d points for a degree-%d interpolation\n", numPoints, funcDegree);
    abort();
  }
  const std::vector<uint8_t> inv = vandermonde_inverse(evalPoints, m);
  for (int i = 0; i < m; ++i) {  // computeMatrixTimesResponse (interpolation.cpp:40-48)
    uint8_t v = 0;
    for (int j = 0; j < m; ++j) v ^= gf_mul_h(evals[j], inv[(size_t)i * m + j]);
    output[i] = v;
  }
}

// client.cpp:211-268 (semi-honest, B == 0): responses[j][round][byte] from the NUM_PARTIES - R
// servers not erased (erasureIndexList[q-1] == 1 for server q, in increasing q), output =
// FILE_SIZE_BYTES of the record.  Round i peels the coefficients recovered in rounds < i off
// the shares, then interpolates each byte position; the evaluation points are the same for
// every byte, so the Vandermonde system is inverted once per round, not once per byte.
void assembleDPFTreeQueryResponses(client* c, uint8_t* erasureIndexList, uint8_t*** responses,
                                   uint8_t* output) {
  (void)c;
  if (B > 0) {
    fprintf(stderr, "pir shim: malicious (B > 0) decoding is outside the engine's scope\n");
    abort();
  }
  const int nr = NUM_PARTIES - R, efs = ENCODED_FILE_SIZE_BYTES, m = K + RHO;
  if (nr < m) {
    fprintf(stderr, "pir shim: %d responses cannot decode degree %d\n", nr, m - 1);
    abort();
  }
  std::vector<uint8_t> acc((size_t)K * efs, 0), pts(nr), sh((size_t)nr);
  for (int i = 0; i < NUM_ROUNDS; ++i) {
    int cur = 1;
    for (int j = 0; j < nr; ++j) {
      while (!erasureIndexList[cur - 1]) ++cur;
      pts[j] = (uint8_t)cur++;
    }
    const std::vector<uint8_t> inv = vandermonde_inverse(pts.data(), m);
    std::vector<uint8_t> peel((size_t)nr * i);  // gf_pow(point_j, K + i - b), b < i
    for (int j = 0; j < nr; ++j)
      for (int b = 0; b < i; ++b) peel[(size_t)j * i + b] = gf_pow_h(pts[j], K + i - b);
    for (int a = 0; a < efs; ++a) {
      for (int j = 0; j < nr; ++j) {
        uint8_t v = responses[j][i][a];
        for (int b = 0; b < i; ++b)
          v ^= gf_mul_h(acc[(size_t)(K - 1 - b) * efs + a], peel[(size_t)j * i + b]);
        sh[j] = v;
      }
      for (int q = 0; q < RHO; ++q) {  // coefficient K+RHO-1-q of the interpolant
        const int row = m - 1 - q;
        uint8_t v = 0;
        for (int j = 0; j < m; ++j) v ^= gf_mul_h(sh[j], inv[(size_t)row * m + j]);
        const int dst = K - 1 - i - q;
        if (dst >= 0) acc[(size_t)dst * efs + a] = v;
      }
    }
  }
  memcpy(output, acc.data(), FILE_SIZE_BYTES);
}

// client.cpp:499-552 (semi-honest, B == 0): the polynomial-PIR decode.  Round i peels the parts
// recovered in earlier rounds off the shares (gf_pow(point, K + T - 1 + i - b)), then reads
// coefficients K+T+RHO-2-q (q < RHO) of the degree-(K+T+RHO-2) interpolant at every byte
// position into part K-1-i-q; one Vandermonde inverse per round.  output = FILE_SIZE_BYTES.
void assembleHollantiResponses(client* c, uint8_t* erasureIndexList, uint8_t*** responses,
                               uint8_t* output) {
  (void)c;
  if (B > 0) {
    fprintf(stderr, "pir shim: malicious (B > 0) decoding is outside the engine's scope\n");
    abort();
  }
  const int nr = NUM_PARTIES - R, efs = ENCODED_FILE_SIZE_BYTES, deg = K + T + RHO - 2;
  const int m = deg + 1;
  if (nr < m) {
    fprintf(stderr, "pir shim: %d responses cannot decode degree %d\n", nr, deg);
    abort();
  }
  std::vector<uint8_t> acc((size_t)K * efs, 0), pts(nr), sh((size_t)nr);
  for (int i = 0; i < NUM_ROUNDS; ++i) {
    int cur = 1;
    for (int j = 0; j < nr; ++j) {
      while (!erasureIndexList[cur - 1]) ++cur;
      pts[j] = (uint8_t)cur++;
    }
    const std::vector<uint8_t> inv = vandermonde_inverse(pts.data(), m);
    std::vector<uint8_t> peel((size_t)nr * i);
    for (int j = 0; j < nr; ++j)
      for (int b = 0; b < i; ++b) peel[(size_t)j * i + b] = gf_pow_h(pts[j], K + T - 1 + i - b);
    for (int a = 0; a < efs; ++a) {
      for (int j = 0; j < nr; ++j) {
        uint8_t v = responses[j][i][a];
        for (int b = 0; b < i; ++b)
          v ^= gf_mul_h(acc[(size_t)(K - 1 - b) * efs + a], peel[(size_t)j * i + b]);
        sh[j] = v;
      }
      for (int q = 0; q < RHO; ++q) {
        const int row = deg - q, dst = K - 1 - i - q;
        uint8_t v = 0;
        for (int j = 0; j < m; ++j) v ^= gf_mul_h(sh[j], inv[(size_t)row * m + j]);
        if (dst >= 0) acc[(size_t)dst * efs + a] = v;
      }
    }
  }
  memcpy(output, acc.data(), FILE_SIZE_BYTES);
}

void pirSetDevice(int device) { g_device = device; }

void pirServerShardChanged(server* s) {
  if (!s || !s->ctx) return;
  ShimState* st = static_cast<ShimState*>(s->ctx);
  std::lock_guard<std::mutex> lk(st->mu);
  if (st->host_stale)  // the caller wrote rows it never read back (see pir_server.h)
    fprintf(stderr, "pir shim: indexList written after a GPU setup without pirServerSyncRows; "
                    "its other rows are zero on the host and now replace the device shard\n");
  st->host_stale = false;
  st->rows_zero = false;
  st->dirty = true;
}

void pirServerSyncRows(server* s) {
  ShimState* st = state_of(s);
  std::lock_guard<std::mutex> lk(st->mu);
  std::unique_lock<std::shared_mutex> excl(st->life);  // no slice pass reads the shard meanwhile
  sync_rows_down(s, st);
}

void pirServerSetRows(server* s, const uint8_t* rows, uint64_t row0, uint64_t nrows,
                      uint32_t rowBytes) {
  ShimState* st = state_of(s);
  std::lock_guard<std::mutex> lk(st->mu);
  if (row0 > st->rows_alloc || nrows > st->rows_alloc - row0 || (!rows && nrows) ||
      rowBytes > st->row_bytes) {
    fprintf(stderr, "pir shim: rows [%llu,%llu) outside the server's %u\n",
            (unsigned long long)row0, (unsigned long long)(row0 + nrows), st->rows_alloc);
    abort();
  }
  {
    std::unique_lock<std::shared_mutex> excl(st->life);
    sync_rows_down(s, st);  // the rows not written here keep the GPU setup's values
  }
  for (uint64_t i = 0; i < nrows; ++i)
    memcpy(s->indexList[row0 + i], rows + i * rowBytes, rowBytes);
  st->rows_zero = false;
  st->dirty = true;
}

int calcOptimizedDPFTreeKeyLength(int p, int log_domainSize, int numQueries) {
  return pir_engine_key_len(p, log_domainSize, numQueries);
}

// params.cpp:12 `int M = 4` (the covering designs' extra-party count) and params.cpp:372 isRss:
// setModeParams(CD) sets M to 2 for K = 2, B = 1 (params.cpp:439-441) and a covering-design
// selection clears isRss (:520-599); the reference never resets either, so a later setup's party
// count and NUM_RSS_KEYS depend on the process's call history.  This shim starts every
// setSystemParams from M = 4, isRss = 1 and the CD532 key counts (NUM_CD_KEYS = 2,
// NUM_CD_KEYS_NEEDED = 4, params.cpp:368-369), as a fresh process would (the Go servers set
// their parameters once).
static int g_cd_m = 4;

// The covering designs of params.cpp:519-599: (T, NUM_PARTIES, M) -> NUM_CD_KEYS,
// NUM_CD_KEYS_NEEDED (the counts of params.cpp:64-362); every mode runs this selection.
static bool select_covering(int t, int p, int m) {
  static const int tab[][5] = {  // p, M, NUM_CD_KEYS, NUM_CD_KEYS_NEEDED  (all with T == 2)
      {5, 1, 2, 4}, {7, 1, 4, 7}, {6, 1, 3, 6}, {8, 1, 7, 11}, {9, 1, 8, 12}, {8, 2, 3, 6},
      {9, 2, 5, 8}, {10, 2, 6, 9}, {12, 4, 3, 6}, {16, 4, 3, 6}, {14, 4, 3, 6}};
  if (t != 2) return false;
  for (const auto& c : tab)
    if (c[0] == p && c[1] == m) {
      NUM_CD_KEYS = c[2];
      NUM_CD_KEYS_NEEDED = c[3];
      return true;
    }
  return false;
}

// params.cpp:467-512 with setModeParams(Tree) (params.cpp:414-418), setModeParams(Multiparty)
// (:419-422), setModeParams(Hollanti) (:430-433) or setModeParams(CD) (:434-447), the covering
// design of :519-599 and the RSS share count of :603-619; the other modes (Shamir, Woodruff,
// Goldberg) abort
void setSystemParams(int logNumFiles, int fileSizeBytes, int t, int k, int r, int b, int rho,
                     int checkMac, int mode) {
  if (mode != 0 && mode != 1 && mode != 3 && mode != 4) {
    fprintf(stderr, "pir shim: mode %d is outside the engine's scope (tree = 0, multiparty = 1, "
            "Hollanti = 3, covering design = 4)\n", mode);
    abort();
  }
  if (mode == 0 && t != 1) {  // params.cpp:415 assert(T == 1)
    fprintf(stderr, "pir shim: tree mode requires t == 1 (got %d)\n", t);
    abort();
  }
  if (mode == 3 && checkMac) {
    fprintf(stderr, "pir shim: CheckMAC setups are outside the engine's scope\n");
    abort();
  }
  RHO = rho; K = k; T = t; R = r; B = b;
  NUM_FILES = 1 << logNumFiles;
  LOG_NUM_FILES = (uint32_t)logNumFiles;
  PAYLOAD_SIZE_BYTES = (uint32_t)fileSizeBytes;
  FILE_SIZE_BYTES = (uint32_t)fileSizeBytes;
  CHECK_MAC = checkMac;
  MODE = mode;
  g_cd_m = 4;
  NUM_CD_KEYS = 2;  // params.cpp:368-369 (CD532) until select_covering picks a design
  NUM_CD_KEYS_NEEDED = 4;
  if (mode == 4) {
    if (K == 4 && B == 2) {
      NUM_PARTIES = 16;
    } else if (K == 3 && B == 2) {
      NUM_PARTIES = 14;
    } else if (K == 2 && B == 1) {
      g_cd_m = 2;
      NUM_PARTIES = 8;
    } else {
      NUM_PARTIES = T + K + R + 2 * B + g_cd_m;
    }
  } else {
    NUM_PARTIES = K + R + T + 2 * B + (mode == 1 ? 0 : RHO - 1);
  }
  ENCODE_ACROSS = mode == 3 ? 0 : 1;
  NUM_RESPONSES = NUM_PARTIES - R;
  if (ENCODE_ACROSS) {
    LOG_NUM_ENCODED_FILES = ceil_log2((NUM_FILES + k - 1) / k);
    NUM_ENCODED_FILES = 1 << LOG_NUM_ENCODED_FILES;
    ENCODED_PAYLOAD_SIZE_BYTES = (int)FILE_SIZE_BYTES;
    ENCODED_FILE_SIZE_BYTES = (int)FILE_SIZE_BYTES;
    if (CHECK_MAC) {
      FILE_SIZE_BYTES += MAC_SIZE_BYTES;
      ENCODED_FILE_SIZE_BYTES += MAC_SIZE_BYTES;
    }
  } else {  // params.cpp:496-507: every file is split into K parts of ceil(f / K) bytes
    NUM_ENCODED_FILES = NUM_FILES;
    LOG_NUM_ENCODED_FILES = logNumFiles;
    ENCODED_PAYLOAD_SIZE_BYTES = (int)((PAYLOAD_SIZE_BYTES + k - 1) / k);
    ENCODED_FILE_SIZE_BYTES = (int)((FILE_SIZE_BYTES + k - 1) / k);
  }
  NUM_ROUNDS = (K == 1) ? 1 : K / RHO;
  const bool is_rss = !select_covering(T, NUM_PARTIES, g_cd_m);
  if (t >= 1 && is_rss) NUM_RSS_KEYS = pir_engine_mp_num_keys(NUM_PARTIES, T);
}

// utils.cpp:105-116
int calcMultiPartyOptDPFKeyLength(int p, int log_domainSize, int t) {
  return pir_engine_mp_key_len(p, log_domainSize, t);
}

// utils.cpp:131-143
int calcShamirDPFKeyLength(int log_domainSize) {
  const int x = log_domainSize / 2 + (log_domainSize % 2 != 0), y = log_domainSize - x;
  return (1 << x) + (1 << y);
}

int calcShamirResponseLength(int log_domainSize, int fileSizeBytes) {
  return (calcShamirDPFKeyLength(log_domainSize) + 2) * fileSizeBytes;
}

void freeParams(void) {}

// server.cpp:17-42: rows are host memory the Go setup path encodes into; the engine (and the
// device copy of the shard) is created on the first query.
void initializeServer(server* s, int partyIndex, uint32_t logNumFiles, uint32_t fileSizeBytes,
                      int isByzantine, int numThreads) {
  auto* st = new ShimState;
  st->row_bytes = fileSizeBytes;
  s->ctx = st;
  s->ctxThreads = nullptr;
  s->partyIndex = partyIndex;
  const uint32_t n = 1u << logNumFiles;
  // one zeroed allocation for all N rows (the reference mallocs each, server.cpp:34-38): the
  // pages are only touched when rows are written, not by a GPU setup
  s->indexList = (uint8_t**)malloc((size_t)n * sizeof(uint8_t*));
  st->row_block = big_alloc((size_t)n * fileSizeBytes);
  if (!s->indexList || !st->row_block) {
    fprintf(stderr, "pir shim: cannot allocate %u rows of %u bytes\n", n, fileSizeBytes);
    abort();
  }
  for (uint32_t i = 0; i < n; ++i) s->indexList[i] = st->row_block + (size_t)i * fileSizeBytes;
  st->rows_alloc = n;
  s->isByzantine = isByzantine;
  s->numThreads = numThreads;
}

// server.cpp:45-52
// No Thread call may start once freeServer has begun (the reference frees the rows under any
// caller alike); one still inside its slice-group pass is waited for (the life lock).  The
// engine teardown and the row block's unmap run on the reaper thread (see Reaper): the call
// returns once nothing can reach them any more, and the next engine created waits for them.
void freeServer(server* s) {
  if (!s || !s->ctx) return;
  ShimState* st = static_cast<ShimState*>(s->ctx);
  pir_engine_t* eng = nullptr;
  {
    std::lock_guard<std::mutex> lk(st->mu);
    std::unique_lock<std::shared_mutex> excl(st->life);
    st->groups.clear();
    st->group_bytes = 0;
    eng = st->eng;
    st->eng = nullptr;
  }
  uint8_t* rows = st->row_block;
  uint8_t** list = s->indexList;
  s->indexList = nullptr;
  s->ctx = nullptr;
  delete st;
  if (getenv("PIR_SHIM_SYNC_FREE")) {  // the synchronous teardown (A/B timing)
    if (eng) pir_engine_destroy(eng);
    big_free(rows);
    free(list);
    return;
  }
  reaper().post([eng, rows, list] {
    if (eng) pir_engine_destroy(eng);
    big_free(rows);
    free(list);
  });
}

// Blocks until every freeServer teardown handed to the reaper has finished (tests, and callers
// that measure device memory).
void pirServerWaitFreed(void) { reaper_wait_idle(); }

// server.cpp:96-134
void runOptimizedDPFTreeQuery(server* s, uint8_t* key, int numQueries, uint8_t** result) {
  ShimState* st = state_of(s);
  std::lock_guard<std::mutex> lk(st->mu);
  pir_engine_t* e = engine_for(s, st, numQueries);
  const size_t efs = (size_t)ENCODED_FILE_SIZE_BYTES;
  std::vector<uint8_t> out((size_t)numQueries * efs);
  if (pir_engine_answer(e, key, out.data()) != PIR_OK) die("runOptimizedDPFTreeQuery");
  for (int a = 0; a < numQueries; ++a) memcpy(result[a], out.data() + a * efs, efs);
}

// How long the first Thread call of a query waits for a second call with the same key before it
// answers its own slice alone ($PIR_SLICE_JOIN_US, default 200 us).  The T goroutines of
// tree.go:60-76 start within microseconds of each other, so a fan-out still meets in one group
// and pays one pass; a lone caller pays this wait plus a 1/T pass.
int64_t slice_join_us() {
  static const int64_t v = [] {
    const char* s = getenv("PIR_SLICE_JOIN_US");
    return s ? std::max<int64_t>(0, atoll(s)) : (int64_t)200;
  }();
  return v;
}

// server.cpp:505-549, intended semantics (see pir_server.h).  The T calls of one query
// (tree.go:60-76: T goroutines, the same key) share ONE engine pass: the first to take the
// server lock opens a slice group and waits up to slice_join_us() for a partner; with one, it
// answers every slice (pir_engine_answer_slices) and the rest copy theirs from it; without, it
// closes the group and answers only its own slice (pir_engine_answer_slice: a 1/T pass).
void runOptimizedDPFTreeQueryThread(server* s, uint8_t* key, int threadNum, int numThreads,
                                    uint8_t** result) {
  ShimState* st = state_of(s);
  std::shared_ptr<SliceGroup> g;
  pir_engine_t* e = nullptr;
  std::shared_lock<std::shared_mutex> pass;  // the computing call's hold on the engine
  bool creator = false;
  const size_t efs = (size_t)ENCODED_FILE_SIZE_BYTES, ans = (size_t)NUM_ROUNDS * efs;
  {
    std::lock_guard<std::mutex> lk(st->mu);
    e = engine_for(s, st, NUM_ROUNDS);
    if (!key || numThreads < 1 || threadNum < 0 || threadNum >= numThreads ||
        (numThreads & (numThreads - 1)) || numThreads > NUM_ENCODED_FILES) {
      fprintf(stderr, "pir shim: thread %d of %d (a power of two <= %d rows)\n", threadNum,
              numThreads, NUM_ENCODED_FILES);
      abort();
    }
    const size_t klen = (size_t)calcOptimizedDPFTreeKeyLength(
        NUM_PARTIES < 2 ? 2 : NUM_PARTIES, LOG_NUM_ENCODED_FILES, NUM_ROUNDS);
    // groups whose every slice was copied out are done
    st->groups.erase(std::remove_if(st->groups.begin(), st->groups.end(),
                                    [st](const std::shared_ptr<SliceGroup>& x) {
                                      const bool done = x->left.load(std::memory_order_acquire) == 0;
                                      if (done) st->group_bytes -= x->parts.size();
                                      return done;
                                    }),
                     st->groups.end());
    for (auto& x : st->groups)
      if (x->num_threads == numThreads && !x->taken[threadNum] &&
          memcmp(x->key.data(), key, klen) == 0) {
        g = x;
        g->joined.fetch_add(1, std::memory_order_acq_rel);
        break;
      }
    if (!g) {  // the first call of this query
      const size_t need = (size_t)numThreads * ans;
      while (!st->groups.empty() && (st->groups.size() >= kMaxSliceGroups ||
                                     st->group_bytes + need > kMaxSliceGroupBytes)) {
        st->group_bytes -= st->groups.front()->parts.size();
        st->groups.erase(st->groups.begin());
      }
      st->group_bytes += need;
      g = std::make_shared<SliceGroup>();
      g->key.assign(key, key + klen);
      g->num_threads = numThreads;
      g->parts.resize((size_t)numThreads * ans);
      g->taken.assign((size_t)numThreads, 0);
      g->left.store(numThreads, std::memory_order_relaxed);
      st->groups.push_back(g);
      creator = true;
    }
    g->taken[threadNum] = 1;
  }
  if (creator) {  // wait (without the lock) for a partner, then decide under it
    const int64_t wait_us = numThreads > 1 ? slice_join_us() : 0;
    const auto t0 = std::chrono::steady_clock::now();
    while (g->joined.load(std::memory_order_acquire) < 2 &&
           std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(wait_us))
      std::this_thread::yield();
    bool solo;
    {
      std::lock_guard<std::mutex> lk(st->mu);
      e = engine_for(s, st, NUM_ROUNDS);  // the engine may have been replaced meanwhile
      solo = g->joined.load(std::memory_order_acquire) < 2;  // partners join under mu
      if (solo) {  // close the group: later calls with this key open their own
        auto it = std::find(st->groups.begin(), st->groups.end(), g);
        if (it != st->groups.end()) {
          st->group_bytes -= g->parts.size();
          st->groups.erase(it);
        }
      }
      pass = std::shared_lock<std::shared_mutex>(st->life);  // no exclusive holder: we hold mu
    }
    if (solo) {  // nobody else asked for this query: a 1/T pass for this slice alone
      std::vector<uint8_t> out(ans);
      const int rc = pir_engine_answer_slice(e, key, threadNum, numThreads, out.data());
      pass.unlock();
      if (rc != PIR_OK) die("runOptimizedDPFTreeQueryThread");
      for (int a = 0; a < NUM_ROUNDS; ++a) memcpy(result[a], out.data() + a * efs, efs);
      return;
    }
    // the one engine pass of the query, outside the server lock
    const int rc = pir_engine_answer_slices(e, key, numThreads, g->parts.data());
    pass.unlock();
    {
      std::lock_guard<std::mutex> gl(g->m);
      g->state.store(rc == PIR_OK ? 1 : -1, std::memory_order_release);
    }
    g->cv.notify_all();
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    while (g->state.load(std::memory_order_acquire) == 0 &&
           std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(5))
      std::this_thread::yield();
    if (g->state.load(std::memory_order_acquire) == 0) {
      std::unique_lock<std::mutex> gl(g->m);
      g->cv.wait(gl, [&] { return g->state.load(std::memory_order_acquire) != 0; });
    }
  }
  if (g->state.load(std::memory_order_acquire) < 0) die("runOptimizedDPFTreeQueryThread");
  const uint8_t* part = g->parts.data() + (size_t)threadNum * ans;
  for (int a = 0; a < NUM_ROUNDS; ++a) memcpy(result[a], part + a * efs, efs);
  g->left.fetch_sub(1, std::memory_order_acq_rel);
}

// RunTreeQuery's fan-out (src/server_util/tree.go:60-80) for callers without Go: numThreads
// pool threads call runOptimizedDPFTreeQueryThread(s, key, t, numThreads, .) concurrently (the
// goroutines), then assemblDPFTreeQueryThreadResults XORs their partials into result.
void pirRunTreeQueryThreads(server* s, uint8_t* key, int numThreads, uint8_t** result) {
  if (numThreads < 1) {
    fprintf(stderr, "pir shim: %d threads\n", numThreads);
    abort();
  }
  const size_t efs = (size_t)ENCODED_FILE_SIZE_BYTES;
  std::vector<uint8_t> buf((size_t)numThreads * NUM_ROUNDS * efs);
  std::vector<uint8_t*> rows((size_t)numThreads * NUM_ROUNDS);
  std::vector<uint8_t**> in((size_t)numThreads);
  for (int t = 0; t < numThreads; ++t) {
    for (int a = 0; a < NUM_ROUNDS; ++a)
      rows[(size_t)t * NUM_ROUNDS + a] = buf.data() + ((size_t)t * NUM_ROUNDS + a) * efs;
    in[t] = rows.data() + (size_t)t * NUM_ROUNDS;
  }
  const std::function<void(int)> job = [&](int t) {
    runOptimizedDPFTreeQueryThread(s, key, t, numThreads, in[t]);
  };
  fanout_pool().run(numThreads, job);
  assemblDPFTreeQueryThreadResults(s, in.data(), numThreads, result);
}

// server.cpp:553-562 (host buffers from the Go caller)
void assemblDPFTreeQueryThreadResults(server* s, uint8_t*** in, int numThreads, uint8_t** out) {
  (void)s;
  for (int a = 0; a < NUM_ROUNDS; ++a) {
    memset(out[a], 0, ENCODED_FILE_SIZE_BYTES);
    for (int t = 0; t < numThreads; ++t)
      for (int j = 0; j < ENCODED_FILE_SIZE_BYTES; ++j) out[a][j] ^= in[t][a][j];
  }
}

// ---- polynomial (Hollanti) PIR: explicit coefficients, scanned on the engine ----------------
// server.cpp:321-343: random answers for a Byzantine server, else the scan of every row
void runHollantiQuery(server* s, uint8_t** key, uint8_t** result) {
  ShimState* st = state_of(s);
  const size_t efs = (size_t)ENCODED_FILE_SIZE_BYTES;
  if (s->isByzantine) {  // gen_rand_bytes (server.cpp:329-332)
    static std::mutex rmu;
    static std::mt19937_64 rng{std::random_device{}()};
    std::lock_guard<std::mutex> lk(rmu);
    for (int a = 0; a < NUM_ROUNDS; ++a)
      for (size_t j = 0; j < efs; ++j) result[a][j] = (uint8_t)rng();
    return;
  }
  std::lock_guard<std::mutex> lk(st->mu);
  pir_engine_t* e = engine_for(s, st, NUM_ROUNDS);
  std::vector<uint8_t> out((size_t)NUM_ROUNDS * efs);
  if (pir_engine_answer_coefs(e, key, 0, (uint64_t)NUM_ENCODED_FILES, out.data()) != PIR_OK)
    die("runHollantiQuery");
  for (int a = 0; a < NUM_ROUNDS; ++a) memcpy(result[a], out.data() + a * efs, efs);
}

// server.cpp:345-371: rows [startIndex, endIndex) (both of the reference's branches compute the
// honest answer)
void runHollantiQueryThread(server* s, uint8_t** keys, int threadNum, int startIndex, int endIndex,
                            uint8_t** result) {
  (void)threadNum;
  ShimState* st = state_of(s);
  if (startIndex < 0 || endIndex < startIndex || endIndex > NUM_ENCODED_FILES) {
    fprintf(stderr, "pir shim: rows [%d,%d) outside [0,%d)\n", startIndex, endIndex,
            NUM_ENCODED_FILES);
    abort();
  }
  std::lock_guard<std::mutex> lk(st->mu);
  pir_engine_t* e = engine_for(s, st, NUM_ROUNDS);
  const size_t efs = (size_t)ENCODED_FILE_SIZE_BYTES;
  std::vector<uint8_t> out((size_t)NUM_ROUNDS * efs);
  if (pir_engine_answer_coefs(e, keys, (uint64_t)startIndex, (uint64_t)(endIndex - startIndex),
                              out.data()) != PIR_OK)
    die("runHollantiQueryThread");
  for (int a = 0; a < NUM_ROUNDS; ++a) memcpy(result[a], out.data() + a * efs, efs);
}

// the reference's per-thread XOR folds: `rows` output rows of `len` bytes
static void xor_fold(uint8_t*** in, int numThreads, uint8_t** out, int rows, size_t len) {
  for (int a = 0; a < rows; ++a) {
    memset(out[a], 0, len);
    for (int t = 0; t < numThreads; ++t)
      for (size_t j = 0; j < len; ++j) out[a][j] ^= in[t][a][j];
  }
}

void assembleHollantiQueryThreadResults(server* s, uint8_t*** in, int numThreads, uint8_t** out) {
  (void)s;  // server.cpp:373-382
  xor_fold(in, numThreads, out, NUM_ROUNDS, (size_t)ENCODED_FILE_SIZE_BYTES);
}

void assembleShamirQueryThreadResults(server* s, uint8_t*** in, int numThreads, uint8_t** out) {
  (void)s;  // server.cpp:304-319
  xor_fold(in, numThreads, out, NUM_ROUNDS,
           (size_t)calcShamirResponseLength(LOG_NUM_ENCODED_FILES, ENCODED_FILE_SIZE_BYTES));
}

// ---- multiparty sqrt(N) DPF PIR: the key's shares evaluated and scanned on the engine -------
static void mp_answer(server* s, uint8_t* key, int threadNum, int numThreads, uint8_t** result,
                      const char* fn) {
  ShimState* st = state_of(s);
  std::lock_guard<std::mutex> lk(st->mu);
  pir_engine_t* e = engine_for(s, st, NUM_RSS_KEYS);
  const size_t efs = (size_t)ENCODED_FILE_SIZE_BYTES;
  std::vector<uint8_t> out((size_t)NUM_RSS_KEYS * efs);
  const int kl = calcMultiPartyOptDPFKeyLength(NUM_PARTIES, LOG_NUM_ENCODED_FILES, T);
  if (pir_engine_answer_mp(e, key, (uint64_t)(kl > 0 ? kl : 0), NUM_PARTIES, T, threadNum,
                           numThreads, out.data()) != PIR_OK)
    die(fn);
  for (int a = 0; a < NUM_RSS_KEYS; ++a) memcpy(result[a], out.data() + a * efs, efs);
}

// server.cpp:136-176: random answers for a Byzantine server, else the whole domain
void runOptimizedMultiPartyDPFQuery(server* s, uint8_t* key, uint8_t** result) {
  state_of(s);
  if (s->isByzantine) {  // gen_rand_bytes (server.cpp:157-160)
    static std::mutex rmu;
    static std::mt19937_64 rng{std::random_device{}()};
    std::lock_guard<std::mutex> lk(rmu);
    for (int a = 0; a < NUM_RSS_KEYS; ++a)
      for (int j = 0; j < ENCODED_FILE_SIZE_BYTES; ++j) result[a][j] = (uint8_t)rng();
    return;
  }
  mp_answer(s, key, 0, 1, result, "runOptimizedMultiPartyDPFQuery");
}

// server.cpp:384-430 (both branches compute the honest answer)
void runOptimizedMultiPartyDPFQueryThread(server* s, uint8_t* key, int threadNum, int numThreads,
                                          uint8_t** result) {
  mp_answer(s, key, threadNum, numThreads, result, "runOptimizedMultiPartyDPFQueryThread");
}

void assembleMultipartyDPFQueryThreadResults(server* s, uint8_t*** in, int numThreads,
                                             uint8_t** out) {
  (void)s;  // server.cpp:432-441
  xor_fold(in, numThreads, out, NUM_RSS_KEYS, (size_t)ENCODED_FILE_SIZE_BYTES);
}

void assembleCDQueryThreadResults(server* s, uint8_t*** in, int numThreads, uint8_t** out) {
  (void)s;  // server.cpp:494-503
  xor_fold(in, numThreads, out, NUM_CD_KEYS, (size_t)ENCODED_FILE_SIZE_BYTES);
}

void assembleWoodruffQueryThreadResults(server* s, uint8_t*** in, int numThreads, uint8_t** out) {
  (void)s;  // server.cpp:647-665
  xor_fold(in, numThreads, out, WOODRUFF_DERIVATIVE ? WOODRUFF_M + 1 : 1,
           (size_t)ENCODED_FILE_SIZE_BYTES);
}

void runOptShamirDPFQueryThread(server*, uint8_t**, int, int, int, uint8_t**) {
  out_of_scope("runOptShamirDPFQueryThread", "Shamir");
}
// server.cpp:443-492 (both branches compute the honest answer): NUM_CD_KEYS shares of the
// covering-design key evaluated on the thread's rows and scanned on the engine
void runCDQueryThread(server* s, uint8_t* key, int threadNum, int numThreads, uint8_t** result) {
  ShimState* st = state_of(s);
  std::lock_guard<std::mutex> lk(st->mu);
  pir_engine_t* e = engine_for(s, st, NUM_CD_KEYS);
  const size_t efs = (size_t)ENCODED_FILE_SIZE_BYTES;
  std::vector<uint8_t> out((size_t)NUM_CD_KEYS * efs);
  const int kl = calcCDDPFKeyLength(NUM_PARTIES, LOG_NUM_ENCODED_FILES, T, NUM_CD_KEYS_NEEDED,
                                    NUM_CD_KEYS);
  if (pir_engine_answer_cd(e, key, (uint64_t)(kl > 0 ? kl : 0), NUM_CD_KEYS_NEEDED, NUM_CD_KEYS,
                           threadNum, numThreads, out.data()) != PIR_OK)
    die("runCDQueryThread");
  for (int a = 0; a < NUM_CD_KEYS; ++a) memcpy(result[a], out.data() + a * efs, efs);
}
void runWoodruffQueryThread(server*, uint8_t*, int, int, int, uint8_t**) {
  out_of_scope("runWoodruffQueryThread", "Woodruff");
}

// client.cpp:16-33 (synthetic DB; MAC tags are outside this engine's scope).  The files share
// one allocation (held in c->ctx, which the reference uses for an unused EVP context) and are
// filled by host threads: the reference's per-file malloc + memset of NUM_FILES rows is most of
// a large setup's host time (2^26 x 1 KiB for configs[4]'s k = 5).
void initialize_client(client* c, uint8_t log_num_files, uint32_t file_size_bytes) {
  (void)file_size_bytes;
  if (CHECK_MAC) {
    fprintf(stderr, "pir shim: CHECK_MAC setups are outside the engine's scope\n");
    abort();
  }
  c->macCtx = nullptr;
  c->macKey = (uint8_t*)"1234567812345678";
  const uint64_t n = 1ull << log_num_files, fb = FILE_SIZE_BYTES;
  c->unencoded_files = (uint8_t**)malloc((size_t)n * sizeof(uint8_t*));
  uint8_t* block = big_alloc((size_t)(n * fb));
  if (!c->unencoded_files || !block) {
    fprintf(stderr, "pir shim: cannot allocate %llu client files of %llu bytes\n",
            (unsigned long long)n, (unsigned long long)fb);
    abort();
  }
  c->ctx = block;
  const uint32_t pb = PAYLOAD_SIZE_BYTES;
  const int T = shim_threads();
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([=] {
      for (uint64_t i = (uint64_t)t; i < n; i += (uint64_t)T) {
        uint8_t* f = block + i * fb;
        c->unencoded_files[i] = f;
        memset(f, (int)(i & 0xff), pb);
        if (fb > pb) memset(f + pb, 0, fb - pb);
        if (i == 1)
          for (uint32_t j = 0; j < pb; ++j) f[j] = (uint8_t)j;
      }
    });
  for (auto& x : th) x.join();
}

void free_client(client* c) {  // client.cpp:35-41
  big_free(c->ctx);  // the files' block
  c->ctx = nullptr;
  free(c->unencoded_files);
  c->unencoded_files = nullptr;
}

// the nq the mode's queries will ask the engine for (engine_for's callers below)
static int setup_nq() { return MODE == 1 ? NUM_RSS_KEYS : (MODE == 4 ? NUM_CD_KEYS : NUM_ROUNDS); }

// A setup encodes on the GPU when the rows are still initializeServer's zeros (the reference
// XORs the encoding INTO the rows, client.cpp:66/88, so that is the whole result); the shard is
// then resident and the first query answers from HBM.  Otherwise, and for servers this shim did
// not initialise, the host encode below.
static bool gpu_setup(server* s, const std::function<int(pir_engine_t*)>& encode) {
  if (!s->ctx || getenv("PIR_SHIM_HOST_SETUP")) return false;
  ShimState* st = static_cast<ShimState*>(s->ctx);
  std::lock_guard<std::mutex> lk(st->mu);
  // a caller may have written indexList directly (legal in the reference, which XORs the
  // encoding into whatever the rows hold) without pirServerSetRows / pirServerShardChanged
  if (st->rows_zero && rows_touched(st)) {
    st->rows_zero = false;
    st->dirty = true;
  }
  if (!st->rows_zero) {  // rows already hold data: the host XOR-encode keeps that data
    std::unique_lock<std::shared_mutex> excl(st->life);
    sync_rows_down(s, st);
    return false;
  }
  pir_engine_t* e = engine_for(s, st, setup_nq(), /*upload=*/false, /*must=*/false);
  if (!e) {  // no usable GPU here: the reference's host encode (queries will refuse loudly)
    st->dirty = true;
    return false;
  }
  // the encode rewrites the whole shard: no slice pass may read it meanwhile, and no slice
  // group computed from the rows before the setup may be served after it
  std::unique_lock<std::shared_mutex> excl(st->life);
  st->groups.clear();
  st->group_bytes = 0;
  if (encode(e) != PIR_OK) die("encode on the GPU");
  st->dirty = false;
  st->host_stale = true;
  st->rows_zero = false;
  // tree mode: one throw-away pass in the server's own Thread shape (an all-zero key), so the
  // first client query does not pay the kernels' first launch and the engine's buffers
  const int T = s->numThreads;
  if (MODE == 0 && getenv("PIR_SHIM_NO_WARM") == nullptr && T >= 1 && (T & (T - 1)) == 0 &&
      T <= NUM_ENCODED_FILES) {
    const int kl = pir_engine_key_len(st->cfg.num_parties, LOG_NUM_ENCODED_FILES, NUM_ROUNDS);
    std::vector<uint8_t> key((size_t)kl, 0), parts((size_t)T * NUM_ROUNDS * ENCODED_FILE_SIZE_BYTES);
    if (pir_engine_answer_slices(e, key.data(), T, parts.data()) != PIR_OK) die("setup warm-up");
  }
  return true;
}

// client.cpp:70-97: row i of party q = XOR_j gf_pow(q, j) * file[encDBsize*j + i]
void encode_across_files_server(client* c, server* s) {
  if (gpu_setup(s, [&](pir_engine_t* e) {
        return pir_engine_encode_across_rows(e, c->unencoded_files, (uint64_t)NUM_FILES, K);
      }))
    return;
  const long encdb = (NUM_FILES + K - 1) / K;
  const int efs = ENCODED_FILE_SIZE_BYTES;
  std::vector<uint8_t> coef(K);
  for (int j = 0; j < K; ++j) coef[j] = gf_pow_h((uint8_t)s->partyIndex, j);
  for (int i = 0; i < NUM_ENCODED_FILES; ++i) {
    uint8_t* row = s->indexList[i];
    for (int j = 0; j < K; ++j) {
      const long src = encdb * j + i;
      if (src >= NUM_FILES) continue;
      const uint8_t* f = c->unencoded_files[src];
      for (int b = 0; b < efs; ++b) row[b] ^= gf_mul_h(f[b], coef[j]);
    }
  }
  shard_written_on_host(s);
}

// client.cpp:43-56, 99-103: row i of party q = XOR_{j<K} gf_pow(q, j) * part j of file i, where
// part j = bytes [j*EFS, (j+1)*EFS) of the file zero-padded to K*EFS (encodeMat[j][q-1] of
// gen_encode_matrix, coding.cpp:64-70).  One 256-entry product table per coefficient.
void encode_within_files_server(client* c, server* s) {
  if (IS_HERMITE) out_of_scope("encode_within_files_server (Hermite rows)", "Shamir");
  if (gpu_setup(s, [&](pir_engine_t* e) {
        return pir_engine_encode_within_rows(e, c->unencoded_files, (uint64_t)NUM_FILES,
                                             FILE_SIZE_BYTES, K, s->partyIndex);
      }))
    return;
  const int efs = ENCODED_FILE_SIZE_BYTES;
  std::vector<uint8_t> tab((size_t)K * 256);
  for (int j = 0; j < K; ++j) {
    const uint8_t cj = gf_pow_h((uint8_t)s->partyIndex, j);
    for (int x = 0; x < 256; ++x) tab[(size_t)j * 256 + x] = gf_mul_h((uint8_t)x, cj);
  }
  for (int i = 0; i < NUM_ENCODED_FILES; ++i) {
    uint8_t* row = s->indexList[i];
    const uint8_t* f = c->unencoded_files[i];
    for (int j = 0; j < K; ++j) {
      const uint8_t* t = &tab[(size_t)j * 256];
      for (int b = 0; b < efs; ++b) {
        const long src = (long)j * efs + b;
        if (src < (long)FILE_SIZE_BYTES) row[b] ^= t[f[src]];
      }
    }
  }
  shard_written_on_host(s);
}

// ---- client-side names of package c (src/client/*.go, src/benchmark/benchmark.go) ----------

// client.cpp:144-153: finalCW = gf_pow(j, RHO*i) ^ 1, keys by genOptimizedDPF
// (dpf_tree.cpp:142-274) -- on the GPU (pir_gen_keys, the engine's own AES), root seeds from the
// OS CSPRNG (the reference: RAND_bytes).  (*keys)[j] receives party j's key.
void generate_opt_DPF_tree_query(client* c, int index, uint8_t*** keys) {
  (void)c;
  if (T != 1) {  // client.cpp:145 assert(T == 1)
    fprintf(stderr, "pir shim: generate_opt_DPF_tree_query needs T == 1 (got %d)\n", T);
    abort();
  }
  const int p = NUM_PARTIES, nq = NUM_ROUNDS, n = LOG_NUM_ENCODED_FILES;
  const int kl = calcOptimizedDPFTreeKeyLength(p, n, nq);
  if (p < 2 || kl <= 0 || index < 0 || index >= NUM_ENCODED_FILES) {
    fprintf(stderr, "pir shim: generate_opt_DPF_tree_query: index %d, p %d, n %d\n", index, p, n);
    abort();
  }
  std::vector<uint8_t> fcw((size_t)nq * (p - 1)), seeds((size_t)p * 16),
      out((size_t)p * kl);
  pir_final_cw(p, nq, RHO, fcw.data());
  os_random(seeds.data(), seeds.size());
  if (pir_gen_keys(device_default(), n, (uint64_t)index, fcw.data(), p, nq, seeds.data(),
                   out.data()) != PIR_OK)
    die("generate_opt_DPF_tree_query");
  for (int j = 0; j < p; ++j) memcpy((*keys)[j], out.data() + (size_t)j * kl, kl);
}

// client.cpp:201-203 -> genHollantiDPF (shamir_dpf.cpp:190-237): for round a and record x a
// random polynomial of t random low coefficients whose coefficient t + (a+1)*RHO - 1 is
// [x == index]; keys[q][a][x] = its value at q + 1 (evalPoly, shamir_dpf.cpp:10-17, Horner).
// The reference's evalPoly is called with degree t + RHO*NUM_ROUNDS on an array of that many
// bytes and so reads one byte past the allocation as the top coefficient; the intended
// polynomial (that byte 0) is computed here.
void generateHollantiQuery(client* c, int index, uint8_t*** keys) {
  (void)c;
  const int p = NUM_PARTIES, nq = NUM_ROUNDS, t = T, rho = RHO;
  const long N = NUM_ENCODED_FILES;
  std::vector<uint8_t> rnd((size_t)N * t);
  for (int a = 0; a < nq; ++a) {
    os_random(rnd.data(), rnd.size());
    const int sec = t + (a + 1) * rho - 1;
    for (int q = 0; q < p; ++q) {
      const uint8_t xq = (uint8_t)(q + 1);
      uint8_t xsec = 1;  // xq^sec
      for (int e = 0; e < sec; ++e) xsec = gf_mul_h(xsec, xq);
      uint8_t* dst = keys[q][a];
      for (long x = 0; x < N; ++x) {
        const uint8_t* r = &rnd[(size_t)x * t];
        uint8_t v = 0;
        for (int m = t - 1; m >= 0; --m) v = gf_mul_h(v, xq) ^ r[m];
        dst[x] = v ^ (x == index ? xsec : 0);
      }
    }
  }
}

// utils.cpp:32-34: HMAC-SHA256 under a 16-byte key.  Like the reference (HMAC() writes the
// whole digest and stores its length through the outputLen argument), 32 bytes are written.
void mac(uint8_t* key, uint8_t* input, int inputLen, unsigned char* output, int outputLen) {
  (void)outputLen;
  hmac_sha256(key, 16, input, (size_t)(inputLen > 0 ? inputLen : 0), output);
}

// utils.cpp:168-174
int choose(int n, int k) { return k == 0 ? 1 : (n * choose(n - 1, k - 1)) / k; }

// utils.cpp:221-223
uint128_t convertInt(int x) { return (uint128_t)x; }

// utils.cpp:118-129 (double pow as in the reference; ceil((double)(n/2)) == n/2)
int calcCDDPFKeyLength(int p, int log_domainSize, int t, int num_cd_keys_needed,
                       int num_cd_keys) {
  (void)t;
  const int n = log_domainSize;
  const uint32_t p2 = (uint32_t)pow(2, num_cd_keys_needed - 1);
  const int mu_pow = n / 2 + 3;
  const uint64_t mu = (uint64_t)pow(2, mu_pow), nu = (uint64_t)pow(2, n - mu_pow);
  return (int)(16 * p2 * nu + num_cd_keys * nu * p2 + p2 * mu);
}

// utils.cpp:145-153: the smallest m >= 3 with choose(m, 2) >= 2^logDomainSize
int calcWoodruffKeyLength(int p, int r, int t, int logDomainSize, int fileSizeBytes) {
  (void)p; (void)r; (void)t; (void)fileSizeBytes;
  int m = 3;
  while (choose(m, 2) < (1 << logDomainSize)) ++m;
  return m;
}

// The other modes' client halves: their server modes are refused at setSystemParams, so a
// client of this engine never reaches them (and the multiparty key generation of the reference
// cannot make a usable key: DESIGN.md, reference defects).
void generateMultiPartyDPFQuery(client*, int, uint8_t***) {
  out_of_scope("generateMultiPartyDPFQuery", "multiparty key generation");
}
void assembleMultiPartyResponses(client*, uint8_t*, uint8_t***, uint8_t*) {
  out_of_scope("assembleMultiPartyResponses", "multiparty decode");
}
void generateCDQuery(client*, int, uint8_t***) { out_of_scope("generateCDQuery", "covering-design"); }
void assembleCDResponses(client*, uint8_t*, uint8_t***, uint8_t*) {
  out_of_scope("assembleCDResponses", "covering-design");
}
void genShamirCoeffs(int, int, int, uint128_t, uint8_t***, uint8_t***) {
  out_of_scope("genShamirCoeffs", "Shamir");
}
void genOptShamirDPF(int, uint128_t, int, int, int, uint8_t***, uint8_t***, uint8_t***) {
  out_of_scope("genOptShamirDPF", "Shamir");
}
void assembleShamirResponses(client*, uint8_t*, uint8_t***, uint8_t*, uint8_t***, uint8_t***) {
  out_of_scope("assembleShamirResponses", "Shamir");
}
void genWoodruffVs(int, int, uint8_t**) { out_of_scope("genWoodruffVs", "Woodruff"); }
void genWoodruffQuery(uint128_t, int, int, int, uint8_t**, uint8_t**) {
  out_of_scope("genWoodruffQuery", "Woodruff");
}
void assembleWoodruffResponses(client*, uint8_t*, uint8_t***, uint8_t*, uint8_t**) {
  out_of_scope("assembleWoodruffResponses", "Woodruff");
}

}  // extern "C"
