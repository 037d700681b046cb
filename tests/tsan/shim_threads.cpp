// TEST INFRASTRUCTURE ONLY (tests/test_tsan_shim.py): the shim's concurrent paths under
// ThreadSanitizer, on the CPU, with the oracle-backed stub engine (stub_engine.cpp).  The
// scenarios are those of tests/test_gpu_threads.py plus the ones the round-4 shim added:
//   1. T = 16 concurrent runOptimizedDPFTreeQueryThread calls of one query (tree.go:60-76)
//   2. two queries' slices interleaved (8 + 8 threads)
//   3. pirServerSetRows and pirServerShardChanged while a query's slice group is in flight,
//      then a clean query
//   4. more than kMaxSliceGroups (8) queries at once: 12 queries x 4 threads (group eviction)
//   5. two pirRunTreeQueryThreads fan-outs at once (the shim's pool)
//   6. a GPU-path setup (encode_across_files_server -> the engine; lazy host rows) with queries
//      and pirServerSyncRows concurrently, then freeServer
//   7. freeServer -> initializeServer + setup + queries while the reaper thread still tears the
//      previous engine down (3 rounds), another server answering fan-outs throughout
//   8. indexList written directly before the setup: the encode XORs into those rows
//   9. lone Thread calls (no partner: the 1/T slice path), alone and beside a fan-out
//  10. a fan-out whose first call answered alone and whose other calls came late
// Exit status 0 when every answer equals the oracle's (or, for 3, one of the two shards').
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <random>
#include <thread>
#include <vector>

#include "../../include/pir_server.h"
extern "C" {
#include "../../oracle/pir_oracle.h"
}

static int g_fail = 0;
#define CHECK(cond, ...)                \
  do {                                  \
    if (!(cond)) {                      \
      fprintf(stderr, "FAIL: " __VA_ARGS__); \
      fprintf(stderr, "\n");            \
      ++g_fail;                         \
    }                                   \
  } while (0)

struct Keys {
  int p, n, nq, kl;
  std::vector<uint8_t> bytes;  // p keys
  const uint8_t* party(int q) const { return bytes.data() + (size_t)(q - 1) * kl; }
};

static Keys make_keys(int p, int n, int nq, uint64_t index, uint64_t seed) {
  Keys k{p, n, nq, orc_key_len(p, n, nq), {}};
  k.bytes.resize((size_t)p * k.kl);
  std::vector<uint8_t> fcw((size_t)nq * (p - 1)), seeds((size_t)p * 16);
  orc_final_cw(p, nq, 1, fcw.data());
  std::mt19937_64 g(seed);
  for (auto& b : seeds) b = (uint8_t)g();
  orc_gen_opt_dpf(n, index, fcw.data(), p, nq, seeds.data(), k.bytes.data());
  return k;
}

// one thread slice into a packed nq x efs buffer
static void slice(server* s, const uint8_t* key, int t, int T, int nq, int efs, uint8_t* out) {
  std::vector<uint8_t*> rows(nq);
  for (int a = 0; a < nq; ++a) rows[a] = out + a * efs;
  runOptimizedDPFTreeQueryThread(s, const_cast<uint8_t*>(key), t, T, rows.data());
}

static std::vector<uint8_t> xor_parts(const std::vector<uint8_t>& parts, int T, size_t ans) {
  std::vector<uint8_t> out(ans, 0);
  for (int t = 0; t < T; ++t)
    for (size_t i = 0; i < ans; ++i) out[i] ^= parts[t * ans + i];
  return out;
}

static std::vector<uint8_t> oracle(const Keys& k, int party, int efs, const std::vector<uint8_t>& shard) {
  std::vector<uint8_t> out((size_t)k.nq * efs);
  orc_answer(k.p, party, k.n, efs, k.nq, k.party(party), shard.data(), out.data());
  return out;
}

int main() {
  const int L = 9, f = 48;
  setSystemParams(L, f, 1, 1, 0, 0, 1, 0, 0);  // tree mode, k = 1: p = 2, NUM_ROUNDS = 1
  const int p = NUM_PARTIES, n = LOG_NUM_ENCODED_FILES, nq = NUM_ROUNDS, efs = ENCODED_FILE_SIZE_BYTES;
  const size_t N = (size_t)1 << n, ans = (size_t)nq * efs;
  std::vector<uint8_t> shard(N * efs);
  orc_xorshift_fill(0x9E3779B97F4A7C15ull, shard.data(), shard.size());

  server s{};
  initializeServer(&s, 1, L, f, 0, 16);
  pirServerSetRows(&s, shard.data(), 0, N, f);

  std::vector<Keys> keys;
  for (int q = 0; q < 12; ++q) keys.push_back(make_keys(p, n, nq, (N / 13) * q + 3, 100 + q));

  {  // 1. one query, T = 16
    const int T = 16;
    std::vector<uint8_t> parts(T * ans);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] { slice(&s, keys[0].party(1), t, T, nq, efs, &parts[t * ans]); });
    for (auto& x : th) x.join();
    CHECK(xor_parts(parts, T, ans) == oracle(keys[0], 1, efs, shard), "scenario 1");
  }
  {  // 2. two queries interleaved, 8 slices each
    const int T = 8;
    std::vector<uint8_t> pa(T * ans), pb(T * ans);
    std::vector<std::thread> th;
    for (int t = 0; t < 2 * T; ++t)
      th.emplace_back([&, t] {
        if (t & 1) slice(&s, keys[2].party(1), t / 2, T, nq, efs, &pb[(t / 2) * ans]);
        else slice(&s, keys[1].party(1), t / 2, T, nq, efs, &pa[(t / 2) * ans]);
      });
    for (auto& x : th) x.join();
    CHECK(xor_parts(pa, T, ans) == oracle(keys[1], 1, efs, shard), "scenario 2a");
    CHECK(xor_parts(pb, T, ans) == oracle(keys[2], 1, efs, shard), "scenario 2b");
  }
  {  // 3. a shard change while a query's slices are in flight, then a clean query
    const int T = 8;
    std::vector<uint8_t> shard2 = shard;
    for (size_t i = 0; i < shard2.size(); i += 7) shard2[i] ^= 0x5a;
    std::vector<uint8_t> parts(T * ans);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] { slice(&s, keys[3].party(1), t, T, nq, efs, &parts[t * ans]); });
    th.emplace_back([&] { pirServerSetRows(&s, shard2.data(), 0, N, f); });
    th.emplace_back([&] { pirServerShardChanged(&s); });  // concurrently with the slice group
    for (auto& x : th) x.join();
    // slices of either shard (the change may fall between the group's pass and a late caller)
    std::vector<uint8_t> sl(ans);
    bool each_ok = true;
    for (int t = 0; t < T; ++t) {
      std::vector<uint8_t> a(ans), b(ans);
      orc_answer_slice(p, 1, n, efs, nq, keys[3].party(1), shard.data(), t, T, a.data());
      orc_answer_slice(p, 1, n, efs, nq, keys[3].party(1), shard2.data(), t, T, b.data());
      const std::vector<uint8_t> got(parts.begin() + t * ans, parts.begin() + (t + 1) * ans);
      each_ok &= got == a || got == b;
    }
    CHECK(each_ok, "scenario 3: a slice of neither shard");
    shard = shard2;
    std::vector<uint8_t> p2(T * ans);
    std::vector<std::thread> th2;
    for (int t = 0; t < T; ++t)
      th2.emplace_back([&, t] { slice(&s, keys[3].party(1), t, T, nq, efs, &p2[t * ans]); });
    for (auto& x : th2) x.join();
    CHECK(xor_parts(p2, T, ans) == oracle(keys[3], 1, efs, shard), "scenario 3 (after the change)");
  }
  {  // 4. 12 queries x 4 threads at once: more slice groups than the shim keeps
    const int T = 4, Q = 12;
    std::vector<uint8_t> parts((size_t)Q * T * ans);
    std::vector<std::thread> th;
    for (int i = 0; i < Q * T; ++i)
      th.emplace_back([&, i] {
        const int q = i % Q, t = i / Q;
        slice(&s, keys[q].party(1), t, T, nq, efs, &parts[((size_t)q * T + t) * ans]);
      });
    for (auto& x : th) x.join();
    for (int q = 0; q < Q; ++q) {
      std::vector<uint8_t> pq(parts.begin() + (size_t)q * T * ans, parts.begin() + (size_t)(q + 1) * T * ans);
      CHECK(xor_parts(pq, T, ans) == oracle(keys[q], 1, efs, shard), "scenario 4, query %d", q);
    }
  }
  {  // 5. two fan-outs through the shim's pool at once
    std::vector<uint8_t> a(ans), b(ans);
    uint8_t* ra[16];
    uint8_t* rb[16];
    for (int i = 0; i < nq; ++i) {
      ra[i] = a.data() + i * efs;
      rb[i] = b.data() + i * efs;
    }
    std::thread t1([&] { pirRunTreeQueryThreads(&s, const_cast<uint8_t*>(keys[4].party(1)), 16, ra); });
    std::thread t2([&] { pirRunTreeQueryThreads(&s, const_cast<uint8_t*>(keys[5].party(1)), 8, rb); });
    t1.join();
    t2.join();
    CHECK(a == oracle(keys[4], 1, efs, shard), "scenario 5a");
    CHECK(b == oracle(keys[5], 1, efs, shard), "scenario 5b");
  }
  freeServer(&s);

#ifndef TSAN_ROUND4_SHIM  // (the round-4 shim has no GPU setup path; see test_tsan_shim.py)
  {  // 6. a GPU-path setup: the engine encodes, indexList is synced lazily
    const int L6 = 10, f6 = 32, k6 = 2;
    setSystemParams(L6, f6, 1, k6, 1, 0, 1, 0, 0);  // p = 4, 2^9 encoded rows, NUM_ROUNDS = 2
    const int p6 = NUM_PARTIES, n6 = LOG_NUM_ENCODED_FILES, nq6 = NUM_ROUNDS, efs6 = ENCODED_FILE_SIZE_BYTES;
    const size_t ans6 = (size_t)nq6 * efs6;
    client c{};
    initialize_client(&c, L6, f6);
    std::vector<uint8_t> files((size_t)1 << L6 << 0);
    files.resize(((size_t)1 << L6) * f6);
    orc_synthetic_db(L6, f6, files.data());
    std::vector<uint8_t> want(((size_t)1 << n6) * efs6);
    orc_encode_across(L6, f6, k6, p6, 2, files.data(), want.data());
    server s6{};
    initializeServer(&s6, 2, L6, f6, 0, 8);
    encode_across_files_server(&c, &s6);
    Keys k6k = make_keys(p6, n6, nq6, 77, 7);
    const int T = 8;
    std::vector<uint8_t> parts(T * ans6);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] { slice(&s6, k6k.party(2), t, T, nq6, efs6, &parts[t * ans6]); });
    th.emplace_back([&] { pirServerSyncRows(&s6); });
    for (auto& x : th) x.join();
    CHECK(xor_parts(parts, T, ans6) == oracle(k6k, 2, efs6, want), "scenario 6 answer");
    bool rows_ok = true;
    for (size_t r = 0; r < ((size_t)1 << n6); ++r)
      rows_ok &= memcmp(s6.indexList[r], &want[r * efs6], efs6) == 0;
    CHECK(rows_ok, "scenario 6 rows after pirServerSyncRows");
    freeServer(&s6);

    // 7. freeServer hands the engine to the reaper thread (the stub's teardown takes 20 ms):
    //    set the next server up and query it while the previous teardown still runs, 3 times,
    //    with a second server answering fan-outs throughout
    server keep{};
    initializeServer(&keep, 2, L6, f6, 0, 4);
    encode_across_files_server(&c, &keep);
    std::atomic<bool> stop{false};
    std::atomic<int> keep_bad{0};
    std::thread busy([&] {
      std::vector<uint8_t> a(ans6);
      uint8_t* ra[8];
      for (int i = 0; i < nq6; ++i) ra[i] = a.data() + i * efs6;
      const std::vector<uint8_t> want_a = oracle(k6k, 2, efs6, want);
      while (!stop.load()) {
        pirRunTreeQueryThreads(&keep, const_cast<uint8_t*>(k6k.party(2)), 4, ra);
        if (a != want_a) keep_bad.fetch_add(1);
      }
    });
    for (int it = 0; it < 3; ++it) {
      server s7{};
      initializeServer(&s7, 2, L6, f6, 0, T);
      encode_across_files_server(&c, &s7);
      std::vector<uint8_t> p7(T * ans6);
      std::vector<std::thread> t7;
      for (int t = 0; t < T; ++t)
        t7.emplace_back([&, t] { slice(&s7, k6k.party(2), t, T, nq6, efs6, &p7[t * ans6]); });
      for (auto& x : t7) x.join();
      CHECK(xor_parts(p7, T, ans6) == oracle(k6k, 2, efs6, want), "scenario 7 answer, round %d", it);
      freeServer(&s7);  // returns before the teardown is done
      CHECK(s7.ctx == nullptr && s7.indexList == nullptr, "scenario 7 server not cleared");
    }
    stop.store(true);
    busy.join();
    CHECK(keep_bad.load() == 0, "scenario 7: %d wrong answers on the other server", keep_bad.load());
    freeServer(&keep);
    pirServerWaitFreed();

    // 8. indexList written directly (no pirServerSetRows / ShardChanged) before the setup: the
    //    encode is XORed into those rows (client.cpp:88), not written over them
    {
      server s8{};
      initializeServer(&s8, 2, L6, f6, 0, T);
      std::vector<uint8_t> mine(((size_t)1 << n6) * efs6), want8(want);
      orc_xorshift_fill(0x51EDull, mine.data(), mine.size());
      for (size_t r = 0; r < ((size_t)1 << n6); ++r) {
        memcpy(s8.indexList[r], &mine[r * efs6], efs6);
        for (int b = 0; b < efs6; ++b) want8[r * efs6 + b] ^= mine[r * efs6 + b];
      }
      encode_across_files_server(&c, &s8);
      std::vector<uint8_t> p8(T * ans6);
      std::vector<std::thread> t8;
      for (int t = 0; t < T; ++t)
        t8.emplace_back([&, t] { slice(&s8, k6k.party(2), t, T, nq6, efs6, &p8[t * ans6]); });
      for (auto& x : t8) x.join();
      CHECK(xor_parts(p8, T, ans6) == oracle(k6k, 2, efs6, want8), "scenario 8 answer");
      bool ok8 = true;
      for (size_t r = 0; r < ((size_t)1 << n6); ++r)
        ok8 &= memcmp(s8.indexList[r], &want8[r * efs6], efs6) == 0;
      CHECK(ok8, "scenario 8 rows");

      // 9. lone Thread calls (no partner within the join window): each answers its own slice,
      //    also while another query's fan-out runs on the same server
      std::vector<uint8_t> one(ans6), ref(ans6);
      slice(&s8, k6k.party(2), 3, T, nq6, efs6, one.data());
      orc_answer_slice(p6, 2, n6, efs6, nq6, k6k.party(2), want8.data(), 3, T, ref.data());
      CHECK(one == ref, "scenario 9 lone slice");
      Keys k9 = make_keys(p6, n6, nq6, 5, 9);
      std::vector<uint8_t> p9(T * ans6), lone(ans6), lref(ans6);
      std::vector<std::thread> t9;
      for (int t = 0; t < T; ++t)
        t9.emplace_back([&, t] { slice(&s8, k9.party(2), t, T, nq6, efs6, &p9[t * ans6]); });
      t9.emplace_back([&] { slice(&s8, k6k.party(2), 6, 2 * T, nq6, efs6, lone.data()); });
      for (auto& x : t9) x.join();
      CHECK(xor_parts(p9, T, ans6) == oracle(k9, 2, efs6, want8), "scenario 9 fan-out beside");
      orc_answer_slice(p6, 2, n6, efs6, nq6, k6k.party(2), want8.data(), 6, 2 * T, lref.data());
      CHECK(lone == lref, "scenario 9 lone slice beside a fan-out");

      // 10. a fan-out whose first call came alone (answered alone after the join window), the
      //     other T - 1 late: they meet in one group (its creator waits for late partners)
      Keys k10 = make_keys(p6, n6, nq6, 200, 10);
      std::vector<uint8_t> p10(T * ans6);
      slice(&s8, k10.party(2), 0, T, nq6, efs6, &p10[0]);
      std::vector<std::thread> t10;
      for (int t = 1; t < T; ++t)
        t10.emplace_back([&, t] { slice(&s8, k10.party(2), t, T, nq6, efs6, &p10[t * ans6]); });
      for (auto& x : t10) x.join();
      CHECK(xor_parts(p10, T, ans6) == oracle(k10, 2, efs6, want8), "scenario 10 late fan-out");
      freeServer(&s8);
    }
    free_client(&c);
  }
#endif
  printf("%s: %d failure(s)\n", g_fail ? "FAIL" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
