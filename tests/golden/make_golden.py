#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/*.json from the REFERENCE itself.

Test infrastructure only.  Requires oracle/_ref/libref.so, i.e. the reference's own
src/c compiled from /root/reference by `make -C oracle ref` (this container only; the
reference never travels to the GPU box -- these JSON files do).  Every expected output
below is produced by a reference symbol (see oracle/ref_driver.cpp); the only thing this
script computes itself is the synthetic shard INPUT (xorshift64, whose SHA-256 is stored so
a different generator is caught).

Root seeds come from the reference's RAND_bytes, so each fixture stores the full key bytes.

    python tests/golden/make_golden.py     # rewrites tests/golden/*.json
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref.so"))
U64 = ctypes.c_uint64
SHARD_SEED = 0x9E3779B97F4A7C15


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def xorshift_bytes(seed, n):
    # x ^= x << 13; x ^= x >> 7; x ^= x << 17 (64-bit), output low byte per step
    out = np.empty(n, np.uint8)
    x = seed & 0xFFFFFFFFFFFFFFFF
    M = 0xFFFFFFFFFFFFFFFF
    for i in range(n):
        x ^= (x << 13) & M
        x ^= x >> 7
        x ^= (x << 17) & M
        out[i] = x & 0xFF
    return out


def final_cw(p, nq, rho, k):
    # client.cpp:144-153 (computed through the reference's gf_pow)
    out = []
    for i in range(1, nq + 1):
        for j in range(2, p + 1):
            out.append(REF.ref_gf_pow(j, rho * i) ^ 1)
    return np.array(out, np.uint8)


def write(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
    print("wrote", name)


def prg_kats():
    cases = []
    rng = np.random.RandomState(1)
    seeds = [bytes(range(16)), bytes(16), bytes(rng.randint(0, 256, 16, dtype=np.uint8))]
    for s in seeds:
        for plen in (16, 33, 34, 48):
            out = np.zeros(plen, np.uint8)
            REF.ref_G(s, plen, ptr(out))
            cases.append({"seed": s.hex(), "plen": plen, "out": out.tobytes().hex()})
    blen = {p: REF.ref_blen(p) for p in range(2, 18)}
    keylen = {f"{p},{n},{nq}": REF.ref_key_len(p, n, nq)
              for (p, n, nq) in [(2, 16, 1), (2, 20, 1), (2, 24, 1), (2, 27, 1), (8, 24, 5),
                                 (3, 10, 1), (5, 12, 4), (8, 12, 5), (9, 10, 1)]}
    write("prg_kat.json", {"G": cases, "blen": blen, "key_len": keylen})


def gf_kats():
    mul = np.array([[REF.ref_gf_mul(a, b) for b in range(256)] for a in range(256)], np.uint8)
    pw = np.array([[REF.ref_gf_pow(a, e) for e in range(256)] for a in range(256)], np.uint8)
    inv = np.array([REF.ref_gf_inv(a) for a in range(256)], np.uint8)
    spot = {"02*80": int(mul[2, 0x80]), "53*ca": int(mul[0x53, 0xCA]), "ff*ff": int(mul[255, 255]),
            "inv02": int(inv[2]), "pow(2,8)": int(pw[2, 8]), "pow(0,5)": int(pw[0, 5])}
    write("gf_kat.json", {"mul_sha256": sha(mul), "pow_sha256": sha(pw), "inv": inv.tobytes().hex(),
                          "spot": spot})


def dpf_and_answers():
    cases = []
    for (p, n, nq, idx) in [(2, 10, 1, 77), (3, 10, 1, 513), (5, 12, 4, 4000), (8, 12, 5, 1234),
                            (9, 10, 1, 1023), (2, 16, 1, 21845)]:
        kl = REF.ref_key_len(p, n, nq)
        fcw = final_cw(p, nq, 1, nq)
        keys = np.zeros(p * kl, np.uint8)
        REF.ref_gen_opt_dpf(n, U64(idx), ptr(fcw), p, nq, ptr(keys))
        N = 1 << n
        parties = []
        for party in range(p):
            c = np.zeros(nq * N, np.uint8)
            REF.ref_eval_all_opt(p, party, n, ptr(keys[party * kl:]), nq, ptr(c))
            ent = {"key": keys[party * kl:(party + 1) * kl].tobytes().hex(), "c_sha256": sha(c)}
            if n <= 10:
                ent["c"] = c.tobytes().hex()
            parties.append(ent)
        answers = {}
        for efs in ((8, 256) if n <= 12 else (256,)):
            shard = xorshift_bytes(SHARD_SEED, N * efs)
            per = []
            for party in range(p):
                h = REF.ref_server_new(p, party + 1, n, efs, nq, ptr(shard), 0, 1)
                res = np.zeros(nq * efs, np.uint8)
                REF.ref_server_answer(ctypes.c_void_p(h), ptr(keys[party * kl:]), ptr(res))
                REF.ref_server_free(ctypes.c_void_p(h))
                per.append(res.tobytes().hex())
            answers[str(efs)] = {"shard_sha256": sha(shard), "answers": per}
        cases.append({"p": p, "n": n, "nq": nq, "index": idx, "final_cw": fcw.tobytes().hex(),
                      "key_len": kl, "parties": parties, "answers": answers})
        print("dpf case", p, n, nq)
    write("dpf_eval.json", {"shard_seed": SHARD_SEED, "cases": cases})


def e2e():
    restype = ctypes.c_int
    REF.ref_e2e.restype = restype
    cases = []
    for (L, f, k, r, idx) in [(10, 8, 1, 1, 5), (10, 8, 2, 1, 300), (12, 16, 4, 2, 77),
                              (12, 16, 5, 2, 501), (11, 32, 3, 1, 100)]:
        rho = 1
        s = (ctypes.c_int * 5)()
        REF.ref_e2e_sizes(L, f, k, r, rho, s)
        p, n, efs, nq, kl = list(s)
        N = 1 << n
        files = np.zeros((1 << L) * f, np.uint8)
        shards = np.zeros(p * N * efs, np.uint8)
        keys = np.zeros(p * kl, np.uint8)
        ans = np.zeros(p * nq * efs, np.uint8)
        dec = np.zeros(f, np.uint8)
        ok = REF.ref_e2e(L, f, k, r, rho, idx, ptr(files), ptr(shards), ptr(keys), ptr(ans), ptr(dec))
        assert ok == 1, (L, f, k, r)
        cases.append({
            "L": L, "f": f, "k": k, "r": r, "rho": rho, "index": idx,
            "p": p, "n": n, "efs": efs, "nq": nq, "key_len": kl,
            "files_sha256": sha(files),
            "shard_sha256": [sha(shards[i * N * efs:(i + 1) * N * efs]) for i in range(p)],
            "keys": [keys[i * kl:(i + 1) * kl].tobytes().hex() for i in range(p)],
            "answers": [ans[i * nq * efs:(i + 1) * nq * efs].tobytes().hex() for i in range(p)],
            "erasure": [0 if i < r else 1 for i in range(p)],
            "decoded": dec.tobytes().hex(),
        })
        print("e2e case", L, f, k, r, "p", p, "nq", nq)
    write("e2e.json", {"cases": cases})


def thread_defect():
    # server.cpp:505-562 as shipped: documents the defect; NOT a parity target.
    p, n, nq, efs, T = 2, 10, 1, 8, 4
    kl = REF.ref_key_len(p, n, nq)
    fcw = final_cw(p, nq, 1, nq)
    keys = np.zeros(p * kl, np.uint8)
    REF.ref_gen_opt_dpf(n, U64(333), ptr(fcw), p, nq, ptr(keys))
    shard = xorshift_bytes(SHARD_SEED, (1 << n) * efs)
    h = REF.ref_server_new(p, 1, n, efs, nq, ptr(shard), 0, T)
    good = np.zeros(nq * efs, np.uint8)
    bad = np.zeros(nq * efs, np.uint8)
    REF.ref_server_answer(ctypes.c_void_p(h), ptr(keys), ptr(good))
    REF.ref_server_answer_threads(ctypes.c_void_p(h), ptr(keys), T, ptr(bad))
    REF.ref_server_free(ctypes.c_void_p(h))
    c_thr = np.zeros(nq * (1 << n), np.uint8)
    REF.ref_eval_all_opt_thread(p, 0, n, ptr(keys), nq, 0, T, ptr(c_thr))
    write("thread_defect.json", {"p": p, "n": n, "nq": nq, "efs": efs, "threads": T,
                                 "key": keys[:kl].tobytes().hex(), "shard_sha256": sha(shard),
                                 "answer_single": good.tobytes().hex(),
                                 "answer_thread_assembled": bad.tobytes().hex(),
                                 "thread0_c_nonzero": int((c_thr != 0).sum())})


def fullsize():
    """Reference answers at BASELINE sizes: configs[1] (2^20 x 1 KiB, p=2) itself, the C5 party
    shape (p=8, NUM_ROUNDS=5) at 2^18 x 1 KiB and the C3 record size at 2^22 x 256 B.  The
    shard INPUT is xorshift64 (the same generator as above, filled by the test oracle's C
    loop for speed; its first bytes are checked against the Python definition here)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    assert np.array_equal(O.xorshift(SHARD_SEED, 4096), xorshift_bytes(SHARD_SEED, 4096))
    cases = []
    for (p, n, efs, nq, idx) in [(2, 20, 1024, 1, (1 << 20) // 3 + 7), (8, 18, 1024, 5, 77777),
                                 (2, 22, 256, 1, (1 << 22) - 12345)]:
        kl = REF.ref_key_len(p, n, nq)
        fcw = final_cw(p, nq, 1, nq)
        keys = np.zeros(p * kl, np.uint8)
        REF.ref_gen_opt_dpf(n, U64(idx), ptr(fcw), p, nq, ptr(keys))
        shard = O.xorshift(SHARD_SEED, (1 << n) * efs)
        parties = sorted({0, 1, p - 1})
        per = {}
        for party in parties:
            h = REF.ref_server_new(p, party + 1, n, efs, nq, ptr(shard), 0, 1)
            res = np.zeros(nq * efs, np.uint8)
            REF.ref_server_answer(ctypes.c_void_p(h), ptr(keys[party * kl:]), ptr(res))
            REF.ref_server_free(ctypes.c_void_p(h))
            per[str(party)] = {"key": keys[party * kl:(party + 1) * kl].tobytes().hex(),
                               "answer": res.tobytes().hex()}
        cases.append({"p": p, "n": n, "efs": efs, "nq": nq, "index": idx,
                      "final_cw": fcw.tobytes().hex(), "shard_sha256": sha(shard),
                      "parties": per})
        print("fullsize case", p, n, efs, nq)
    write("fullsize.json", {"shard_seed": SHARD_SEED, "cases": cases})


FULL24_CASES = [  # name, p, n, efs, nq, shard seed, [(index, [parties])]
    ("c24", 2, 24, 1024, 1, 0xC24, [((1 << 24) // 3, [0, 1]), ((1 << 24) - 1, [0])]),
    ("c5", 8, 24, 1024, 5, 0xC5, [((1 << 24) // 3 + 5, [0, 1, 7]), (1234567, [0])]),
    ("c3", 2, 24, 256, 1, 0xC3, [(0, [0, 1]), ((1 << 24) - 1, [0]), (9876543, [0, 1]),
                                 ((1 << 23) + 3, [0])]),
]


def fullsize24():
    """Reference answers at the full 2^24-row BASELINE shapes: north_star's 2^24 x 1 KiB (p=2),
    configs[4]'s per-server shape (2^24 x 1 KiB, p=8, NUM_ROUNDS=5) and configs[2]'s
    2^24 x 256 B.  The shard INPUT is the engine's device generator (fill_shard_random,
    k_fill_shard: splitmix64 per 8 bytes), restated by the oracle (orc_splitmix_fill) so the GPU
    tests fill the shard in HBM instead of uploading 16 GiB; the answers are the reference's own
    runOptimizedDPFTreeQuery over that shard (ref_server_view, one thread per call)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    REF.ref_server_view.restype = ctypes.c_void_p
    cases = []
    for (name, p, n, efs, nq, seed, keyspec) in FULL24_CASES:
        N = 1 << n
        kl = REF.ref_key_len(p, n, nq)
        fcw = final_cw(p, nq, 1, nq)
        shard = O.splitmix_shard(seed, 0, N, efs)
        h = REF.ref_server_view(p, 1, n, efs, nq, ptr(shard))
        keys, calls = [], []
        for (idx, parties) in keyspec:
            kk = np.zeros(p * kl, np.uint8)
            REF.ref_gen_opt_dpf(n, U64(idx), ptr(fcw), p, nq, ptr(kk))
            keys.append(kk)
            calls += [(len(keys) - 1, party) for party in parties]
        kbuf = np.concatenate([keys[q][party * kl:(party + 1) * kl] for (q, party) in calls])
        p1 = (ctypes.c_int * len(calls))(*[party + 1 for (_, party) in calls])
        res = np.zeros(len(calls) * nq * efs, np.uint8)
        t0 = __import__("time").time()
        REF.ref_server_answer_many(ctypes.c_void_p(h), ptr(kbuf), kl, p1, len(calls), ptr(res))
        dt = __import__("time").time() - t0
        REF.ref_server_view_free(ctypes.c_void_p(h))
        queries = []
        for q, (idx, _) in enumerate(keyspec):
            per = {}
            for c, (qq, party) in enumerate(calls):
                if qq == q:
                    per[str(party)] = {"key": keys[q][party * kl:(party + 1) * kl].tobytes().hex(),
                                       "answer": res[c * nq * efs:(c + 1) * nq * efs].tobytes().hex()}
            queries.append({"index": idx, "parties": per})
        # a few rows of the input, so the device generator is checked where it is used
        rows = sorted({0, 1, N // 2 + 1, N - 1, keyspec[0][0]})
        cases.append({"name": name, "p": p, "n": n, "efs": efs, "nq": nq, "shard_seed": seed,
                      "final_cw": fcw.tobytes().hex(), "key_len": kl,
                      "shard_sha256_first_mib": sha(shard[:1 << 20]),
                      "sample_rows": {str(r): sha(shard[r * efs:(r + 1) * efs]) for r in rows},
                      "queries": queries, "ref_seconds_parallel": round(dt, 1)})
        del shard
        print("fullsize24 case", name, "calls", len(calls), "%.1f s" % dt)
    write("fullsize24.json", {"generator": "k_fill_shard splitmix64 (oracle orc_splitmix_fill)",
                              "cases": cases})


def hollanti():
    """Polynomial (Hollanti) PIR, mode 3: keys from generateHollantiQuery, encode-within shards,
    every party's runHollantiQuery answer and its T-thread assembled form, the decode."""
    REF.ref_hollanti_e2e.restype = ctypes.c_int
    cases = []
    for (L, f, t, k, r, rho, idx, T) in [(10, 64, 1, 2, 1, 1, 77, 4), (12, 100, 2, 3, 2, 1, 1234, 8),
                                         (11, 48, 1, 4, 1, 1, 5, 2), (9, 33, 1, 1, 0, 1, 511, 1)]:
        s = (ctypes.c_int * 3)()
        REF.ref_hollanti_sizes(L, f, t, k, r, rho, s)
        p, efs, nq = list(s)
        N = 1 << L
        shards = np.zeros(p * N * efs, np.uint8)
        keys = np.zeros(p * nq * N, np.uint8)
        ans = np.zeros(p * nq * efs, np.uint8)
        thr = np.zeros(p * nq * efs, np.uint8)
        dec = np.zeros(f, np.uint8)
        ok = REF.ref_hollanti_e2e(L, f, t, k, r, rho, idx, T, ptr(shards), ptr(keys), ptr(ans),
                                  ptr(thr), ptr(dec))
        assert ok == 1, (L, f, t, k, r, rho)
        assert np.array_equal(ans, thr)
        cases.append({
            "L": L, "f": f, "t": t, "k": k, "r": r, "rho": rho, "index": idx, "threads": T,
            "p": p, "efs": efs, "nq": nq,
            "shard_sha256": [sha(shards[i * N * efs:(i + 1) * N * efs]) for i in range(p)],
            "keys": [keys[i * nq * N:(i + 1) * nq * N].tobytes().hex() for i in range(p)],
            "answers": [ans[i * nq * efs:(i + 1) * nq * efs].tobytes().hex() for i in range(p)],
            "erasure": [0 if i < r else 1 for i in range(p)],
            "decoded": dec.tobytes().hex(),
        })
        print("hollanti case", L, f, t, k, r, rho, "p", p, "nq", nq, "efs", efs)
    write("hollanti.json", {"cases": cases,
                            "shamir_key_len": {str(n): REF.ref_shamir_key_len(n) for n in (1, 2, 7, 10, 20, 25)}})


def client_kats():
    """The client/benchmark names of package c with deterministic outputs: mac (HMAC-SHA256,
    utils.cpp:32-34), choose, calcCDDPFKeyLength, calcWoodruffKeyLength."""
    rng = np.random.RandomState(7)
    macs = []
    for n in (0, 1, 31, 64, 100, 1000):
        key = bytes(rng.randint(0, 256, 16, dtype=np.uint8))
        msg = bytes(rng.randint(0, 256, n, dtype=np.uint8))
        out = np.zeros(32, np.uint8)
        REF.ref_mac(key, msg, n, ptr(out))
        macs.append({"key": key.hex(), "msg": msg.hex(), "mac": out.tobytes().hex()})
    choose = {f"{n},{k}": REF.ref_choose(n, k) for n in range(0, 17) for k in range(0, n + 1)}
    cd = {f"{p},{n},{t},{a},{b}": REF.ref_cd_key_len(p, n, t, a, b)
          for (p, n, t, a, b) in [(5, 10, 3, 4, 2), (7, 12, 3, 6, 3), (8, 16, 3, 5, 3),
                                  (16, 11, 8, 6, 3)]}
    wd = {f"{p},{r},{t},{n},{f}": REF.ref_woodruff_key_len(p, r, t, n, f)
          for (p, r, t, n, f) in [(4, 1, 1, 4, 8), (6, 2, 2, 10, 64), (3, 0, 1, 16, 32),
                                  (5, 1, 2, 20, 1024)]}
    write("client_kat.json", {"mac": macs, "choose": choose, "cd_key_len": cd,
                              "woodruff_key_len": wd})


MP_CASES = [  # (p, t, n, efs, threads): shares per record 2/3/4/5/9, short rows, mu_pow > n
    (3, 1, 10, 64, 4), (3, 1, 11, 37, 2), (4, 1, 12, 48, 8), (4, 2, 9, 20, 1), (3, 1, 4, 16, 1),
    (3, 1, 3, 8, 1), (5, 1, 10, 32, 2), (3, 2, 10, 64, 1), (6, 1, 8, 16, 2), (7, 1, 4, 8, 1),
    (10, 1, 10, 16, 1)]


def mp():
    """Multiparty sqrt(N) DPF server path (mode 1) on synthetic keys (tests/_oracle.mp_key: the
    reference's own keygen leaves the toggle bytes unset): the shares of evalAllOptMultiPartyDPF
    and of its Thread form, runOptimizedMultiPartyDPFQuery, and the thread-assembled answer."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    REF.ref_mp_key_len.restype = ctypes.c_int
    cases = []
    for (p, t, n, efs, T) in MP_CASES:
        z = O.mp_sizes(p, n, t)
        nrk, N = z["nrk"], 1 << n
        assert REF.ref_mp_key_len(p, n, t) == z["key_len"]
        kseed, sseed = 0x5EED0000 + 97 * n + p, 0xD00D0000 + 13 * n + t
        key = O.mp_key(p, n, t, kseed)
        shard = O.xorshift(sseed, N * efs)
        shares = np.zeros(nrk * N, np.uint8)
        REF.ref_mp_eval(p, n, t, nrk, ptr(key), 0, 0, ptr(shares))
        thr_shares = []
        for th in range(T):
            o = np.zeros(nrk * N, np.uint8)
            REF.ref_mp_eval(p, n, t, nrk, ptr(key), th, T, ptr(o))
            thr_shares.append(sha(o))
        h = REF.ref_server_new(p, 1, n, efs, nrk, ptr(shard), 0, T)
        ans = np.zeros(nrk * efs, np.uint8)
        REF.ref_mp_server_answer(ctypes.c_void_p(h), p, t, nrk, ptr(key), 0, ptr(ans))
        tans = np.zeros(nrk * efs, np.uint8)
        REF.ref_mp_server_answer(ctypes.c_void_p(h), p, t, nrk, ptr(key), T, ptr(tans))
        REF.ref_server_free(ctypes.c_void_p(h))
        cases.append({"p": p, "t": t, "n": n, "efs": efs, "threads": T, "key_seed": kseed,
                      "shard_seed": sseed, "sizes": z, "key_sha256": sha(key),
                      "shares_sha256": sha(shares), "thread_shares_sha256": thr_shares,
                      "answer": ans.tobytes().hex(), "thread_answer": tans.tobytes().hex()})
        print("mp case", p, t, n, efs, T, z)
    sizes = []
    for (L, f, t, k, r, b, rho) in [(10, 64, 1, 1, 1, 0, 1), (12, 100, 1, 2, 1, 0, 1),
                                    (11, 48, 2, 1, 1, 0, 1), (10, 32, 1, 1, 0, 1, 1)]:
        s = (ctypes.c_int * 5)()
        REF.ref_mp_sizes(L, f, t, k, r, b, rho, s)
        sizes.append({"L": L, "f": f, "t": t, "k": k, "r": r, "b": b, "rho": rho,
                      "p": s[0], "n": s[1], "efs": s[2], "nrk": s[3], "key_len": s[4]})
    write("multiparty.json", {"cases": cases, "setup_sizes": sizes})


CD_CASES = [  # (L, f, t, k, r, b, rho, index, threads, decode): P = 8 (CD842, the reference's
    # own runCDPirTests setup, correctness_tests.cpp:1236), 16 (CD1682), 14 (CD1472), 12 (CD1262).
    # genCDDPF puts index a at row gamma = a >> (n/2), column delta = a mod 2^(n/2)
    # (multiparty_dpf.cpp:283-284) and reads s[gamma] of nu = 2^(n - n/2 - 3) rows: an index with
    # gamma >= nu reads past its seed array, so the indices below keep gamma < nu (gamma > 0 in
    # the last three, decode off: their point is record gamma*mu + delta, not a)
    (15, 8, 2, 2, 0, 1, 1, 1, 4, 1), (12, 64, 2, 4, 0, 2, 1, 3 * 32 + 5, 2, 0),
    (13, 40, 2, 3, 1, 2, 1, 6 * 64 + 9, 8, 0), (11, 33, 2, 4, 0, 1, 1, 2 * 16 + 3, 1, 0)]


def cd():
    """Covering-design sqrt(N) DPF PIR (mode 4): the reference's own CD harness with its own key
    generation (generateCDQuery -> genCDDPF), encode-across shards, every party's answer from
    runCDQueryThread slices + assembleCDQueryThreadResults, and the decode.  Keys are kept for
    three parties per case (first, middle, last) to bound the fixture's size."""
    REF.ref_cd_sizes.restype = None
    cases = []
    for (L, f, t, k, r, b, rho, idx, T, dec_ok) in CD_CASES:
        s = (ctypes.c_int * 6)()
        REF.ref_cd_sizes(L, f, t, k, r, b, rho, s)
        p, n, efs, nck, qn, kl = list(s)
        N = 1 << n
        shards = np.zeros(p * N * efs, np.uint8)
        keys = np.zeros(p * kl, np.uint8)
        ans = np.zeros(p * nck * efs, np.uint8)
        dec = np.zeros(f, np.uint8)
        ok = REF.ref_cd_e2e(L, f, t, k, r, b, rho, idx, T, int(dec_ok), ptr(shards), ptr(keys), ptr(ans), ptr(dec))
        kept = sorted({0, p // 2, p - 1})
        cases.append({
            "L": L, "f": f, "t": t, "k": k, "r": r, "b": b, "rho": rho, "index": idx, "threads": T,
            "p": p, "n": n, "efs": efs, "num_cd_keys": nck, "num_cd_keys_needed": qn,
            "key_len": kl, "decoded_ok": int(ok),  # -1: decode not run
            "shard_sha256": [sha(shards[i * N * efs:(i + 1) * N * efs]) for i in range(p)],
            "key_sha256": [sha(keys[i * kl:(i + 1) * kl]) for i in range(p)],
            "keys": {str(i + 1): keys[i * kl:(i + 1) * kl].tobytes().hex() for i in kept},
            "answers": [ans[i * nck * efs:(i + 1) * nck * efs].tobytes().hex() for i in range(p)],
        })
        print("cd case", L, f, t, k, r, b, "p", p, "n", n, "keys", nck, "/", qn, "kl", kl, "ok", ok)
    write("cd.json", {"cases": cases})


if __name__ == "__main__":
    REF.ref_server_new.restype = ctypes.c_void_p
    REF.ref_blen.restype = ctypes.c_uint32
    for fn in (REF.ref_gf_mul, REF.ref_gf_pow, REF.ref_gf_inv):
        fn.restype = ctypes.c_uint8
    what = sys.argv[1:] or ["prg", "gf", "dpf", "e2e", "thread", "fullsize", "hollanti", "mp", "client", "cd"]
    if "prg" in what: prg_kats()
    if "gf" in what: gf_kats()
    if "dpf" in what: dpf_and_answers()
    if "e2e" in what: e2e()
    if "thread" in what: thread_defect()
    if "fullsize" in what: fullsize()
    if "fullsize24" in what: fullsize24()
    if "client" in what: client_kats()
    if "hollanti" in what: hollanti()
    if "mp" in what: mp()
    if "cd" in what: cd()
