"""Covering-design (CD) sqrt(N) DPF PIR, mode 4 -- SURVEY.md 8(f) item 4 ("the multiparty/CD
sqrt(N) DPF"): evalAllCDThread (src/c/multiparty_dpf.cpp:617-690) + the GF(2^8) shard scan of
runCDQueryThread (src/c/server.cpp:443-492) on the engine (pir_engine_answer_cd, the shim's
runCDQueryThread).  The evaluation is the multiparty one on another layout: NUM_CD_KEYS shares,
2^(NUM_CD_KEYS_NEEDED-1) seeds a row, mu = 2^(n/2 + 3) records a row.

Fixtures (tests/golden/cd.json, tests/golden/make_golden.py cd): the reference's own CD harness
(runCDPirTests, correctness_tests.cpp:568-715 -- its one active test, main :1236) compiled in
oracle/_ref: setSystemParams(mode 4), its own key generation (generateCDQuery -> genCDDPF), the
encode-across shards, every party's T-thread assembled answer, and (first case) the decode.
Cases: the reference's P = 8 (CD842) setup and P = 16 / 14 / 12 (CD1682 / CD1472 / CD1262).
"""
import numpy as np
import pytest

import _oracle as O

CASES = O.golden("cd.json")["cases"]


def _shard(c, party):
    files = O.synthetic_db(c["L"], c["f"])
    return O.encode_across(c["L"], c["f"], c["k"], c["p"], party, files)


def _ans(c, party):
    return np.frombuffer(bytes.fromhex(c["answers"][party - 1]), np.uint8).reshape(
        c["num_cd_keys"], c["efs"])


def _key(c, party):
    return np.frombuffer(bytes.fromhex(c["keys"][str(party)]), np.uint8).copy()


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_oracle_matches_reference(ci):
    """The C restatement (orc_cd_*) reproduces the reference's answers from its own keys and
    shards, whole-domain and as the XOR of the T thread slices (pins the GPU tests' checker)."""
    c = CASES[ci]
    n, qn, nck, efs, T = c["n"], c["num_cd_keys_needed"], c["num_cd_keys"], c["efs"], c["threads"]
    assert O.cd_sizes(n, qn, nck)["key_len"] == c["key_len"]
    assert c["decoded_ok"] in (1, -1)
    for party in map(int, c["keys"]):
        shard, key = _shard(c, party), _key(c, party)
        assert O.sha(shard) == c["shard_sha256"][party - 1]
        assert O.sha(key) == c["key_sha256"][party - 1]
        assert np.array_equal(O.cd_answer(n, qn, nck, efs, key, shard), _ans(c, party)), party
        acc = np.zeros((nck, efs), np.uint8)
        for th in range(T):
            acc ^= O.cd_answer(n, qn, nck, efs, key, shard, th, T)
        assert np.array_equal(acc, _ans(c, party)), party


def test_reference_answers_reconstruct_the_record():
    """The first case's answers decode to the record in the reference (decoded_ok), and the
    parties' shares of it are consistent: every key's shares XOR, over the covering design, to
    a point function -- here checked as: the answers are not all zero and differ by party."""
    c = CASES[0]
    assert c["decoded_ok"] == 1
    assert len({a for a in c["answers"]}) == c["p"]


def test_sizes_match_reference():
    """setSystemParams(mode 4) sizing + covering-design selection (params.cpp:434-447,
    :519-599) and calcCDDPFKeyLength == the reference's; host code only."""
    import erasurecodedpir_amd as pir
    from erasurecodedpir_amd import _lib, server as S
    for c in CASES:
        S.setSystemParams(c["L"], c["f"], c["t"], c["k"], c["r"], c["b"], c["rho"], 0, 4)
        got = [_lib.global_int(g) for g in ("NUM_PARTIES", "LOG_NUM_ENCODED_FILES",
                                            "ENCODED_FILE_SIZE_BYTES", "NUM_CD_KEYS",
                                            "NUM_CD_KEYS_NEEDED", "ENCODE_ACROSS")]
        assert got == [c["p"], c["n"], c["efs"], c["num_cd_keys"], c["num_cd_keys_needed"], 1], c
        assert S.calcCDDPFKeyLength(c["p"], c["n"], c["t"], c["num_cd_keys_needed"],
                                    c["num_cd_keys"]) == c["key_len"]
        assert pir.cd_key_len(c["p"], c["n"], c["t"], c["num_cd_keys_needed"],
                              c["num_cd_keys"]) == c["key_len"]
    # every setSystemParams starts from M = 4 (as a fresh reference process would): the M = 2 of
    # the K = 2, B = 1 setup does not leak into the next one
    S.setSystemParams(15, 8, 2, 2, 0, 1, 1, 0, 4)
    assert _lib.global_int("NUM_PARTIES") == 8
    S.setSystemParams(11, 33, 2, 4, 0, 1, 1, 0, 4)
    assert _lib.global_int("NUM_PARTIES") == 12 and _lib.global_int("NUM_CD_KEYS") == 3
    # mu > 2^n: no rows (the reference's (uint64_t)pow(2, negative) == 0), a zero answer
    assert O.cd_sizes(4, 6, 3)["nu"] == 0
    assert pir.cd_key_len(8, 4, 2, 6, 3) == O.cd_sizes(4, 6, 3)["key_len"]


# ------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_gpu_cd_matches_reference(ci):
    """Engine answer from the reference's own key == the reference's assembled answer (whole
    domain, and the XOR of the T thread slices, each slice == the oracle's)."""
    import erasurecodedpir_amd as pir
    c = CASES[ci]
    n, qn, nck, efs, T = c["n"], c["num_cd_keys_needed"], c["num_cd_keys"], c["efs"], c["threads"]
    for party in map(int, c["keys"]):
        shard, key = _shard(c, party), _key(c, party)
        with pir.Engine(2, 1, n, efs, nck) as e:
            e.set_shard(shard)
            full = e.answer_cd(key, qn, nck)
            parts = [e.answer_cd(key, qn, nck, th, T) for th in range(T)]
        assert np.array_equal(full, _ans(c, party)), party
        acc = np.zeros_like(full)
        for th, a in enumerate(parts):
            assert np.array_equal(a, O.cd_answer(n, qn, nck, efs, key, shard, th, T)), (party, th)
            acc ^= a
        assert np.array_equal(acc, _ans(c, party)), party


@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_gpu_cd_shim_matches_reference(ci):
    """The Go-bound names (cd732.go:64): setSystemParams(mode 4), a server whose shard the shim's
    encode_across_files_server computes on the GPU, T runCDQueryThread slices +
    assembleCDQueryThreadResults == the reference's answer for every kept party."""
    from erasurecodedpir_amd import server as S
    c = CASES[ci]
    T = c["threads"]
    S.setSystemParams(c["L"], c["f"], c["t"], c["k"], c["r"], c["b"], c["rho"], 0, 4)
    cl = S.Client(c["L"], c["f"])
    for party in map(int, c["keys"]):
        sv = S.Server(party, c["n"], c["efs"], 0, T)
        cl.encode_across_files_server(sv)
        key = _key(c, party)
        parts = np.stack([sv.runCDQueryThread(key, th, T) for th in range(T)])
        asm = S.assembleCDQueryThreadResults(sv, parts)
        sv.freeServer()
        assert np.array_equal(asm, _ans(c, party)), party
    cl.free_client()


@pytest.mark.gpu
@pytest.mark.parametrize("n,qn,nck,efs,T", [
    (14, 11, 7, 64, 4),    # CD832: 1024 seeds a row, 7 shares (8-byte share records)
    (13, 12, 8, 40, 2),    # CD932: 2048 seeds a row, 8 shares
    (9, 8, 5, 33, 1),      # CD942, odd n and ragged rows
    (18, 6, 3, 256, 8),    # 2^18 x 256 B, 64 rows of 4096 records
    (6, 4, 2, 16, 1),      # mu = 2^6 = the whole domain: one row
    (4, 6, 3, 16, 1),      # mu > 2^n: no rows, zero answer
])
def test_gpu_cd_synthetic_keys(n, qn, nck, efs, T):
    """Synthetic keys over the other covering designs' counts (seed counts up to 2^11, 5-8
    shares) and the edge layouts: engine == oracle, whole and per slice; device-key form from an
    unaligned pointer == the host form."""
    import erasurecodedpir_amd as pir
    key = O.cd_key(n, qn, nck, 1000 * n + qn)
    shard = O.xorshift(31 * n + nck, (1 << n) * efs)
    with pir.Engine(2, 1, n, efs, nck) as e:
        e.set_shard(shard)
        full = e.answer_cd(key, qn, nck)
        parts = [e.answer_cd(key, qn, nck, th, T) for th in range(T)]
        d_k = e.alloc_dev(key.size + 1)
        d_r = e.alloc_dev(nck * efs)
        e.h2d(d_k + 1, key)
        e.answer_cd_dev(d_k + 1, qn, nck, d_r)
        e.sync()
        dev = e.d2h(d_r, nck * efs).reshape(nck, efs)
    want = O.cd_answer(n, qn, nck, efs, key, shard)
    assert np.array_equal(full, want)
    assert np.array_equal(dev, want)
    for th in range(T):
        assert np.array_equal(parts[th], O.cd_answer(n, qn, nck, efs, key, shard, th, T)), th
    if O.cd_sizes(n, qn, nck)["nu"] == 0:
        assert not full.any()


@pytest.mark.gpu
def test_gpu_cd_rejects_bad_arguments():
    import erasurecodedpir_amd as pir
    key = O.cd_key(12, 6, 3, 5)
    with pir.Engine(2, 1, 12, 64, 3) as e:
        with pytest.raises(pir.PirError):
            e.answer_cd(key, 6, 2)  # 2 shares, engine has 3 rounds
        with pytest.raises(pir.PirError):
            e.answer_cd(key[:100], 6, 3)  # shorter than the evaluation reads
        with pytest.raises(pir.PirError):
            e.answer_cd(key, 6, 3, 4, 4)  # thread 4 of 4
        with pytest.raises(pir.PirError):
            e.answer_cd(key, 0, 3)  # no layout


@pytest.mark.gpu
@pytest.mark.parametrize("kind,a,b,nrk,n,efs", [
    # n >= 19: k_query takes a domain of >= 2 tiles of 1024 leaves per CU (fused_tile)
    ("cd", 6, 3, 3, 19, 1024),    # CD842 counts: 32 seeds a row of 4096 records, 3 shares
    ("cd", 7, 4, 4, 20, 512),     # CD732 counts: 64 seeds, 4 shares (the four-Russians k_query)
    ("mp", 3, 1, 2, 19, 1024),    # multiparty p = 3, t = 1: 4 seeds a row of 2048 records
    ("mp", 4, 1, 3, 19, 1040),    # p = 4: 8 seeds, 3 shares, ragged records
])
def test_gpu_sqrtn_in_k_query(kind, a, b, nrk, n, efs, monkeypatch):
    """Whole-domain multiparty / covering-design answers through k_query's sqrt(N) mode
    ($PIR_MP_FUSED=2: forced, an answer it cannot take fails; the tree waves build each tile's
    shares from the key, mp_tile) == the two-kernel path ($PIR_MP_FUSED=0: k_mp_shares + the
    scan) == the oracle, twice on one engine."""
    import erasurecodedpir_amd as pir
    if kind == "cd":
        key = O.cd_key(n, a, b, 77 * n + a)
        want = lambda k, sh: O.cd_answer(n, a, b, efs, k, sh)  # noqa: E731
    else:
        key = O.mp_key(a, n, b, 55 * n + a)
        want = lambda k, sh: O.mp_answer(a, b, n, efs, k, sh)  # noqa: E731
    shard = O.xorshift(3 * n + nrk, (1 << n) * efs)
    got = {}
    for mode in ("2", "0"):
        monkeypatch.setenv("PIR_MP_FUSED", mode)
        with pir.Engine(2, 1, n, efs, nrk) as e:
            e.set_shard(shard)
            ans = (lambda k: e.answer_cd(k, a, b)) if kind == "cd" else (lambda k: e.answer_mp(k, a, b))
            got[mode] = [ans(key), ans(key)]
    assert np.array_equal(got["2"][0], got["2"][1])
    assert np.array_equal(got["2"][0], got["0"][0])
    assert np.array_equal(got["2"][0], want(key, shard))


@pytest.mark.gpu
@pytest.mark.parametrize("kind,a,b,nrk", [
    ("cd", 6, 3, 3),   # the bench's ccd: CD842 counts, four-Russians k_query at 3 shares
    ("cd", 7, 4, 4),   # ccd7: CD732 counts
    ("mp", 4, 1, 3),   # cm4: multiparty p = 4, t = 1
])
def test_gpu_sqrtn_fullsize(kind, a, b, nrk, monkeypatch):
    """At the bench shape (2^24 x 1 KiB, device-generated shard): k_query's sqrt(N) mode (the
    default for >= 3 shares) == the two-kernel path == the XOR of 4 thread slices (which always
    take the two-kernel path) -- the same answer by three routes; the oracle pins both paths at
    2^19-2^20 (test_gpu_sqrtn_in_k_query)."""
    import erasurecodedpir_amd as pir
    n, efs = 24, 1024
    key = O.cd_key(n, a, b, 5 + a) if kind == "cd" else O.mp_key(a, n, b, 9 + a)
    with pir.Engine(2, 1, n, efs, nrk) as e:
        e.fill_shard_random(11)
        ans = (lambda *s: e.answer_cd(key, a, b, *s)) if kind == "cd" else (lambda *s: e.answer_mp(key, a, b, *s))
        monkeypatch.setenv("PIR_MP_FUSED", "2")
        fused = ans()
        monkeypatch.setenv("PIR_MP_FUSED", "0")
        two = ans()
        monkeypatch.delenv("PIR_MP_FUSED")
        dflt = ans()
        sl = [ans(t, 4) for t in range(4)]
    acc = np.zeros_like(two)
    for s in sl:
        acc ^= s
    assert fused.any()
    assert np.array_equal(fused, two)
    assert np.array_equal(dflt, fused)
    assert np.array_equal(acc, two)
