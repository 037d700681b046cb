"""Polynomial (Hollanti) PIR, mode 3 -- SURVEY.md 8(f) item 4: the explicit-coefficient scan on
the engine's GF(2^8) kernel (runHollantiQuery / runHollantiQueryThread, src/c/server.cpp:321-382)
and the shim's setup / client pieces around it (encode_within_files_server, client.cpp:99-103;
assembleHollantiResponses, client.cpp:499-552).

Golden fixtures (tests/golden/hollanti.json) are the reference's own outputs: keys from its
generateHollantiQuery (RAND_bytes, so stored), shard hashes from its encode_within_files_server,
answers from its runHollantiQuery (and the same from its T-thread form), the decode of the
answers with the first r servers erased.  CPU tests pin the host pieces; -m gpu tests the scan.
"""
import numpy as np
import pytest

import _oracle as O


def _setup(case):
    from erasurecodedpir_amd import server as S
    S.setSystemParams(case["L"], case["f"], case["t"], case["k"], case["r"], 0, case["rho"], 0, 3)
    return S


def _keys(case, party):
    N = 1 << case["L"]
    return np.frombuffer(bytes.fromhex(case["keys"][party]), np.uint8).reshape(case["nq"], N)


def _answers(case, party):
    return np.frombuffer(bytes.fromhex(case["answers"][party]), np.uint8).reshape(case["nq"], case["efs"])


@pytest.mark.parametrize("ci", range(4))
def test_encode_within_matches_reference(ci):
    """The shim's encode_within_files_server rows == the reference's (per-party shard hash)."""
    case = O.golden("hollanti.json")["cases"][ci]
    S = _setup(case)
    cl = S.Client(case["L"], case["f"])
    N = 1 << case["L"]
    for party in range(case["p"]):
        sv = S.Server(party + 1, case["L"], case["efs"])
        cl.encode_within_files_server(sv)
        rows = np.stack([sv.read_row(i) for i in range(N)])
        assert O.sha(rows) == case["shard_sha256"][party], party
        sv.freeServer()
    cl.free_client()


@pytest.mark.parametrize("ci", range(4))
def test_decode_reference_answers(ci):
    """assembleHollantiResponses on the reference's answers, first r servers erased == the
    reference's decode == the file; also with the LAST r servers erased."""
    case = O.golden("hollanti.json")["cases"][ci]
    S = _setup(case)
    p, r = case["p"], case["r"]
    ans = [_answers(case, q) for q in range(p)]
    files = O.synthetic_db(case["L"], case["f"]).reshape(-1, case["f"])
    want = files[case["index"]]
    for er in (case["erasure"], [1] * (p - r) + [0] * r):
        kept = np.stack([ans[q] for q in range(p) if er[q]])
        dec = S.assembleHollantiResponses(er, kept)
        assert np.array_equal(dec, want)
    assert dec.tobytes().hex() == case["decoded"] or r == 0


def test_scan_oracle_matches_reference_answers():
    """The oracle's explicit-coefficient scan reproduces the reference answers (pins the
    checker used by the GPU tests below)."""
    case = O.golden("hollanti.json")["cases"][0]
    S = _setup(case)
    cl = S.Client(case["L"], case["f"])
    for party in range(case["p"]):
        sv = S.Server(party + 1, case["L"], case["efs"])
        cl.encode_within_files_server(sv)
        shard = np.stack([sv.read_row(i) for i in range(1 << case["L"])]).reshape(-1)
        got = O.scan(_keys(case, party), shard, case["efs"])
        assert np.array_equal(got, _answers(case, party))
        sv.freeServer()
    cl.free_client()


# ------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(4))
def test_gpu_hollanti_golden_end_to_end(ci):
    """setSystemParams(mode 3) -> encode_within_files_server -> runHollantiQuery on the GPU ==
    the reference's answers; T runHollantiQueryThread slices + assemble == the same; decode."""
    case = O.golden("hollanti.json")["cases"][ci]
    S = _setup(case)
    p, T, N = case["p"], case["threads"], 1 << case["L"]
    cl = S.Client(case["L"], case["f"])
    got = []
    for party in range(p):
        sv = S.Server(party + 1, case["L"], case["efs"], 0, T)
        cl.encode_within_files_server(sv)
        keys = _keys(case, party)
        a = sv.runHollantiQuery(keys)
        assert a.tobytes().hex() == case["answers"][party], party
        sl = N // T
        parts = np.stack([sv.runHollantiQueryThread(keys, t, t * sl, (t + 1) * sl) for t in range(T)])
        assert np.array_equal(S.assembleHollantiQueryThreadResults(sv, parts), a)
        got.append(a)
        sv.freeServer()
    cl.free_client()
    kept = np.stack([got[q] for q in range(p) if case["erasure"][q]])
    assert S.assembleHollantiResponses(case["erasure"], kept).tobytes().hex() == case["decoded"]


@pytest.mark.gpu
@pytest.mark.parametrize("n,efs,nq", [(10, 64, 1), (12, 1024, 3), (13, 100, 16), (16, 256, 2),
                                      (14, 8, 5), (18, 1056, 4),
                                      # k_scan_uni shapes: VEC 4 -> 2 fallback (512 B, 3 rounds),
                                      # several column groups (2 KiB, 1040 B), plane-table rounds
                                      # 6-8, VEC 1 for 9-16, a 1-row range
                                      (11, 512, 3), (11, 2048, 3), (12, 1040, 2), (11, 1024, 7),
                                      (10, 1024, 8), (9, 2048, 12), (13, 4096, 1), (7, 1024, 3),
                                      # one dword per lane, 4-8 rounds: four-Russians folds
                                      (12, 256, 5), (11, 300, 8), (12, 400, 4), (10, 256, 6),
                                      (7, 256, 7),
                                      # two dwords per lane, 4-5 rounds: the 768-thread kernel
                                      (12, 1024, 5), (11, 512, 4), (10, 2048, 5), (9, 1040, 5),
                                      # 3 rounds, 256-511 B: one record per row at VEC 1
                                      (11, 256, 3), (10, 300, 3), (10, 508, 3)])
def test_gpu_answer_coefs_vs_oracle(n, efs, nq):
    import erasurecodedpir_amd as pir
    rng = np.random.default_rng(n * 131 + nq)
    shard = rng.integers(0, 256, (1 << n) * efs, dtype=np.uint8)
    coefs = rng.integers(0, 256, (nq, 1 << n), dtype=np.uint8)
    with pir.Engine(2, 1, n, efs, nq) as e:
        e.set_shard(shard)
        full = e.answer_coefs(coefs)
        lo, hi = (1 << n) // 3, (1 << n) - 7
        part = e.answer_coefs(coefs, lo, hi - lo)
        empty = e.answer_coefs(coefs, 5, 0)
        one = e.answer_coefs(coefs, 77, 1)
    assert np.array_equal(full, O.scan(coefs, shard, efs))
    assert np.array_equal(part, O.scan(coefs, shard, efs, lo, hi))
    assert np.array_equal(one, O.scan(coefs, shard, efs, 77, 78))
    assert not empty.any()


@pytest.mark.gpu
def test_gpu_answer_coefs_full_size_linearity():
    """2^24 x 1 KiB, 3 rounds: changing one coefficient by x changes that round's answer by
    x * record (GF(2^8) linearity, size-independent); the device-resident form agrees."""
    import erasurecodedpir_amd as pir
    n, efs, nq = 24, 1024, 3
    N = 1 << n
    rng = np.random.default_rng(24)
    coefs = rng.integers(0, 256, (nq, N), dtype=np.uint8)
    i, a, x = 12345678, 1, 0x5B
    with pir.Engine(2, 1, n, efs, nq) as e:
        e.fill_shard_random(0x401)
        base = e.answer_coefs(coefs)
        c2 = coefs.copy()
        c2[a, i] ^= x
        moved = e.answer_coefs(c2)
        rec = e.shard_row(i)
        d_c = e.alloc_dev(nq * N)
        d_r = e.alloc_dev(nq * efs)
        e.h2d(d_c, coefs.reshape(-1))
        e.answer_coefs_dev(d_c, N, 0, N, d_r)
        e.sync()
        dev = e.d2h(d_r, nq * efs).reshape(nq, efs)
    tab = np.array([O.gf_mul(x, v) for v in range(256)], np.uint8)
    delta = base ^ moved
    assert np.array_equal(delta[a], tab[rec])
    assert not delta[[r for r in range(nq) if r != a]].any()
    assert np.array_equal(dev, base)


# ---------------------------------------------------------- the Hollanti shard on the GPU
@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(4))
def test_gpu_encode_within_matches_reference(ci):
    """k_encode_within (pir_engine_encode_within_dev: the server setup of MODE 3 in pir_serve)
    == the reference's encode_within_files_server rows (per-party shard hash), from the
    synthetic database and from explicit files."""
    import erasurecodedpir_amd as pir
    case = O.golden("hollanti.json")["cases"][ci]
    L, f, efs, k, nq = case["L"], case["f"], case["efs"], case["k"], case["nq"]
    files = O.synthetic_db(L, f).reshape(1 << L, f)
    for party in range(case["p"]):
        with pir.Engine(2, 1, L, efs, nq) as e:
            e.encode_within(1 << L, f, k, party=party + 1)
            assert O.sha(e.get_shard()) == case["shard_sha256"][party], party
            e.encode_within(1 << L, f, k, files=files, party=party + 1)
            assert O.sha(e.get_shard()) == case["shard_sha256"][party], party


@pytest.mark.gpu
def test_gpu_encode_within_random_files_and_partitions():
    """Random files, a file size that is not a multiple of k, split-shard partitions: the GPU
    rows equal a numpy restatement of client.cpp:99-103 (coefficients gf_pow(party, j))."""
    import erasurecodedpir_amd as pir
    L, f, k, party = 12, 1000, 3, 4
    efs = -(-f // k)
    rng = np.random.default_rng(9)
    files = rng.integers(0, 256, (1 << L, f), dtype=np.uint8)
    pad = np.zeros((1 << L, k * efs), np.uint8)
    pad[:, :f] = files
    want = np.zeros((1 << L, efs), np.uint8)
    for j in range(k):
        c = O.gf_pow(party, j)
        tab = np.array([O.gf_mul(x, c) for x in range(256)], np.uint8)
        want ^= tab[pad[:, j * efs:(j + 1) * efs]]
    G = 2
    rows = (1 << L) >> G
    for part in range(1 << G):
        with pir.Engine(2, 1, L, efs, 1, log_num_partitions=G, partition_index=part) as e:
            e.encode_within(1 << L, f, k, files=files, party=party)
            assert np.array_equal(e.get_shard(), want[part * rows:(part + 1) * rows]), part
