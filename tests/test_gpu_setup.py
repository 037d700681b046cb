"""The drop-in's SETUP on the GPU (src/server/server.go:299-331: setSystemParams ->
initialize_client -> initializeServer -> encode_{across,within}_files_server): the shim encodes
the shard from the client's HOST file rows on the engine (pir_engine_encode_*_rows: pinned,
double-buffered, multi-threaded staging) and leaves it resident in HBM, so the first query is a
device-resident answer; indexList is materialised from the device copy only when the host rows
are read or written (pirServerSyncRows, pirServerSetRows, an engine re-creation, a second
encode).  Checked against the plain-C oracle's encode (oracle/pir_oracle.c, pinned to the
reference's shard hashes) and against the reference's host encode path ($PIR_SHIM_HOST_SETUP=1).
"""
import ctypes

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def S():
    import erasurecodedpir_amd as pir
    pir.load()
    from erasurecodedpir_amd import server
    return server


def _tree_setup(S, L, f, k, r):
    S.setSystemParams(L, f, 1, k, r, 0, 1, 0, 0)
    prm = S.params()
    return (prm["NUM_PARTIES"], prm["LOG_NUM_ENCODED_FILES"], prm["NUM_ROUNDS"],
            prm["ENCODED_FILE_SIZE_BYTES"])


def _rows(sv, n):
    return np.stack([sv.read_row(i) for i in range(1 << n)])


@pytest.mark.parametrize("L,f,k,r", [(12, 64, 1, 1), (13, 1024, 4, 2), (12, 100, 5, 2)])
def test_gpu_setup_matches_oracle_encode(S, L, f, k, r):
    """The GPU-encoded shard (read back through pirServerSyncRows) and every party's first
    answers equal the oracle's encode of the reference's synthetic database and its answers."""
    import erasurecodedpir_amd as pir
    p, n, nq, efs = _tree_setup(S, L, f, k, r)
    cl = S.Client(L, f)
    files = O.synthetic_db(L, f)
    keys = pir.gen_keys(n, (1 << n) // 3, p, nq, fcw=O.final_cw(p, nq, 1))
    for party in sorted({1, 2, p}):
        sv = S.Server(party, L, efs, 0, 4)
        cl.encode_across_files_server(sv)
        want = O.encode_across(L, f, k, p, party, files)
        # first query straight after the setup: the device-resident shard
        got = sv.runOptimizedDPFTreeQuery(keys[party - 1], nq)
        assert np.array_equal(got, O.answer(p, party, n, efs, nq, keys[party - 1], want)), party
        assert np.array_equal(_rows(sv, n).reshape(-1), want), party
        sv.freeServer()
    cl.free_client()


def test_gpu_setup_equals_host_setup(S, monkeypatch):
    """$PIR_SHIM_HOST_SETUP=1 (the reference's host encode into indexList, uploaded on the first
    query) and the GPU setup give the same rows and the same T-thread answers."""
    import erasurecodedpir_amd as pir
    L, f, k, r, T = 14, 256, 5, 2, 8
    p, n, nq, efs = _tree_setup(S, L, f, k, r)
    cl = S.Client(L, f)
    keys = pir.gen_keys(n, 77, p, nq, fcw=O.final_cw(p, nq, 1))
    out = {}
    for mode in ("gpu", "host"):
        if mode == "host":
            monkeypatch.setenv("PIR_SHIM_HOST_SETUP", "1")
        sv = S.Server(3, L, efs, 0, T)
        cl.encode_across_files_server(sv)
        out[mode] = (sv.runTreeQueryThreads(keys[2], T), _rows(sv, n))
        sv.freeServer()
    cl.free_client()
    assert np.array_equal(out["gpu"][0], out["host"][0])
    assert np.array_equal(out["gpu"][1], out["host"][1])


def test_gpu_setup_then_set_rows_keeps_other_rows(S):
    """pirServerSetRows after a GPU setup first syncs the device shard down, so the rows it does
    not write keep the encoded values (and the next answer sees both)."""
    import erasurecodedpir_amd as pir
    L, f, k, r = 12, 128, 2, 1
    p, n, nq, efs = _tree_setup(S, L, f, k, r)
    cl = S.Client(L, f)
    want = O.encode_across(L, f, k, p, 2, O.synthetic_db(L, f)).reshape(-1, efs)
    sv = S.Server(2, L, efs)
    cl.encode_across_files_server(sv)
    new = np.random.default_rng(5).integers(0, 256, (16, efs), dtype=np.uint8)
    sv.write_rows(new, row0=100)
    want[100:116] = new
    assert np.array_equal(_rows(sv, n), want)
    key = pir.gen_keys(n, 105, p, nq, fcw=O.final_cw(p, nq, 1))[1]
    assert np.array_equal(sv.runOptimizedDPFTreeQuery(key, nq),
                          O.answer(p, 2, n, efs, nq, key, want.reshape(-1)))
    sv.freeServer()
    cl.free_client()


def test_gpu_setup_survives_engine_recreation(S):
    """An engine re-creation after a GPU setup (here: isByzantine toggled in the server struct,
    a config change) first syncs the only copy of the shard down into indexList, then the new
    engine uploads it: honest answers before and after are the oracle's."""
    import erasurecodedpir_amd as pir
    L, f, k, r = 12, 64, 1, 1
    p, n, nq, efs = _tree_setup(S, L, f, k, r)
    cl = S.Client(L, f)
    shard = O.encode_across(L, f, k, p, 1, O.synthetic_db(L, f))
    key = pir.gen_keys(n, 9, p, nq)[0]
    want = O.answer(p, 1, n, efs, nq, key, shard)
    sv = S.Server(1, L, efs)
    cl.encode_across_files_server(sv)
    assert np.array_equal(sv.runOptimizedDPFTreeQuery(key, nq), want)
    sv.s.isByzantine = 1
    byz = sv.runOptimizedDPFTreeQuery(key, nq)  # random answers (server.cpp:116-119)
    assert byz.shape == want.shape
    sv.s.isByzantine = 0
    assert np.array_equal(sv.runOptimizedDPFTreeQuery(key, nq), want)
    assert np.array_equal(_rows(sv, n).reshape(-1), shard)
    sv.freeServer()
    cl.free_client()


def test_second_encode_xors_like_the_reference(S):
    """The reference XORs an encode INTO the rows (client.cpp:88): a second
    encode_across_files_server on the same server leaves all-zero rows; the shim takes the host
    path for it (after syncing the GPU setup's rows down)."""
    L, f, k, r = 11, 32, 1, 1
    p, n, nq, efs = _tree_setup(S, L, f, k, r)
    cl = S.Client(L, f)
    sv = S.Server(1, L, efs)
    cl.encode_across_files_server(sv)
    cl.encode_across_files_server(sv)
    assert not _rows(sv, n).any()
    sv.freeServer()
    cl.free_client()


@pytest.mark.parametrize("ci", range(4))
def test_gpu_setup_encode_within_matches_reference(S, ci):
    """Mode 3 (Hollanti) setup on the GPU from host rows: the reference's own shard hashes."""
    case = O.golden("hollanti.json")["cases"][ci]
    S.setSystemParams(case["L"], case["f"], case["t"], case["k"], case["r"], 0, case["rho"], 0, 3)
    cl = S.Client(case["L"], case["f"])
    for party in range(case["p"]):
        sv = S.Server(party + 1, case["L"], case["efs"])
        cl.encode_within_files_server(sv)
        assert O.sha(_rows(sv, case["L"])) == case["shard_sha256"][party], party
        sv.freeServer()
    cl.free_client()


def test_engine_rows_roundtrip(S):
    """pir_engine_set_shard_rows / pir_engine_get_shard_rows (the staged copies) over row
    pointers with a ragged chunk count: what goes up comes back."""
    import erasurecodedpir_amd as pir
    from erasurecodedpir_amd import _lib
    n, efs = 17, 200  # 2^17 x 200 B: 26 MiB, several staging chunks with a partial last one
    with pir.Engine(2, 1, n, efs, 1) as e:
        lib = _lib.load()
        rows = np.random.default_rng(3).integers(0, 256, (1 << n, efs), dtype=np.uint8)
        ptrs = (ctypes.c_void_p * (1 << n))(*[rows.ctypes.data + i * efs for i in range(1 << n)])
        _lib.check(lib.pir_engine_set_shard_rows(e._h, ptrs, 0, 1 << n), "set_shard_rows")
        assert np.array_equal(e.get_shard(0, 1 << n).reshape(-1, efs), rows)
        back = np.zeros_like(rows)
        bptrs = (ctypes.c_void_p * (1 << n))(*[back.ctypes.data + i * efs for i in range(1 << n)])
        _lib.check(lib.pir_engine_get_shard_rows(e._h, bptrs, 0, 1 << n), "get_shard_rows")
        assert np.array_equal(back, rows)


def test_setup_free_setup_again(S):
    """SETUP -> query -> freeServer -> SETUP -> query, three times (tree.go:90-100 frees the
    server after every query): freeServer hands the engine teardown to the reaper thread and
    returns at once; the next setup's engine waits for it; every answer is the oracle's."""
    import time
    import erasurecodedpir_amd as pir
    L, f, k, r = 13, 256, 2, 1
    p, n, nq, efs = _tree_setup(S, L, f, k, r)
    cl = S.Client(L, f)
    shard = O.encode_across(L, f, k, p, 2, O.synthetic_db(L, f))
    keys = [pir.gen_keys(n, i * 311 + 5, p, nq, fcw=O.final_cw(p, nq, 1))[1] for i in range(3)]
    frees = []
    for i in range(3):
        sv = S.Server(2, L, efs, 0, 4)
        cl.encode_across_files_server(sv)
        assert np.array_equal(sv.runOptimizedDPFTreeQuery(keys[i], nq),
                              O.answer(p, 2, n, efs, nq, keys[i], shard)), i
        assert np.array_equal(sv.runTreeQueryThreads(keys[i], 4),
                              O.answer(p, 2, n, efs, nq, keys[i], shard)), i
        t0 = time.perf_counter()
        sv.freeServer()
        frees.append(time.perf_counter() - t0)
        assert not sv.s.ctx and not sv.s.indexList
    S.wait_freed()
    cl.free_client()
    assert max(frees) < 0.05, frees  # the engine teardown is not on the caller's path


def test_setup_over_directly_written_rows(S):
    """indexList written directly (no pirServerSetRows / pirServerShardChanged) before the
    setup: the encode is XORed INTO those rows as the reference does (client.cpp:88) -- the shim
    sees the touched pages (mincore) and keeps the host encode; answers and rows are the
    oracle's of (caller rows XOR encoding)."""
    import erasurecodedpir_amd as pir
    L, f, k, r = 12, 96, 2, 1
    p, n, nq, efs = _tree_setup(S, L, f, k, r)
    cl = S.Client(L, f)
    enc = O.encode_across(L, f, k, p, 3, O.synthetic_db(L, f)).reshape(-1, efs)
    mine = np.random.default_rng(8).integers(0, 256, enc.shape, dtype=np.uint8)
    sv = S.Server(3, L, efs, 0, 4)
    for i in range(1 << n):  # straight through the row pointers, as a C caller would
        ctypes.memmove(sv.s.indexList[i], mine[i].ctypes.data, efs)
    cl.encode_across_files_server(sv)
    want = mine ^ enc
    key = pir.gen_keys(n, 1234, p, nq, fcw=O.final_cw(p, nq, 1))[2]
    assert np.array_equal(sv.runOptimizedDPFTreeQuery(key, nq),
                          O.answer(p, 3, n, efs, nq, key, want.reshape(-1)))
    assert np.array_equal(_rows(sv, n), want)
    sv.freeServer()
    cl.free_client()


@pytest.mark.parametrize("chunk", [7 * 1000, 65536 + 40])
def test_staging_many_chunks(S, monkeypatch, chunk):
    """$PIR_STAGE_CHUNK_BYTES splits the staged copies into many small chunks with a ragged
    last one: the double-buffer reuse (chunk c waits for c - 2's copy), get_shard_rows'
    enqueue-ahead and encode_across_rows' per-chunk block mapping (blocks at j*n, file
    encdb*j + row) are exercised; rows round-trip and both encodes equal the oracle's."""
    import erasurecodedpir_amd as pir
    from erasurecodedpir_amd import _lib
    monkeypatch.setenv("PIR_STAGE_CHUNK_BYTES", str(chunk))
    n, efs = 12, 200
    with pir.Engine(2, 1, n, efs, 1) as e:
        lib = _lib.load()
        rows = np.random.default_rng(chunk).integers(0, 256, (1 << n, efs), dtype=np.uint8)
        assert (1 << n) * efs // chunk >= 3  # several chunks
        ptrs = (ctypes.c_void_p * (1 << n))(*[rows.ctypes.data + i * efs for i in range(1 << n)])
        _lib.check(lib.pir_engine_set_shard_rows(e._h, ptrs, 0, 1 << n), "set_shard_rows")
        assert np.array_equal(e.get_shard(0, 1 << n).reshape(-1, efs), rows)
        back = np.zeros_like(rows)
        bptrs = (ctypes.c_void_p * (1 << n))(*[back.ctypes.data + i * efs for i in range(1 << n)])
        _lib.check(lib.pir_engine_get_shard_rows(e._h, bptrs, 0, 1 << n), "get_shard_rows")
        assert np.array_equal(back, rows)
    # encode across (k = 5: the last block past NUM_FILES is zero) and within, shim setups
    L, f, k, r = 12, 100, 5, 2
    p, n, nq, efs = _tree_setup(S, L, f, k, r)
    cl = S.Client(L, f)
    for party in (1, p):
        sv = S.Server(party, L, efs)
        cl.encode_across_files_server(sv)
        assert np.array_equal(_rows(sv, n).reshape(-1),
                              O.encode_across(L, f, k, p, party, O.synthetic_db(L, f))), party
        sv.freeServer()
    cl.free_client()
    case = O.golden("hollanti.json")["cases"][0]
    S.setSystemParams(case["L"], case["f"], case["t"], case["k"], case["r"], 0, case["rho"], 0, 3)
    cl = S.Client(case["L"], case["f"])
    sv = S.Server(1, case["L"], case["efs"])
    cl.encode_within_files_server(sv)
    assert O.sha(_rows(sv, case["L"])) == case["shard_sha256"][0]
    sv.freeServer()
    cl.free_client()
