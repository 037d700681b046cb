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
