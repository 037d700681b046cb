"""The wire boundary: `pir_serve` (C++, TLS + msgpack framing of src/server/server.go:53-125)
and the Python client of erasurecodedpir_amd/wire.py (src/client/tree.go).  On the CPU: the
TLS handshake, the request framing and the TEST echo, and that a setup without a GPU fails
loudly.  On the GPU: the configs[0] loopback (2 servers, 2^16 x 256 B, one query) and an
erasure-coded setup with a server down, decoded from the remaining answers."""
import os
import socket
import subprocess
import time

import numpy as np
import pytest

from erasurecodedpir_amd import wire

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SERVE = os.path.join(ROOT, "erasurecodedpir_amd", "pir_serve")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class Servers:
    def __init__(self, p, byzantine=(), parties=None):
        self.procs, self.addrs = [], []
        for party in parties or range(1, p + 1):
            port = _free_port()
            args = [SERVE, "--port", str(port), "--party", str(party)]
            if party in byzantine:
                args += ["--byzantine", "1"]
            self.procs.append(subprocess.Popen(args, stderr=subprocess.PIPE))
            self.addrs.append(("127.0.0.1", port))
        for addr in self.addrs:  # wait until listening
            for _ in range(200):
                try:
                    socket.create_connection(addr, timeout=1).close()
                    break
                except OSError:
                    time.sleep(0.05)

    def stop(self, i):
        self.procs[i].terminate()
        self.procs[i].wait(timeout=30)

    def close(self):
        for pr in self.procs:
            if pr.poll() is None:
                pr.terminate()
                try:
                    pr.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    pr.kill()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


@pytest.fixture(scope="module")
def serve_bin():
    if not os.path.exists(SERVE):
        pytest.fail("pir_serve not built (make -C erasurecodedpir_amd/csrc)")
    return SERVE


def test_tls_framing_and_echo(serve_bin):
    with Servers(1) as sv:
        with wire.Conn(*sv.addrs[0]) as c:
            for msg in ("", "hello", "x" * 5000):
                assert c.call(wire.TEST_REQUEST, {"Msg": msg}) == {"Msg": msg}


def test_setup_without_gpu_fails_loudly(serve_bin):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with Servers(1) as sv:
        with pytest.raises(wire.WireError):
            wire.setup(sv.addrs[0], 10, 16, 1, 0)
        with pytest.raises(wire.WireError):  # no engine: a query is refused, not answered
            wire.tree_search(sv.addrs[0], b"\0" * 100)


def _synthetic(v, f):  # client.cpp:16-33
    return np.arange(f, dtype=np.uint8) if v == 1 else np.full(f, v & 0xFF, np.uint8)


@pytest.mark.gpu
def test_loopback_configs0(serve_bin):
    """BASELINE configs[0]: 2-server loopback, 2^16 x 256 B database, queries decoded."""
    L, f, k, r = 16, 256, 1, 0
    with Servers(2) as sv:
        for addr in sv.addrs:
            resp = wire.setup(addr, L, f, k, r)
            assert resp["ServerLatency"] >= 0
        for idx in (1, 5, 40000, (1 << L) - 1):
            rec, resps, er = wire.tree_query(sv.addrs, idx, L, f, k, r)
            assert er == [1, 1]
            assert np.array_equal(rec, _synthetic(idx, f)), idx
            assert {r_["PartyIndex"] for r_ in resps} == {1, 2}


@pytest.mark.gpu
def test_erasure_coded_servers_with_one_down(serve_bin):
    """k=3, r=1 -> p=5 servers, NUM_ROUNDS=3; one server killed before the query."""
    L, f, k, r = 14, 128, 3, 1
    with Servers(5) as sv:
        for addr in sv.addrs:
            wire.setup(addr, L, f, k, r)
        sv.stop(2)
        encdb = -(-(1 << L) // k)
        for row in (1, 7, encdb - 1):
            rec, _, er = wire.tree_query(sv.addrs, row, L, f, k, r)
            assert er[2] == 0 and sum(er) == 4
            assert np.array_equal(rec, _synthetic(row, f)), row


@pytest.mark.gpu
def test_multiparty_over_the_wire(serve_bin):
    """Mode 1 (multiparty sqrt(N) DPF): SETUP encodes across files on the GPU (k = 2, so each
    server's own evaluation point matters: parties 1 and 3), each MULTIPARTY_SEARCH answer ==
    the CPU restatement on that party's encoded shard; a tree request to a multiparty setup is
    refused with an error."""
    import _oracle as O
    L, f, t, k, r = 12, 64, 1, 2, 1
    p = t + k + r
    key = O.mp_key(p, L - 1, t, 31337)  # k = 2: the domain is the 2^(L-1) encoded rows
    files = O.synthetic_db(L, f)
    with Servers(2, parties=(1, 3)) as sv:  # party 3: its own encode-across evaluation point
        for addr in sv.addrs:
            wire.setup(addr, L, f, k, r, mode=1, t=t)
        resps = [wire.multiparty_search(addr, key) for addr in sv.addrs]
        with pytest.raises(wire.WireError):
            wire.tree_search(sv.addrs[0], b"\0" * 64)
    n = L - 1  # k = 2: 2^(L-1) encoded rows
    for party, resp in zip((1, 3), resps):
        got = np.stack([np.frombuffer(b, np.uint8) for b in resp["Results"]])
        shard = O.encode_across(L, f, k, p, party, files)
        assert np.array_equal(got, O.mp_answer(p, t, n, f, key, shard)), party
        assert "PartyIndex" not in resp and resp["ServerLatency"] >= 0


@pytest.mark.gpu
def test_hollanti_over_the_wire(serve_bin):
    """Mode 3 (polynomial PIR): SETUP encodes within files, a HOLLANTI_SEARCH answer with
    NUM_ROUNDS coefficient vectors == their scan of the encoded rows (CPU restatement)."""
    import _oracle as O
    from erasurecodedpir_amd import server as S
    L, f, t, k, r = 11, 96, 1, 2, 1
    S.setSystemParams(L, f, t, k, r, 0, 1, 0, 3)
    prm = S.params()
    nq, efs, N = prm["NUM_ROUNDS"], prm["ENCODED_FILE_SIZE_BYTES"], 1 << L
    cl = S.Client(L, f)
    srv = S.Server(2, L, efs)
    cl.encode_within_files_server(srv)
    shard = np.stack([srv.read_row(i) for i in range(N)]).reshape(-1)
    srv.freeServer()
    cl.free_client()
    keys = np.random.default_rng(3).integers(0, 256, (nq, N), dtype=np.uint8)
    with Servers(2) as sv:
        wire.setup(sv.addrs[1], L, f, k, r, mode=3, t=t)
        resp = wire.hollanti_search(sv.addrs[1], keys)
    got = np.stack([np.frombuffer(b, np.uint8) for b in resp["Results"]])
    assert np.array_equal(got, O.scan(keys, shard, efs))


@pytest.mark.gpu
def test_cd_over_the_wire(serve_bin):
    """Mode 4 (covering-design sqrt(N) DPF): three servers (parties 1, 5, 8 of the reference's
    own P = 8 CD842 setup, correctness_tests.cpp:1236) set up over the wire encode across files
    on the GPU; their CD732_SEARCH answers to the reference's genCDDPF keys == the reference's
    answers (tests/golden/cd.json)."""
    import _oracle as O
    c = O.golden("cd.json")["cases"][0]
    parties = sorted(map(int, c["keys"]))
    with Servers(len(parties), parties=parties) as sv:
        for addr in sv.addrs:
            wire.setup(addr, c["L"], c["f"], c["k"], c["r"], c["rho"], mode=4, t=c["t"], b=c["b"])
        resps = [wire.cd_search(addr, bytes.fromhex(c["keys"][str(q)]))
                 for addr, q in zip(sv.addrs, parties)]
        with pytest.raises(wire.WireError):
            wire.multiparty_search(sv.addrs[0], b"\0" * 64)
    for q, resp in zip(parties, resps):
        assert b"".join(resp["Results"]).hex() == c["answers"][q - 1], q
