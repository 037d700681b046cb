"""Client side of the reference's wire protocol, against `pir_serve` (or the reference's Go
server): TLS (no certificate check, src/common/network.go:27-30), one request-type byte then
a msgpack request; the server answers msgpack(error) then msgpack(response)
(src/server/server.go:53-125).  Structs are msgpack maps keyed by the Go field names of
src/common/common.go:51-81.

`tree_query` is src/client/tree.go:17-175: generate the p keys, send one to every server in
parallel, keep the first NUM_PARTIES - R answers, decode (client.cpp:211-268).
"""
import socket
import ssl
import threading

import msgpack
import numpy as np

# common.go:147-154
SETUP_REQUEST, TREE_SEARCH_REQUEST, MULTIPARTY_SEARCH_REQUEST, HOLLANTI_SEARCH_REQUEST = 0, 1, 3, 4
CD732_SEARCH_REQUEST, TEST_REQUEST = 5, 7


class WireError(RuntimeError):
    pass


class Conn:
    """One TLS connection to a server (network.go:24-50)."""

    def __init__(self, host, port, timeout=120.0):
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
        raw = socket.create_connection((host, int(port)), timeout=timeout)
        self.sock = ctx.wrap_socket(raw, server_hostname=host)
        self.unpacker = msgpack.Unpacker(raw=False, strict_map_key=False)

    def _next(self):
        for obj in self.unpacker:
            return obj
        while True:
            data = self.sock.recv(1 << 16)
            if not data:
                raise EOFError("connection closed")
            self.unpacker.feed(data)
            for obj in self.unpacker:
                return obj

    def call(self, req_type, req):
        """SendMessageWithConnection (network.go:72-100): returns the response map; a non-nil
        error from the server raises WireError."""
        self.sock.sendall(bytes([req_type]) + msgpack.packb(req, use_bin_type=True))
        err = self._next()
        resp = self._next()
        if err:
            raise WireError(err if isinstance(err, str) else repr(err))
        return resp

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def setup(addr, log_num_files, file_size_bytes, k, r, rho=1, num_threads=1, is_byzantine=0,
          mode=0, t=1, b=0):
    """SETUP_REQUEST with the fields of common.go:51-65 (no MAC): mode 0 tree, 1 multiparty,
    3 Hollanti, 4 covering design."""
    host, port = addr
    req = {"BenchmarkDir": "", "LogNumFiles": log_num_files, "FileSizeBytes": file_size_bytes,
           "T": t, "K": k, "R": r, "B": b, "Rho": rho, "Mode": mode, "IsByzantine": is_byzantine,
           "DelayTime": 0, "NumThreads": num_threads, "CheckMAC": 0}
    with Conn(host, port) as c:
        return c.call(SETUP_REQUEST, req)


def tree_search(addr, key):
    host, port = addr
    with Conn(host, port) as c:
        return c.call(TREE_SEARCH_REQUEST, {"Key": bytes(key)})


def multiparty_search(addr, key):
    """MULTIPARTY_SEARCH_REQUEST (client/multiparty.go:76-90): Results = NUM_RSS_KEYS answers."""
    host, port = addr
    with Conn(host, port) as c:
        return c.call(MULTIPARTY_SEARCH_REQUEST, {"Key": bytes(key)})


def cd_search(addr, key):
    """CD732_SEARCH_REQUEST (server_util/cd732.go:16-100): Results = NUM_CD_KEYS answers."""
    host, port = addr
    with Conn(host, port) as c:
        return c.call(CD732_SEARCH_REQUEST, {"Key": bytes(key)})


def hollanti_search(addr, keys):
    """HOLLANTI_SEARCH_REQUEST: keys = NUM_ROUNDS coefficient vectors of NUM_FILES bytes."""
    host, port = addr
    with Conn(host, port) as c:
        return c.call(HOLLANTI_SEARCH_REQUEST, {"Key": [bytes(np.asarray(k, np.uint8)) for k in keys]})


def tree_query(addrs, index, log_num_files, file_size_bytes, k, r, rho=1, device=0):
    """src/client/tree.go:17-175 for one record: returns (record bytes, per-server responses,
    erasure list).  Needs the sizing globals of setSystemParams (set here) and a GPU for key
    generation (pir_client.h)."""
    from . import client as C
    from . import server as S
    S.setSystemParams(log_num_files, file_size_bytes, 1, k, r, 0, rho, 0, 0)
    prm = S.params()
    p, n, nq, R = prm["NUM_PARTIES"], prm["LOG_NUM_ENCODED_FILES"], prm["NUM_ROUNDS"], prm["R"]
    if len(addrs) != p:
        raise ValueError(f"{len(addrs)} server addresses for {p} parties")
    keys = C.gen_keys(n, index, p, nq, fcw=C.final_cw(p, nq, rho), device=device)
    resps, errs = [None] * p, [None] * p
    done = threading.Condition()
    order = []

    def ask(i):
        try:
            resps[i] = tree_search(addrs[i], keys[i])
        except Exception as ex:  # an unreachable / failing server is an erasure
            errs[i] = ex
        with done:
            order.append(i)
            done.notify()

    threads = [threading.Thread(target=ask, args=(i,), daemon=True) for i in range(p)]
    for t in threads:
        t.start()
    with done:  # the first p - R good answers (tree.go:104-120)
        while True:
            arrived = [i for i in order if errs[i] is None]
            if len(arrived) >= p - R or len(order) == p:
                break
            done.wait()
    good = sorted(arrived[: p - R])
    if len(good) < p - R:
        raise WireError("Not enough valid responses")
    erasure = [1 if i in good else 0 for i in range(p)]
    kept = np.stack([np.stack([np.frombuffer(b, np.uint8) for b in resps[i]["Results"]])
                     for i in good])
    record = S.assembleDPFTreeQueryResponses(erasure, kept)
    return record, resps, erasure
