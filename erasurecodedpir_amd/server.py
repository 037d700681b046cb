"""The reference's server-side API for the tree-DPF path, by its own names, over the
server.h-compatible shim (include/pir_server.h) -- what the Go server binds through cgo
(src/server_util/tree.go:65,76; src/server/server.go:299-331).  Parity tests use this module
the way src/c/correctness_tests.cpp:230-372 drives src/c.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import CClient, CServer, c_u8_p


def setSystemParams(logNumFiles, fileSizeBytes, t, k, r, b, rho, checkMac, mode):
    _lib.load().setSystemParams(logNumFiles, fileSizeBytes, t, k, r, b, rho, checkMac, mode)


def params():
    """The sizing globals of src/c/params.h:9-33 as a dict."""
    return {n: _lib.global_int(n) for n in _lib.GLOBALS_INT + _lib.GLOBALS_U32}


def calcOptimizedDPFTreeKeyLength(p, log_domain_size, num_queries):
    return _lib.load().calcOptimizedDPFTreeKeyLength(p, log_domain_size, num_queries)


def _row_ptrs(arr2d):
    rows = arr2d.shape[0]
    base = arr2d.ctypes.data
    ptrs = (c_u8_p * rows)()
    for i in range(rows):
        ptrs[i] = ctypes.cast(base + i * arr2d.strides[0], c_u8_p)
    return ptrs


class Server:
    """A `server` struct (src/c/server.h:13-25) owned by the shim."""

    def __init__(self, partyIndex, logNumFiles, fileSizeBytes, isByzantine=0, numThreads=1):
        self._lib = _lib.load()
        self.s = CServer()
        self._lib.initializeServer(ctypes.byref(self.s), partyIndex, logNumFiles, fileSizeBytes,
                                   isByzantine, numThreads)
        self.rows = 1 << logNumFiles
        self.file_size = fileSizeBytes

    @property
    def partyIndex(self):
        return self.s.partyIndex

    def write_rows(self, rows, row0=0):
        """Copy (nrows, file_size) bytes into indexList[row0 ..] (as a test harness would) and
        mark the shard changed (pirServerSetRows)."""
        rows = np.ascontiguousarray(rows, dtype=np.uint8).reshape(-1, self.file_size)
        self._lib.pirServerSetRows(ctypes.byref(self.s), rows.ctypes.data, row0, rows.shape[0],
                                   self.file_size)

    def read_row(self, i):
        """indexList[i] (after a GPU setup the rows are first synced from the device shard:
        pirServerSyncRows, a no-op once they are current)."""
        self._lib.pirServerSyncRows(ctypes.byref(self.s))
        return np.ctypeslib.as_array(self.s.indexList[i], (self.file_size,)).copy()

    def runOptimizedDPFTreeQuery(self, key, numQueries):
        efs = _lib.global_int("ENCODED_FILE_SIZE_BYTES")
        out = np.zeros((numQueries, efs), np.uint8)
        k = np.frombuffer(bytes(key), np.uint8).copy()
        self._lib.runOptimizedDPFTreeQuery(ctypes.byref(self.s), k.ctypes.data_as(ctypes.c_void_p),
                                           numQueries, _row_ptrs(out))
        return out

    def runOptimizedDPFTreeQueryThread(self, key, threadNum, numThreads):
        efs = _lib.global_int("ENCODED_FILE_SIZE_BYTES")
        nq = _lib.global_int("NUM_ROUNDS")
        out = np.zeros((nq, efs), np.uint8)
        k = np.frombuffer(bytes(key), np.uint8).copy()
        self._lib.runOptimizedDPFTreeQueryThread(ctypes.byref(self.s),
                                                 k.ctypes.data_as(ctypes.c_void_p), threadNum,
                                                 numThreads, _row_ptrs(out))
        return out

    def runTreeQueryThreads(self, key, numThreads):
        """RunTreeQuery's fan-out (src/server_util/tree.go:60-80) in the library: numThreads
        concurrent runOptimizedDPFTreeQueryThread calls + assemblDPFTreeQueryThreadResults."""
        efs = _lib.global_int("ENCODED_FILE_SIZE_BYTES")
        nq = _lib.global_int("NUM_ROUNDS")
        out = np.zeros((nq, efs), np.uint8)
        k = np.frombuffer(bytes(key), np.uint8).copy()
        self._lib.pirRunTreeQueryThreads(ctypes.byref(self.s), k.ctypes.data_as(ctypes.c_void_p),
                                         numThreads, ctypes.cast(_row_ptrs(out), ctypes.c_void_p))
        return out

    def runHollantiQuery(self, keys):
        """keys: (NUM_ROUNDS, NUM_ENCODED_FILES) coefficient vectors (server.cpp:321-343)."""
        return self._hollanti(keys, None)

    def runHollantiQueryThread(self, keys, threadNum, startIndex, endIndex):
        """Rows [startIndex, endIndex) (server.cpp:345-371)."""
        return self._hollanti(keys, (threadNum, startIndex, endIndex))

    def _hollanti(self, keys, thread):
        efs = _lib.global_int("ENCODED_FILE_SIZE_BYTES")
        nq = _lib.global_int("NUM_ROUNDS")
        N = _lib.global_int("NUM_ENCODED_FILES")
        k = np.ascontiguousarray(np.asarray(keys, np.uint8))
        if k.size != nq * N:  # the shim reads NUM_ROUNDS rows of NUM_ENCODED_FILES bytes
            raise ValueError(f"Hollanti keys of {k.size} bytes, expected {nq} x {N}")
        k = k.reshape(nq, N)
        out = np.zeros((nq, efs), np.uint8)
        kp = _row_ptrs(k)
        if thread is None:
            self._lib.runHollantiQuery(ctypes.byref(self.s), kp, _row_ptrs(out))
        else:
            self._lib.runHollantiQueryThread(ctypes.byref(self.s), kp, *thread, _row_ptrs(out))
        return out

    def runOptimizedMultiPartyDPFQuery(self, key):
        """Multiparty sqrt(N) DPF answer (server.cpp:136-176): (NUM_RSS_KEYS, EFS)."""
        return self._mp(key, None)

    def runOptimizedMultiPartyDPFQueryThread(self, key, threadNum, numThreads):
        """Rows of thread threadNum of numThreads (server.cpp:384-430)."""
        return self._mp(key, (threadNum, numThreads))

    def _mp(self, key, thread):
        efs = _lib.global_int("ENCODED_FILE_SIZE_BYTES")
        out = np.zeros((_lib.global_int("NUM_RSS_KEYS"), efs), np.uint8)
        k = np.frombuffer(bytes(key), np.uint8).copy()
        need = calcMultiPartyOptDPFKeyLength(_lib.global_int("NUM_PARTIES"),
                                             _lib.global_int("LOG_NUM_ENCODED_FILES"),
                                             _lib.global_int("T"))
        if k.size < need:  # the shim reads calcMultiPartyOptDPFKeyLength bytes
            raise ValueError(f"multiparty key of {k.size} bytes, expected {need}")
        kp = k.ctypes.data_as(ctypes.c_void_p)
        if thread is None:
            self._lib.runOptimizedMultiPartyDPFQuery(ctypes.byref(self.s), kp, _row_ptrs(out))
        else:
            self._lib.runOptimizedMultiPartyDPFQueryThread(ctypes.byref(self.s), kp, *thread,
                                                           _row_ptrs(out))
        return out

    def runCDQueryThread(self, key, threadNum, numThreads):
        """Covering-design answer over thread threadNum's rows (server.cpp:443-492):
        (NUM_CD_KEYS, EFS)."""
        efs = _lib.global_int("ENCODED_FILE_SIZE_BYTES")
        out = np.zeros((_lib.global_int("NUM_CD_KEYS"), efs), np.uint8)
        k = np.frombuffer(bytes(key), np.uint8).copy()
        need = calcCDDPFKeyLength(_lib.global_int("NUM_PARTIES"),
                                  _lib.global_int("LOG_NUM_ENCODED_FILES"), _lib.global_int("T"),
                                  _lib.global_int("NUM_CD_KEYS_NEEDED"),
                                  _lib.global_int("NUM_CD_KEYS"))
        if k.size < need:  # the shim reads calcCDDPFKeyLength bytes
            raise ValueError(f"covering-design key of {k.size} bytes, expected {need}")
        self._lib.runCDQueryThread(ctypes.byref(self.s), k.ctypes.data_as(ctypes.c_void_p),
                                   threadNum, numThreads, _row_ptrs(out))
        return out

    def freeServer(self):
        """Returns once the server is unreachable; the engine teardown runs in the background
        (pirServerWaitFreed / wait_freed() waits for it)."""
        if self.s.ctx:
            self._lib.freeServer(ctypes.byref(self.s))


def wait_freed():
    """Block until every freeServer's background teardown has finished (pirServerWaitFreed)."""
    _lib.load().pirServerWaitFreed()

    def __del__(self):
        try:
            self.freeServer()
        except Exception:
            pass


def assemblDPFTreeQueryThreadResults(server, parts):
    """parts: (numThreads, NUM_ROUNDS, EFS) -> (NUM_ROUNDS, EFS) (src/c/server.cpp:553-562)."""
    parts = np.ascontiguousarray(parts, dtype=np.uint8)
    T, nq, efs = parts.shape
    ins = (ctypes.POINTER(c_u8_p) * T)()
    keep = []
    for t in range(T):
        rp = _row_ptrs(parts[t])
        keep.append(rp)
        ins[t] = ctypes.cast(rp, ctypes.POINTER(c_u8_p))
    out = np.zeros((nq, efs), np.uint8)
    _lib.load().assemblDPFTreeQueryThreadResults(ctypes.byref(server.s), ins, T, _row_ptrs(out))
    return out


def assembleHollantiQueryThreadResults(server, parts):
    """parts: (numThreads, NUM_ROUNDS, EFS) -> (NUM_ROUNDS, EFS) (src/c/server.cpp:373-382)."""
    return _assemble("assembleHollantiQueryThreadResults", server, parts)


def assembleMultipartyDPFQueryThreadResults(server, parts):
    """parts: (numThreads, NUM_RSS_KEYS, EFS) -> (NUM_RSS_KEYS, EFS) (server.cpp:432-441)."""
    return _assemble("assembleMultipartyDPFQueryThreadResults", server, parts)


def assembleCDQueryThreadResults(server, parts):
    """parts: (numThreads, NUM_CD_KEYS, EFS) -> (NUM_CD_KEYS, EFS) (server.cpp:494-503)."""
    return _assemble("assembleCDQueryThreadResults", server, parts)


def calcCDDPFKeyLength(p, log_domain_size, t, num_cd_keys_needed, num_cd_keys):
    """utils.cpp:118-129."""
    return _lib.load().calcCDDPFKeyLength(p, log_domain_size, t, num_cd_keys_needed, num_cd_keys)


def calcMultiPartyOptDPFKeyLength(p, log_domain_size, t):
    """utils.cpp:105-116."""
    return _lib.load().calcMultiPartyOptDPFKeyLength(p, log_domain_size, t)


def _assemble(fn, server, parts):
    parts = np.ascontiguousarray(parts, dtype=np.uint8)
    T, nq, efs = parts.shape
    ins = (ctypes.POINTER(c_u8_p) * T)()
    keep = []
    for t in range(T):
        rp = _row_ptrs(parts[t])
        keep.append(rp)
        ins[t] = ctypes.cast(rp, ctypes.POINTER(c_u8_p))
    out = np.zeros((nq, efs), np.uint8)
    getattr(_lib.load(), fn)(ctypes.byref(server.s), ins, T, _row_ptrs(out))
    return out


class Client:
    """The synthetic-DB client of src/c/client.cpp:16-41 (server setup path)."""

    def __init__(self, log_num_files, file_size_bytes):
        self._lib = _lib.load()
        self.c = CClient()
        self._lib.initialize_client(ctypes.byref(self.c), log_num_files, file_size_bytes)

    def encode_across_files_server(self, server):
        self._lib.encode_across_files_server(ctypes.byref(self.c), ctypes.byref(server.s))

    def encode_within_files_server(self, server):
        self._lib.encode_within_files_server(ctypes.byref(self.c), ctypes.byref(server.s))

    def assembleDPFTreeQueryResponses(self, erasure, responses):
        """Client decode (client.cpp:211-268); see the module function of the same name."""
        return assembleDPFTreeQueryResponses(erasure, responses, self.c)

    def generate_opt_DPF_tree_query(self, index):
        """client.cpp:144-153 (src/client/tree.go:55): NUM_PARTIES keys (GPU key generation)."""
        return generate_opt_DPF_tree_query(index, self.c)

    def generateHollantiQuery(self, index):
        """client.cpp:201-203 (src/client/hollanti.go:37): (NUM_PARTIES, NUM_ROUNDS,
        NUM_ENCODED_FILES) coefficient vectors."""
        return generateHollantiQuery(index, self.c)

    def free_client(self):
        if self.c.unencoded_files:
            self._lib.free_client(ctypes.byref(self.c))


def generate_opt_DPF_tree_query(index, c=None):
    """The client's keys for record `index` under the current setSystemParams(mode 0): a list of
    NUM_PARTIES calcOptimizedDPFTreeKeyLength-byte keys (client.cpp:144-153)."""
    lib = _lib.load()
    prm = params()
    p = prm["NUM_PARTIES"]
    kl = lib.calcOptimizedDPFTreeKeyLength(p, prm["LOG_NUM_ENCODED_FILES"], prm["NUM_ROUNDS"])
    keys = np.zeros((p, kl), np.uint8)
    kp = _row_ptrs(keys)
    arr = ctypes.cast(kp, ctypes.POINTER(c_u8_p))  # the Go caller's `keys` (**byte); it passes &keys
    cl = c if c is not None else CClient()
    lib.generate_opt_DPF_tree_query(ctypes.byref(cl), int(index), ctypes.pointer(arr))
    return [keys[j].tobytes() for j in range(p)]


def generateHollantiQuery(index, c=None):
    """Polynomial-PIR query for record `index` under the current setSystemParams(mode 3):
    (NUM_PARTIES, NUM_ROUNDS, NUM_ENCODED_FILES) (client.cpp:201-203)."""
    lib = _lib.load()
    prm = params()
    p, nq, N = prm["NUM_PARTIES"], prm["NUM_ROUNDS"], prm["NUM_ENCODED_FILES"]
    keys = np.zeros((p, nq, N), np.uint8)
    rows = [_row_ptrs(keys[q]) for q in range(p)]
    outer = (ctypes.POINTER(c_u8_p) * p)(*[ctypes.cast(r, ctypes.POINTER(c_u8_p)) for r in rows])
    cl = c if c is not None else CClient()
    lib.generateHollantiQuery(ctypes.byref(cl), int(index), outer)
    return keys


def mac(key16, msg):
    """utils.cpp:32-34: HMAC-SHA256 of msg under the 16-byte key (32 bytes)."""
    k = np.frombuffer(bytes(key16), np.uint8).copy()
    m = np.frombuffer(bytes(msg), np.uint8).copy() if len(msg) else np.zeros(1, np.uint8)
    out = np.zeros(32, np.uint8)
    _lib.load().mac(k.ctypes.data_as(ctypes.c_void_p), m.ctypes.data_as(ctypes.c_void_p),
                    len(msg), out.ctypes.data_as(ctypes.c_void_p), 32)
    return out.tobytes()


def assembleDPFTreeQueryResponses(erasure, responses, c=None):
    """Client erasure decode of one tree-mode query (client.cpp:211-268) under the current
    setSystemParams: erasure[q-1] = 1 for the servers whose answers are given, responses =
    [NUM_PARTIES - R][NUM_ROUNDS][ENCODED_FILE_SIZE_BYTES] in increasing server order.  Returns
    the FILE_SIZE_BYTES record.  The decode reads no client state, so `c` may be omitted."""
    lib = _lib.load()
    prm = params()
    nr, nq, efs = prm["NUM_PARTIES"] - prm["R"], prm["NUM_ROUNDS"], prm["ENCODED_FILE_SIZE_BYTES"]
    resp = np.ascontiguousarray(np.asarray(responses, np.uint8).reshape(nr, nq, efs))
    er = np.ascontiguousarray(np.asarray(erasure, np.uint8))
    rows = [(c_u8_p * nq)(*[resp[j, i].ctypes.data_as(c_u8_p) for i in range(nq)]) for j in range(nr)]
    outer = (ctypes.POINTER(c_u8_p) * nr)(*[ctypes.cast(r, ctypes.POINTER(c_u8_p)) for r in rows])
    out = np.zeros(_lib.global_int("FILE_SIZE_BYTES"), np.uint8)
    cl = c if c is not None else CClient()
    lib.assembleDPFTreeQueryResponses(ctypes.byref(cl), er.ctypes.data_as(ctypes.c_void_p), outer,
                                      out.ctypes.data_as(ctypes.c_void_p))
    return out


def assembleHollantiResponses(erasure, responses, c=None):
    """Client decode of one polynomial (Hollanti) query (client.cpp:499-552) under the current
    setSystemParams(mode 3): responses = [NUM_PARTIES - R][NUM_ROUNDS][EFS]."""
    lib = _lib.load()
    prm = params()
    nr, nq, efs = prm["NUM_PARTIES"] - prm["R"], prm["NUM_ROUNDS"], prm["ENCODED_FILE_SIZE_BYTES"]
    resp = np.ascontiguousarray(np.asarray(responses, np.uint8).reshape(nr, nq, efs))
    er = np.ascontiguousarray(np.asarray(erasure, np.uint8))
    rows = [(c_u8_p * nq)(*[resp[j, i].ctypes.data_as(c_u8_p) for i in range(nq)]) for j in range(nr)]
    outer = (ctypes.POINTER(c_u8_p) * nr)(*[ctypes.cast(r, ctypes.POINTER(c_u8_p)) for r in rows])
    out = np.zeros(_lib.global_int("FILE_SIZE_BYTES"), np.uint8)
    cl = c if c is not None else CClient()
    lib.assembleHollantiResponses(ctypes.byref(cl), er.ctypes.data_as(ctypes.c_void_p), outer,
                                  out.ctypes.data_as(ctypes.c_void_p))
    return out
