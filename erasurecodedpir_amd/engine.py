"""Python host mirror of the engine C ABI (include/pir_engine.h).

`Engine` is one PIR server's shard -- or one 2^-G partition of it -- resident in the HBM of one
MI355X, answering tree-DPF queries with the HIP kernels of csrc/pir_kernels.hip.  Method names
follow the reference's server operations (src/c/server.h:27-53):

    Engine.answer        runOptimizedDPFTreeQuery        (src/c/server.cpp:96-134)
    Engine.answer_slice  runOptimizedDPFTreeQueryThread  (src/c/server.cpp:505-549, intended)
    Engine.eval_all      evalAllOptimizedDPF             (src/c/dpf_tree.cpp:473-598)
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check


def _buf(b):
    if isinstance(b, (bytes, bytearray)):
        b = np.frombuffer(bytes(b), dtype=np.uint8)
    b = np.ascontiguousarray(b, dtype=np.uint8)
    return b, b.ctypes.data_as(ctypes.c_void_p)


def key_len(num_parties, log_num_records, num_rounds):
    """calcOptimizedDPFTreeKeyLength (src/c/utils.cpp:85-90)."""
    return _lib.load().pir_engine_key_len(num_parties, log_num_records, num_rounds)


class Engine:
    def __init__(self, num_parties, party_index, log_num_records, record_bytes, num_rounds=1,
                 device=0, log_num_partitions=0, partition_index=0, is_byzantine=False):
        lib = _lib.load()
        self._lib = lib
        cfg = _lib.PirConfig(device, num_parties, party_index, log_num_records, record_bytes,
                             num_rounds, log_num_partitions, partition_index, int(is_byzantine))
        h = ctypes.c_void_p()
        check(lib.pir_engine_create(ctypes.byref(cfg), ctypes.byref(h)), "pir_engine_create")
        self._h = h
        self.num_parties = num_parties
        self.party_index = party_index
        self.n = log_num_records
        self.record_bytes = record_bytes
        self.num_rounds = num_rounds
        self.log_num_partitions = log_num_partitions
        self.partition_index = partition_index
        self.key_len = key_len(num_parties, log_num_records, num_rounds)
        self.num_rows = int(lib.pir_engine_num_rows(h))
        self.answer_bytes = num_rounds * record_bytes

    # -- lifetime ------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._lib.pir_engine_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- shard -----------------------------------------------------------------------------
    def set_shard(self, rows, row0=0):
        """rows: (nrows, record_bytes) uint8 array (or a flat buffer of whole rows)."""
        arr = np.ascontiguousarray(rows, dtype=np.uint8).reshape(-1, self.record_bytes)
        check(self._lib.pir_engine_set_shard(self._h, arr.ctypes.data_as(ctypes.c_void_p), row0,
                                             arr.shape[0], self.record_bytes),
              "pir_engine_set_shard")

    def fill_shard_random(self, seed):
        check(self._lib.pir_engine_fill_shard_random(self._h, seed), "fill_shard_random")

    def encode_across(self, num_files, k, files=None):
        """The erasure-coded shard computed on the GPU (client.cpp:70-97): from `files`
        (num_files x record_bytes host array) or, files=None, the reference's synthetic
        database (client.cpp:16-33)."""
        d_f, pitch = None, 0
        if files is not None:
            f = np.ascontiguousarray(np.asarray(files, np.uint8).reshape(num_files, -1))
            pitch = f.shape[1]
            d_f = self.alloc_dev(f.size)
        try:
            if d_f is not None:
                self.h2d(d_f, f.reshape(-1))
            check(self._lib.pir_engine_encode_across_dev(self._h, d_f, pitch, num_files, k),
                  "encode_across")
        finally:
            if d_f is not None:
                self.free_dev(d_f)

    def encode_within(self, num_files, file_bytes, k, files=None, party=0):
        """The Hollanti-mode shard (encoded within files) computed on the GPU (client.cpp:43-56,
        99-103): from `files` (num_files x file_bytes host array) or, files=None, the
        reference's synthetic database (client.cpp:16-33).  party: the server's party index
        (0: the engine's)."""
        d_f, pitch = None, 0
        if files is not None:
            f = np.ascontiguousarray(np.asarray(files, np.uint8).reshape(num_files, -1))
            pitch = f.shape[1]
            d_f = self.alloc_dev(f.size)
        try:
            if d_f is not None:
                self.h2d(d_f, f.reshape(-1))
            check(self._lib.pir_engine_encode_within_dev(self._h, d_f, pitch, num_files,
                                                         file_bytes, k, party), "encode_within")
        finally:
            if d_f is not None:
                self.free_dev(d_f)

    def shard_row(self, i):
        out = np.empty(self.record_bytes, np.uint8)
        check(self._lib.pir_engine_get_shard_row(self._h, i, out.ctypes.data_as(ctypes.c_void_p)),
              "get_shard_row")
        return out

    def get_shard(self, row0=0, nrows=None):
        nrows = self.num_rows - row0 if nrows is None else nrows
        out = np.empty((nrows, self.record_bytes), np.uint8)
        check(self._lib.pir_engine_get_shard(self._h, row0, nrows,
                                             out.ctypes.data_as(ctypes.c_void_p)), "get_shard")
        return out

    # -- answers ---------------------------------------------------------------------------
    def _check_key(self, key):
        k, kp = _buf(key)
        if k.size != self.key_len:
            raise ValueError(f"key has {k.size} bytes, expected {self.key_len}")
        return k, kp

    def answer(self, key):
        """(num_rounds, record_bytes) answer of this engine (XOR over ranks if a comm is
        attached)."""
        k, kp = self._check_key(key)
        out = np.empty((self.num_rounds, self.record_bytes), np.uint8)
        check(self._lib.pir_engine_answer(self._h, kp, out.ctypes.data_as(ctypes.c_void_p)),
              "pir_engine_answer")
        return out

    def answer_batch(self, keys):
        """(num_keys, num_rounds, record_bytes) answers of keys (a sequence of key_len-byte
        keys, or a (num_keys, key_len) uint8 array), batch_group keys per shard pass."""
        ks = [_buf(k)[0] for k in keys]
        for k in ks:
            if k.size != self.key_len:
                raise ValueError(f"key of {k.size} bytes, expected {self.key_len}")
        nk = len(ks)
        flat = np.ascontiguousarray(np.concatenate(ks) if nk else np.zeros(0, np.uint8),
                                    dtype=np.uint8)
        out = np.empty((nk, self.num_rounds, self.record_bytes), np.uint8)
        check(self._lib.pir_engine_answer_batch(self._h, flat.ctypes.data_as(ctypes.c_void_p), nk,
                                                out.ctypes.data_as(ctypes.c_void_p)),
              "pir_engine_answer_batch")
        return out

    @property
    def batch_group(self):
        """Keys answered per pass over the shard."""
        return self._lib.pir_engine_batch_group(self._h)

    @batch_group.setter
    def batch_group(self, g):
        check(self._lib.pir_engine_set_batch_group(self._h, int(g)), "set_batch_group")

    def answer_slice(self, key, thread_num, num_threads):
        k, kp = self._check_key(key)
        out = np.empty((self.num_rounds, self.record_bytes), np.uint8)
        check(self._lib.pir_engine_answer_slice(self._h, kp, thread_num, num_threads,
                                                out.ctypes.data_as(ctypes.c_void_p)),
              "pir_engine_answer_slice")
        return out

    def answer_slices(self, key, num_threads):
        """Every thread slice of one query at once, (num_threads, num_rounds, record_bytes):
        row t = answer_slice(key, t, num_threads) -- the T concurrent
        runOptimizedDPFTreeQueryThread calls of src/server_util/tree.go:60-76, from one tree and
        one pass over the shard where the shape allows."""
        k, kp = self._check_key(key)
        out = np.empty((num_threads, self.num_rounds, self.record_bytes), np.uint8)
        check(self._lib.pir_engine_answer_slices(self._h, kp, num_threads,
                                                 out.ctypes.data_as(ctypes.c_void_p)),
              "pir_engine_answer_slices")
        return out

    def answer_slices_dev(self, d_key, num_threads, d_results, stream=None):
        check(self._lib.pir_engine_answer_slices_dev(self._h, d_key, num_threads, d_results,
                                                     stream), "answer_slices_dev")

    def fold_gathered_dev(self, d_gathered, nranks, bytes_per_rank, d_result, stream=None):
        """The split-shard combine after the RCCL all-gather: d_result = XOR over r of the
        rank-r block of d_gathered (pir_engine_fold_gathered_dev)."""
        check(self._lib.pir_engine_fold_gathered_dev(self._h, d_gathered, nranks, bytes_per_rank,
                                                     d_result, stream), "fold_gathered_dev")

    def answer_coefs(self, coefs, row0=0, nrows=None):
        """Explicit-coefficient answer (runHollantiQuery[Thread], src/c/server.cpp:321-371):
        coefs is (num_rounds, rows) uint8 -- coefficient of engine row r in round a at
        coefs[a][r]; rows [row0, row0 + nrows) are answered.  (num_rounds, record_bytes)."""
        c = np.ascontiguousarray(np.asarray(coefs, np.uint8).reshape(self.num_rounds, -1))
        nrows = c.shape[1] - row0 if nrows is None else nrows
        ptrs = (ctypes.c_void_p * self.num_rounds)(*[c[a].ctypes.data for a in range(self.num_rounds)])
        out = np.empty((self.num_rounds, self.record_bytes), np.uint8)
        check(self._lib.pir_engine_answer_coefs(self._h, ptrs, row0, nrows,
                                                out.ctypes.data_as(ctypes.c_void_p)),
              "pir_engine_answer_coefs")
        return out

    def answer_coefs_dev(self, d_coefs, coef_pitch, row0, nrows, d_result, stream=None):
        check(self._lib.pir_engine_answer_coefs_dev(self._h, d_coefs, coef_pitch, row0, nrows,
                                                    d_result, stream), "answer_coefs_dev")

    def answer_mp(self, key, p, t, thread_num=0, num_threads=1):
        """Multiparty sqrt(N) DPF answer (runOptimizedMultiPartyDPFQuery[Thread], src/c/
        server.cpp:136-176, :384-430): the key's NUM_RSS_KEYS shares of every record (the
        layout of multiparty_dpf.cpp:467-539) scanned against the shard.  The engine's
        num_rounds must be mp_num_keys(p, t).  -> (num_rounds, record_bytes)."""
        k = np.frombuffer(bytes(key), np.uint8) if not isinstance(key, np.ndarray) else \
            np.ascontiguousarray(key, np.uint8)
        out = np.empty((self.num_rounds, self.record_bytes), np.uint8)
        check(self._lib.pir_engine_answer_mp(self._h, k.ctypes.data_as(ctypes.c_void_p), k.size,
                                             p, t, thread_num, num_threads,
                                             out.ctypes.data_as(ctypes.c_void_p)),
              "pir_engine_answer_mp")
        return out

    def answer_mp_dev(self, d_key, p, t, d_result, thread_num=0, num_threads=1, stream=None):
        check(self._lib.pir_engine_answer_mp_dev(self._h, d_key, p, t, thread_num, num_threads,
                                                 d_result, stream), "answer_mp_dev")

    def answer_cd(self, key, num_cd_keys_needed, num_cd_keys, thread_num=0, num_threads=1):
        """Covering-design sqrt(N) DPF answer (runCDQueryThread, src/c/server.cpp:443-492): the
        key's NUM_CD_KEYS shares (evalAllCDThread's layout, multiparty_dpf.cpp:617-690) scanned
        against the shard.  The engine's num_rounds must be num_cd_keys.
        -> (num_rounds, record_bytes)."""
        k = np.frombuffer(bytes(key), np.uint8) if not isinstance(key, np.ndarray) else \
            np.ascontiguousarray(key, np.uint8)
        out = np.empty((self.num_rounds, self.record_bytes), np.uint8)
        check(self._lib.pir_engine_answer_cd(self._h, k.ctypes.data_as(ctypes.c_void_p), k.size,
                                             num_cd_keys_needed, num_cd_keys, thread_num,
                                             num_threads, out.ctypes.data_as(ctypes.c_void_p)),
              "pir_engine_answer_cd")
        return out

    def answer_cd_dev(self, d_key, num_cd_keys_needed, num_cd_keys, d_result, thread_num=0,
                      num_threads=1, stream=None):
        check(self._lib.pir_engine_answer_cd_dev(self._h, d_key, num_cd_keys_needed, num_cd_keys,
                                                 thread_num, num_threads, d_result, stream),
              "answer_cd_dev")

    def eval_all(self, key):
        """(num_rounds, rows) DPF shares dataShare[a][i]."""
        k, kp = self._check_key(key)
        out = np.empty((self.num_rounds, self.num_rows), np.uint8)
        check(self._lib.pir_engine_eval_all(self._h, kp, out.ctypes.data_as(ctypes.c_void_p)),
              "pir_engine_eval_all")
        return out

    # -- device-resident path ----------------------------------------------------------------
    def alloc_dev(self, nbytes):
        p = ctypes.c_void_p()
        check(self._lib.pir_engine_alloc_dev(self._h, nbytes, ctypes.byref(p)), "alloc_dev")
        return p.value

    def free_dev(self, d_ptr):
        check(self._lib.pir_engine_free_dev(self._h, d_ptr), "free_dev")

    def set_party(self, party_index):
        """Answer later queries as party `party_index` over the same resident shard
        (server.partyIndex, src/c/server.h:16)."""
        check(self._lib.pir_engine_set_party_index(self._h, int(party_index)), "set_party_index")
        self.party_index = int(party_index)

    def h2d(self, d_ptr, host):
        h, hp = _buf(host)
        check(self._lib.pir_engine_memcpy_h2d(self._h, d_ptr, hp, h.size), "memcpy_h2d")

    def d2h(self, d_ptr, nbytes):
        out = np.empty(nbytes, np.uint8)
        check(self._lib.pir_engine_memcpy_d2h(self._h, out.ctypes.data_as(ctypes.c_void_p),
                                              d_ptr, nbytes), "memcpy_d2h")
        return out

    def answer_dev(self, d_key, d_result, stream=None):
        check(self._lib.pir_engine_answer_dev(self._h, d_key, d_result, stream), "answer_dev")

    def answer_batch_dev(self, d_keys, num_keys, d_result, stream=None):
        check(self._lib.pir_engine_answer_batch_dev(self._h, d_keys, num_keys, d_result, stream),
              "answer_batch_dev")

    def answer_stream_dev(self, d_keys, num_keys, d_result, stream=None):
        """A queue of independent queries, each its own tree and full shard pass, answered
        back to back in one launch (device pointers; asynchronous)."""
        check(self._lib.pir_engine_answer_stream_dev(self._h, d_keys, num_keys, d_result, stream),
              "answer_stream_dev")

    def reserve_queue(self, num_keys):
        """Pre-size the work buffers for queues of up to num_keys queries (no allocation, and
        so no device synchronisation, inside later answer_stream_dev calls)."""
        check(self._lib.pir_engine_reserve_queue(self._h, num_keys), "reserve_queue")

    def answer_stream(self, keys):
        """Host form of answer_stream_dev: [num_keys, num_rounds, record_bytes]."""
        keys = [bytes(k) for k in keys]
        nk = len(keys)
        d_k = self.alloc_dev(max(1, nk * self.key_len))
        try:
            d_r = self.alloc_dev(max(1, nk * self.answer_bytes))
            try:
                if nk:
                    self.h2d(d_k, b"".join(keys))
                self.answer_stream_dev(d_k, nk, d_r)
                self.sync()
                out = self.d2h(d_r, nk * self.answer_bytes)
            finally:
                self.free_dev(d_r)
        finally:
            self.free_dev(d_k)
        return out.reshape(nk, self.num_rounds, self.record_bytes)

    @property
    def stream(self):
        return self._lib.pir_engine_stream(self._h)

    def sync(self):
        check(self._lib.pir_engine_sync(self._h), "pir_engine_sync")

    def set_profiling(self, slots=64):
        """Record per-phase HIP events for up to `slots` answers (0 turns profiling off)."""
        check(self._lib.pir_engine_set_profiling(self._h, int(slots)), "set_profiling")

    def last_timings(self):
        """{phase: mean ms} over the answers recorded since the previous call."""
        arr = (_lib.PirKernelTime * 16)()
        n = self._lib.pir_engine_last_timings(self._h, arr, 16)
        if n < 0:
            check(n, "last_timings")
        return {arr[i].name.decode(): float(arr[i].ms) for i in range(n)}

    def profile_phases(self, d_key, iters=10):
        """Each phase alone (diagnostics): {phase: mean ms}."""
        out = (ctypes.c_float * 5)()
        check(self._lib.pir_engine_profile_phases(self._h, d_key, iters, out), "profile_phases")
        names = ["key_prep", "tree_frontier", "tree_stages", "scan", "reduce"]
        return {n: float(out[i]) for i, n in enumerate(names)}

    TRACE_PHASES = ["start", "key_parsed", "first_tile_root", "tile0_ready", "last_tile_ready",
                    "scan_done", "end"]

    def trace_query(self, d_key, num_keys=1):
        """One single-launch answer of a queue of num_keys keys (at d_key, key_len apart) with
        per-workgroup phase stamps (diagnostics): an array [workgroups, 256] of microseconds
        since the earliest workgroup start (layout: pir_engine_trace_query in
        include/pir_engine.h; 0 = stamp not reached; columns 56-57, 59-61, 128-159 and 192-255
        are raw shader-clock ticks or counts, divided by 100 like the rest)."""
        out = np.zeros((4096, 256), np.uint64)
        n = self._lib.pir_engine_trace_query(self._h, d_key, num_keys,
                                             out.ctypes.data_as(ctypes.c_void_p), 4096)
        check(min(n, 0), "trace_query")
        return out[:n].astype(np.float64) / 100.0

    # -- split shard ---------------------------------------------------------------------------
    def attach_comm(self, unique_id, nranks, rank):
        uid, up = _buf(unique_id)
        check(self._lib.pir_comm_attach(self._h, up, nranks, rank), "pir_comm_attach")

    def detach_comm(self):
        """Drop the communicator (aborted): this engine answers its partition alone again."""
        check(self._lib.pir_comm_detach(self._h), "pir_comm_detach")

    def comm_info(self):
        """RCCL's own view of this engine's communicator (ncclCommCount, ncclCommUserRank,
        ncclCommCuDevice; -1 when none is attached) and the engine device's PCI bus id."""
        ci = _lib.PirCommInfo()
        check(self._lib.pir_comm_info(self._h, ctypes.byref(ci)), "pir_comm_info")
        return {"attached": bool(ci.attached), "rccl_count": ci.count,
                "rccl_user_rank": ci.user_rank, "rccl_device": ci.device,
                "engine_device": ci.engine_device,
                "pci_bus_id": ci.pci_bus_id.decode(errors="replace")}


def mp_num_keys(p, t):
    """NUM_RSS_KEYS = choose(p, t) * (p - t) / p (params.cpp:618): shares per multiparty key."""
    return _lib.load().pir_engine_mp_num_keys(p, t)


def mp_key_len(p, n, t):
    """calcMultiPartyOptDPFKeyLength (utils.cpp:105-116)."""
    return _lib.load().pir_engine_mp_key_len(p, n, t)


def cd_key_len(p, n, t, num_cd_keys_needed, num_cd_keys):
    """calcCDDPFKeyLength (utils.cpp:118-129) = the bytes evalAllCDThread reads; 0: no layout."""
    return _lib.load().pir_engine_cd_key_len(p, n, t, num_cd_keys_needed, num_cd_keys)


def mp_eval_bytes(p, n, t):
    """Key bytes the multiparty evaluation reads (multiparty_dpf.cpp:485-511); -1: no layout."""
    return _lib.load().pir_engine_mp_eval_bytes(p, n, t)


def comm_unique_id():
    out = np.zeros(128, np.uint8)
    check(_lib.load().pir_comm_unique_id(out.ctypes.data_as(ctypes.c_void_p)), "pir_comm_unique_id")
    return out.tobytes()
