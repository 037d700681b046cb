#!/usr/bin/env python3
"""Benchmark of the MI355X tree-DPF PIR answer path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c24|c2|c3|c5|c4|c3b]

A step = one PIR query answered against the device-resident shard: key parse -> DPF
full-domain evaluation (AES-128 PRG tree) -> GF(2^8) inner product over every record ->
partial-answer reduce (-> RCCL all-gather + XOR fold across GPUs when N > 1).  Inputs (shard,
keys) are resident in HBM before the timed region; the answers stay in HBM.  The K timed steps
are K independent queries (distinct keys) answered as a queue: one launch of the query kernel,
each query still its own tree and its own full shard pass, the tree of query k+1 built while
query k's rows stream.  W warm-up queries (a queue of W) run before it.  The same K queries
answered one launch at a time are reported as `single_query` (the per-query latency).

Workloads:
  N = 1, default "c24": the north_star target shape, one shard of 2^24 x 1 KiB (16 GiB),
         p = 2.  The same line carries configs[1] (2^20 x 1 KiB, batch = 1) as `configs1_c2`
         and the N = 1 point of the split-shard curve (the 2^27 x 1 KiB logical shard as one
         128 GiB engine) as `c4_single_engine`.
  N > 1, default "c4": BASELINE configs[3], one logical server of 2^27 x 1 KiB split over the
         N GPUs (strong scaling: rank r holds rows [r 2^27/N, (r+1) 2^27/N) and evaluates the DPF
         subtree of its partition); the partial answers are combined by ONE RCCL all-gather +
         XOR fold per queue.  Rank 0 then answers the same queries with the whole shard on its
         own GPU (`n1_reference`), so the line carries the speedup over one GPU.
  --config c2|c3|c5 at N > 1: weak scaling (2^n rows per GPU of a 2^(n + log2 N) logical shard).
Launched per the driver contract with torch.distributed.run (gloo carries the barrier, the
timing max and the RCCL unique id).

rank 0 also prints the roofline of the dominant kernel (k_query: algorithmic bytes = K x
records x record_bytes per launch over the HIP-event duration of that launch) and a CPU
baseline: the reference src/c (oracle/_ref/libref.so, compiled from the reference's own
sources) on one host core answering one query of the SAME workload at full size, checked
bit-exactly against the GPU answer, plus an all-cores aggregate (one reference process per
core over one shared copy of the shard).
"""
import argparse
import ctypes
import json
import math
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident shard GiB/s per PIR query, 1/2/4/8 MI355X; bit-exact vs CPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured copy)
# best streaming read of 16 GiB (16-B non-temporal loads, any rows-in-flight / blocks-per-CU
# variant): tools/micro/read_bw.hip, profiles/r02_micro/read_bw.log
HBM_READ_MEASURED_GBS = 6762.0
GIB = float(1 << 30)
SHARD_SEED = 0xC0FFEE

CONFIGS = {
    # name: (log records, record bytes, parties, rounds, strong, workload text)
    # strong=False: 2^n rows per GPU (weak scaling); strong=True: 2^n rows in all
    "c24": (24, 1024, 2, 1, False, "north_star target shape: one shard 2^24 x 1 KiB, DPF depth 24, p=2"),
    "c2": (20, 1024, 2, 1, False, "configs[1]: 1 MI355X, one shard 2^20 x 1 KiB, DPF depth 20, batch=1 query"),
    "c3": (24, 256, 2, 1, False, "configs[2] shape per query: one shard 2^24 x 256 B (queries answered one at a time)"),
    "c5": (24, 1024, 8, 5, False, "configs[4] per-GPU server: 2^24 x 1 KiB shard, p=8 (k=5, r=2), NUM_ROUNDS=5"),
    "c4": (27, 1024, 2, 1, True, "configs[3]: one logical server, 2^27 x 1 KiB split over the GPUs, RCCL all-gather + XOR fold"),
}
# explicit-coefficient (polynomial / Hollanti) answers: a step = one query's NUM_ROUNDS
# coefficient vectors (device-resident) scanned against the shard (server.cpp:321-371)
COEF_CONFIGS = {
    "ch": (24, 1024, 1, "polynomial (Hollanti) PIR: 2^24 x 1 KiB shard, 1 round, explicit coefficient vector"),
    "ch3": (24, 1024, 3, "polynomial (Hollanti) PIR: 2^24 x 1 KiB shard, 3 rounds (k=3), explicit coefficient vectors"),
    "ch5": (24, 1024, 5, "polynomial (Hollanti) PIR: 2^24 x 1 KiB shard, 5 rounds (k=5), explicit coefficient vectors"),
}
# multiparty sqrt(N) DPF answers: a step = one query's key (device-resident) evaluated into
# NUM_RSS_KEYS shares and scanned against the shard (server.cpp:136-176)
MP_CONFIGS = {
    "cm": (24, 1024, 3, 1, "multiparty sqrt(N) DPF PIR (mode 1): 2^24 x 1 KiB shard, p=3, t=1 (2 shares, 4 seeds per row of 8192 records)"),
    "cm4": (24, 1024, 4, 1, "multiparty sqrt(N) DPF PIR (mode 1): 2^24 x 1 KiB shard, p=4, t=1 (3 shares, 8 seeds per row of 8192 records)"),
}
# covering-design sqrt(N) DPF answers (mode 4, runCDQueryThread, server.cpp:443-492): the same
# evaluation + scan on evalAllCDThread's layout -- (n, efs, NUM_CD_KEYS_NEEDED, NUM_CD_KEYS)
CD_CONFIGS = {
    "ccd": (24, 1024, 6, 3, "covering-design sqrt(N) DPF PIR (mode 4): 2^24 x 1 KiB shard, CD842 (the reference's P = 8 setup: 3 shares, 32 seeds per row of 32768 records)"),
    "ccd7": (24, 1024, 7, 4, "covering-design sqrt(N) DPF PIR (mode 4): 2^24 x 1 KiB shard, CD732 (4 shares, 64 seeds per row of 32768 records)"),
}
# batched configs: a step answers `batch` keys (distinct indices) against the shard
BATCH_CONFIGS = {
    "c3b": (24, 256, 2, 1, 128, "configs[2]: 1 MI355X, one shard 2^24 x 256 B, 128 batched queries"),
}


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return world, rank, local


# ------------------------------------------------------------------------------- CPU baseline
def _ref_lib():
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref.so"))
    L.ref_server_view.restype = ctypes.c_void_p
    L.ref_server_view.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p]
    L.ref_server_view_free.argtypes = [ctypes.c_void_p]
    L.ref_server_time.restype = ctypes.c_double
    L.ref_server_time.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    return L


def dump_shard(eng, path, chunk_rows=1 << 20):
    """The engine's rows -> a host file, in chunks (no full-size host copy)."""
    with open(path, "wb") as f:
        for r0 in range(0, eng.num_rows, chunk_rows):
            eng.get_shard(r0, min(chunk_rows, eng.num_rows - r0)).tofile(f)


def shard_file_path(nbytes):
    """A file for the shard copy the CPU processes share: /dev/shm when it has room."""
    d = "/dev/shm"
    if not (os.path.isdir(d) and os.access(d, os.W_OK)):
        d = None
    else:
        st = os.statvfs(d)
        if st.f_bavail * st.f_frsize < nbytes + (1 << 30):
            d = None
    return os.path.join(d or tempfile.gettempdir(), f"pir_bench_shard_{os.getpid()}.bin")


def cpu_baseline(path, n, efs, p, nq, key, gpu_answer, budget_s, cores):
    """The reference runOptimizedDPFTreeQuery (oracle/_ref/libref.so) on this host over the same
    shard (a read-only mapping of `path`): one core, then `cores` processes at once."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libref.so")
    if not os.path.exists(ref_so):
        return _cpu_port(path, n, efs, p, nq, key, gpu_answer)
    L = _ref_lib()
    shard = np.memmap(path, np.uint8, mode="r")
    keyb = np.frombuffer(bytes(key), np.uint8).copy()
    res = np.zeros(nq * efs, np.uint8)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    h = L.ref_server_view(p, 1, n, efs, nq, P(shard))
    t1 = L.ref_server_time(h, P(keyb), P(res), 1)
    reps = max(0, min(8, int(budget_s / max(t1, 1e-3)) - 1))  # first call doubles as warm-up
    t = L.ref_server_time(h, P(keyb), P(res), reps) / reps if reps else t1
    L.ref_server_view_free(h)
    del shard
    parity = bool(np.array_equal(res.reshape(nq, efs), gpu_answer))
    all_cores = None
    if cores > 1:
        try:
            all_cores = _cpu_all_cores(path, keyb, n, efs, p, nq, res, cores)
        except (OSError, RuntimeError, ValueError) as exc:  # a reported baseline: never fatal
            all_cores = {"error": f"{type(exc).__name__}: {exc}"}
    return {
        "value": ((1 << n) * efs / GIB) / t,
        "unit": "GiB/s",
        "cores": 1,
        "kind": "reference",
        "sample": f"{1 + reps} queries of the same workload at full size (2^{n} x {efs} B, p={p}, "
                  f"NUM_ROUNDS={nq}) on 1 host core, {t:.3f} s per query"
                  + (" (the first one timed)" if not reps else " (first one untimed)")
                  + "; oracle/_ref/libref.so: the reference src/c runOptimizedDPFTreeQuery "
                    "(OpenSSL EVP AES, log/exp gf_mul) over indexList rows pointing into a "
                    "read-only mapping of the shard",
        "s_per_query": t,
        "bit_exact_vs_gpu": parity,
        "host_cpu": _cpu_model(),
        "all_cores": all_cores,
    }


def _cpu_port(path, n, efs, p, nq, key, gpu_answer):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    shard = np.memmap(path, np.uint8, mode="r")
    t0 = time.perf_counter()
    res = O.answer(p, 1, n, efs, nq, key, shard)
    t = time.perf_counter() - t0
    return {"value": ((1 << n) * efs / GIB) / t, "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"1 query at full size on 1 host core; oracle/liboracle.so (plain-C "
                      f"restatement); {t:.3f} s", "s_per_query": t,
            "bit_exact_vs_gpu": bool(np.array_equal(res, gpu_answer)), "host_cpu": _cpu_model()}


def _cpu_all_cores(path, keyb, n, efs, p, nq, ref_answer, ncores):
    """All-cores reference aggregate: `ncores` worker PROCESSES, each a reference server over
    the same read-only shard mapping answering one query, started together.  Processes, not
    threads: in one process the reference's per-node EVP_EncryptInit_ex (utils.cpp:42)
    serialises on OpenSSL 3's shared cipher-fetch locks (16 threads answer no faster than 1)."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-worker", path, str(n), str(efs),
           str(p), str(nq), keyb.tobytes().hex()]
    procs = []
    try:
        procs = [subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
                 for _ in range(ncores)]
        for pr in procs:
            if pr.stdout.readline().strip() != "ready":
                raise RuntimeError("cpu worker failed to start")
        t0 = time.perf_counter()
        for pr in procs:
            pr.stdin.write("go\n")
            pr.stdin.flush()
        outs = [pr.stdout.readline().split() for pr in procs]
        wall = time.perf_counter() - t0
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
            pr.wait()
    agree = all(len(o) == 2 and o[1] == ref_answer.tobytes().hex() for o in outs)
    per = [float(o[0]) for o in outs if o]
    shard_bytes = (1 << n) * efs
    return {
        "value": ncores * (shard_bytes / GIB) / wall, "unit": "GiB/s", "cores": ncores,
        "sample": f"{ncores} worker processes over one shared read-only copy of the shard, one "
                  f"full-size query each, started together: {wall:.3f} s wall (per-process "
                  f"{min(per):.3f}-{max(per):.3f} s)",
        "answers_agree": bool(agree),
    }


def _cpu_worker(argv):
    """Child of _cpu_all_cores (never touches the GPU): a reference server over the shared shard
    file, one runOptimizedDPFTreeQuery on "go"; prints seconds and the answer hex."""
    path, n, efs, p, nq, keyhex = argv[0], *map(int, argv[1:5]), argv[5]
    L = _ref_lib()
    shard = np.memmap(path, np.uint8, mode="r")
    key = np.frombuffer(bytes.fromhex(keyhex), np.uint8).copy()
    res = np.zeros(nq * efs, np.uint8)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    h = L.ref_server_view(p, 1, n, efs, nq, P(shard))
    print("ready", flush=True)
    sys.stdin.readline()
    t = L.ref_server_time(h, P(key), P(res), 1)
    print(f"{t:.6f} {res.tobytes().hex()}", flush=True)
    L.ref_server_view_free(h)


def _host_cores():
    """Host processes for the all-cores CPU leg: this process's CPU share (the GPU box grants
    16 per GPU; nproc there shows the whole machine), capped by the affinity mask; one core is
    left to this (GPU) process, which also keeps within the box's 16-process guard."""
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    aff = len(os.sched_getaffinity(0))
    return max(1, (min(share, aff) if share > 0 else min(aff, 16)) - 1)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# --------------------------------------------------------------------------------- GPU legs
def _gf_table(c):
    t = np.zeros(256, np.uint8)
    for x in range(256):
        a, b, r = c, x, 0
        while b:
            if b & 1:
                r ^= a
            a = ((a << 1) ^ (0x11D if a & 0x80 else 0)) & 0xFF
            b >>= 1
        t[x] = r
    return t


class Ctx:
    """Distributed context: barrier + device sync around timed regions, max over ranks."""

    def __init__(self, world, rank, local):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world, self.rank, self.local = world, rank, local
        self.rehearsal = False
        self.host_fold = False  # no RCCL communicator: partition answers XORed over gloo

    def fold(self, arr):
        """Host-fold runs only (rehearsal, or the RCCL-init fallback): XOR of every rank's
        partition answer (gloo all-gather)."""
        if not self.host_fold:
            return arr
        t = self.torch.from_numpy(np.ascontiguousarray(arr))
        parts = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        out = parts[0].numpy().copy()
        for p in parts[1:]:
            out ^= p.numpy()
        return out

    def timed(self, eng, fn):
        self.sync(eng)
        t0 = time.perf_counter()
        fn()
        self.sync(eng)
        dt = time.perf_counter() - t0
        if self.world > 1:
            tt = self.torch.tensor([dt], dtype=self.torch.float64)
            self.dist.all_reduce(tt, op=self.dist.ReduceOp.MAX)
            dt = float(tt.item())
        return dt

    def sync(self, eng):
        eng.sync()
        self.torch.cuda.synchronize()
        if self.world > 1:
            self.dist.barrier()


def make_keys(pir, n, p, nq, count, rng, device, first=None):
    """count independent queries (distinct indices): [(index, [key of party 1, ..., p])]."""
    idxs = [int(i) for i in rng.choice(1 << n, count, replace=False)]
    if first is not None:
        idxs[0] = first
    fcw = pir.final_cw(p, nq, 1)
    return [(i, pir.gen_keys(n, i, p, nq, fcw=fcw,
                             seeds=rng.integers(0, 256, 16 * p, dtype=np.uint8).tobytes(),
                             device=device)) for i in idxs], fcw


def measure(ctx, eng, keys, W, K, single=True):
    """Warm-up queue of W, then the timed queue of K (HIP events around the query kernel), then
    the same K queries one launch each.  keys: party-1 keys (W + K of them)."""
    kl, ab = eng.key_len, eng.answer_bytes
    nkeys = W + K
    if len(keys) < nkeys:
        raise ValueError(f"measure: {len(keys)} keys for a warm-up of {W} and {K} timed queries")
    keys = keys[:nkeys]  # callers may pass more (the 1-GPU reference reuses the N-GPU key set)
    d_keys = eng.alloc_dev(kl * nkeys)
    d_res = eng.alloc_dev(ab * nkeys)
    eng.h2d(d_keys, b"".join(keys))
    d_kq, d_rq = d_keys + W * kl, d_res + W * ab
    eng.reserve_queue(max(W, K, 1))  # queue buffers sized at setup, as a server would
    if W:
        eng.answer_stream_dev(d_keys, W, d_res)
    box = {}
    if ctx.host_fold:
        # no device exchange: the answers go to the host and are XORed over gloo INSIDE the
        # timed region (the exchange a split-shard query cannot skip)
        def run_queue():
            eng.answer_stream_dev(d_kq, K, d_rq)
            box["q"] = ctx.fold(eng.d2h(d_rq, ab * K))
    else:
        def run_queue():
            eng.answer_stream_dev(d_kq, K, d_rq)
    eng.set_profiling(1)
    dt = ctx.timed(eng, run_queue)
    phases = eng.last_timings()
    eng.set_profiling(0)
    queue = (box["q"] if ctx.host_fold else eng.d2h(d_rq, ab * K)).reshape(
        K, eng.num_rounds, eng.record_bytes)
    out = {"ms": dt / K * 1e3, "phases": phases, "answers": queue}
    if single:
        for i in range(max(1, min(W, 5))):  # warm the one-query kernel (its own code object)
            eng.answer_dev(d_keys + (i % nkeys) * kl, d_res + (i % nkeys) * ab)
        if ctx.host_fold:
            def run_singles():
                box["s"] = [ctx.fold(eng.answer_dev(d_kq + i * kl, d_rq + i * ab) or
                                     eng.d2h(d_rq + i * ab, ab)) for i in range(K)]
            dt1 = ctx.timed(eng, run_singles)
            singles = np.stack(box["s"]).reshape(K, eng.num_rounds, eng.record_bytes)
        else:
            dt1 = ctx.timed(eng, lambda: [eng.answer_dev(d_kq + i * kl, d_rq + i * ab)
                                          for i in range(K)])
            singles = eng.d2h(d_rq, ab * K).reshape(K, eng.num_rounds, eng.record_bytes)
        eng.set_profiling(max(K, 1))
        for i in range(K):
            eng.answer_dev(d_kq + i * kl, d_rq + i * ab)
        out.update(ms1=dt1 / K * 1e3, phases1=eng.last_timings(), singles=singles)
        eng.set_profiling(0)
    eng.free_dev(d_keys)
    eng.free_dev(d_res)
    return out


def pir_check(ctx, eng, keyset, fcw, q_answers, n, g, parties=(2,)):
    """Full-size PIR property on every rank: for each party j (1-based) in `parties`, round r of
    the party-1 answers (from the queue) XOR round r of party j's answers of the same queries ==
    finalCW[r][j] * record (the key structure of dpf_tree.cpp:142-274; finalCW[r][j] at
    fcw[r * (p - 1) + j - 2], client.cpp:144-153)."""
    import erasurecodedpir_amd as pir  # noqa: F401
    nq, p1 = eng.num_rounds, len(keyset[0][1]) - 1
    ok = True
    for j in parties:
        eng.set_party(j)
        for q, (idx, ks) in enumerate(keyset):
            aj = ctx.fold(eng.answer(ks[j - 1]))
            owner = idx >> (n - g) if g else 0
            rec = eng.shard_row(idx - owner * eng.num_rows) if ctx.rank == owner else None
            if ctx.world > 1:
                rec = broadcast_from(rec, owner, eng.record_bytes)
            for r in range(nq):
                tab = _gf_table(int(fcw[r * p1 + j - 2]))
                ok &= bool(np.array_equal(q_answers[q][r] ^ aj[r], tab[rec]))
    eng.set_party(1)
    return ok


def roofline(kern_ms, local_bytes, K, config, world):
    algo = local_bytes * K
    achieved = algo / (kern_ms / 1e3) / 1e9 if kern_ms == kern_ms and kern_ms > 0 else None
    traffic, src = _pmc_traffic(config, world, K)
    return {
        "bound": "hbm",
        "kernel": f"k_query (DPF tree + GF(2^8) shard scan, {K} queries per launch)",
        "achieved": round(achieved, 1) if achieved else None,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
        "read_ceiling_measured": HBM_READ_MEASURED_GBS,
        "frac_of_read_ceiling": round(achieved / HBM_READ_MEASURED_GBS, 4) if achieved else None,
        "traffic": traffic,
        "traffic_source": src,
        "algorithmic_bytes_per_launch": int(algo),
        "algorithmic_bytes_per_query": int(local_bytes),
        "kernel_ms_per_launch": round(kern_ms, 5),
    }


VALU_PEAK_SPEC_T = 256 * 128 * 2.4e9 / 1e12  # lane-ops/s: 256 CUs x 4 SIMD-32 x 2.4 GHz
VALU_PEAK_MEASURED_T = 47.0  # 2-VGPR-source bitwise ops, all CUs (profiles/r02_micro/valu_rate.log)


def _lib_sha256():
    import hashlib
    h = hashlib.sha256()
    with open(os.path.join(ROOT, "erasurecodedpir_amd", "libpir_engine.so"), "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def _pmc_current(d):
    """A committed counter summary describes the loaded library only if it carries its sha."""
    return d.get("lib_sha256") is not None and d.get("lib_sha256") == _lib_sha256()


def _valu_roofline(config, world, kern_ms, queries_per_launch, leaves_per_query):
    """Integer-VALU ceiling of the dominant kernel (the AES tree's secondary
    roofline): VALU lane-ops per launch from the committed rocprofv3 --pmc SQ_INSTS_VALU pass
    (wave instructions x 64 lanes), over this run's measured kernel time."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if world != 1 or not os.path.exists(path) or not kern_ms or kern_ms != kern_ms:
        return None
    try:
        d = json.load(open(path))
        if not _pmc_current(d):  # counters of another build: not quoted
            return None
        c = d.get("counters_per_launch", {})
        insts = c.get("SQ_INSTS_VALU")
        if not insts:
            return None
        q_prof = d.get("queries_per_launch", queries_per_launch)
        ops_q = insts * 64 / q_prof
        lds_q = c.get("SQ_INSTS_LDS", 0) * 64 / q_prof
        achieved = ops_q * queries_per_launch / (kern_ms / 1e3) / 1e12
        return {"bound": "valu", "unit": "T lane-ops/s",
                "lane_ops_per_query": int(ops_q), "lane_ops_per_leaf": round(ops_q / leaves_per_query, 1),
                "lds_lane_ops_per_leaf": round(lds_q / leaves_per_query, 1),
                "achieved": round(achieved, 2), "peak_spec": round(VALU_PEAK_SPEC_T, 1),
                "peak_measured": VALU_PEAK_MEASURED_T,
                "frac_of_measured": round(achieved / VALU_PEAK_MEASURED_T, 3),
                "source": f"profiles/pmc_{config}.json (SQ_INSTS_VALU, SQ_INSTS_LDS per launch)"}
    except (OSError, ValueError, KeyError):
        return None


def _pmc_traffic(config, world, queries_per_launch):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 --pmc passes
    (profiles/pmc_<config>.json: bytes per query, measured), scaled to the launch's queries.
    Not measured inside this run (PMC collection needs its own profiler passes)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if world != 1 or not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
        per_q = d.get("hbm_bytes_per_query")
        if not per_q:
            return None, None
        src = (f"profiles/pmc_{config}.json (rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE, gfx950 "
               f"corrections), bytes per query x {queries_per_launch}")
        if not _pmc_current(d):
            src = "stale: " + src + " -- taken from a different libpir_engine.so build"
        return int(per_q * queries_per_launch), src
    except (OSError, ValueError):
        return None, None


def _c3b_ceilings():
    """configs[2]'s bound, from the committed per-kernel counters (profiles/pmc_c3b.json,
    tools/pmc_kernels.py; quoted only when they were taken on the loaded library): the leaf stage
    (k_subtree, ~77 % of the step) is LDS-lookup-bound -- its conflict-free LDS-array cycles over
    its duration -- and k_scan_t is LDS-bound through bank conflicts."""
    path = os.path.join(ROOT, "profiles", "pmc_c3b.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    cur = _pmc_current(d)
    ks = d.get("kernels", {})
    leaf, scan = ks.get("k_subtree<false", {}), ks.get("k_scan_t", {})
    if not leaf.get("ceilings"):
        return None
    lc, sc = leaf["ceilings"], scan.get("ceilings", {})
    return {"bound": "lds", "unit": "fraction of the LDS-array ceiling (32 lookups/clk/CU)",
            "kernel": "k_subtree leaf stage (8 keys x 2^24 leaves per launch)",
            "frac": lc.get("lds_frac_of_ceiling"),
            "lds_lookups_per_leaf": leaf.get("derived", {}).get("lds_lane_ops_per_leaf"),
            "valu_frac": lc.get("valu_frac_of_ceiling"),
            "scan_kernel": "k_scan_t (transposed four Russians, 64 planes)",
            "scan_lds_busy_with_conflicts": sc.get("lds_busy_share_with_conflicts"),
            "scan_lds_conflict_share": scan.get("derived", {}).get("lds_bank_conflict_share_of_lds_cycles"),
            "source": "profiles/pmc_c3b.json" + ("" if cur else " (stale: another libpir_engine.so build)")}


def r5(x):
    return round(float(x), 5)


def trace_stats(eng, keys, nk):
    """One traced k_query launch (pir_engine_trace_query: per-workgroup wall-clock stamps and
    s_memtime shader-clock stamps) of a queue of nk of `keys`, after the timed legs: the shader
    clock this box ran the kernel at (s_memtime ticks between the first and last stamped tile
    over the 100 MHz wall clock between them, median over workgroups) and, for the first query,
    when tile 0 was ready (the head before the first row can be folded).  None when the shape
    does not run k_query."""
    nk = max(1, min(nk, len(keys)))
    kl = eng.key_len
    try:
        d = eng.alloc_dev(kl * nk)
        try:
            eng.h2d(d, b"".join(keys[:nk]))
            tr = eng.trace_query(d, nk)
        finally:
            eng.free_dev(d)
    except Exception:  # noqa: BLE001 - shape without k_query, or no trace support
        return None
    if not len(tr):
        return None
    raw = tr * 100.0  # wall stamps back to 100 MHz ticks; shader-clock columns back to ticks
    g = [i for i in range(32) if tr[:, 64 + i].all() and tr[:, 128 + i].all()]
    if len(g) >= 2:
        ghz = (raw[:, 128 + g[-1]] - raw[:, 128 + g[0]]) / ((tr[:, 64 + g[-1]] - tr[:, 64 + g[0]]) * 1e3)
        span = f"tiles {g[0]}..{g[-1]} of a traced queue of {nk} queries"
    else:
        ghz = (raw[:, 57] - raw[:, 56]) / ((tr[:, 2] - tr[:, 0]) * 1e3)
        span = "start -> first tile root of one traced query"
    ghz = ghz[np.isfinite(ghz) & (ghz > 0)]
    return {"shader_clock_ghz": {"median": round(float(np.median(ghz)), 3),
                                 "min": round(float(ghz.min()), 3), "max": round(float(ghz.max()), 3),
                                 "source": "k_query s_memtime vs 100 MHz wall-clock stamps, " + span},
            "tile0_ready_us_median": round(float(np.median(tr[:, 3])), 2),
            "first_tile_root_us_median": round(float(np.median(tr[:, 2])), 2),
            "launch_end_us_max": round(float(tr[:, 6].max()), 2)}


def _pmc_issue(config, queries_per_launch, kern_ms, clock_ghz):
    """Issue-port ceilings of a compute-bound k_query from its committed, sha-stamped counters
    (profiles/pmc_<config>.json: SQ_INSTS_SALU / SQ_INSTS_VALU per launch): the share of the
    CUs' scalar issue (1 SALU per CU-clock) and vector issue (0.5 VALU per SIMD-clock, 4 SIMDs)
    this run's kernel time implies, at the clock this run measured (else the counters' implied
    clock).  None unless the counters describe the loaded library."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    if not _pmc_current(d) or not kern_ms or kern_ms != kern_ms:
        return None
    c = d.get("counters_per_launch", {})
    q_prof = d.get("queries_per_launch", queries_per_launch)
    f = clock_ghz or d.get("issue", {}).get("shader_clock_GHz_implied")
    if not f or not c.get("SQ_INSTS_SALU"):
        return None
    cyc = kern_ms / 1e3 * f * 1e9  # CU clocks of this run's launch
    salu = c["SQ_INSTS_SALU"] / q_prof * queries_per_launch
    valu = c.get("SQ_INSTS_VALU", 0) / q_prof * queries_per_launch
    return {"salu_issue_frac": round(salu / (256 * cyc), 4),
            "valu_issue_frac": round(valu / (256 * 4 * 0.5 * cyc), 4),
            "salu_insts_per_query": int(salu / queries_per_launch),
            "valu_insts_per_query": int(valu / queries_per_launch),
            "clock_ghz_used": round(f, 3),
            "clock_source": "this run's k_query stamps" if clock_ghz else "counters' implied clock",
            "source": f"profiles/pmc_{config}.json (SQ_INSTS_SALU / SQ_INSTS_VALU per launch, "
                      "sha-stamped at this library)"}


def single_phases(ph, ms_per_query):
    """The per-query phases of a lone answer, from the profiled pass (HIP events on the engine
    stream).  On the k_query path (fused == 2) key parse, tree and scan are ONE kernel, so the
    phases are what exists: launch (answer start -> k_query start), k_query, k_reduce, and the
    exchange / tail; they sum to the profiled answer, quoted beside the unprofiled ms_per_query
    (the two runs differ by the profiling events' own dispatch cost)."""
    if ph.get("fused") == 2.0:
        names = {"launch": "launch", "scan": "k_query", "reduce": "k_reduce",
                 "comm_fold": "exchange_and_tail"}
        phases = {names[k]: r5(ph[k]) for k in names if k in ph}
        total = ph.get("total", sum(phases.values()))
        return {"phases_ms": phases, "phases_sum_ms": r5(sum(phases.values())),
                "profiled_ms_per_query": r5(total),
                "phases_sum_over_ms_per_query": round(sum(phases.values()) / ms_per_query, 4)
                if ms_per_query else None,
                "phases_path": "k_query (key parse + DPF tree + scan in one launch) + k_reduce"}
    return {"phases_ms": {k: r5(v) for k, v in ph.items() if k not in ("chunks", "fused")},
            "phases_path": "multi-kernel (k_frontier / k_expand / k_fused or k_scan) + k_reduce"}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--cpu-worker":
        return _cpu_worker(sys.argv[2:])
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default=None,
                    choices=sorted(CONFIGS) + sorted(BATCH_CONFIGS) + sorted(COEF_CONFIGS) + sorted(MP_CONFIGS) + sorted(CD_CONFIGS),
                    help="default: c24 on one GPU, c4 (split shard) on several")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-budget", type=float, default=20.0,
                    help="seconds of single-core reference work (at least one full query)")
    ap.add_argument("--cpu-cores", type=int, default=-1,
                    help="processes of the all-cores reference leg (-1: this process's CPU "
                         "share minus one; 0 or 1: skip)")
    ap.add_argument("--no-extras", action="store_true",
                    help="N=1: skip the configs[1] and 2^27 single-engine extra legs")
    ap.add_argument("--queue-only", action="store_true",
                    help="profiling passes: only the warm-up and timed queues of the main "
                         "workload (run with --warmup equal to --steps so every launch of the "
                         "query kernel answers the same number of queries)")
    args = ap.parse_args()

    world, rank, local = dist_env()
    if world == 1 and args.gpus > 1:
        raise SystemExit("--gpus N>1 must be launched with torch.distributed.run")
    import torch
    import torch.distributed as dist

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    # PIR_BENCH_REHEARSAL=1 (diagnostics, N > 1 on a box with fewer GPUs): ranks share the
    # visible GPUs, no RCCL communicator is attached, and the partition answers are XOR-folded
    # over gloo on the host inside the timed region (the host-fold exchange below)
    rehearsal = world > 1 and os.environ.get("PIR_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    ctx = Ctx(world, rank, local)
    ctx.rehearsal = ctx.host_fold = rehearsal

    import erasurecodedpir_amd as pir
    from erasurecodedpir_amd.dist import broadcast_bytes, log2_exact

    config = args.config or ("c24" if world == 1 else "c4")
    if config in BATCH_CONFIGS:
        return run_batch(args, ctx, config)
    if config in COEF_CONFIGS:
        return run_coefs(args, ctx, config)
    if config in MP_CONFIGS or config in CD_CONFIGS:
        return run_mp(args, ctx, config)
    n_cfg, efs, p, nq, strong, workload = CONFIGS[config]
    g = log2_exact(world)
    n = n_cfg if strong else n_cfg + g  # logical tree depth
    W, K = args.warmup, args.steps
    seed = int.from_bytes(broadcast_bytes(os.urandom(8) if rank == 0 else None)
                          if world > 1 else os.urandom(8), "little")
    rng = np.random.default_rng(seed)
    keyset, fcw = make_keys(pir, n, p, nq, W + K, rng, local)

    eng = pir.Engine(p, 1, n, efs, nq, device=local, log_num_partitions=g, partition_index=rank)
    eng.fill_shard_random(SHARD_SEED)
    comm_err = None
    if world > 1 and not rehearsal:
        comm_err = attach_or_fallback(pir, eng, world, rank)
        ctx.host_fold = comm_err is not None
    m = measure(ctx, eng, [ks[0] for _, ks in keyset], W, K, single=not args.queue_only)
    ms = m["ms"]
    shard_bytes = float(1 << n) * efs  # logical shard (all ranks)
    value = shard_bytes / GIB / (ms / 1e3)
    if args.queue_only:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": round(value, 3), "unit": "GiB/s",
                              "ms_per_step": r5(ms), "steps": K, "warmup": W,
                              "config": {"workload": workload},
                              "mode": "queue-only profiling pass"}), flush=True)
        eng.close()
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    timed = keyset[W:]
    # PIR correctness at full size on every rank (the party-2 answers come from the same
    # resident shard, answered as party 2)
    pir_ok = pir_check(ctx, eng, timed[:4] if p == 2 else timed[:2], fcw, m["answers"], n, g,
                       parties=sorted({2, p}))
    # host API (key H2D + answer D2H + sync): the PCIe-inclusive rate
    k0 = timed[0][1][0]
    incl_steps = min(20, K)
    t1 = time.perf_counter()
    for _ in range(incl_steps):
        a1 = eng.answer(k0)
    a1 = ctx.fold(a1)
    incl_ms = (time.perf_counter() - t1) / incl_steps * 1e3
    same = bool(np.array_equal(a1, m["singles"][0]))
    queue_same = bool(np.array_equal(m["answers"], m["singles"]))

    ph = m["phases"]
    local_bytes = float(eng.num_rows) * efs
    kern_ms = ph.get("scan", float("nan"))  # the k_query launch (all K queries)
    path = {2.0: "k_query", 1.0: "k_fused", 0.0: "k_expand+k_scan"}.get(ph.get("fused"), "?")
    rl = roofline(kern_ms, local_bytes, K, config, world)
    rl["kernel"] = rl["kernel"].replace("k_query", path)
    if world == 1:  # the clock this box ran the kernel at (a traced queue of 2 after the timing)
        ts = trace_stats(eng, [ks[0] for _, ks in keyset[W:]], 2)
        rl["shader_clock_ghz"] = ts["shader_clock_ghz"] if ts else None
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": r5(ms),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": workload if world == 1 or strong else
            f"split shard, weak scaling: {world} x 2^{n_cfg} x {efs} B partitions of one 2^{n} x {efs} B logical shard (RCCL all-gather + XOR fold)",
            "records": 1 << n, "record_bytes": efs, "parties": p, "num_rounds": nq,
            "records_per_gpu": int(eng.num_rows), "dpf_depth": n,
            "parallelism": (f"split-shard x{world}" + (
                " (REHEARSAL: shared GPU, no RCCL, host gloo fold inside the timed region)"
                if rehearsal else (" (host gloo exchange inside the timed region: RCCL "
                                   "communicator init failed)" if comm_err else "")))
                           if world > 1 else "single",
            "step": "one PIR query: its own DPF key and tree, one full pass over the shard",
            "mode": "query queue: the K timed queries (distinct keys) are answered back to back "
                    "in one launch, the tree of query k+1 built while query k streams",
        },
        "roofline": rl,
        "roofline_valu": _valu_roofline(config, world, kern_ms, K, float(eng.num_rows)),
        "single_query": {
            "ms_per_query": r5(m["ms1"]),
            "value": round(shard_bytes / GIB / (m["ms1"] / 1e3), 3),
            "unit": "GiB/s",
            "note": "answer_dev per step (one launch per query, nothing queued behind it)",
            **single_phases(m["phases1"], m["ms1"]),
        },
        "inclusive_h2d_key_d2h_answer": {"ms_per_query": round(incl_ms, 4),
                                         "value": round(shard_bytes / GIB / (incl_ms / 1e3), 3),
                                         "unit": "GiB/s"},
        "parity": {"pir_record_recovered": pir_ok, "host_api_equals_device_api": same,
                   "queue_equals_one_at_a_time": queue_same},
    }
    if world > 1:  # per-rank kernel and exchange times of the timed queue
        rl_rank = roofline(kern_ms, local_bytes, K, config, world)  # this rank's own kernel time
        mine = {"rank": rank, "k_query_ms": r5(kern_ms), "reduce_ms": r5(ph.get("reduce", 0)),
                "allgather_xor_fold_ms": r5(ph.get("comm_fold", 0)),
                "queue_total_ms": r5(ph.get("total", 0)),
                "roofline": {k: rl_rank[k] for k in ("bound", "achieved", "peak", "unit", "frac",
                                                     "traffic", "algorithmic_bytes_per_launch")},
                "rccl": eng.comm_info()}
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        out["per_rank"] = allr
        out.update(exchange_fields(allr, world, ctx.host_fold, comm_err))
    cpu_path = None
    threads_leg = rank == 0 and world == 1 and not args.no_extras and config == "c24"
    if rank == 0 and world == 1 and (not args.no_cpu or threads_leg):
        cpu_path = shard_file_path(int(local_bytes))
        dump_shard(eng, cpu_path)
    cpu_key, cpu_want = k0, m["singles"][0]
    if threads_leg:
        try:
            out["threads_c24"] = thread_leg(ctx, pir, eng, [ks[0] for _, ks in timed],
                                            list(m["singles"]), cpu_path, n, efs)
        except Exception:
            os.unlink(cpu_path)
            raise
    eng.close()

    if strong and world > 1:
        # the same K queries answered by ONE GPU holding the whole logical shard (rank 0's GPU,
        # after its partition engine is freed): the 1-GPU point of the strong-scaling curve
        if rank == 0:
            e1 = pir.Engine(p, 1, n, efs, nq, device=local)
            e1.fill_shard_random(SHARD_SEED)
            solo = Ctx(1, 0, local)
            W1 = min(W, 2)  # the same K timed queries as the split-shard run (keys W .. W+K-1)
            m1 = measure(solo, e1, [ks[0] for _, ks in keyset][W - W1:], W1, K, single=False)
            e1.close()
            v1 = shard_bytes / GIB / (m1["ms"] / 1e3)
            out["n1_reference"] = {
                "ms_per_query": r5(m1["ms"]), "value": round(v1, 3), "unit": "GiB/s",
                "k_query_ms": r5(m1["phases"].get("scan", 0)),
                "answers_equal_split_shard": bool(np.array_equal(m1["answers"], m["answers"])),
                "note": "the same K queries answered by one engine holding the whole 2^27 x 1 KiB "
                        "shard (128 GiB) on rank 0's GPU"}
            out["speedup_vs_1gpu"] = round(value / v1, 3)
        dist.barrier()

    if rank == 0 and world == 1 and not args.no_extras:
        # the drop-in's setup -> first answer (north_star shape; configs[4]'s per-server shape)
        out["setup_c24"] = setup_leg(ctx, pir, 24, 1024, 1, 0)  # k = 1, r = 0: p = 2
        out["setup_c5"] = setup_leg(ctx, pir, 26, 1024, 5, 2, party=3)
        out["configs1_c2"] = batch1_first(extra_leg(ctx, pir, "c2", W, K, rng, trace=1))
        if config != "c4":
            out["c4_single_engine"] = extra_leg(ctx, pir, "c4", min(W, 2), min(K, 16), rng,
                                                single=False)
        if config != "c5":
            out["configs4_c5"] = extra_leg(ctx, pir, "c5", min(W, 3), min(K, 20), rng,
                                           single=False, trace=2)
        b = measure_batch(min(K, 8), min(W, 2), ctx, "c3b")
        out["configs2_c3b"] = {k: b[k] for k in ("value", "unit", "value_kind", "steps", "warmup",
                                                 "ms_per_step", "ms_per_key", "keys_per_s",
                                                 "shard_passes_per_step", "parity")}
        out["configs2_c3b"]["workload"] = b["config"]["workload"]
        out["configs2_c3b"]["roofline"] = _c3b_ceilings()
    if cpu_path and args.no_cpu:
        os.unlink(cpu_path)
    elif cpu_path:
        try:
            cores = _host_cores() if args.cpu_cores < 0 else args.cpu_cores
            out["cpu_baseline"] = cpu_baseline(cpu_path, n, efs, p, nq, cpu_key, cpu_want,
                                               args.cpu_budget, cores)
            out["parity"]["gpu_equals_cpu_reference"] = out["cpu_baseline"]["bit_exact_vs_gpu"]
        finally:
            os.unlink(cpu_path)
        if not args.no_extras and os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref.so")):
            out["cpu_baselines"] = per_config_cpu(ctx, pir, rng, out["cpu_baseline"])
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def attach_or_fallback(pir, eng, world, rank):
    """Attach the RCCL communicator on every rank, or fall back together: the engine's init is
    non-blocking and bounded ($PIR_COMM_INIT_TIMEOUT, pir_comm_attach), every rank reports its
    outcome over gloo, and if any rank failed every rank detaches (an engine without a
    communicator answers its partition) and the run exchanges the partial answers over gloo on
    the host inside the timed region, labelled in the line -- returns the error, or None.
    $PIR_BENCH_NO_FALLBACK=1: all ranks exit with status 3 and the message instead (no retry,
    no re-exec)."""
    import torch.distributed as dist
    from erasurecodedpir_amd.dist import broadcast_bytes

    err, uid = None, None
    if rank == 0:
        try:
            uid = pir.comm_unique_id()
        except Exception as ex:  # noqa: BLE001 -- reported below, on every rank
            err = f"ncclGetUniqueId: {ex}"
    uid = broadcast_bytes(uid)
    if uid is None and err is None:
        err = "no unique id from rank 0"
    if err is None:
        try:
            eng.attach_comm(uid, world, rank)
        except Exception as ex:  # noqa: BLE001
            err = f"{type(ex).__name__}: {ex}"
    errs = [None] * world
    dist.all_gather_object(errs, err)
    bad = [(r, e) for r, e in enumerate(errs) if e]
    if not bad:
        return None
    msg = (f"RCCL communicator init failed on {len(bad)} of {world} ranks: "
           + "; ".join(f"rank {r}: {e}" for r, e in bad))
    if rank == 0:
        print(f"bench.py: {msg}", file=sys.stderr, flush=True)
    if os.environ.get("PIR_BENCH_NO_FALLBACK") == "1":
        eng.close()
        dist.destroy_process_group()
        sys.exit(3)
    if err is None:
        eng.detach_comm()  # this rank joined a communicator the others did not
    return msg[:300]


def rccl_ranks_ok(per_rank, world):
    """True iff RCCL itself reports the run's `world` ranks: every rank has a communicator
    attached, ncclCommCount == world and ncclCommUserRank == the rank on every rank, and the
    ranks' devices are `world` distinct GPUs (distinct PCI bus ids)."""
    if len(per_rank) != world:
        return False
    infos = [(r.get("rank"), r.get("rccl") or {}) for r in per_rank]
    if not all(i.get("attached") and i.get("rccl_count") == world and i.get("rccl_user_rank") == rk
               for rk, i in infos):
        return False
    bus = [i.get("pci_bus_id") for _, i in infos]
    return all(bus) and len(set(bus)) == world


def exchange_fields(per_rank, world, host_fold, comm_err):
    """Top-level fields of an N > 1 line saying what carried the exchange.  A host-fold run
    (rehearsal, or the RCCL-init fallback) is labelled so that its value cannot be read as an
    RCCL number."""
    ok = rccl_ranks_ok(per_rank, world) and not host_fold
    out = {"rccl_ranks_ok": bool(ok),
           "exchange": ("rccl all-gather + k_xor_fold" if not host_fold else
                        "host: D2H + gloo all-gather + numpy XOR" +
                        (f" (RCCL init failed: {comm_err})" if comm_err else " (rehearsal)"))}
    if host_fold:
        out["value_kind"] = ("HOST-FOLD FALLBACK: the partition answers were XORed on the host over "
                             "gloo inside the timed region -- NOT an RCCL/xGMI measurement")
    elif not ok:
        out["value_kind"] = ("RCCL communicator attached, but RCCL's own view does not show "
                             f"{world} ranks on {world} distinct GPUs (per_rank[].rccl)")
    return out


def extra_leg(ctx, pir, config, W, K, rng, single=True, trace=0):
    """Another workload on this GPU (N = 1): queue and single-query rates; trace > 0: one traced
    queue of `trace` queries after the timed runs (shader clock, tile-0 head: trace_stats)."""
    n, efs, p, nq, _, workload = CONFIGS[config]
    keyset, fcw = make_keys(pir, n, p, nq, W + K, rng, ctx.local)
    eng = pir.Engine(p, 1, n, efs, nq, device=ctx.local)
    eng.fill_shard_random(SHARD_SEED)
    m = measure(ctx, eng, [ks[0] for _, ks in keyset], W, K, single=single)
    tstats = trace_stats(eng, [ks[0] for _, ks in keyset[W:]], trace) if trace else None
    # every round's share property against parties 2 and p (all of them for p = 2)
    ok = pir_check(ctx, eng, keyset[W:W + 2], fcw, m["answers"], n, 0,
                   parties=sorted({2, p}))
    # queue == one launch per query (the first two timed keys, when the leg times no singles)
    q1 = None if single else all(np.array_equal(eng.answer(keyset[W + i][1][0]), m["answers"][i])
                                 for i in range(min(2, K)))
    eng.close()
    gib = float(1 << n) * efs / GIB
    kern = m["phases"].get("scan", float("nan"))
    res = {"workload": workload, "steps": K, "warmup": W, "ms_per_query": r5(m["ms"]),
           "value": round(gib / (m["ms"] / 1e3), 3), "unit": "GiB/s",
           "k_query_ms_per_launch": r5(kern),
           "roofline_frac": round(gib * GIB * K / (kern / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if kern > 0 else None,
           "pir_record_recovered": ok}
    if tstats:
        res["trace"] = tstats
    if config == "c5":  # compute-bound: the issue ports beside HBM
        ck = tstats["shader_clock_ghz"]["median"] if tstats else None
        iss = _pmc_issue(config, K, kern, ck)
        res["roofline"] = {
            "bound": "issue: the four-Russians fold's own instruction stream (4 per plane per "
                     "scan wave; neither the scalar nor the vector port saturates -- "
                     "profiles/r06/r6b_fold_mix.txt)",
            "hbm_frac": res["roofline_frac"], "hbm_peak_GBps": HBM_PEAK_GBS,
            **(iss or {"counters": "profiles/pmc_c5.json is not stamped with this library: "
                                   "no issue fractions quoted"}),
            "shader_clock_ghz": ck,
            "note": "per plane of the fold: s_bfe_u32 + s_set_gpr_idx_idx (SALU) + 2 indexed "
                    "v_xor (VALU); salu/valu_issue_frac = the launch's SALU / VALU instructions "
                    "over the port capacity at this run's clock (1 SALU per CU-clock; 0.5 VALU "
                    "per SIMD-clock x 4 SIMDs)"}
    if single:
        res["single_query"] = {"ms_per_query": r5(m["ms1"]),
                               "value": round(gib / (m["ms1"] / 1e3), 3), "unit": "GiB/s",
                               "note": "batch = 1: one launch per query",
                               "k_query_ms": r5(m["phases1"].get("scan", float("nan"))),
                               "k_reduce_ms": r5(m["phases1"].get("reduce", float("nan")))}
        if config == "c2" and tstats:  # the lone query's floor model (Bounds)
            head_ms = tstats["tile0_ready_us_median"] / 1e3
            stream_ms = float(1 << n) * efs / (HBM_READ_MEASURED_GBS * 1e9) * 1e3
            red_ms = m["phases1"].get("reduce", 0.0)
            floor = head_ms + stream_ms + red_ms
            res["single_query"]["roofline"] = {
                "bound": "latency + stream: the dependent PRG head before the first row, then "
                         "the shard at the measured read ceiling, then k_reduce",
                "head_ms": r5(head_ms), "stream_ms": r5(stream_ms), "reduce_ms": r5(red_ms),
                "floor_ms": r5(floor), "achieved_ms": r5(m["ms1"]),
                "frac_of_floor": round(floor / m["ms1"], 4),
                "hbm_frac": round(float(1 << n) * efs / (m["ms1"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "read_ceiling_GBps": HBM_READ_MEASURED_GBS,
                "source": "head = median tile-0-ready stamp of this run's traced launch "
                          "(key parse + 10-level descent + tile 0's 10 levels); stream = 1 GiB at "
                          "profiles/r02_micro/read_bw.log's ceiling; reduce = this run's k_reduce"}
        res["queue_equals_one_at_a_time"] = bool(np.array_equal(m["answers"], m["singles"]))
    else:
        res["queue_equals_one_at_a_time"] = bool(q1)
    return res


def cpu_sample(ctx, pir, rng, n, efs, p, nq, full_n, what):
    """The reference (oracle/_ref/libref.so) answering one query of a BASELINE config's shape on
    one host core, at 2^n rows (full_n: the config's own size), bit-exact against the GPU's
    answer of the same key over the same shard.  Its GiB/s is size-independent to first order
    (the reference's tree and scan are both linear in the rows), so a sample at fewer rows is
    reported as that config's rate, labelled."""
    keyset, _ = make_keys(pir, n, p, nq, 1, rng, ctx.local)
    key = keyset[0][1][0]
    eng = pir.Engine(p, 1, n, efs, nq, device=ctx.local)
    try:
        eng.fill_shard_random(SHARD_SEED)
        want = eng.answer(key)
        path = shard_file_path((1 << n) * efs)
        dump_shard(eng, path)
    finally:
        eng.close()
    try:
        L = _ref_lib()
        shard = np.memmap(path, np.uint8, mode="r")
        keyb = np.frombuffer(bytes(key), np.uint8).copy()
        res = np.zeros(nq * efs, np.uint8)
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        h = L.ref_server_view(p, 1, n, efs, nq, P(shard))
        t = L.ref_server_time(h, P(keyb), P(res), 1)
        L.ref_server_view_free(h)
        del shard
    finally:
        os.unlink(path)
    gib = (1 << n) * efs / GIB
    return {"workload": what, "value": round(gib / t, 4), "unit": "GiB/s", "cores": 1,
            "kind": "reference", "s_per_query": round(t, 4),
            "s_per_query_at_full_size": round(t * (1 << (full_n - n)), 2),
            "sample": (f"1 query at 2^{n} x {efs} B, p={p}, NUM_ROUNDS={nq} on 1 host core"
                       + ("" if n == full_n else f" (the config has 2^{full_n} rows: the full-size "
                                                 f"time is scaled by 2^{full_n - n})")),
            "bit_exact_vs_gpu": bool(np.array_equal(res.reshape(nq, efs), want))}


def per_config_cpu(ctx, pir, rng, main_leg):
    """BASELINE.md section 3's per-config CPU figures: the reference src/c path
    (runOptimizedDPFTreeQuery, server.cpp:96-134) on one host core for every config shape."""
    out = {
        "configs1_c2": cpu_sample(ctx, pir, rng, 20, 1024, 2, 1, 20,
                                  "configs[1]: 2^20 x 1 KiB, p=2, one query (full size)"),
        "configs2_c3_per_key": cpu_sample(ctx, pir, rng, 20, 256, 2, 1, 24,
                                          "configs[2]: 2^24 x 256 B, p=2 -- per key (the "
                                          "reference has no batched answer: 128 keys = 128 queries)"),
        "configs4_c5": cpu_sample(ctx, pir, rng, 18, 1024, 8, 5, 24,
                                  "configs[4] per server: 2^24 x 1 KiB, p=8, NUM_ROUNDS=5"),
    }
    t24 = main_leg.get("s_per_query")
    if t24:
        out["configs3_c4"] = {
            "workload": "configs[3]: one logical 2^27 x 1 KiB server (8 x 2^24 partitions)",
            "value": round(128.0 / (8 * t24), 4), "unit": "GiB/s", "cores": 1, "kind": "reference",
            "s_per_query_at_full_size": round(8 * t24, 2),
            "sample": "derived: 8 x the 2^24 x 1 KiB query timed in cpu_baseline (the reference "
                      "cannot evaluate a depth-27 tree: int overflow, dpf_tree.cpp:484-485)"}
    return out


def batch1_first(res):
    """configs[1] is defined at batch = 1 (BASELINE.json configs[1]): its value and ms_per_query
    are the one-launch-per-query figures; the queue's stay beside them as `queue`."""
    sq = res.pop("single_query")
    res["queue"] = {"ms_per_query": res.pop("ms_per_query"), "value": res.pop("value"),
                    "unit": "GiB/s", "k_query_ms_per_launch": res.pop("k_query_ms_per_launch"),
                    "roofline_frac": res.pop("roofline_frac"),
                    "note": "the same K queries answered as ONE queued launch"}
    res.update(ms_per_query=sq["ms_per_query"], value=sq["value"], unit="GiB/s",
               value_kind="batch = 1: one launch per query (answer_dev), K queries back to back",
               k_query_ms=sq.get("k_query_ms"), k_reduce_ms=sq.get("k_reduce_ms"))
    if "roofline" in sq:
        res["roofline"] = sq["roofline"]
    return res


def setup_leg(ctx, pir, L, f, k, r, party=1, T=16, check=True):
    """The drop-in's SETUP -> first answer through the reference's names (pir_server.h), as the
    Go server runs it: setup() of src/server/server.go:299-331 (setSystemParams,
    initialize_client, initializeServer with LOG_NUM_FILES rows, encode_across_files_server --
    the shim encodes from the client's host files on the GPU and leaves the shard in HBM), then
    RunTreeQuery's T-goroutine query (src/server_util/tree.go:17-101: T concurrent
    runOptimizedDPFTreeQueryThread calls + assemblDPFTreeQueryThreadResults, here the shim's C++
    pool), then FreeServer (tree.go:96).  Host wall clock of each step."""
    from erasurecodedpir_amd import server as S
    steps = {}
    t0 = time.perf_counter()
    S.setSystemParams(L, f, 1, k, r, 0, 1, 0, 0)
    prm = S.params()
    p, n, nq, efs = (prm["NUM_PARTIES"], prm["LOG_NUM_ENCODED_FILES"], prm["NUM_ROUNDS"],
                     prm["ENCODED_FILE_SIZE_BYTES"])
    cl = S.Client(L, f)
    t1 = time.perf_counter()
    sv = S.Server(party, prm["LOG_NUM_FILES"], efs, 0, T)
    t2 = time.perf_counter()
    cl.encode_across_files_server(sv)
    t3 = time.perf_counter()
    steps.update(set_params_and_initialize_client_s=t1 - t0, initialize_server_s=t2 - t1,
                 encode_across_files_server_s=t3 - t2)
    fcw = pir.final_cw(p, nq, 1)
    idx = (1 << n) // 3 + 5
    keys = pir.gen_keys(n, idx, p, nq, fcw=fcw, device=ctx.local)  # the client's, not timed
    q0 = time.perf_counter()
    a1 = sv.runTreeQueryThreads(keys[party - 1], T)
    q1 = time.perf_counter()
    a2 = sv.runTreeQueryThreads(keys[party - 1], T)
    q2 = time.perf_counter()
    parity = {"second_query_equals_first": bool(np.array_equal(a1, a2))}
    if check:
        # the setup's rows (pirServerSyncRows) against the encode of the reference's synthetic
        # database (client.cpp:16-33, :70-97) for a few rows, computed here on the host
        def file_bytes(v):
            return np.arange(f, dtype=np.uint8) if v == 1 else np.full(f, v & 0xFF, np.uint8)
        encdb = -(-(1 << L) // k)
        ok = True
        for row in (0, 1, idx, (1 << n) - 1):
            want = np.zeros(efs, np.uint8)
            for j in range(k):
                src = encdb * j + row
                if src < (1 << L):
                    want ^= _gf_table(_gf_pow(party, j))[file_bytes(src)]
            ok &= bool(np.array_equal(sv.read_row(row), want))
        parity["setup_rows_match_host_encode"] = ok
        if k == 1 and p == 2:  # a second server: ans_1 ^ ans_2 == finalCW * record (PIR property)
            sv2 = S.Server(2, prm["LOG_NUM_FILES"], efs, 0, T)
            cl.encode_across_files_server(sv2)
            b = sv2.runTreeQueryThreads(keys[1], T)
            sv2.freeServer()
            parity["pir_record_recovered"] = bool(np.array_equal(
                a1[0] ^ b[0], _gf_table(int(fcw[0]))[file_bytes(idx)]))
    q3 = time.perf_counter()
    sv.freeServer()
    q4 = time.perf_counter()
    S.wait_freed()  # the teardown freeServer handed to the reaper thread (off the answer path)
    q5 = time.perf_counter()
    cl.free_client()
    return {"workload": f"server setup -> first answer through pir_server.h: setSystemParams(L={L}, "
                        f"f={f}, k={k}, r={r}) -> p={p}, 2^{n} x {efs} B shard, NUM_ROUNDS={nq}; "
                        f"party {party}; T={T} Thread calls per query",
            "setup_s": round(t3 - t0, 4), "steps_s": {kk: round(v, 4) for kk, v in steps.items()},
            "first_query_ms": round((q1 - q0) * 1e3, 4),
            "second_query_ms": round((q2 - q1) * 1e3, 4),
            "free_server_ms": round((q4 - q3) * 1e3, 4),
            "free_server_background_teardown_ms": round((q5 - q4) * 1e3, 4),
            "client_files_gib": round((1 << L) * f / GIB, 3),
            "parity": parity,
            "note": "host wall clock; the setup encodes on the GPU from the client's host files "
                    "(pinned, double-buffered, multi-threaded staging) and leaves the shard in HBM, "
                    "so the first query is a device-resident answer"}


def _gf_pow(a, e):
    r = 1
    for _ in range(e):
        r = int(_gf_table(a)[r]) if a else r  # gf_pow(0, e) == 1 (isa-l log-table quirk)
    return r


def thread_leg(ctx, pir, eng, keys, want, shard_path, n, efs, T=16, K=10):
    """The reference's own call shape for a query (src/server_util/tree.go:60-76): T goroutines
    each call runOptimizedDPFTreeQueryThread(s, key, t, T) on ONE server (T = 16: the AWS
    config's threads, bench/run_tests.py:180), then assemblDPFTreeQueryThreadResults -- here T
    persistent Python threads through the pir_server.h shim (ctypes drops the GIL), released
    together per query.  The shim answers every slice of a query from one engine pass
    (pir_engine_answer_slices).  Host-API times (key upload, answer download, sync) like
    `inclusive_h2d_key_d2h_answer`; beside it the same queries as one runOptimizedDPFTreeQuery
    call, and as T serialised per-slice engine answers (the round-3 behaviour of the shim)."""
    import threading
    from erasurecodedpir_amd import server as S
    S.setSystemParams(n, efs, 1, 1, 0, 0, 1, 0, 0)  # tree mode, k = 1: p = 2, NUM_ROUNDS = 1
    sv = S.Server(1, n, efs, 0, T)
    try:
        sv.write_rows(np.memmap(shard_path, np.uint8, mode="r"))
        K = min(K, len(keys))
        parts = np.zeros((T, 1, efs), np.uint8)
        cur = {"key": None}
        start, done = threading.Barrier(T + 1), threading.Barrier(T + 1)
        stop = []

        def worker(t):
            while True:
                start.wait()
                if stop:
                    return
                parts[t] = sv.runOptimizedDPFTreeQueryThread(cur["key"], t, T)
                done.wait()

        ths = [threading.Thread(target=worker, args=(t,), daemon=True) for t in range(T)]
        for th in ths:
            th.start()

        def query(k):
            cur["key"] = k
            start.wait()
            done.wait()
            return S.assemblDPFTreeQueryThreadResults(sv, parts)

        got = query(keys[0])  # engine creation + the 16 GiB upload + warm-up
        query(keys[1 % len(keys)])
        t0 = time.perf_counter()
        outs = [query(keys[q]) for q in range(K)]
        py_ms = (time.perf_counter() - t0) / K * 1e3
        stop.append(1)
        start.wait()
        for th in ths:
            th.join(10)
        ok_py = all(np.array_equal(outs[q], want[q]) for q in range(K))
        ok_py &= bool(np.array_equal(got, want[0]))
        # the same fan-out from C++ threads (pirRunTreeQueryThreads: a persistent pool, as the
        # Go runtime's goroutines run on its own threads): the library's cost without the
        # Python harness's per-call and wake-up overheads
        sv.runTreeQueryThreads(keys[0], T)
        t0 = time.perf_counter()
        outs = [sv.runTreeQueryThreads(keys[q], T) for q in range(K)]
        thr_ms = (time.perf_counter() - t0) / K * 1e3
        ok = all(np.array_equal(outs[q], want[q]) for q in range(K))
        sv.runOptimizedDPFTreeQuery(keys[0], 1)
        t0 = time.perf_counter()
        whole = [sv.runOptimizedDPFTreeQuery(keys[q], 1) for q in range(K)]
        one_ms = (time.perf_counter() - t0) / K * 1e3
        ok_one = all(np.array_equal(whole[q], want[q]) for q in range(K))
        # a lone Thread call (no partner within $PIR_SLICE_JOIN_US): the shim answers that
        # slice alone, a 1/T pass; the fan-out's slice t of the same key is the check
        sv.runOptimizedDPFTreeQueryThread(keys[-1], 5, T)  # a key the timed calls do not repeat
        t0 = time.perf_counter()
        lone = [sv.runOptimizedDPFTreeQueryThread(keys[q], 5, T) for q in range(K)]
        lone_ms = (time.perf_counter() - t0) / K * 1e3
    finally:
        sv.freeServer()
        S.wait_freed()  # its teardown (host rows, device shard) done before the next leg starts
    # the round-3 shim: T per-slice engine answers one after another (each its own descent,
    # tile-0 latency, reduce and sync)
    Ks = min(3, K)
    eng.answer_slice(keys[0], 0, T)
    t0 = time.perf_counter()
    ser = [np.bitwise_xor.reduce(np.stack([eng.answer_slice(keys[q], t, T) for t in range(T)]), 0)
           for q in range(Ks)]
    ser_ms = (time.perf_counter() - t0) / Ks * 1e3
    ok_ser = all(np.array_equal(ser[q], want[q]) for q in range(Ks))
    ok_lone = all(np.array_equal(lone[q], eng.answer_slice(keys[q], 5, T)) for q in range(min(2, K)))
    gib = float(1 << n) * efs / GIB
    return {"workload": f"the reference call shape (tree.go:60-76) at the north_star shape: 2^{n} x {efs} B, "
                        f"p=2, T={T} concurrent runOptimizedDPFTreeQueryThread calls per query "
                        "+ assemblDPFTreeQueryThreadResults (tree.go:60-76)",
            "threads": T, "steps": K, "ms_per_query": r5(thr_ms),
            "value": round(gib / (thr_ms / 1e3), 3), "unit": "GiB/s",
            "one_call_ms_per_query": r5(one_ms),
            "ratio_vs_one_call": round(thr_ms / one_ms, 4),
            "python_threads_ms_per_query": r5(py_ms),
            "serialised_per_slice_ms_per_query": r5(ser_ms),
            "lone_thread_call_ms": r5(lone_ms),
            "lone_thread_call_over_one_call": round(lone_ms / one_ms, 4),
            "note": "host-buffer API through the pir_server.h shim (key upload, answer download, "
                    "sync); ms_per_query = T threads of pirRunTreeQueryThreads (C++ pool, the "
                    "goroutines of tree.go:60-76); python_threads = the same calls from T Python "
                    "threads through ctypes; one_call = runOptimizedDPFTreeQuery on the same "
                    "server; serialised_per_slice = T pir_engine_answer_slice calls in a row "
                    "(the shim's round-3 behaviour); lone_thread_call = ONE "
                    "runOptimizedDPFTreeQueryThread(t=5, T) with no partner call: the join wait "
                    "($PIR_SLICE_JOIN_US, 200 us) + a 1/T pass",
            "parity": {"assembled_equals_device_answer": bool(ok),
                       "python_threads_assembled_equal": bool(ok_py),
                       "one_call_equals_device_answer": bool(ok_one),
                       "serialised_slices_equal": bool(ok_ser),
                       "lone_slice_equals_engine_slice": bool(ok_lone)}}


def run_coefs(args, ctx, config):
    """Polynomial-PIR answers (answer_coefs_dev): each step scans one query's device-resident
    coefficient vectors against the shard.  N = 1 only (replicas on more GPUs)."""
    import erasurecodedpir_amd as pir
    n, efs, nq, workload = COEF_CONFIGS[config]
    N = 1 << n
    eng = pir.Engine(2, 1, n, efs, nq, device=ctx.local)
    eng.fill_shard_random(SHARD_SEED)
    rng = np.random.default_rng(7)
    K, W = args.steps, args.warmup
    nkeys = max(2, min(K, 4))  # distinct queries, cycled
    d_c = eng.alloc_dev(nkeys * nq * N)
    d_r = eng.alloc_dev(K * nq * efs)
    for q in range(nkeys):
        eng.h2d(d_c + q * nq * N, rng.integers(0, 256, nq * N, dtype=np.uint8))
    for i in range(W):
        eng.answer_coefs_dev(d_c + (i % nkeys) * nq * N, N, 0, N, d_r)
    dt = ctx.timed(eng, lambda: [eng.answer_coefs_dev(d_c + (i % nkeys) * nq * N, N, 0, N,
                                                      d_r + i * nq * efs) for i in range(K)])
    ms = dt / K * 1e3
    # correctness at full size: one coefficient changed by x moves its round's answer by x*record
    host = eng.d2h(d_c, nq * N).reshape(nq, N)
    base = eng.answer_coefs(host)
    i, x = N // 3, 0x35
    host[nq - 1, i] ^= x
    moved = eng.answer_coefs(host)
    ok = bool(np.array_equal((base ^ moved)[nq - 1], _gf_table(x)[eng.shard_row(i)]))
    eng.close()
    gib = float(N) * efs / GIB
    algo = float(N) * (efs + nq)  # shard + the query's coefficients
    out = {"metric": METRIC, "value": round(gib / (ms / 1e3), 3), "unit": "GiB/s", "n_gpus": 1,
           "steps": K, "warmup": W, "ms_per_step": r5(ms), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
           "config": {"workload": workload, "records": N, "record_bytes": efs, "num_rounds": nq,
                      "step": "one query: interleave its coefficient vectors + GF(2^8) scan + reduce"},
           "roofline": {"bound": "hbm", "kernel": "k_interleave_coefs + k_scan + k_reduce",
                        "achieved": round(algo / (ms / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(algo / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": None, "algorithmic_bytes_per_query": int(algo),
                        "note": "wall time per query over the device work of all three launches"},
           "parity": {"coefficient_linearity": ok}}
    if ctx.rank == 0:
        print(json.dumps(out), flush=True)


def run_mp(args, ctx, config):
    """Multiparty (MP_CONFIGS) or covering-design (CD_CONFIGS) sqrt(N) DPF answers
    (answer_mp_dev / answer_cd_dev): each step evaluates one query's key into its shares
    (k_mp_shares) and scans them against the shard.  Keys are random bytes in the evaluation's
    layout (toggle bytes 0/1): the reference's multiparty key generation leaves them unset
    (params.cpp:613-617); its CD key generation is client code outside the server path
    (tests/test_cd.py pins the engine on genCDDPF's own keys).  N = 1 only (replicas on more
    GPUs)."""
    import erasurecodedpir_amd as pir
    cd = config in CD_CONFIGS
    if cd:
        n, efs, qn, nrk, workload = CD_CONFIGS[config]
        eb = pir.cd_key_len(0, n, 0, qn, nrk)
        mu, p2 = 1 << (n // 2 + 3), 1 << (qn - 1)
    else:
        n, efs, p, t, workload = MP_CONFIGS[config]
        nrk = pir.mp_num_keys(p, t)
        eb = pir.mp_eval_bytes(p, n, t)
        mu = 1 << int(np.ceil(np.log2(np.ceil(2 ** (n / 2) * 2 ** ((p - 1) / 2)))))
        p2 = 1 << (math.comb(p, t) - 1)
    N = 1 << n
    rng = np.random.default_rng(11)
    K, W = args.steps, args.warmup
    nkeys = max(2, min(K, 4))
    nu = N // mu
    tog = nu * 16 * p2
    keys = rng.integers(0, 256, (nkeys, eb), dtype=np.uint8)
    keys[:, tog:tog + nrk * nu * p2] = rng.integers(0, 2, (nkeys, nrk * nu * p2), dtype=np.uint8)
    if cd:
        ans_dev = lambda dk, dr: eng.answer_cd_dev(dk, qn, nrk, dr)  # noqa: E731
        ans = lambda k: eng.answer_cd(k, qn, nrk)  # noqa: E731
    else:
        ans_dev = lambda dk, dr: eng.answer_mp_dev(dk, p, t, dr)  # noqa: E731
        ans = lambda k: eng.answer_mp(k, p, t)  # noqa: E731
    # the engine's default (answer_mp_locked): k_query's sqrt(N) mode for >= 3 shares or <= 8
    # seeds a row, at most 32 seeds a row (64 when forced)
    fv = os.environ.get("PIR_MP_FUSED", "1")
    fused = (fv == "2" and p2 <= 64) or (fv not in ("0", "2") and p2 <= 32 and (nrk >= 3 or p2 <= 8))
    eng = pir.Engine(2, 1, n, efs, nrk, device=ctx.local)
    eng.fill_shard_random(SHARD_SEED)
    d_k = eng.alloc_dev(nkeys * eb)
    d_r = eng.alloc_dev(K * nrk * efs)
    eng.h2d(d_k, keys.reshape(-1))
    for i in range(W):
        ans_dev(d_k + (i % nkeys) * eb, d_r)
    dt = ctx.timed(eng, lambda: [ans_dev(d_k + (i % nkeys) * eb, d_r + i * nrk * efs)
                                 for i in range(K)])
    ms = dt / K * 1e3
    # correctness at full size: flipping cw[j][x] by d moves share a's answer by
    # d * XOR of the records i*mu + x of the rows whose toggle (a, i, j) is set
    j, x, d = 1, 777, 0x5A
    cwo = tog + nrk * nu * p2
    k0 = keys[0].copy()
    base = ans(k0)
    k0[cwo + j * mu + x] ^= d
    moved = ans(k0)
    tab = _gf_table(d)
    ok = True
    for a in range(nrk):
        acc = np.zeros(efs, np.uint8)
        for i in range(nu):
            if keys[0][tog + a * nu * p2 + i * p2 + j]:
                acc ^= eng.shard_row(i * mu + x)
        ok &= bool(np.array_equal((base ^ moved)[a], tab[acc]))
    dev0 = eng.d2h(d_r, nrk * efs).reshape(nrk, efs)
    ok_dev = bool(np.array_equal(dev0, ans(keys[0])))
    eng.close()
    gib = float(N) * efs / GIB
    algo = float(N) * efs + eb  # shard + the key
    # HBM bytes of the sqrt(N) k_query from its committed counters (profiles/pmc_<config>.json,
    # one query per launch; the shares never leave the CU), stamped with the library sha
    traffic, tsrc = _pmc_traffic(config, ctx.world, 1) if fused else (None, None)
    out = {"metric": METRIC, "value": round(gib / (ms / 1e3), 3), "unit": "GiB/s", "n_gpus": 1,
           "steps": K, "warmup": W, "ms_per_step": r5(ms), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
           "config": {"workload": workload, "records": N, "record_bytes": efs,
                      **({"num_cd_keys_needed": qn} if cd else {"parties": p, "threshold": t}),
                      "shares": nrk, "seeds_per_row": p2, "row_records": mu,
                      "rows": nu, "key_bytes_read": eb,
                      "step": "one query: >= 3 shares or <= 8 seeds a row: k_query in its "
                              "sqrt(N) mode (share waves build each tile's shares -- AES-CTR per "
                              "seed, toggled into the shares -- while the scan waves stream the "
                              "shard) + k_reduce; else or PIR_MP_FUSED=0: k_mp_shares + "
                              "k_scan_uni + k_reduce",
                      "mp_fused": fused},
           "roofline": {"bound": "hbm", "kernel": "k_query (sqrt(N) mode) + k_reduce" if fused
                        else "k_mp_shares + k_scan_uni + k_reduce",
                        "achieved": round(algo / (ms / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(algo / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": traffic, "traffic_source": tsrc,
                        "algorithmic_bytes_per_query": int(algo),
                        "note": "wall time per query over the device work of the launches"},
           "parity": {"correction_word_linearity": ok, "device_equals_host_api": ok_dev}}
    if ctx.rank == 0:
        print(json.dumps(out), flush=True)


def run_batch(args, ctx, config):
    """A step = `batch` keys answered against the device-resident shard (answer_batch_dev: one
    shard pass per group of keys, one DPF tree per key).  value = effective GiB/s = keys x
    logical shard bytes / time (every key's answer covers the whole shard)."""
    out = measure_batch(args.steps, args.warmup, ctx, config)
    if ctx.rank == 0:
        print(json.dumps(out), flush=True)
    if ctx.world > 1:
        ctx.dist.barrier()
        ctx.dist.destroy_process_group()


def measure_batch(steps, warmup, ctx, config):
    import erasurecodedpir_amd as pir
    from erasurecodedpir_amd.dist import broadcast_bytes, log2_exact

    world, rank, local = ctx.world, ctx.rank, ctx.local
    n_local, efs, p, nq, nk, workload = BATCH_CONFIGS[config]
    g = log2_exact(world)
    n = n_local + g
    eng = pir.Engine(p, 1, n, efs, nq, device=local, log_num_partitions=g, partition_index=rank)
    eng.fill_shard_random(SHARD_SEED)
    if os.environ.get("PIR_BENCH_BATCH_G"):  # diagnostics: keys per shard pass
        eng.batch_group = int(os.environ["PIR_BENCH_BATCH_G"])
    if world > 1 and not getattr(ctx, "rehearsal", False):
        # no host-fold variant of the batched answer: a rank that cannot join RCCL ends the run
        os.environ["PIR_BENCH_NO_FALLBACK"] = "1"
        attach_or_fallback(pir, eng, world, rank)
    rng = np.random.default_rng(int.from_bytes(
        broadcast_bytes(os.urandom(8) if rank == 0 else None) if world > 1 else os.urandom(8), "little"))
    keyset, fcw = make_keys(pir, n, p, nq, nk, rng, local)
    d_keys = eng.alloc_dev(eng.key_len * nk)
    d_res = eng.alloc_dev(eng.answer_bytes * nk)
    eng.h2d(d_keys, b"".join(ks[0] for _, ks in keyset))
    for _ in range(warmup):
        eng.answer_batch_dev(d_keys, nk, d_res)
    eng.set_profiling(max(1, steps))
    dt = ctx.timed(eng, lambda: [eng.answer_batch_dev(d_keys, nk, d_res) for _ in range(steps)])
    eng.set_profiling(0)
    ms = dt / steps * 1e3
    alone = eng.profile_phases(d_keys, 5)
    got = eng.d2h(d_res, eng.answer_bytes * nk).reshape(nk, nq, efs)
    # correctness at full size: party-1 batch ^ party-2 batch == finalCW * record, every key
    eng.set_party(2)
    got2 = eng.answer_batch([ks[1] for _, ks in keyset])
    eng.set_party(1)
    tab = _gf_table(int(fcw[0]))
    ok = True
    for q, (i, _) in enumerate(keyset):
        owner = i >> (n - g) if g else 0
        rec = eng.shard_row(i - owner * eng.num_rows) if rank == owner else None
        if world > 1:
            rec = broadcast_from(rec, owner, efs)
        ok &= bool(np.array_equal(got[q][0] ^ got2[q][0], tab[rec]))
    shard_bytes = float(1 << n) * efs
    out = {
        "metric": METRIC,
        "value": round(nk * shard_bytes / GIB / (ms / 1e3), 3),
        "unit": "GiB/s",
        "value_kind": "effective: keys x logical shard bytes / batch time",
        "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": workload, "records": 1 << n, "record_bytes": efs, "parties": p,
                   "num_rounds": nq, "batch": nk, "keys_per_shard_pass": eng.batch_group,
                   "records_per_gpu": int(eng.num_rows), "dpf_depth": n,
                   "parallelism": "split-shard" if world > 1 else "single"},
        "ms_per_key": round(ms / nk, 5),
        "keys_per_s": round(nk / (ms / 1e3), 1),
        "shard_passes_per_step": -(-nk // eng.batch_group),
        "single_key_phases_alone_ms": {k: r5(v) for k, v in alone.items()},
        "parity": {"pir_record_recovered_all_keys": ok},
    }
    eng.close()
    return out


def broadcast_from(arr, src, nbytes):
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(arr.copy()) if arr is not None else torch.zeros(nbytes, dtype=torch.uint8)
    dist.broadcast(t, src=src)
    return t.numpy()


if __name__ == "__main__":
    main()
