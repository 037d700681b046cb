"""bench.py's CPU-baseline leg on a small shape (CPU only): the 1-core reference timing and the
all-cores aggregate (worker processes over one shared read-only mapping of the shard, one
reference server and one query each) agree on the answer with each other and with the plain-C
oracle."""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref.so")
sys.path.insert(0, ROOT)


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built")
def test_cpu_baseline_legs_agree(monkeypatch, tmp_path):
    import bench
    import _oracle as O

    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    L = ctypes.CDLL(REF_SO)
    n, efs, p, nq = 12, 64, 2, 1
    kl = L.ref_key_len(p, n, nq)
    keys = np.zeros(p * kl, np.uint8)
    fcw = np.array([3], np.uint8)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    L.ref_gen_opt_dpf(n, ctypes.c_uint64(1234), P(fcw), p, nq, P(keys))
    shard = np.random.default_rng(7).integers(0, 256, (1 << n) * efs, dtype=np.uint8)
    want = O.answer(p, 1, n, efs, nq, keys[kl:].tobytes(), shard).reshape(nq, efs)
    path = str(tmp_path / "shard.bin")
    shard.tofile(path)
    assert bench._host_cores() == 2  # the share minus the GPU process's own core
    r = bench.cpu_baseline(path, n, efs, p, nq, keys[kl:].tobytes(), want, 0.5,
                           bench._host_cores())
    assert r["kind"] == "reference" and r["bit_exact_vs_gpu"]
    ac = r["all_cores"]
    assert ac["cores"] == 2 and ac["answers_agree"] and ac["value"] > 0


def _rank(r, world, bus=None, attached=True, count=None, user=None):
    return {"rank": r, "rccl": {"attached": attached, "rccl_count": world if count is None else count,
                                "rccl_user_rank": r if user is None else user, "rccl_device": 0,
                                "engine_device": r, "pci_bus_id": bus or f"0000:{r:02x}:00.0"}}


def test_rccl_self_check_fields():
    """The N > 1 line's self-check (bench.rccl_ranks_ok / exchange_fields): true only when RCCL
    reports every rank, its own rank number and N distinct GPUs; a host-fold run is labelled as
    not an RCCL measurement whatever the communicator says."""
    import bench
    w = 8
    good = [_rank(r, w) for r in range(w)]
    assert bench.rccl_ranks_ok(good, w)
    f = bench.exchange_fields(good, w, host_fold=False, comm_err=None)
    assert f["rccl_ranks_ok"] and f["exchange"].startswith("rccl") and "value_kind" not in f
    # two ranks on one GPU, a wrong count, a wrong user rank, a rank without a communicator
    dup = [_rank(r, w, bus="0000:01:00.0" if r < 2 else None) for r in range(w)]
    assert not bench.rccl_ranks_ok(dup, w)
    assert not bench.rccl_ranks_ok([_rank(r, w, count=4) for r in range(w)], w)
    assert not bench.rccl_ranks_ok([_rank(r, w, user=(r + 1) % w) for r in range(w)], w)
    assert not bench.rccl_ranks_ok([_rank(r, w, attached=r != 3) for r in range(w)], w)
    assert not bench.rccl_ranks_ok(good[:4], w)
    bad = bench.exchange_fields(dup, w, host_fold=False, comm_err=None)
    assert not bad["rccl_ranks_ok"] and "does not show" in bad["value_kind"]
    hf = bench.exchange_fields(good, w, host_fold=True, comm_err="ncclCommInitRank failed")
    assert not hf["rccl_ranks_ok"] and "NOT an RCCL" in hf["value_kind"]
    assert "RCCL init failed" in hf["exchange"]
    reh = bench.exchange_fields([_rank(r, w, attached=False, count=-1, user=-1) for r in range(w)],
                                w, host_fold=True, comm_err=None)
    assert not reh["rccl_ranks_ok"] and reh["exchange"].endswith("(rehearsal)")


class _FakeTraceEngine:
    """trace_query's layout (include/pir_engine.h): wall stamps in us, shader-clock columns in
    ticks / 100."""
    key_len = 4

    def __init__(self, ghz, nwg=8, tiles=6):
        tr = np.zeros((nwg, 256))
        tr[:, 0], tr[:, 2], tr[:, 3], tr[:, 6] = 0.0, 14.0, 43.0, 200.0
        tr[:, 56], tr[:, 57] = 0.0, 14.0 * ghz * 1e3 / 100  # start -> first root
        for g in range(tiles):
            tr[:, 64 + g] = 43.0 + 35.0 * g
            tr[:, 128 + g] = tr[:, 64 + g] * ghz * 1e3 / 100
        self.tr = tr

    def alloc_dev(self, n):
        return 1

    def free_dev(self, d):
        pass

    def h2d(self, d, b):
        pass

    def trace_query(self, d, nk):
        return self.tr


def test_leg_ceilings_and_clock_fields(monkeypatch, tmp_path):
    """The per-leg ceilings the line carries: the shader clock from
    k_query's stamps (trace_stats), configs[4]'s issue-port fractions from sha-stamped counters
    (_pmc_issue, refused for another build), and the k_query phases that sum to the answer."""
    import json
    import bench
    st = bench.trace_stats(_FakeTraceEngine(2.1), [b"k" * 4] * 4, 3)
    assert abs(st["shader_clock_ghz"]["median"] - 2.1) < 1e-6
    assert "tiles 0..5" in st["shader_clock_ghz"]["source"]
    assert st["tile0_ready_us_median"] == 43.0
    one = bench.trace_stats(_FakeTraceEngine(1.8, tiles=1), [b"k" * 4], 1)
    assert abs(one["shader_clock_ghz"]["median"] - 1.8) < 1e-6 and "first tile root" in \
        one["shader_clock_ghz"]["source"]
    # counters: 2e9 SALU and 4e9 VALU per launch of 2 queries, stamped with the loaded library
    root = tmp_path
    (root / "profiles").mkdir()
    d = {"lib_sha256": "abc", "queries_per_launch": 2,
         "counters_per_launch": {"SQ_INSTS_SALU": 2e9, "SQ_INSTS_VALU": 4e9},
         "issue": {"shader_clock_GHz_implied": 1.9}}
    (root / "profiles" / "pmc_c5.json").write_text(json.dumps(d))
    monkeypatch.setattr(bench, "ROOT", str(root))
    monkeypatch.setattr(bench, "_lib_sha256", lambda: "abc")
    iss = bench._pmc_issue("c5", 20, 70.0, 2.0)  # 20 queries in 70 ms at 2 GHz
    cyc = 70e-3 * 2e9
    assert abs(iss["salu_issue_frac"] - 2e10 / (256 * cyc)) < 1e-4
    assert abs(iss["valu_issue_frac"] - 4e10 / (256 * 2 * cyc)) < 1e-4
    assert iss["clock_source"] == "this run's k_query stamps"
    assert bench._pmc_issue("c5", 20, 70.0, None)["clock_ghz_used"] == 1.9
    monkeypatch.setattr(bench, "_lib_sha256", lambda: "other build")
    assert bench._pmc_issue("c5", 20, 70.0, 2.0) is None
    # k_query phases: launch + k_query + k_reduce + tail == the profiled answer
    ph = {"launch": 0.004, "scan": 2.85, "reduce": 0.005, "comm_fold": 0.001, "total": 2.86,
          "fused": 2.0}
    sp = bench.single_phases(ph, 2.87)
    assert set(sp["phases_ms"]) == {"launch", "k_query", "k_reduce", "exchange_and_tail"}
    assert abs(sp["phases_sum_ms"] - 2.86) < 1e-9
    assert abs(sp["phases_sum_over_ms_per_query"] - 2.86 / 2.87) < 1e-4
    old = bench.single_phases({"key_prep": 0.1, "scan": 1.0, "chunks": 4, "fused": 0.0}, 1.2)
    assert "chunks" not in old["phases_ms"] and "fused" not in old["phases_ms"]
