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
