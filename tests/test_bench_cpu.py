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
