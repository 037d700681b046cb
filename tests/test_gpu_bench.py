"""bench.py's measurement helpers on the GPU (the driver runs bench.py at round end): measure()
takes a key list longer than its warm-up + timed window (the 1-GPU reference leg of
`bench.py --gpus N` reuses the N-GPU key set) and times exactly keys[W : W + K]."""
import os
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Ctx:
    """bench.Ctx without torch (one process: the engine's own sync brackets the timing)."""
    world, rank, local, rehearsal, host_fold = 1, 0, 0, False, False

    def fold(self, arr):
        return arr

    def timed(self, eng, fn):
        eng.sync()
        t0 = time.perf_counter()
        fn()
        eng.sync()
        return time.perf_counter() - t0


def test_measure_uses_its_key_window():
    sys.path.insert(0, ROOT)
    import bench
    import erasurecodedpir_amd as pir
    n, efs, p, nq = 14, 256, 2, 1
    rng = np.random.default_rng(5)
    keyset, _ = bench.make_keys(pir, n, p, nq, 9, rng, 0)
    keys = [ks[0] for _, ks in keyset]
    ctx = _Ctx()
    with pir.Engine(p, 1, n, efs, nq) as e:
        e.fill_shard_random(3)
        m_a = bench.measure(ctx, e, keys, 5, 3, single=False)          # timed: keys 5..7
        m_b = bench.measure(ctx, e, keys[3:], 2, 3, single=False)      # timed: keys 5..7
        want = np.stack([e.answer(k) for k in keys[5:8]])
    assert np.array_equal(m_a["answers"], want)
    assert np.array_equal(m_b["answers"], want)
    with pir.Engine(p, 1, n, efs, nq) as e2, pytest.raises(ValueError):
        bench.measure(ctx, e2, keys[:4], 2, 3, single=False)


def test_measure_host_fold_path():
    """The host-fold exchange (bench.py's fallback when RCCL cannot be set up, and rehearsals):
    answers copied back and folded inside the timed region, queue and single legs -- here with
    one rank, so the fold is the identity and the answers equal the device path's."""
    sys.path.insert(0, ROOT)
    import bench
    import erasurecodedpir_amd as pir
    n, efs, p, nq = 14, 256, 2, 1
    rng = np.random.default_rng(6)
    keyset, _ = bench.make_keys(pir, n, p, nq, 8, rng, 0)
    keys = [ks[0] for _, ks in keyset]
    ctx = _Ctx()
    ctx.host_fold = True
    with pir.Engine(p, 1, n, efs, nq) as e:
        e.fill_shard_random(4)
        m = bench.measure(ctx, e, keys, 4, 4, single=True)
        want = np.stack([e.answer(k) for k in keys[4:8]])
    assert np.array_equal(m["answers"], want)
    assert np.array_equal(m["singles"], want)
    assert m["ms"] > 0 and m["ms1"] > 0
