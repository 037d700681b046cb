"""Diagnostics: per-round / per-coefficient-bit comparison of answer_coefs with the oracle on the
four-Russians shapes (which planes a broken fold gets wrong)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import _oracle as O  # noqa: E402
import erasurecodedpir_amd as pir  # noqa: E402

for n, efs, nq in [(12, 400, 4), (12, 256, 5), (10, 256, 6), (11, 300, 8), (11, 512, 4), (12, 1024, 5)]:
    rng = np.random.default_rng(n * 131 + nq)
    shard = rng.integers(0, 256, (1 << n) * efs, dtype=np.uint8)
    res = []
    for bit in range(8):  # coefficients with one bit set: only plane (a, bit) may be nonzero
        coefs = (rng.integers(0, 2, (nq, 1 << n), dtype=np.uint8) << bit).astype(np.uint8)
        with pir.Engine(2, 1, n, efs, nq) as e:
            e.set_shard(shard)
            got = e.answer_coefs(coefs)
        want = O.scan(coefs, shard, efs)
        res.append("".join("." if np.array_equal(got[a], want[a]) else "X" for a in range(nq)))
    coefs = rng.integers(0, 256, (nq, 1 << n), dtype=np.uint8)
    with pir.Engine(2, 1, n, efs, nq) as e:
        e.set_shard(shard)
        got = e.answer_coefs(coefs)
    want = O.scan(coefs, shard, efs)
    ok = [bool(np.array_equal(got[a], want[a])) for a in range(nq)]
    print(f"n={n} efs={efs} nq={nq}: per bit (rounds) {' '.join(res)}  random: {ok}", flush=True)
