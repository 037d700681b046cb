#!/usr/bin/env python3
"""Queue vs one-at-a-time answers: ms per query for a few shapes (diagnostics)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import erasurecodedpir_amd as pir  # noqa: E402


def run(n, efs, p, nq, nk, reps=3):
    e = pir.Engine(p, 1, n, efs, nq)
    e.fill_shard_random(5)
    rng = np.random.default_rng(0)
    keys = [pir.gen_keys(n, int(i), p, nq)[0] for i in rng.choice(1 << n, nk, replace=False)]
    d_k = e.alloc_dev(nk * e.key_len)
    d_r = e.alloc_dev(nk * e.answer_bytes)
    e.h2d(d_k, b"".join(keys))
    e.answer_stream_dev(d_k, nk, d_r)
    e.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        e.answer_stream_dev(d_k, nk, d_r)
    e.sync()
    ts = (time.perf_counter() - t0) / reps / nk
    for k in range(min(nk, 4)):
        e.answer_dev(d_k + k * e.key_len, d_r)
    e.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        for k in range(nk):
            e.answer_dev(d_k + k * e.key_len, d_r + k * e.answer_bytes)
    e.sync()
    t1 = (time.perf_counter() - t0) / reps / nk
    gib = (1 << n) * efs / 2**30
    print(f"n={n} efs={efs} p={p} nq={nq} nk={nk}: queue {ts*1e3:.4f} ms/query ({gib/ts:.0f} GiB/s)  "
          f"single {t1*1e3:.4f} ms/query ({gib/t1:.0f} GiB/s)", flush=True)
    e.close()


if __name__ == "__main__":
    run(20, 1024, 2, 1, 50)
    run(24, 1024, 2, 1, 8)
    run(24, 1024, 8, 5, 4)
    run(24, 256, 2, 1, 16)
