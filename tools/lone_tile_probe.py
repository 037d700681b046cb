#!/usr/bin/env python3
"""Lone-query latency by first-tile size (diagnostics): configs[1] (2^20 x 1 KiB, p=2), one
query per launch, for PIR_QUERY_TILE1 = 1024 / 512 / 256 leaves per tile; answers must agree.

    python tools/lone_tile_probe.py [--n 20] [--efs 1024] [--reps 50]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--efs", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--tiles", default="1024,512,256")
    ap.add_argument("--fused", default="1", help="PIR_FUSED_REDUCE values to try")
    a = ap.parse_args()
    import torch
    import erasurecodedpir_amd as pir
    torch.cuda.set_device(0)
    rng = np.random.default_rng(5)
    keys = [pir.gen_keys(a.n, int(i), 2, 1)[0] for i in rng.choice(1 << a.n, a.reps, replace=False)]
    res = {}
    ref = None
    for t, fr in [(int(x), f) for x in a.tiles.split(",") for f in a.fused.split(",")]:
        os.environ["PIR_QUERY_TILE1"] = str(t)
        os.environ["PIR_FUSED_REDUCE"] = fr
        with pir.Engine(2, 1, a.n, a.efs, 1) as e:
            e.fill_shard_random(0xC0FFEE)
            kl, ab = e.key_len, e.answer_bytes
            d_k = e.alloc_dev(kl * a.reps)
            d_r = e.alloc_dev(ab * a.reps)
            e.h2d(d_k, b"".join(keys))
            for i in range(5):
                e.answer_dev(d_k + i * kl, d_r + i * ab)
            e.sync()
            t0 = time.perf_counter()
            for i in range(a.reps):
                e.answer_dev(d_k + i * kl, d_r + i * ab)
            e.sync()
            ms = (time.perf_counter() - t0) / a.reps * 1e3
            e.set_profiling(a.reps)
            for i in range(a.reps):
                e.answer_dev(d_k + i * kl, d_r + i * ab)
            ph = e.last_timings()
            e.set_profiling(0)
            out = e.d2h(d_r, ab * a.reps)
            tr = e.trace_query(d_k, 1)
        if ref is None:
            ref = out
        first_scan_us = float(np.median(tr[:, 3]))  # tile 0 shares ready (us after the start)
        res[f"{t}/fused{fr}"] = {"ms_per_query": round(ms, 5), "kernel_ms": round(ph.get("scan", 0), 5),
                  "tile0_ready_us_median": round(first_scan_us, 2),
                  "answers_equal_tile1024": bool(np.array_equal(out, ref))}
        print(t, fr, res[f"{t}/fused{fr}"], flush=True)
    print(json.dumps({"probe": "lone query by first-tile size", "n": a.n, "efs": a.efs,
                      "results": res}))


if __name__ == "__main__":
    main()
