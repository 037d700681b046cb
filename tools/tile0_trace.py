#!/usr/bin/env python3
"""Lone-query timeline (diagnostics): configs[1] (2^20 x 1 KiB, p=2) answered once with k_query's
phase stamps; prints the median over workgroups of: key staged, each descent level, descent end,
each tile-0 level, tile 0 ready, last tile ready, end of scan (microseconds from kernel start).

    python tools/tile0_trace.py [--n 20] [--efs 1024]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--efs", type=int, default=1024)
    a = ap.parse_args()
    import erasurecodedpir_amd as pir
    key = pir.gen_keys(a.n, 12345, 2, 1)[0]
    with pir.Engine(2, 1, a.n, a.efs, 1) as e:
        e.fill_shard_random(1)
        d_k = e.alloc_dev(e.key_len)
        e.h2d(d_k, key)
        for _ in range(3):
            tr = e.trace_query(d_k, 1)
    med = lambda c: float(np.median(tr[:, c])) if np.any(tr[:, c]) else None
    rows = [("key staged", 1)] + [(f"descent level {d}", 8 + d) for d in range(32) if np.any(tr[:, 8 + d])]
    rows += [("descent end", 2)] + [(f"tile-0 level {l}", 40 + l) for l in range(16) if np.any(tr[:, 40 + l])]
    rows += [("tile 0 ready", 3), ("last tile ready", 4), ("scan end", 5)]
    prev = 0.0
    for name, c in rows:
        v = med(c)
        if v is None:
            continue
        print(f"{name:18s} {v:8.2f} us  (+{v - prev:6.2f})")
        prev = v


if __name__ == "__main__":
    main()
