#!/usr/bin/env python3
"""Lone-query launch gaps (diagnostics): configs[1] (2^20 x 1 KiB, p=2), R queries answered one
launch each, back to back on the engine stream.  Run under

    rocprofv3 --kernel-trace -d gpurun_out/gap -o run --output-format csv -- python tools/lone_gap_probe.py
    python tools/lone_gap_probe.py --analyse gpurun_out/gap

The analysis prints the median k_query and k_reduce durations and the idle gaps between them
(k_query end -> k_reduce start, k_reduce end -> next k_query start) over the timed queries."""
import argparse
import csv
import glob
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(a):
    import erasurecodedpir_amd as pir
    p, nq = 2, 1
    keys = [pir.gen_keys(a.n, (i * 7919) % (1 << a.n), p, nq)[0] for i in range(a.reps + 5)]
    with pir.Engine(p, 1, a.n, a.efs, nq) as e:
        e.fill_shard_random(5)
        kl, ab = e.key_len, e.answer_bytes
        d_k = e.alloc_dev(kl * len(keys))
        d_r = e.alloc_dev(ab * len(keys))
        e.h2d(d_k, b"".join(keys))
        for i in range(5):
            e.answer_dev(d_k + i * kl, d_r + i * ab)
        e.sync()
        t0 = time.perf_counter()
        for i in range(5, len(keys)):
            e.answer_dev(d_k + i * kl, d_r + i * ab)
        e.sync()
        dt = (time.perf_counter() - t0) / a.reps
        print(f"lone queries: {dt * 1e3:.4f} ms per query (wall, {a.reps} back to back)")


def analyse(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ev = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
          if "k_query" in r["Kernel_Name"] or "k_reduce" in r["Kernel_Name"]]
    ev = ev[-2 * 40:]  # the timed tail
    q = [(s, e) for n, s, e in ev if "k_query" in n]
    rd = [(s, e) for n, s, e in ev if "k_reduce" in n]
    m = min(len(q), len(rd))
    qd = [e - s for s, e in q[:m]]
    rdd = [e - s for s, e in rd[:m]]
    g1 = [rd[i][0] - q[i][1] for i in range(m)]
    g2 = [q[i + 1][0] - rd[i][1] for i in range(m - 1)]
    per = [q[i + 1][0] - q[i][0] for i in range(m - 1)]
    med = lambda v: float(np.median(v)) / 1e3  # noqa: E731
    print(f"k_query {med(qd):.2f} us | gap {med(g1):.2f} | k_reduce {med(rdd):.2f} | gap {med(g2):.2f}"
          f" | period {med(per):.2f} us  ({m} queries)")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--efs", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--analyse", default=None)
    a = ap.parse_args()
    if a.analyse:
        analyse(a.analyse)
    else:
        run(a)
