#!/usr/bin/env python3
"""Per-phase cycle breakdown of k_query's four-Russians scan waves (diagnostics, not product).

Needs the stamp build: `make -C erasurecodedpir_amd/csrc diag` (libpir_engine_diag.so, compiled
with -DPIR_FOLD_STAMPS=1; loaded here through $PIR_ENGINE_LIB).  Each scan wave adds the shader
cycles (s_memtime) of every phase of its loop into counters that the trace returns:

    0 tree      waiting for the tile's shares (the tree waves)
    1 index     coefficient words from the LDS ring, the 40 plane indices, the DPP pack
    2 rows      waiting for the group's 4 rows (s_waitcnt vmcnt)
    3 fold      the asm fold: 32 combinations + 40 indexed planes (m4r_fold4p)
    4 loads     issuing the 4 refill loads
    6 other     per-tile bookkeeping, end-of-query plane fold and slab store

    python tools/fold_phases.py [--n 24] [--p 8] [--nq 5] [--queue 4]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PHASES = {0: "tree", 1: "index", 2: "rows", 3: "fold", 4: "loads", 6: "other"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=24)
    ap.add_argument("--efs", type=int, default=1024)
    ap.add_argument("--p", type=int, default=8)
    ap.add_argument("--nq", type=int, default=5)
    ap.add_argument("--queue", type=int, default=4)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    os.environ.setdefault("PIR_ENGINE_LIB", os.path.join(ROOT, "erasurecodedpir_amd",
                                                         "libpir_engine_diag.so"))
    import erasurecodedpir_amd as pir
    print("library:", os.environ["PIR_ENGINE_LIB"])
    e = pir.Engine(a.p, 1, a.n, a.efs, a.nq)
    e.fill_shard_random(1)
    keys = [pir.gen_keys(a.n, (1 << a.n) // 3 + 17 * k, a.p, a.nq)[0] for k in range(a.queue)]
    d_key = e.alloc_dev(e.key_len * a.queue)
    e.h2d(d_key, b"".join(keys))
    for _ in range(2):
        e.answer(keys[0])
    for r in range(a.reps):
        tr = e.trace_query(d_key, a.queue) * 100.0  # back to raw counts
        st = tr[:, 192:256].reshape(tr.shape[0], 8, 8)  # [workgroup, scan wave, counter]
        groups = st[:, :, 7]
        if not groups.any():
            print("no fold stamps: not the stamp build, or not the four-Russians k_query")
            return 1
        tot = st[:, :, [0, 1, 2, 3, 4, 6]].sum(axis=2)
        wall_us = (tr[:, 6] - tr[:, 0]).max() / 100.0 if tr[:, 6].any() else float("nan")
        print(f"n={a.n} efs={a.efs} p={a.p} nq={a.nq} queue={a.queue} rep {r}: {tr.shape[0]} "
              f"workgroups x 8 scan waves, {np.median(groups):.0f} groups per wave")
        print(f"  cycles per wave: median {np.median(tot):.0f}  (min {tot.min():.0f} max {tot.max():.0f})")
        for k, name in PHASES.items():
            share = st[:, :, k] / tot
            per_g = st[:, :, k] / np.maximum(groups, 1)
            print(f"  {k} {name:6s} share med {np.median(share):6.3f}  "
                  f"(min {share.min():6.3f} max {share.max():6.3f})   cycles per group med {np.median(per_g):8.1f}")
        print(f"  all phases per group: {np.median(tot / np.maximum(groups, 1)):.1f} cycles")
    e.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
