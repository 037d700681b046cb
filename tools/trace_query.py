#!/usr/bin/env python3
"""Phase timeline of one single-launch answer (k_query), from per-workgroup wall-clock stamps.

    python tools/trace_query.py [--n 20] [--efs 1024] [--p 2] [--nq 1]

Prints, for each phase stamp, min / median / max over workgroups in microseconds since the
earliest workgroup start (diagnostics; not part of the product path)."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--efs", type=int, default=1024)
    ap.add_argument("--p", type=int, default=2)
    ap.add_argument("--nq", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--queue", type=int, default=1, help="keys in the traced queue")
    a = ap.parse_args()
    import erasurecodedpir_amd as pir
    e = pir.Engine(a.p, 1, a.n, a.efs, a.nq)
    e.fill_shard_random(1)
    keys = [pir.gen_keys(a.n, (1 << a.n) // 3 + 17 * k, a.p, a.nq) for k in range(a.queue)]
    d_key = e.alloc_dev(e.key_len * a.queue)
    e.h2d(d_key, b"".join(k[0] for k in keys))
    keys = keys[0]
    for _ in range(3):
        e.answer(keys[0])
    for r in range(a.reps):
        tr = e.trace_query(d_key, a.queue)
        print(f"n={a.n} efs={a.efs} p={a.p} nq={a.nq}: {tr.shape[0]} workgroups (rep {r})")
        for i, name in enumerate(e.TRACE_PHASES):
            col = tr[:, i]
            print(f"  {name:16s} min {col.min():8.2f}  med {np.median(col):8.2f}  max {col.max():8.2f} us")
        med = np.median(tr, axis=0)
        desc = [med[8 + d] for d in range(32) if tr[:, 8 + d].all()]
        lev = [med[40 + k] for k in range(16) if tr[:, 40 + k].all()]
        print("  descent level ends (med us):", " ".join(f"{v:.1f}" for v in desc))
        print("  tile-0 level ends  (med us):", " ".join(f"{v:.1f}" for v in lev))
        raw = tr * 100.0  # back to ticks for the clock columns
        ghz = (raw[:, 57] - raw[:, 56]) / ((tr[:, 2] - tr[:, 0]) * 1e3)
        print(f"  shader clock start->first root: med {np.median(ghz):.3f} GHz (min {ghz.min():.3f} max {ghz.max():.3f})")
        # workgroup b runs on XCD b % 8 under round-robin dispatch: per-XCD medians of the late
        # phases and of the clock, and the spread of the end stamp within each XCD
        names = list(e.TRACE_PHASES)
        il, ie = names.index("last_tile_ready"), names.index("end")
        xcd = np.arange(tr.shape[0]) % 8
        for x in range(8):
            m = xcd == x
            print(f"  xcd {x}: last_tile_ready med {np.median(tr[m, il]):8.1f}  end med {np.median(tr[m, ie]):8.1f}"
                  f" (min {tr[m, ie].min():8.1f} max {tr[m, ie].max():8.1f})  clock med {np.median(ghz[m]):.3f} GHz")
        print(f"  corr(end, clock) over workgroups: {np.corrcoef(tr[:, ie], ghz)[0, 1]:+.2f}")
        # end-of-query work stealing (a lone query): chunk counts are raw (not ticks)
        cnt = np.rint(raw[:, 59:62]).astype(np.int64)
        if cnt.any():
            print(f"  stealing: chunks of others folded by tree waves {cnt[:, 0].sum()} "
                  f"(max {cnt[:, 0].max()}/wg), own by tree waves {cnt[:, 1].sum()}, own by scan "
                  f"waves {cnt[:, 2].sum()}; tree waves done med {np.median(tr[:, 58]):.1f} "
                  f"max {tr[:, 58].max():.1f} us")
        print(f"  end spread: med {np.median(tr[:, ie]):.1f}  p90 {np.percentile(tr[:, ie], 90):.1f}"
              f"  max {tr[:, ie].max():.1f} us")
        rd = [med[64 + g] for g in range(32) if tr[:, 64 + g].all()]
        cs = [med[96 + g] for g in range(32) if tr[:, 96 + g].all()]
        if a.queue == 1 and len(rd) > 1:
            print("  tile ready    (med us):", " ".join(f"{v:.1f}" for v in rd))
            print("  tile consumed (med us):", " ".join(f"{v:.1f}" for v in cs))
        if a.queue > 1:
            cs = [med[96 + g] for g in range(32) if tr[:, 96 + g].all()]
            print("  queue tile ready    (med us):", " ".join(f"{v:.0f}" for v in rd))
            print("  queue tile consumed (med us):", " ".join(f"{v:.0f}" for v in cs))
            ck = [(tr[:, 128 + g + 1] - tr[:, 128 + g]) * 100 / ((tr[:, 64 + g + 1] - tr[:, 64 + g]) * 1e3)
                  for g in range(len(rd) - 1)]
            print("  shader clock between ready stamps (GHz):", " ".join(f"{np.median(c):.2f}" for c in ck))
            t1 = [med[176]] + [med[160 + k] for k in range(16) if tr[:, 160 + k].all()]
            print("  tile-1 root + level ends (med us, tree waves beside the scan):",
                  " ".join(f"{v:.1f}" for v in t1), f"| ready {med[65]:.1f}")
            # diagnostics build (-DPIR_TRACE_TREE_TILES=1) with $PIR_TRACE_TILES=a,b: two queue
            # tiles' tree phases (wave 0 of the tree team): slot wait, entry, inputs, levels, leaf, ready
            tv = os.environ.get("PIR_TRACE_TILES")
            if tv:
                for t, g in enumerate(int(x) for x in tv.split(",")[:2]):
                    base = 224 + 16 * t
                    col = lambda k: tr[:, base + k]
                    if not col(0).all():
                        continue
                    lev = [k for k in range(2, 14) if col(k).all()]
                    parts = [("slot_wait", 15), ("entry", 0), ("inputs", 1)] + [(f"L{k - 1}", k) for k in lev] + [("leaf", 14)]
                    print(f"  tree tile {g}: " + "  ".join(f"{n} {np.median(col(k)):.1f}" for n, k in parts)
                          + f"  ready {med[64 + g]:.1f}  consumed[{g - 1}] {med[96 + g - 1]:.1f}  consumed[{g}] {med[96 + g]:.1f}")
                    if tr[:, 208 + 8 * t:216 + 8 * t].all():
                        sw = np.median(tr[:, 208 + 8 * t:216 + 8 * t], axis=0)
                        blk = tr[:, 208 + 8 * t:216 + 8 * t]
                        spread = blk.max(axis=1) - blk.min(axis=1)
                        print(f"    scan waves' consumed[{g}] (med us, sw 0-7): " + " ".join(f"{v:.1f}" for v in sw)
                              + f"  | per-workgroup spread med {np.median(spread):.1f} max {spread.max():.1f} us,"
                              + f" slowest sw histogram {np.bincount(blk.argmax(axis=1), minlength=8).tolist()}")
    e.close()


if __name__ == "__main__":
    main()
