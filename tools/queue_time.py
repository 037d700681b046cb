#!/usr/bin/env python3
"""ms per query of a K-query k_query queue (diagnostics; A/B of library builds through
$PIR_ENGINE_LIB): 2^n x efs shard, p parties, nq rounds, W warm-up queries, R repetitions.
    python tools/queue_time.py [n] [efs] [p] [nq] [K] [R]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import erasurecodedpir_amd as pir
    n, efs, p, nq, K, R = (int(x) for x in (sys.argv[1:7] + ["24", "1024", "8", "5", "20", "3"][len(sys.argv[1:7]):]))
    W = 5
    rng = np.random.default_rng(1)
    fcw = pir.final_cw(p, nq, 1)
    keys = [pir.gen_keys(n, int(i), p, nq, fcw=fcw,
                         seeds=rng.integers(0, 256, 16 * p, dtype=np.uint8).tobytes())[0]
            for i in rng.choice(1 << n, W + K, replace=False)]
    with pir.Engine(p, 1, n, efs, nq) as e:
        e.fill_shard_random(7)
        kl, ab = e.key_len, e.answer_bytes
        dk = e.alloc_dev(kl * (W + K))
        dr = e.alloc_dev(ab * (W + K))
        e.h2d(dk, b"".join(keys))
        e.reserve_queue(K)
        out = []
        for _ in range(R):
            e.answer_stream_dev(dk, W, dr)
            e.sync()
            t0 = time.perf_counter()
            e.answer_stream_dev(dk + W * kl, K, dr + W * ab)
            e.sync()
            out.append((time.perf_counter() - t0) / K * 1e3)
        lib = os.path.basename(os.environ.get("PIR_ENGINE_LIB", "libpir_engine.so"))
        lib += "".join(f" {k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("PIR_") and k != "PIR_ENGINE_LIB")
        o = sorted(out)
        print(f"{lib} n={n} efs={efs} p={p} nq={nq} K={K}: ms/query "
              + (" ".join(f"{v:.4f}" for v in out) if R <= 4 else f"median {o[len(o) // 2]:.4f} min {o[0]:.4f} (of {R})")
              + f" (TB/s at min {(1 << n) * efs / min(out) / 1e9:.3f})", flush=True)


if __name__ == "__main__":
    main()
