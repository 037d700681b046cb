#!/usr/bin/env python3
"""k_query queue rate by round count (diagnostics): 2^24 x 1 KiB, p = NQ + 1 parties so that the
tree-DPF key has NQ output bytes per leaf, K queued queries per launch; prints ms per query and
TB/s for NQ = 1..5 -- the scan speed a fused share generator would run at."""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))


def main():
    import erasurecodedpir_amd as pir
    n, efs, K, W = 24, 1024, 10, 3
    rng = np.random.default_rng(1)
    for nq in (1, 2, 3, 4, 5):
        p = 2 if nq == 1 else nq + 1
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
            e.answer_stream_dev(dk, W, dr)
            e.sync()
            t0 = time.perf_counter()
            e.answer_stream_dev(dk + W * kl, K, dr + W * ab)
            e.sync()
            ms = (time.perf_counter() - t0) / K * 1e3
            print(f"NQ={nq} p={p}: {ms:.3f} ms per query, {(1 << n) * efs / ms / 1e9:.3f} TB/s", flush=True)


if __name__ == "__main__":
    main()
