#!/usr/bin/env python3
"""Does throughput sag under sustained load?  Mean per-launch time of the GF scan alone and of
the tree stages alone, over short and long back-to-back runs (diagnostics)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import erasurecodedpir_amd as pir  # noqa: E402


def main():
    n, efs, p, nq = 20, 1024, 2, 1
    e = pir.Engine(p, 1, n, efs, nq)
    e.fill_shard_random(5)
    k = pir.gen_keys(n, 12345, p, nq)[0]
    d_k = e.alloc_dev(e.key_len)
    e.h2d(d_k, k)
    for iters in (10, 100, 1000, 10):
        ph = e.profile_phases(d_k, iters)
        gbs = (1 << n) * efs / (ph["scan"] * 1e-3) / 1e9
        print(f"iters={iters:5d}: scan alone {ph['scan']*1e3:7.1f} us ({gbs:6.0f} GB/s)  "
              f"tree stages alone {ph['tree_stages']*1e3:7.1f} us  frontier {ph['tree_frontier']*1e3:6.1f} us", flush=True)
    e.close()


if __name__ == "__main__":
    main()
