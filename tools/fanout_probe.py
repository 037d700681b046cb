#!/usr/bin/env python3
"""Per-query times of the reference's T-thread call shape through the shim (diagnostics, GPU
box): a 2^L x 1 KiB tree-mode server set up on the GPU, then Q fan-outs of T
runOptimizedDPFTreeQueryThread calls from the shim's C++ pool (pirRunTreeQueryThreads), each
timed, beside Q single runOptimizedDPFTreeQuery calls; once per $PIR_SLICE_JOIN_US value given.
A bimodal distribution means some fan-outs did not meet in one slice group.
    python tools/fanout_probe.py [L] [T] [Q] [join_us ...]
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(L, T, Q):
    import numpy as np
    import erasurecodedpir_amd as pir
    from erasurecodedpir_amd import server as S
    pir.load()
    S.setSystemParams(L, 1024, 1, 1, 0, 0, 1, 0, 0)
    prm = S.params()
    p, n, nq = prm["NUM_PARTIES"], prm["LOG_NUM_ENCODED_FILES"], prm["NUM_ROUNDS"]
    cl = S.Client(L, 1024)
    sv = S.Server(1, L, 1024, 0, T)
    cl.encode_across_files_server(sv)
    keys = [pir.gen_keys(n, 1000 + 37 * i, p, nq, fcw=pir.final_cw(p, nq, 1))[0] for i in range(Q)]
    for i in range(3):
        sv.runTreeQueryThreads(keys[i], T)
        sv.runOptimizedDPFTreeQuery(keys[i], nq)
    fan, single = [], []
    for i in range(Q):
        t0 = time.perf_counter()
        a = sv.runTreeQueryThreads(keys[i], T)
        t1 = time.perf_counter()
        b = sv.runOptimizedDPFTreeQuery(keys[i], nq)
        t2 = time.perf_counter()
        assert np.array_equal(a, b)
        fan.append((t1 - t0) * 1e3)
        single.append((t2 - t1) * 1e3)
    sv.freeServer()
    cl.free_client()
    f = sorted(fan)
    print(f"join={os.environ.get('PIR_SLICE_JOIN_US', 'default')}: fan-out T={T} median {np.median(fan):.3f} "
          f"mean {np.mean(fan):.3f} ms (sorted: {' '.join(f'{x:.2f}' for x in f)}); single median "
          f"{np.median(single):.3f} mean {np.mean(single):.3f} ms", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        one(*map(int, sys.argv[2:5]))
        sys.exit(0)
    L, T, Q = (int(x) for x in (sys.argv[1:4] + ["24", "16", "20"][len(sys.argv[1:4]):]))
    joins = sys.argv[4:] or [None]
    for j in joins:
        env = dict(os.environ)
        if j is not None:
            env["PIR_SLICE_JOIN_US"] = j
        subprocess.run([sys.executable, __file__, "--one", str(L), str(T), str(Q)], env=env, check=True)
