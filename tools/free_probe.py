#!/usr/bin/env python3
"""Where freeServer's remaining milliseconds go (diagnostics, GPU box): a shim server set up at
the given shape (the bench's setup_leg path), one T-thread query, then freeServer timed around
the ctypes call -- with the reaper's defer at its default and at 2 s (so that no teardown runs
while the call is timed), and the background teardown timed by pirServerWaitFreed.
    python tools/free_probe.py [L] [k] [r]
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(L, k, r):
    import erasurecodedpir_amd as pir
    from erasurecodedpir_amd import server as S
    pir.load()
    S.setSystemParams(L, 1024, 1, k, r, 0, 1, 0, 0)
    prm = S.params()
    p, n, nq, efs = prm["NUM_PARTIES"], prm["LOG_NUM_ENCODED_FILES"], prm["NUM_ROUNDS"], prm["ENCODED_FILE_SIZE_BYTES"]
    cl = S.Client(L, 1024)
    out = []
    for rep in range(3):
        sv = S.Server(1, prm["LOG_NUM_FILES"], efs, 0, 16)
        cl.encode_across_files_server(sv)
        key = pir.gen_keys(n, 12345, p, nq, fcw=pir.final_cw(p, nq, 1))[0]
        sv.runTreeQueryThreads(key, 16)
        t0 = time.perf_counter()
        sv.freeServer()
        t1 = time.perf_counter()
        S.wait_freed()
        t2 = time.perf_counter()
        out.append((round((t1 - t0) * 1e3, 3), round((t2 - t1) * 1e3, 1)))
    cl.free_client()
    print(f"L={L} k={k} r={r} defer={os.environ.get('PIR_REAPER_DEFER_MS', 'default')}: "
          f"(freeServer ms, teardown ms) x3 = {out}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        one(*map(int, sys.argv[2:5]))
        sys.exit(0)
    args = sys.argv[1:4] or ["24", "1", "0"]
    for defer in (None, "2000"):
        env = dict(os.environ)
        if defer:
            env["PIR_REAPER_DEFER_MS"] = defer
        subprocess.run([sys.executable, __file__, "--one", *args], env=env, check=True)
