#!/usr/bin/env python3
"""BASELINE configs[0] end to end over the wire: start p `pir_serve` processes on localhost
(TLS + msgpack, the protocol of src/server/server.go), SETUP each with the reference's synthetic
database, then query records through the client flow of src/client/tree.go (GPU key generation,
parallel requests, erasure decode) and check them.  The equivalent of the
scripts/run_end_to_end.sh that the reference's README names but does not ship.

    python tools/run_end_to_end.py [--L 16] [--f 256] [--k 1] [--r 0] [--queries 4] [--down 0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=16)
    ap.add_argument("--f", type=int, default=256)
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--r", type=int, default=0)
    ap.add_argument("--queries", type=int, default=4)
    ap.add_argument("--down", type=int, default=0, help="servers to stop before querying (<= r)")
    a = ap.parse_args()
    from erasurecodedpir_amd import server as S
    from erasurecodedpir_amd import wire
    from test_wire import Servers, _synthetic
    S.setSystemParams(a.L, a.f, 1, a.k, a.r, 0, 1, 0, 0)
    p = S.params()["NUM_PARTIES"]
    encdb = -(-(1 << a.L) // a.k)
    rng = np.random.default_rng(0)
    rows = [1] + [int(x) for x in rng.integers(0, encdb, a.queries - 1)]
    out = {"config": f"configs[0]-style loopback: {p} pir_serve processes, 2^{a.L} files x {a.f} B, "
                      f"k={a.k}, r={a.r}, {a.down} server(s) down"}
    with Servers(p) as sv:
        t0 = time.perf_counter()
        for addr in sv.addrs:
            wire.setup(addr, a.L, a.f, a.k, a.r)
        out["setup_s"] = round(time.perf_counter() - t0, 3)
        for i in range(a.down):
            sv.stop(p - 1 - i)
        ok, lat = [], []
        for row in rows:
            t0 = time.perf_counter()
            rec, resps, er = wire.tree_query(sv.addrs, row, a.L, a.f, a.k, a.r)
            lat.append(time.perf_counter() - t0)
            ok.append(bool(np.array_equal(rec, _synthetic(row, a.f))))
        out.update({"queries": len(rows), "decoded_ok": ok, "all_ok": all(ok),
                    "client_query_ms": [round(x * 1e3, 2) for x in lat],
                    "server_latency_us": [round(r_["ServerLatency"] / 1e3, 1) for r_ in resps if r_]})
    print(json.dumps(out), flush=True)
    sys.exit(0 if all(ok) else 1)


if __name__ == "__main__":
    main()
