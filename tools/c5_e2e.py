#!/usr/bin/env python3
"""BASELINE configs[4] end to end on ONE MI355X: 8 PIR servers (k=5, r=2 -> p=8, NUM_ROUNDS=5;
SURVEY.md 8(d): tree mode forces p = k + r + 1), each holding its own 2^24 x 1 KiB
erasure-coded shard (8 x 16 GiB in HBM), encoded on the GPU from the reference's synthetic
database (client.cpp:16-33, 70-97); the client's key for one record goes to every server, two
servers are dropped, and the client decodes the record from the other six answers
(client.cpp:211-268).  Prints one JSON line (timings, correctness).

    python tools/c5_e2e.py [--L 26] [--f 1024] [--k 5] [--r 2] [--drop 2,6]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def synthetic_record(v, f):  # client.cpp:16-33
    return np.arange(f, dtype=np.uint8) if v == 1 else np.full(f, v & 0xFF, np.uint8)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=26)
    ap.add_argument("--f", type=int, default=1024)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--r", type=int, default=2)
    ap.add_argument("--drop", default="2,6")
    ap.add_argument("--queries", type=int, default=4)
    a = ap.parse_args()
    import erasurecodedpir_amd as pir
    from erasurecodedpir_amd import server as S
    S.setSystemParams(a.L, a.f, 1, a.k, a.r, 0, 1, 0, 0)
    prm = S.params()
    p, n, nq, efs = prm["NUM_PARTIES"], prm["LOG_NUM_ENCODED_FILES"], prm["NUM_ROUNDS"], prm["ENCODED_FILE_SIZE_BYTES"]
    encdb = -(-(1 << a.L) // a.k)
    rng = np.random.default_rng(26)
    rows = [1] + [int(x) for x in rng.integers(2, encdb, a.queries - 1)]
    fcw = pir.final_cw(p, nq, 1)
    t0 = time.perf_counter()
    keys = [pir.gen_keys(n, row, p, nq, fcw=fcw) for row in rows]
    t_keys = time.perf_counter() - t0
    engines, t_enc = [], []
    for party in range(1, p + 1):
        e = pir.Engine(p, party, n, efs, nq)
        t0 = time.perf_counter()
        e.encode_across(1 << a.L, a.k)
        t_enc.append(time.perf_counter() - t0)
        engines.append(e)
    # every server answers the queue of queries (one launch per server)
    answers, t_ans = [], []
    for party, e in enumerate(engines):
        e.answer_stream([k[party] for k in keys[:1]])  # warm-up
        t0 = time.perf_counter()
        answers.append(e.answer_stream([k[party] for k in keys]))
        t_ans.append((time.perf_counter() - t0) / len(keys))
    drop = [int(x) for x in a.drop.split(",") if x != ""]
    er = [0 if i in drop else 1 for i in range(p)]
    ok, t_dec = [], []
    for q, row in enumerate(rows):
        kept = np.stack([answers[i][q] for i in range(p) if er[i]])
        t0 = time.perf_counter()
        dec = S.assembleDPFTreeQueryResponses(er, kept)
        t_dec.append(time.perf_counter() - t0)
        ok.append(bool(np.array_equal(dec, synthetic_record(row, a.f))))
    for e in engines:
        e.close()
    shard_gib = (1 << n) * efs / 2**30
    print(json.dumps({
        "workload": f"configs[4]: {p} PIR servers (k={a.k}, r={a.r}) on one MI355X, 2^{n} x {efs} B "
                    f"shard each ({p * shard_gib:.0f} GiB of HBM), servers {drop} dropped",
        "parties": p, "num_rounds": nq, "records_per_shard": 1 << n, "record_bytes": efs,
        "queries": len(rows), "decoded_equals_record": ok, "all_ok": all(ok),
        "gpu_keygen_ms_per_query": round(t_keys / len(rows) * 1e3, 3),
        "encode_ms_per_shard": [round(t * 1e3, 2) for t in t_enc],
        "answer_ms_per_query_per_server": [round(t * 1e3, 3) for t in t_ans],
        "answer_GiB_s_per_server": [round(shard_gib / t, 1) for t in t_ans],
        "client_decode_ms": round(float(np.mean(t_dec)) * 1e3, 3),
    }), flush=True)
    sys.exit(0 if all(ok) else 1)


if __name__ == "__main__":
    main()
