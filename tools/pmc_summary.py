#!/usr/bin/env python3
"""Summarise the rocprofv3 passes of tools/gpu_profile.sh into profiles/pmc_<cfg>.json.

    python tools/pmc_summary.py CFG QUERIES_PER_LAUNCH RECORDS RECORD_BYTES

Reads gpurun_out/prof_<cfg>/run_kernel_stats.csv (kernel trace + stats pass) and the
counter_collection CSVs of the separate --pmc FETCH_SIZE / --pmc WRITE_SIZE passes
(gpurun_out/pmcf_<cfg>, gpurun_out/pmcw_<cfg>).  The dominant kernel is the k_query instance
with the largest total duration.  HBM read bytes = 2 x FETCH_SIZE x 1024 (gfx950: FETCH_SIZE
counts half the bytes of 16-B-per-lane streaming reads, MI355X_MICROARCH.md §HBM)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main():
    cfg, qpl, nrec, efs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    base = os.path.join(ROOT, "gpurun_out")
    stats = rows(os.path.join(base, f"prof_{cfg}", "**", "*kernel_stats.csv"))
    dom = max((r for r in stats if "k_query" in r["Name"]), key=lambda r: float(r["TotalDurationNs"]))
    name = dom["Name"]
    avg_ns = float(dom["AverageNs"])

    def counter(pass_dir, cname):
        vals = {}
        for r in rows(os.path.join(base, pass_dir, "**", "*counter_collection.csv")):
            if r.get("Kernel_Name") == name and r.get("Counter_Name") == cname:
                key = r.get("Dispatch_Id") or r.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
        return sum(vals.values()) / len(vals) if vals else None, len(vals)

    fetch_kb, nf = counter(f"pmcf_{cfg}", "FETCH_SIZE")
    write_kb, nw = counter(f"pmcw_{cfg}", "WRITE_SIZE")
    algo = nrec * efs * qpl
    read_b = 2 * fetch_kb * 1024 if fetch_kb is not None else None
    hbm = (read_b or 0) + (write_kb or 0) * 1024
    out = {
        "config": cfg,
        "kernel": name.split("(")[0],
        "queries_per_launch": qpl,
        "launches_profiled": {"FETCH_SIZE": nf, "WRITE_SIZE": nw},
        "FETCH_SIZE_KB_per_launch": fetch_kb,
        "WRITE_SIZE_KB_per_launch": write_kb,
        "correction": "gfx950 FETCH_SIZE reports 1/2 of wide coalesced streaming reads "
                      "(MI355X_MICROARCH.md HBM): read bytes = 2 x FETCH_SIZE x 1024",
        "hbm_bytes_per_launch": int(hbm),
        "hbm_bytes_per_query": int(hbm / qpl),
        "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": round(hbm / algo, 4),
        "kernel_avg_ns_rocprof": avg_ns,
        "achieved_GBps_rocprof": round(algo / avg_ns, 1),
    }
    dst = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
