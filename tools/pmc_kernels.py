#!/usr/bin/env python3
"""Per-kernel counter summary of the rocprofv3 --pmc passes of tools/gpu_pmc.sh (any config).

    python tools/pmc_kernels.py CFG OUT.json KERNEL=UNITS:UNITNAME ...

Also written (round 5): the library the passes ran (lib_sha256, from tools/gpu_pmc.sh's
gpurun_out/pmc_<CFG>_lib_sha256.txt), each kernel's average duration in the kernel-trace pass
(gpurun_out/prof_<CFG>/run_kernel_stats.csv) and its LDS and VALU floors at the clock the counters
imply: conflict-free LDS-array cycles per CU ((SQ_LDS_IDX_ACTIVE - SQ_LDS_BANK_CONFLICT) / 256)
and VALU issue cycles per SIMD (SQ_INSTS_VALU / 1024 x 2: a wave64 op holds a SIMD-32 for 2
cycles), each over the kernel's duration -- the kernel's fraction of its LDS / VALU ceiling.

For each named kernel (a substring of its demangled name) every counter of every pass
gpurun_out/pmc_<CFG>_*/run_counter_collection.csv is averaged over that kernel's launches, and
derived per unit of work: VALU / SALU / LDS lane-ops per unit (SQ_INSTS_* x 64 / units per launch),
HBM bytes per launch (2 x FETCH_SIZE KiB + WRITE_SIZE KiB on gfx950, MI355X_MICROARCH.md § HBM),
LDS bank-conflict cycles per LDS-array cycle.  UNITS = units of work per launch (e.g. leaves).
GRBM_GUI_ACTIVE is per XCD, summed over the 8 (tools/pmc_summary.py)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    cfg, out = sys.argv[1], sys.argv[2]
    specs = []
    for a in sys.argv[3:]:
        name, rest = a.split("=", 1)
        units, uname = rest.split(":", 1)
        specs.append((name, float(eval(units, {}, {})), uname))  # noqa: S307 -- our own CLI
    vals = {s[0]: defaultdict(list) for s in specs}
    durs = {s[0]: [] for s in specs}
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{cfg}_*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            for name, _, _ in specs:
                if name in r["Kernel_Name"]:
                    vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
                    durs[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    res = {"config": cfg, "source": f"gpurun_out/pmc_{cfg}_*/ (rocprofv3 --pmc, one pass per counter set)",
           "kernels": {}}
    for name, units, uname in specs:
        avg = {k: sum(v) / len(v) for k, v in vals[name].items()}
        d = {"launches_seen": max((len(v) for v in vals[name].values()), default=0),
             "units_per_launch": units, "unit": uname, "counters_avg_per_launch": avg}
        per = {}
        for k, lab in (("SQ_INSTS_VALU", "valu_lane_ops"), ("SQ_INSTS_SALU", "salu_insts_x64"),
                       ("SQ_INSTS_LDS", "lds_lane_ops"), ("SQ_INSTS_VMEM_RD", "vmem_rd_lane_ops")):
            if k in avg:
                per[f"{lab}_per_{uname}"] = round(avg[k] * 64 / units, 2)
        if "FETCH_SIZE" in avg:
            rd = 2 * avg["FETCH_SIZE"] * 1024
            wr = avg.get("WRITE_SIZE", 0) * 1024
            per["hbm_read_bytes_per_launch"] = rd
            per["hbm_write_bytes_per_launch"] = wr
        if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"]:
            per["lds_bank_conflict_share_of_lds_cycles"] = round(avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"], 4)
        if "GRBM_GUI_ACTIVE" in avg and "SQ_INSTS_VALU" in avg:
            gui = avg["GRBM_GUI_ACTIVE"] / 8
            per["valu_insts_per_simd_per_cycle"] = round(avg["SQ_INSTS_VALU"] / (256 * 4) / gui, 4)
        d["derived"] = per
        res["kernels"][name] = d
    shaf = os.path.join(ROOT, "gpurun_out", f"pmc_{cfg}_lib_sha256.txt")
    if os.path.exists(shaf):
        res["lib_sha256"] = open(shaf).read().split()[0]
    stats = os.path.join(ROOT, "gpurun_out", f"prof_{cfg}", "run_kernel_stats.csv")
    if os.path.exists(stats):
        rows = list(csv.DictReader(open(stats)))
        for name, _, _ in specs:
            hit = [r for r in rows if name in r["Name"]]
            d = res["kernels"][name]
            if not hit:
                continue
            avg_ns = float(hit[0]["AverageNs"])
            a = d["counters_avg_per_launch"]
            d["kernel_avg_ns_trace"] = avg_ns
            if "GRBM_GUI_ACTIVE" in a:
                # the counter passes' own clock: their cycles over the traced duration
                gui = a["GRBM_GUI_ACTIVE"] / 8
                ghz = gui / avg_ns
                c = {"shader_clock_GHz_implied": round(ghz, 3)}
                if "SQ_LDS_IDX_ACTIVE" in a:
                    lds = (a["SQ_LDS_IDX_ACTIVE"] - a.get("SQ_LDS_BANK_CONFLICT", 0.0)) / 256
                    c["lds_floor_ns"] = round(lds / ghz, 1)
                    c["lds_frac_of_ceiling"] = round(lds / gui, 4)
                    c["lds_busy_share_with_conflicts"] = round(a["SQ_LDS_IDX_ACTIVE"] / 256 / gui, 4)
                if "SQ_INSTS_VALU" in a:
                    valu = a["SQ_INSTS_VALU"] / 1024 * 2
                    c["valu_floor_ns"] = round(valu / ghz, 1)
                    c["valu_frac_of_ceiling"] = round(valu / gui, 4)
                d["ceilings"] = c
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: {**v["derived"], **v.get("ceilings", {})} for k, v in res["kernels"].items()},
                     indent=1))


if __name__ == "__main__":
    main()
