#!/usr/bin/env python3
"""Per-kernel counter summary of the rocprofv3 --pmc passes of tools/gpu_pmc.sh (any config).

    python tools/pmc_kernels.py CFG OUT.json KERNEL=UNITS:UNITNAME ...

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
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v["derived"] for k, v in res["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
