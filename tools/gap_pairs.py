"""Kernel-pair gaps and durations of a rocprofv3 --kernel-trace csv (diagnostics for
tools/micro/dispatch_gap.hip): per launch-order segment of SEG kernels, the median gap before
and the median duration of each kernel name.
usage: python tools/gap_pairs.py DIR SEG,SEG,..."""
import csv
import glob
import statistics as st
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
R = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ev = [(r["Kernel_Name"].split("(")[0].replace("void ", ""), int(r["Start_Timestamp"]),
       int(r["End_Timestamp"])) for r in R if not r["Kernel_Name"].startswith("__amd")]
segs = [int(x) for x in sys.argv[2].split(",")]
i = 0
for m, n in enumerate(segs):
    part = ev[i:i + n]
    prev_end = ev[i - 1][2] if i else None
    out = {}
    for k, (name, s, e) in enumerate(part):
        pe = part[k - 1][2] if k else prev_end
        if pe is None:
            continue
        out.setdefault(name, ([], []))
        out[name][0].append((s - pe) / 1000)
        out[name][1].append((e - s) / 1000)
    print(f"mode {m}: " + "; ".join(f"{nm} gap {st.median(g):5.2f} dur {st.median(d):6.2f} us"
                                     for nm, (g, d) in out.items()))
    i += n
