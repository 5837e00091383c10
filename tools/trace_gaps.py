"""Busy time vs. idle gaps of the LAST pipeline in a rocprofv3 kernel trace
(gpurun_out/prof/run_kernel_trace.csv), split into stages by marker kernels:
where the GPU waits on the host (launch-bound phases, host syncs).
usage: python tools/trace_gaps.py [trace.csv]"""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "prof", "run_kernel_trace.csv")
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = [i for i, r in enumerate(rows) if "k_clean_symmetrize" in r["Kernel_Name"]]
seg = rows[first[-1]:]
# stage starts: the first kernel of each stage
marks = [("mask", "k_clean_symmetrize"), ("cor", "k_xtx"), ("pca", "k_rand_block"), ("sweep", "k_pt_pairs")]


def name(r):
    return r["Kernel_Name"].replace("void ", "").split("(")[0]


starts = []
for st, key in marks:
    j = next((i for i, r in enumerate(seg) if key in r["Kernel_Name"]), None)
    if j is not None:
        starts.append((st, j))
starts.append(("end", len(seg)))
t_end = int(seg[-1]["End_Timestamp"])
for (st, a), (_, b) in zip(starts, starts[1:]):
    part = seg[a:b]
    t0 = int(part[0]["Start_Timestamp"])
    t1 = int(seg[b]["Start_Timestamp"]) if b < len(seg) else t_end
    busy, cur_end, gaps = 0, t0, []
    for r in part:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > cur_end:
            gaps.append((s - cur_end, name(r)))
        busy += max(0, e - max(s, cur_end))
        cur_end = max(cur_end, e)
    gsum = sum(g for g, _ in gaps)
    print(f"{st:6s} span {(t1 - t0) / 1e3:9.1f} us  busy {busy / 1e3:9.1f}  gaps {gsum / 1e3:8.1f} "
          f"({len(gaps)} gaps, {sum(1 for g, _ in gaps if g > 20000)} > 20 us)  launches {len(part)}")
    big = sorted(gaps, reverse=True)[:6]
    for g, nm in big:
        print(f"         gap {g / 1e3:8.1f} us before {nm}")
