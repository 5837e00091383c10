"""Per-kernel (name, grid) totals of the LAST pipeline in a rocprofv3 kernel
trace (gpurun_out/prof/run_kernel_trace.csv): where one pipeline's time goes.
usage: python tools/trace_top.py [first-kernel-of-pipeline-substring] [rows]"""
import collections
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
mark = sys.argv[1] if len(sys.argv) > 1 else "k_clean_symmetrize"
nrows = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = list(csv.DictReader(open(os.path.join(ROOT, "gpurun_out", "prof", "run_kernel_trace.csv"))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
seg = rows[idx[-1]:]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    key = (r["Kernel_Name"].replace("void ", "").split("(")[0], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
    agg[key][0] += 1
    agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
print(f"pipeline: {len(seg)} launches, kernel time {tot:.1f} us, span {span:.1f} us")
for (name, wg), (cnt, us) in sorted(agg.items(), key=lambda x: -x[1][1])[:nrows]:
    print(f"{us:9.1f} us {cnt:4d} x {us / cnt:8.1f}  wg {wg:6d}  {name}")
