"""Kernel time of the last pipeline's PCA in a rocprofv3 kernel trace, split
into the Krylov steps, the small problem and the final products.
usage: python tools/pca_phases.py [trace.csv]"""
import collections
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "prof", "run_kernel_trace.csv")
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
first = [i for i, r in enumerate(rows) if "k_clean_symmetrize" in r["Kernel_Name"]]
seg = rows[first[-1]:]
a = next(i for i, r in enumerate(seg) if "k_rand_block" in r["Kernel_Name"])
b = next(i for i, r in enumerate(seg) if "k_pt_pairs" in r["Kernel_Name"])
part = seg[a:b]
rb = [i for i, r in enumerate(part) if "k_rand_block" in r["Kernel_Name"]]
sel = [i for i, r in enumerate(part) if "k_select_rev" in r["Kernel_Name"]]


def nm(r):
    return r["Kernel_Name"].replace("void ", "").split("(")[0][:48]


def summarize(lo, hi, label):
    c, t = collections.Counter(), collections.Counter()
    for r in part[lo:hi]:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        c[nm(r)] += 1
        t[nm(r)] += d
    span = (int(part[hi - 1]["End_Timestamp"]) - int(part[lo]["Start_Timestamp"])) / 1e3
    print(f"== {label}: span {span:.1f} us, busy {sum(t.values()) / 1e3:.1f}")
    for k, v in t.most_common(14):
        print(f"   {v / 1e3:8.1f} us {c[k]:4d}x {k}")


s = rb[1] if len(rb) > 1 else 1
summarize(0, s, "Krylov steps (+ T)")
summarize(s, sel[-1] + 1, "small problem")
summarize(sel[-1] + 1, len(part), "final")
