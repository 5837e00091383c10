"""Per-pipeline timeline from a rocprofv3 kernel trace (csv): the last complete
pipeline (k_clean_symmetrize .. the last k_ch) split into stages, with kernel
busy time vs wall time (the gaps are launch/dependency bubbles).
python tools/timeline.py gpurun_out/prof/run_kernel_trace.csv [top gaps] [pipeline index]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""),
             int(r["Stream_Id"]) if r.get("Stream_Id") else 0) for r in rows)
starts = [i for i, e in enumerate(ev) if "k_clean_symmetrize" in e[2]]
if len(starts) < 2:
    sys.exit("need two pipelines in the trace")
# pipeline index (default 1: the first timed step after the warmup; the bench's
# last pipelines time kernel classes with extra events)
pi = int(sys.argv[3]) if len(sys.argv) > 3 else 1
seg = ev[starts[pi]:starts[pi + 1]] if pi + 1 < len(starts) else ev[starts[pi]:]
# stage boundaries by marker kernels
marks = [("mask", "k_clean_symmetrize"), ("cor", "k_xtx"), ("pca", "k_pd_digits_cm"), ("sweep", "k_pt_pairs")]
bounds = []
for name, key in marks:
    for i, e in enumerate(seg):
        if key in e[2]:
            bounds.append((name, i))
            break
bounds.append(("end", len(seg)))
t0 = seg[0][0]
print(f"pipeline wall {(seg[-1][1] - t0) / 1e3:.1f} us, kernels {len(seg)}")
for (name, i0), (_, i1) in zip(bounds, bounds[1:]):
    part = seg[i0:i1]
    if not part:
        continue
    wall = (seg[i1][0] if i1 < len(seg) else part[-1][1]) - part[0][0]
    # busy = union of kernel intervals
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in part:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    gaps = defaultdict(float)
    cnt = defaultdict(int)
    for a, b in zip(part, part[1:]):
        g = b[0] - max(a[1], a[0])
        if g > 0:
            gaps[a[2][:28] + " -> " + b[2][:28]] += g
            cnt[a[2][:28] + " -> " + b[2][:28]] += 1
    print(f"{name:6s} wall {wall / 1e3:8.1f} us  busy {busy / 1e3:8.1f} us  gaps {(wall - busy) / 1e3:7.1f} us  "
          f"kernels {len(part)}")
    for k, v in sorted(gaps.items(), key=lambda kv: -kv[1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 6]:
        print(f"         gap {v / 1e3:7.1f} us  x{cnt[k]:3d}  {k}")
big = [(b[0] - a[1], a[2][:30], b[2][:30], i) for i, (a, b) in enumerate(zip(seg, seg[1:])) if b[0] - a[1] > 20000]
for g, a, b, i in big:
    print(f"gap {g / 1e3:7.1f} us at kernel {i}: {a} -> {b}")
