"""Per-stream kernel breakdown of the last call in a rocprofv3 --kernel-trace
CSV: python tools/trace_streams.py <run_kernel_trace.csv> [gap_ms | kernel]
(calls are split at idle gaps longer than gap_ms, default 20, or at each
launch of the named kernel, e.g. k_clean_symmetrize)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
arg = sys.argv[2] if len(sys.argv) > 2 else "20"
ts = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]) for r in rows)
if arg.replace(".", "").isdigit():
    gap = float(arg) * 1e6
    calls, end = [[ts[0]]], ts[0][1]
    for t in ts[1:]:
        if t[0] - end > gap:
            calls.append([])
        calls[-1].append(t)
        end = max(end, t[1])
    c = calls[-1]
else:
    t_start = max(t[0] for t in ts if arg in t[2])
    c = [t for t in ts if t[0] >= t_start]
t0 = c[0][0]
print("call span %.2f ms, %d kernels" % ((max(e for _, e, _, _ in c) - t0) / 1e6, len(c)))
bys = collections.defaultdict(list)
for s, e, k, q in c:
    bys[q].append((s, e, k))
for q, l in sorted(bys.items(), key=lambda x: x[1][0][0]):
    print("stream %s: %d kernels, %.2f..%.2f ms, busy %.2f ms" % (
        q, len(l), (l[0][0] - t0) / 1e6, max(e for _, e, _ in l) / 1e6 - t0 / 1e6, sum(e - s for s, e, _ in l) / 1e6))
    agg = collections.defaultdict(lambda: [0, 0.0, 1e18, 0.0])
    for s, e, k in l:
        a = agg[k.split("(")[0][:52]]
        a[0] += 1
        a[1] += (e - s) / 1e6
        a[2] = min(a[2], (s - t0) / 1e6)
        a[3] = max(a[3], (e - t0) / 1e6)
    for k, a in sorted(agg.items(), key=lambda x: -x[1][1])[:10]:
        print("   %-52s n=%4d %8.2f ms  [%7.2f .. %7.2f]" % (k, a[0], a[1], a[2], a[3]))
