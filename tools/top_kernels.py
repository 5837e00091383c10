"""Top kernels of a rocprofv3 --stats CSV: python tools/top_kernels.py <kernel_stats.csv> [calls_divisor]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
    t = float(r["TotalDurationNs"])
    print(f"{r['Name'].split('(')[0].replace('void ', '')[:60]:60s} calls {int(r['Calls']) / div:7.1f} "
          f"ms {t / 1e6 / div:8.3f} avg_us {float(r['AverageNs']) / 1e3:9.1f} {100 * t / tot:5.1f}%")
print(f"total ms {tot / 1e6 / div:.3f}")
