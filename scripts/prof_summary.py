"""Summarise a rocprofv3 kernel_stats.csv: per-kernel total / calls / mean, and per-step
totals when the number of profiled steps is given.  usage: prof_summary.py stats.csv [steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.3f} ms over {steps} step(s) = {tot / 1e6 / steps:.3f} ms/step")
print(f"{'ms/step':>8} {'calls/step':>10} {'mean us':>8}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
    t = float(r["TotalDurationNs"])
    print(f"{t / 1e6 / steps:8.3f} {int(r['Calls']) / steps:10.1f} {float(r['AverageNs']) / 1e3:8.1f}  {r['Name'][:100]}")
