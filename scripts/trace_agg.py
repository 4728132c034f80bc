"""Per-kernel totals of one step of a rocprofv3 kernel trace (same step window as
step_trace.py): python scripts/trace_agg.py <kernel_trace.csv> [anchor]"""
import collections
import csv
import re
import sys

path = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "gather_batch_k"
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if anchor in r['Kernel_Name']]
i, j = idx[-3], idx[-2]
agg = collections.defaultdict(lambda: [0, 0.0, []])
for r in rows[i:j]:
    n = re.sub(r'damd::|\(anonymous namespace\)::|void ', '', r['Kernel_Name'])
    k = re.match(r'[\w:]+(<[^()]*>)?', n).group(0)
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000
    agg[k][0] += 1
    agg[k][1] += d
    agg[k][2].append(round(d, 1))
tot = sum(v[1] for v in agg.values())
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{v[1]:8.1f} {100 * v[1] / tot:5.1f}% {v[0]:4d}  {k[:60]:60s} {v[2][:10]}")
print(f"{tot:8.1f} us in {sum(v[0] for v in agg.values())} launches")
