"""Summarise rocprofv3 --pmc counter CSVs per kernel (median over dispatches) for the
fused MNIST step: python scripts/pmc_summary.py gpurun_out/pmc_mnist"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main(root):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch]
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(lambda: defaultdict(float))
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r.get("Kernel_Name", "?")
                if "convnet" not in k:
                    continue
                short = "fwd" if "fwdI" in k else "bwd" if "bwdI" in k else k.split("(")[0][-30:]
                per[(short, r.get("Dispatch_Id"))][r["Counter_Name"]] += float(r["Counter_Value"])
        for (k, _), cs in per.items():
            for c, v in cs.items():
                vals[k][c].append(v)
    for k in sorted(vals):
        print(k)
        for c in sorted(vals[k]):
            print(f"   {c:24s} {statistics.median(vals[k][c]):14.1f}  (n={len(vals[k][c])})")


if __name__ == "__main__":
    main(sys.argv[1])
