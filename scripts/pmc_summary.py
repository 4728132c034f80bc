"""Summarise rocprofv3 --pmc results (the run_results.db sqlite files of each pass) per
kernel, median over dispatches, for the fused MNIST step kernels, plus derived ratios:
    python scripts/pmc_summary.py gpurun_out/pmc_mnist"""
import glob
import os
import sqlite3
import statistics
import sys
from collections import defaultdict


def short(k):
    return "fwd" if "convnet2::fwd" in k else "bwd" if "convnet2::bwd" in k else None


def main(root):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per dispatch]
    for db in sorted(glob.glob(os.path.join(root, "*", "*.db"))):
        con = sqlite3.connect(db)
        per = defaultdict(float)
        q = "select dispatch_id, kernel_name, counter_name, value from counters_collection"
        for d, k, c, v in con.execute(q):
            s = short(k or "")
            if s:
                per[(s, d, c)] += v
        for (s, _, c), v in per.items():
            vals[s][c].append(v)
    for k in sorted(vals):
        m = {c: statistics.median(v) for c, v in vals[k].items()}
        print(k)
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:14.1f}  (n={len(vals[k][c])})")
        w = m.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM", "SQ_INSTS_MFMA"):
                if c in m:
                    print(f"   per wave {c:19s} {m[c] / w:10.1f}")
        for a, b in (("SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES"), ("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
                     ("SQ_WAIT_ANY", "SQ_WAVE_CYCLES"), ("SQ_ACTIVE_INST_LDS", "SQ_WAVE_CYCLES"),
                     ("SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS")):
            if a in m and b in m and m[b]:
                print(f"   {a} / {b}: {m[a] / m[b]:.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
