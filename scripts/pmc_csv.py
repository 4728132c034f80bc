"""Per-kernel PMC summary of rocprofv3 --pmc CSV output (every *counter_collection.csv
under DIR), median over dispatches of each counter summed per dispatch, plus the MFMA-busy
share of the chip's SIMD cycles:  python scripts/pmc_csv.py DIR [kernel-substring ...]"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main(root, subs):
    per = defaultdict(float)  # (kernel, dispatch, counter) -> value
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if subs and not any(s in k for s in subs):
                continue
            k = k.split("(")[0].replace("void ", "").replace("damd::(anonymous namespace)::", "")
            per[(k, f, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    vals = defaultdict(lambda: defaultdict(list))
    for (k, _, _, c), v in per.items():
        vals[k][c].append(v)
    for k in sorted(vals):
        m = {c: statistics.median(v) for c, v in vals[k].items()}
        print(k)
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:16.1f}  (n={len(vals[k][c])})")
        g = m.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            # GRBM_GUI_ACTIVE sums the 8 XCDs: kernel cycles = /8; 256 CUs x 4 SIMDs
            print(f"   MFMA busy share of SIMD cycles: {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.3f}")
        for a, b in (("SQ_WAIT_ANY", "SQ_WAVE_CYCLES"), ("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
                     ("SQ_ACTIVE_INST_LDS", "SQ_WAVE_CYCLES"), ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE")):
            if a in m and b in m and m[b]:
                print(f"   {a} / {b}: {m[a] / m[b]:.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
