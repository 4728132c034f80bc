"""Split a rocprofv3 kernel_stats.csv by origin: the framework's own kernels (csrc/), RCCL,
runtime copies / fills, and anything else (PyTorch / vendor libraries)."""
import csv
import sys


def origin(name: str) -> str:
    n = name.lower()
    if "rccl" in n or "nccl" in n:
        return "rccl"
    if "__amd_rocclr" in n:
        return "runtime copy/fill"
    if "at::native" in n or "at::" in n or "c10::" in n or "void at" in n:
        return "pytorch"
    if any(k in n for k in ("miopen", "cijk", "rocblas", "hipblaslt", "ck::", "ck_tile")):
        return "vendor"
    return "damd"


def main(path):
    rows = list(csv.DictReader(open(path)))
    by = {}
    for r in rows:
        o = origin(r["Name"])
        by.setdefault(o, []).append(r)
    for o, rs in sorted(by.items()):
        calls = sum(int(r["Calls"]) for r in rs)
        ns = sum(float(r["TotalDurationNs"]) for r in rs)
        print(f"{o:20s} kernels {len(rs):3d} calls {calls:7d} time {ns / 1e6:9.3f} ms")
        if o != "damd":
            for r in sorted(rs, key=lambda r: -float(r["TotalDurationNs"])):
                print(f"    {int(r['Calls']):6d}  {float(r['TotalDurationNs']) / 1e3:10.1f} us  {r['Name'][:110]}")


if __name__ == "__main__":
    main(sys.argv[1])
