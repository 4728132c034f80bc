"""Per-kernel occupancy report from a rocprofv3 kernel trace (--kernel-trace CSV).

For every distinct kernel: its register / LDS footprint as the hardware allocated it
(VGPR_Count + Accum_VGPR_Count, LDS_Block_Size from the trace), the resident waves per
SIMD and workgroups per CU those allow on gfx950 (MI355X: 4 SIMDs per CU, a 512-entry
unified VGPR+AGPR file per SIMD lane allocated in 8-register granules, at most 8 waves per
SIMD; 160 KiB LDS per CU), which resource binds, and the launch's workgroup count against
the 256 CUs (one full wave of workgroups = 256 x workgroups-per-CU).  Mean duration per
launch is from the same trace.  Caveat: the trace's LDS_Block_Size can read 0 for kernels
whose LDS is all dynamic (the fused MNIST kernels size theirs at launch), so their LDS
limit is not applied here.

usage: python scripts/occupancy.py <kernel_trace.csv> [out.txt]
"""
from __future__ import annotations

import collections
import csv
import re
import sys

CUS, SIMDS, VGPR_FILE, MAX_WAVES_SIMD, LDS_CU = 256, 4, 512, 8, 160 * 1024


def short(name: str) -> str:
    n = name.replace("void ", "").replace("damd::(anonymous namespace)::", "").replace("damd::", "")
    n = re.sub(r"\(.*", "", n) if not n.startswith("(") else n
    return n[:64]


def occupancy(vgpr: int, agpr: int, lds: int, wg: int):
    regs = -(-(vgpr + agpr) // 8) * 8 or 8
    w_reg = min(MAX_WAVES_SIMD, VGPR_FILE // regs)
    waves_wg = -(-wg // 64)
    per_simd_wg = -(-waves_wg // SIMDS)           # waves of one workgroup on each SIMD
    wg_reg = (w_reg * SIMDS) // waves_wg if waves_wg else 0
    wg_lds = LDS_CU // lds if lds else 1 << 30
    wg_wave = (MAX_WAVES_SIMD * SIMDS) // waves_wg
    wg_cu = max(0, min(wg_reg, wg_lds, wg_wave))
    bind = min((wg_reg, "VGPR"), (wg_lds, "LDS"), (wg_wave, "wave slots"))[1]
    return wg_cu, wg_cu * waves_wg / SIMDS, bind, per_simd_wg


def main():
    path = sys.argv[1]
    out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
    rows = list(csv.DictReader(open(path)))
    agg = collections.OrderedDict()
    for r in rows:
        if "rocclr" in r["Kernel_Name"] or "at::native" in r["Kernel_Name"]:
            continue
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        key = (short(r["Kernel_Name"]), grid // wg)
        d = agg.setdefault(key, dict(n=0, t=0.0, v=int(r["VGPR_Count"]), a=int(r["Accum_VGPR_Count"]),
                                     l=int(r["LDS_Block_Size"]), wg=wg, s=int(r["Scratch_Size"])))
        d["n"] += 1
        d["t"] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{'kernel':64s} {'WGs':>7s} {'thr':>4s} {'vgpr':>4s} {'agpr':>4s} {'lds':>6s} {'scr':>4s} "
          f"{'WG/CU':>5s} {'waves/SIMD':>10s} {'bound by':>10s} {'WG waves':>8s} {'mean us':>8s}", file=out)
    for (k, nwg), d in sorted(agg.items(), key=lambda kv: -kv[1]["t"]):
        wg_cu, wps, bind, _ = occupancy(d["v"], d["a"], d["l"], d["wg"])
        full = CUS * max(wg_cu, 1)
        print(f"{k:64s} {nwg:7d} {d['wg']:4d} {d['v']:4d} {d['a']:4d} {d['l']:6d} {d['s']:4d} {wg_cu:5d} "
              f"{wps:10.1f} {bind:>10s} {nwg / full:8.2f} {d['t'] / d['n']:8.1f}", file=out)


if __name__ == "__main__":
    main()
