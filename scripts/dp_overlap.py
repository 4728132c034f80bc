#!/usr/bin/env python
"""Overlap of the gradient-bucket all-reduces with the backward, from a rocprofv3 kernel
trace (--kernel-trace --output-format csv) of `bench.py --model resnet18 --gpus 2` with the
ranks sharing one GPU (scripts/prof_resnet_dp.sh).

usage: dp_overlap.py <kernel_trace.csv> <out.txt>

One step of one rank's process (the second-to-last complete step: between two
gather_batch_k launches, the step's first kernel): every kernel with start / duration /
HIP queue, then per bucket all-reduce (peer_allreduce_k) the compute time of the SAME
process inside its span, and the exposed tail (the last all-reduce's end minus the last
backward kernel's end)."""
import csv
import sys
from collections import defaultdict


def main():
    path, out = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(path)))
    pid_key = next((k for k in ("Process_Id", "Pid", "PID") if k in rows[0]), None)
    q_key = next((k for k in ("Queue_Id", "Queue_ID", "Stream_Id") if k in rows[0]), None)
    by_pid = defaultdict(list)
    for r in rows:
        by_pid[r[pid_key] if pid_key else "0"].append(r)
    # the rank with the most kernels (a rank process, not the spawning parent)
    pid, rs = max(by_pid.items(), key=lambda kv: len(kv[1]))
    rs.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rs) if "gather_batch_k" in r["Kernel_Name"]]
    i, j = idx[-3], idx[-2]
    step = rs[i:j]
    t0 = int(step[0]["Start_Timestamp"])
    span = lambda r: ((int(r["Start_Timestamp"]) - t0) / 1000, (int(r["End_Timestamp"]) - t0) / 1000)
    ar = [r for r in step if "peer_allreduce_k" in r["Kernel_Name"] or "AllReduce" in r["Kernel_Name"]]
    comp = [r for r in step if r not in ar]
    lines = [f"# one step of process {pid} ({len(step)} kernels); q = HIP queue", "start_us  dur_us  q  kernel"]
    for r in step:
        a, b = span(r)
        lines.append(f"{a:8.1f} {b - a:7.1f} {r[q_key] if q_key else '-':>2}  {r['Kernel_Name'][:84]}")
    lines.append("")
    tot_ar = ov_tot = 0.0
    last_comp_end = max(span(r)[1] for r in comp if "opt_step" not in r["Kernel_Name"])
    for r in ar:
        a, b = span(r)
        ov = sum(max(0.0, min(b, span(c)[1]) - max(a, span(c)[0])) for c in comp)
        n = sum(1 for c in comp if min(b, span(c)[1]) > max(a, span(c)[0]))
        tot_ar += b - a
        ov_tot += min(ov, b - a)
        lines.append(f"bucket all-reduce at {a:8.1f} us, {b - a:6.1f} us long: {n} compute kernels overlap it "
                     f"({ov:.1f} us of compute inside its span)")
    end_ar = max(span(r)[1] for r in ar) if ar else 0.0
    lines.append(f"step span {span(step[-1])[1]:.1f} us; {len(ar)} bucket all-reduces, {tot_ar:.1f} us total, "
                 f"{ov_tot:.1f} us of compute overlapped with them; exposed tail after the last backward kernel "
                 f"{max(0.0, end_ar - last_comp_end):.1f} us")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[-(len(ar) + 1):]))


if __name__ == "__main__":
    main()
