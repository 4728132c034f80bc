#!/usr/bin/env python
"""Which branches of a captured HIP graph run concurrently?  (ResNet data-parallel overlap:
in profiles/r04_resnet18_dp a bucket all-reduce node on the side branch ran with no
backward kernel beside it.)

A main chain of NC "compute" kernels (spin_stamp: every block holds its CU for T_C us) and
NB "all-reduce" kernels (16 blocks, T_A us) forked off the chain after compute kernels
F_1..F_NB and joined at the end -- captured with torch.cuda.graph exactly like the native
graph engine's step (engine/native_graph.py _bucket_progress), in several fork layouts:

  chain   -- one comm stream, every all-reduce queued behind the previous one (the engine's)
  fresh   -- a new side stream per all-reduce
  fresh+dep -- a new side stream per all-reduce that also waits for the previous one (the
             all-reduces stay ordered: one communicator / staging buffer)
  eager   -- no graph (the streams as launched)

For each all-reduce kernel: how much compute ran inside its span.  Run it under different
GPU_MAX_HW_QUEUES values (a child process per value: the HIP runtime reads it at start-up).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NC, T_C, NB, T_A = 24, 20.0, 5, 60.0
FORKS = [4, 9, 14, 19, 23]


def one(layout):
    import torch

    from distributed_amd.native import require_C

    C = require_C()
    dev = torch.device("cuda", 0)
    st = torch.zeros(2 * (NC + NB), dtype=torch.int64, device=dev)
    main = torch.cuda.Stream(dev)
    comm = torch.cuda.Stream(dev)

    def body():
        m = torch.cuda.current_stream(dev)
        sides = []
        for i in range(NC):
            C.spin_stamp(int(T_C * 100), 1024, st.data_ptr(), i, m.cuda_stream)
            if i in FORKS:
                b = FORKS.index(i)
                cs = comm if layout == "chain" else torch.cuda.Stream(dev)
                cs.wait_stream(m)
                if layout == "fresh+dep" and sides:
                    cs.wait_stream(sides[-1])  # all-reduces still in order, each on its own stream
                C.spin_stamp(int(T_A * 100), 16, st.data_ptr(), NC + b, cs.cuda_stream)
                sides.append(cs)
        for cs in sides:
            m.wait_stream(cs)

    if layout == "eager":
        with torch.cuda.stream(main):
            body()
            body()
    else:
        g = torch.cuda.CUDAGraph()
        main.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(main):
            with torch.cuda.graph(g, stream=main):
                body()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        g.replay()
    torch.cuda.synchronize()
    s = st.cpu().view(-1, 2).tolist()
    t0 = min(a for a, _ in s)
    comp = [((a - t0) / 100, (b - t0) / 100) for a, b in s[:NC]]
    out = []
    for k, (a, b) in enumerate(s[NC:]):
        a, b = (a - t0) / 100, (b - t0) / 100
        ov = sum(max(0.0, min(b, y) - max(a, x)) for x, y in comp)
        out.append({"bucket": k, "start_us": round(a, 1), "len_us": round(b - a, 1), "compute_inside_us": round(ov, 1)})
    span = max(y for _, y in comp + [(a, b) for a, b in [((x - t0) / 100, (y - t0) / 100) for x, y in s[NC:]]])
    return {"layout": layout, "span_us": round(span, 1), "buckets": out}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        res = [one(l) for l in ("chain", "fresh", "fresh+dep")]
        print(json.dumps({"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "res": res}))
        return
    for q in (sys.argv[1:] or ["4", "8"]):
        env = dict(os.environ, GPU_MAX_HW_QUEUES=q)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True,
                           text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode or not line:
            print(f"GPU_MAX_HW_QUEUES={q}: rc {r.returncode}\n{r.stderr[-2000:]}")
            continue
        j = json.loads(line[0])
        print(f"== GPU_MAX_HW_QUEUES={q}  (compute chain: {NC} x {T_C} us; all-reduces {NB} x {T_A} us)")
        for lay in j["res"]:
            bs = "  ".join(f"[{b['start_us']:.0f}+{b['len_us']:.0f}: {b['compute_inside_us']:.0f} cmp]"
                           for b in lay["buckets"])
            print(f"  {lay['layout']:9s} span {lay['span_us']:7.1f} us  {bs}")


if __name__ == "__main__":
    main()
