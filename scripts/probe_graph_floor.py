"""Per-kernel floor of a captured hipGraph on this GPU: N dependent 1-element torch
kernels replayed as one graph; wall time / N.  usage: python scripts/probe_graph_floor.py"""
import time

import torch


def main():
    x = torch.zeros(1, device="cuda")
    big = torch.zeros(1 << 20, device="cuda")
    for n, t in ((200, x), (200, big)):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for _ in range(3):
                t.add_(1.0)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                t.add_(1.0)
        g.replay()
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / (reps * n)
        print(f"{n} dependent kernels on {t.numel()} floats: {dt * 1e6:.2f} us per kernel", flush=True)


if __name__ == "__main__":
    main()
