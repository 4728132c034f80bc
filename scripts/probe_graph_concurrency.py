"""Do independent branches of a captured hipGraph run concurrently on MI355X?  Times one
replay of N small GEMMs (few workgroups each) captured (a) on one stream and (b) forked
over two streams (event fork/join), plus the same eagerly.  usage: python
scripts/probe_graph_concurrency.py"""
import time

import torch

dev = torch.device("cuda:0")
N = 40
a = [torch.randn(512, 2048, device=dev, dtype=torch.bfloat16) for _ in range(2)]
b = [torch.randn(2048, 512, device=dev, dtype=torch.bfloat16) for _ in range(2)]
out = [torch.empty(512, 512, device=dev, dtype=torch.bfloat16) for _ in range(2)]


def work(i):
    for _ in range(N):
        torch.matmul(a[i], b[i], out=out[i])


def capture(forked):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    s2 = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        work(0)
        work(1)  # warm-up (cuBLAS handles etc.)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            if forked:
                s2.wait_stream(s)
                work(0)
                with torch.cuda.stream(s2):
                    work(1)
                s.wait_stream(s2)
            else:
                work(0)
                work(1)
    torch.cuda.synchronize()
    return g


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


g1 = capture(False)
g2 = capture(True)
print(f"serial graph: {timeit(g1.replay):.1f} us, forked graph: {timeit(g2.replay):.1f} us, "
      f"eager one stream: {timeit(lambda: (work(0), work(1))):.1f} us", flush=True)
