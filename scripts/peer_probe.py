"""Intrinsic cost of the xGMI peer all-reduce protocol, measured on ONE GPU: W "ranks"
live in this process (link_local, no IPC), each on its own HIP stream, all captured in
one graph with fork/join, so the W kernels run truly concurrently.  Peers' buffers are
local HBM here, so this is a lower bound for the xGMI version (remote loads/stores add
link latency).  usage: python scripts/peer_probe.py [W] [blocks] [floats]"""
import sys
import time

import os
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_amd.native as nat

C = nat.require_C()
W = int(sys.argv[1]) if len(sys.argv) > 1 else 4
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 64
N = int(sys.argv[3]) if len(sys.argv) > 3 else 347152
dev = torch.device("cuda:0")
pas = [C.PeerAllreduce(W, r, 0, N, NB, 1.0) for r in range(W)]
for p in pas:
    p.link_local(pas)
xs = [torch.randn(N, device=dev) for _ in range(W)]
want = sum(x.clone() for x in xs)
streams = [torch.cuda.Stream(dev) for _ in range(W)]
main = torch.cuda.current_stream(dev)


# one single-stream graph of REPS all-reduces per rank, the W graphs launched on W streams
# (HIP runs a graph's nodes in order on its launch stream; concurrency comes from the
# streams' hardware queues -- at most 4 here, so W <= 4)
REPS = 100
for r in range(W):
    pas[r].allreduce(xs[r].data_ptr(), N, streams[r].cuda_stream)
torch.cuda.synchronize()
ok = all(torch.allclose(x, want, rtol=1e-5, atol=1e-5) for x in xs)
graphs = []
for r in range(W):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(streams[r]):
        with torch.cuda.graph(g, stream=streams[r]):
            for _ in range(REPS):
                pas[r].allreduce(xs[r].data_ptr(), N, streams[r].cuda_stream)
    graphs.append(g)
torch.cuda.synchronize()


def run():
    for r in range(W):
        with torch.cuda.stream(streams[r]):
            graphs[r].replay()
    torch.cuda.synchronize()


run()
t = time.perf_counter()
for _ in range(3):
    run()
us = (time.perf_counter() - t) / (3 * REPS) * 1e6
print(f'{{"peer_probe": {{"world": {W}, "blocks": {NB}, "floats": {N}, "us_per_allreduce": {us:.2f}, '
      f'"correct": {str(ok).lower()}, "status": {max(p.status() for p in pas)}}}}}', flush=True)
