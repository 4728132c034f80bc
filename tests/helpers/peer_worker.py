"""Worker for the xGMI peer all-reduce tests: N ranks (processes) that may share one GPU.
Checks the native kernel against an fp32 host reduction in the kernel's fixed peer order
(bitwise), eager and replayed from a captured HIP graph.  Writes rank<r>.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import distributed_amd as tf  # noqa: E402
from distributed_amd.parallel import runtime  # noqa: E402
from distributed_amd.parallel.communicator import make_peer_allreduce  # noqa: E402


def main():
    out = os.environ["DAMD_TEST_OUT"]
    strategy = tf.distribute.experimental.MultiWorkerMirroredStrategy()
    comm = strategy.communicator
    W, r = comm.world_size, comm.rank
    dev = strategy.device
    cap = 347152 + 2 * 320
    pa = make_peer_allreduce(comm, dev.index or 0, cap, blocks=int(os.environ.get("DAMD_PEER_BLOCKS", "64")),
                             timeout_s=30.0)
    res = {"ok": pa is not None, "rank": r, "world": W, "errors": []}
    if pa is not None:
        g = torch.Generator().manual_seed(1000 + r)
        s = torch.cuda.current_stream(dev)
        for n in (4, 1000, 4096 * 3 + 4, cap):
            for rep in range(2):
                x = torch.randn(n, generator=g) * (1 + rep)
                xs = comm.allgather_object(x)  # host copies of every rank's input
                want = xs[0].clone()
                for p in range(1, W):
                    want += xs[p]
                d = x.to(dev)
                pa.allreduce(d.data_ptr(), n, s.cuda_stream)
                torch.cuda.synchronize(dev)
                if not torch.equal(d.cpu(), want):
                    res["errors"].append(f"eager n={n} rep={rep} maxdiff={(d.cpu() - want).abs().max().item()}")
        # fp32 values + an int64 segment (the 2-launch step's fixed-point conv gradient):
        # the integers are summed exactly, including carries across the 32-bit halves
        for n, n64 in ((1000, 320), (347152, 320), (6, 3)):
            x = torch.randn(n, generator=g)
            q = torch.randint(-(2 ** 60), 2 ** 60, (n64,), generator=g, dtype=torch.int64)
            xs, qs = comm.allgather_object(x), comm.allgather_object(q)
            want_x = xs[0].clone()
            for p in range(1, W):
                want_x += xs[p]
            want_q = sum(qs[1:], qs[0].clone())
            dx, dq = x.to(dev), q.to(dev)
            pa.allreduce(dx.data_ptr(), n, s.cuda_stream, dq.data_ptr(), n64)
            torch.cuda.synchronize(dev)
            if not (torch.equal(dx.cpu(), want_x) and torch.equal(dq.cpu(), want_q)):
                res["errors"].append(f"int64 segment n={n} n64={n64}")
        # captured: 3 all-reduces per graph, replayed twice
        n = cap
        buf = torch.zeros(n, device=dev)
        graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            with torch.cuda.graph(graph, stream=side):
                for _ in range(3):
                    pa.allreduce(buf.data_ptr(), n, side.cuda_stream)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        for rep in range(2):
            x = torch.randint(-8, 8, (n,), generator=g).float()
            xs = comm.allgather_object(x)
            want = sum(xs[1:], xs[0].clone()) * float(W) ** 2  # small integers: exact
            buf.copy_(x.to(dev))
            torch.cuda.synchronize(dev)
            graph.replay()
            torch.cuda.synchronize(dev)
            if not torch.equal(buf.cpu(), want):
                res["errors"].append(f"graph rep={rep}")
        # latency of one replayed all-reduce of the MNIST gradient (ranks sharing one GPU:
        # a protocol-latency probe, not an xGMI bandwidth number)
        import time

        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            with torch.cuda.graph(g2, stream=side):
                for _ in range(50):
                    pa.allreduce(buf.data_ptr(), n, side.cuda_stream)
        torch.cuda.synchronize(dev)
        comm.barrier()
        g2.replay()
        torch.cuda.synchronize(dev)
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(4):
            g2.replay()
        torch.cuda.synchronize(dev)
        res["us_per_allreduce"] = (time.perf_counter() - t0) / 200 * 1e6
        res["status"] = int(pa.status())
        digest = float(buf.double().sum().item())
        res["digest"] = digest
    with open(os.path.join(out, f"rank{r}.json"), "w") as f:
        json.dump(res, f)
    runtime.shutdown()


if __name__ == "__main__":
    main()
