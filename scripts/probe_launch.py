"""Fixed per-call overhead of the fused MNIST step on one GPU: wall time of run(k) for
several k, graph lengths and eager launches (each timed like bench.py: sync, run, flush,
sync).  usage: python scripts/probe_launch.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

import distributed_amd as tf


def main():
    rng = np.random.default_rng(0)
    x = rng.random((60000, 28, 28, 1), dtype=np.float32)
    y = rng.integers(0, 10, 60000)
    for gs in (20, 10, 5):
        os.environ["DAMD_GRAPH_STEPS"] = str(gs)
        m = tf.models.mnist_cnn()
        tf.models.compile_reference(m, 0.001)
        eng = m._get_engine(64, 64)
        eng.bind(x, y)
        eng.start_epoch(0, True, wrap_steps=len(x) // 64)
        eng.run(50)
        eng.prepare(2000)
        eng.sync()
        for k in (20, 40, 200, 2000):
            ts = []
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                eng.run(k)
                eng._flush()
                eng.sync()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            print(f"graph_steps {gs:3d} k {k:5d}: " + " ".join(f"{t * 1e6 / k:7.2f}" for t in ts) + " us/step"
                  f"  (first call total {ts[0] * 1e6:.0f} us)", flush=True)
        # eager launches of the same steps
        eng.use_graph = False
        for k in (20, 200):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(k)
            eng._flush()
            eng.sync()
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            print(f"eager k {k}: {t * 1e6 / k:.2f} us/step", flush=True)
        eng.use_graph = True
        eng.finish()
    # bare costs
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        torch.cuda.synchronize()
    print(f"empty synchronize: {(time.perf_counter() - t0) * 1e4:.1f} us")


if __name__ == "__main__":
    main()
