"""Where the fixed cost of a short timed MNIST run goes (bench.py --steps 20 --warmup 5):
host time to enqueue the graph replays + flush, then the wait in torch.cuda.synchronize,
for several graph lengths, with and without the flush, optionally with the HIP device in
spin-wait scheduling (PROBE_SPIN=1: hipSetDeviceFlags(hipDeviceScheduleSpin) before the
first HIP call).  usage: [PROBE_SPIN=1] python scripts/probe_overhead.py"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if os.environ.get("PROBE_SPIN") == "1":
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin):", hip.hipSetDeviceFlags(ctypes.c_uint(1)), flush=True)

import numpy as np
import torch

import distributed_amd as tf


def main():
    rng = np.random.default_rng(0)
    x = rng.random((60000, 28, 28, 1), dtype=np.float32)
    y = rng.integers(0, 10, 60000)
    for gs in (5, 10, 20):
        os.environ["DAMD_GRAPH_STEPS"] = str(gs)
        m = tf.models.mnist_cnn()
        tf.models.compile_reference(m, 0.001)
        eng = m._get_engine(64, 64)
        eng.bind(x, y)
        eng.start_epoch(0, True, wrap_steps=len(x) // 64)
        eng.prepare(20)
        eng.run(5)
        eng.sync()
        for flush in (True, False):
            for k in (20, 2000):
                rows = []
                for _ in range(5):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    eng.run(k)
                    if flush:
                        eng._flush()
                    t1 = time.perf_counter()
                    torch.cuda.synchronize()
                    t2 = time.perf_counter()
                    rows.append(((t1 - t0) * 1e6, (t2 - t0) * 1e6))
                    eng._flush()
                    eng.sync()
                best = min(rows, key=lambda r: r[1])
                med = sorted(r[1] for r in rows)[len(rows) // 2]
                print(f"graph {gs:3d} flush {int(flush)} k {k:5d}: enqueue {best[0]:8.1f} us, total best {best[1]:9.1f} "
                      f"med {med:9.1f} us = {best[1] / k:6.2f} us/step (best), {med / k:6.2f} (median)", flush=True)
        eng.finish()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        torch.cuda.synchronize()
    print(f"empty synchronize: {(time.perf_counter() - t0) * 1e4:.1f} us", flush=True)
    s = torch.cuda.Stream()
    a = torch.zeros(16, device="cuda")
    ts = []
    for _ in range(50):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            a.add_(1)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    print(f"one tiny kernel launch + synchronize: min {min(ts):.1f} med {sorted(ts)[25]:.1f} us", flush=True)


if __name__ == "__main__":
    main()
