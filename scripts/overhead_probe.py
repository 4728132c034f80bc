"""Fixed cost of a timed MNIST window: wall time of one final graph (K steps + the flush)
between device synchronizes, for several K, median of 7; the fit t = a + b K separates the
per-window overhead a (launch, first-kernel start, sync wake-up, flush) from the per-step
time b.  GPU box:  python scripts/overhead_probe.py"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import distributed_amd as tf  # noqa: E402


def main():
    B = 64
    (x, y), _ = tf.keras.datasets.mnist.load_data()
    x = x.reshape(len(x), 28, 28, 1) / 255.0
    m = tf.models.mnist_cnn()
    tf.models.compile_reference(m, 0.001)
    eng = m._get_engine(B, B)
    eng.bind(x, y)
    eng.start_epoch(0, True, wrap_steps=len(x) // B)
    eng.prepare(200)
    eng.run(200)
    eng.sync()
    # bare sync round trip
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(f"bare synchronize: {statistics.median(ts) * 1e6:.1f} us")
    ks, ms = [], []
    for K in (1, 2, 5, 10, 20, 50, 100, 200):
        ok = eng.prepare_final(K)
        eng.run(20)
        torch.cuda.synchronize()
        ts, tl = [], []
        for _ in range(7):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run_and_flush(K)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            tl.append(t1 - t0)
            eng.run(3)  # a pending update again, as before a real window
        t = statistics.median(ts)
        ks.append(K)
        ms.append(t * 1e6)
        print(f"K={K:4d} final_graph={ok}  window {t * 1e6:8.1f} us  = {t * 1e6 / K:6.2f} us/step"
              f"  (first window {ts[0] * 1e6:8.1f} us; host launch call {statistics.median(tl) * 1e6:7.1f} us)",
              flush=True)
    b, a = np.polyfit(ks, ms, 1)
    print(f"fit: window = {a:.1f} us + {b:.2f} us x K")


if __name__ == "__main__":
    main()
