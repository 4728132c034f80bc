"""Cost of a captured step graph's FIRST replay vs later replays (MNIST fused step), and of
the final graph (k steps + flush) replayed cold, after a disabled-node warm replay
(StepExecutor::warm_final), and warm.  usage: python scripts/probe_cold_graph.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import distributed_amd as tf  # noqa: E402


def timed(f):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6


def main():
    rng = np.random.default_rng(0)
    x = (rng.integers(0, 256, size=(60000, 28, 28, 1)) / 255.0).astype(np.float32)
    y = rng.integers(0, 10, 60000)
    os.environ["DAMD_GRAPH_STEPS"] = "5"
    m = tf.models.mnist_cnn()
    tf.models.compile_reference(m, 0.001)
    eng = m._get_engine(64, 64)
    eng.bind(x, y)
    eng.start_epoch(0, True, wrap_steps=len(x) // 64)
    tr = eng.trainer
    tr.capture(5)
    for rep in range(3):
        print(f"rep {rep}: 4 x 5-step graph: {timed(lambda: tr.run(20)):.1f} us", flush=True)
    for k, warm in ((20, False), (19, True), (18, True)):
        tr.capture_final(k)
        if warm:
            print(f"  warm_final({k}): {tr.warm_final(k)}", flush=True)
        for rep in range(3):
            print(f"final {k}-step graph (warm replay first: {warm}) replay {rep}: "
                  f"{timed(lambda: tr.run_final(k)):.1f} us", flush=True)
    eng.finish()


if __name__ == "__main__":
    main()
