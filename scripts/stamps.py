"""Phase-stamp diagnostics of the fused ConvNet step (DAMD_STAMPS=1).

Runs warm steps, then one more step, and prints per kernel / per phase the median
(over blocks) time since that kernel's earliest block start, in microseconds
(s_memrealtime ticks at 100 MHz)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DAMD_STAMPS"] = "1"
os.environ.setdefault("DAMD_GRAPH", "1")
os.environ.setdefault("DAMD_GRAPH_STEPS", "10")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import distributed_amd as tf  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    (x, y), _ = tf.keras.datasets.mnist.load_data()
    x = x.reshape(len(x), 28, 28, 1) / 255.0
    m = tf.models.mnist_cnn()
    tf.models.compile_reference(m)
    eng = m._get_engine(B, B)
    eng.bind(x, y)
    eng.start_epoch(0, True, wrap_steps=len(x) // B)
    eng.run(50)
    eng.sync()
    eng.stamps.zero_()
    eng.run(10)  # one captured 10-step graph; the stamps keep the last step's values
    eng.sync()
    st = eng.stamps.cpu().numpy()
    NS = eng.trainer.num_slices
    grids = {"fwd": (0, NS * ((B + 15) // 16)), "bwd": (2, eng.trainer.num_slices_bwd)}
    names = {"fwd": ["start", "loads+sgd", "xs staged", "conv done", "atomics issued", "conv setup", "conv pool",
                     "pooled/code out", "dense-1 mfma", "dense-1 barrier"],
             "bwd": ["start", "loads staged", "head done", "mfma", "convgrad", "end", "h", "softmax", "dh",
                     "logit operands", "logit mfma+max/sum", "lse/argmax", "w0 softmax stored",
                     "w4 body stored"]}
    t0 = None
    for kn, (k, n) in grids.items():
        a = st[k, :n].astype(np.int64)
        base = a[:, 0][a[:, 0] > 0].min()
        t0 = base if t0 is None else t0
        print(f"{kn}: grid {n}, first block start at +{(base - t0) / 100:.2f} us")
        for j, nm in enumerate(names[kn]):
            col = a[:, j]
            col = col[col > 0]
            if len(col) == 0:
                continue
            d = (col - base) / 100.0
            print(f"   {j} {nm:14s} median {statistics.median(d):7.2f}  min {d.min():7.2f}  max {d.max():7.2f} us")


if __name__ == "__main__":
    main()
