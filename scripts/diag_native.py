"""Per-variable comparison of one native-graph training step vs the fp32 generic engine
(diagnostics for tests/test_native_graph_gpu.py)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_amd as tf  # noqa: E402
from tests.test_native_graph_gpu import _data, _small_resnet, _train  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "resnet"
    if which == "resnet":
        build, shape = _small_resnet, (32, 32, 3)
    else:
        from distributed_amd.models import resnet18

        def build():
            return resnet18(classes=10, input_shape=(32, 32, 3), widths=(16, 32, 32, 64), blocks=(1, 1, 1, 1))
    x, y = _data(64, shape, 10)
    tf.keras.backend.clear_session()
    m0 = build()
    init = m0.get_weights()
    names = [w.name for w in m0.weights]
    wn, hn, _ = _train(build, x, y, init, 32, 1, native=True)
    wg, hg, _ = _train(build, x, y, init, 32, 1, native=False)
    wr, hr, _ = _train(build, x, y, init, 32, 1, native=False, device="cpu")
    print("loss native %.6f gpu-generic %.6f cpu %.6f" % (hn["loss"][0], hg["loss"][0], hr["loss"][0]))
    for w0, a, g, b, nm in zip(init, wn, wg, wr, names):
        da, dg, db = (a - w0).ravel(), (g - w0).ravel(), (b - w0).ravel()
        nb = np.linalg.norm(db) + 1e-30

        def st(d):
            return float(d @ db / (np.linalg.norm(d) * nb + 1e-30)), float(np.linalg.norm(d - db) / nb)
        print("%-28s |d|=%.3e native cos %.4f rel %.4f | gpu-generic cos %.4f rel %.4f" % ((nm, nb) + st(da) + st(dg)))


if __name__ == "__main__":
    main()
