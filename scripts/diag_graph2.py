import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_amd as tf  # noqa: E402
from tests.test_native_graph_gpu import _data, _small_resnet, _train  # noqa: E402

x, y = _data(128, (32, 32, 3), 10, seed=2)
tf.keras.backend.clear_session()
m0 = _small_resnet()
init = m0.get_weights()
names = [w.name for w in m0.weights]
for steps in (1, 2, 4):
    wg, hg, _ = _train(_small_resnet, x, y, init, 32, steps, native=True, momentum=0.9, graph=True)
    we, he, _ = _train(_small_resnet, x, y, init, 32, steps, native=True, momentum=0.9, graph=False)
    we2, he2, _ = _train(_small_resnet, x, y, init, 32, steps, native=True, momentum=0.9, graph=False)
    print("steps", steps, "loss graph", hg["loss"], "eager", he["loss"], "eager2", he2["loss"])
    for a, b, c, nm in list(zip(wg, we, we2, names))[:6]:
        print(f"  {nm:30s} graph-eager {np.abs(a - b).max():.3e} eager-eager {np.abs(b - c).max():.3e}")
