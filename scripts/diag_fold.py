"""BN -> ReLU -> conv fold (DAMD_BN_CONV_FOLD) diagnostics: run-to-run and fold-vs-unfold
weight differences per tensor for a few small-ResNet geometries.  GPU box."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["DAMD_CONV3_MIN_WG"] = "1"

import numpy as np  # noqa: E402

import distributed_amd as tf  # noqa: E402
from distributed_amd.models import resnet18  # noqa: E402
from test_native_graph_gpu import _data, _train  # noqa: E402


def diff(tag, wa, wb, names):
    bad = [(nm, int((a != b).sum()), a.size, float(np.abs(a - b).max())) for a, b, nm in zip(wa, wb, names)
           if not np.array_equal(a, b)]
    print(f"{tag}: {len(bad)} tensors differ", bad[:12], flush=True)


for shape, blocks in (((64, 64, 3), (2, 1, 1, 1)), ((128, 128, 3), (1, 1, 1, 1)), ((64, 64, 3), (1, 1, 1, 1))):
    def build():
        return resnet18(classes=10, input_shape=shape, widths=(64, 64, 128, 128), blocks=blocks)

    x, y = _data(64, shape, 10, seed=7)
    tf.keras.backend.clear_session()
    m = build()
    m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tf.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9))
    e = m._get_engine(32, 32)
    print(shape, blocks, "folded:", [nd.layer.name for nd in e.nodes if "bnin" in nd.attrs], flush=True)
    names = [w.name for w in m.weights]
    init = m.get_weights()
    for steps in (1, 2):
        wf, _, _ = _train(build, x, y, init, 32, steps, native=True, momentum=0.9)
        wf2, _, _ = _train(build, x, y, init, 32, steps, native=True, momentum=0.9)
        wu, _, _ = _train(build, x, y, init, 32, steps, native=True, momentum=0.9, extra_env={"DAMD_BN_CONV_FOLD": "0"})
        wu2, _, _ = _train(build, x, y, init, 32, steps, native=True, momentum=0.9, extra_env={"DAMD_BN_CONV_FOLD": "0"})
        diff(f"  {steps} steps fold vs fold", wf, wf2, names)
        diff(f"  {steps} steps unfold vs unfold", wu, wu2, names)
        diff(f"  {steps} steps fold vs unfold", wf, wu, names)
