"""Graph replay vs eager for the native graph engine: run step 1 eagerly, step 2 either
eagerly or by replaying a captured graph, and report the first buffers that differ."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_amd as tf  # noqa: E402
from tests.test_native_graph_gpu import _data, _small_resnet  # noqa: E402

os.environ["DAMD_FUSED"] = "0"
x, y = _data(128, (32, 32, 3), 10, seed=2)


def make():
    tf.keras.backend.clear_session()
    tf.set_seed(5)
    m = _small_resnet()
    m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tf.keras.optimizers.SGD(learning_rate=0.1, momentum=0.9), metrics=["accuracy"])
    e = m._get_engine(32, 32)
    e.bind(x, y)
    e.start_epoch(0, False)
    return m, e


def snap(e):
    torch.cuda.synchronize()
    d = {"P": e.P.clone(), "G": e.G.clone(), "V": e.V.clone(), "ctrl": e.ctrl.clone(), "x0": e.x0.buf.clone(),
         "labels": e.labels.clone(), "logits": e.logits.clone(), "dlogits": e.dlogits.clone()}
    for i, nd in enumerate(e.nodes):
        r = nd.out.root()
        if r.buf is not None:
            d[f"{i}:{nd.layer.name}:out"] = r.buf.clone()
        if r.grad is not None:
            d[f"{i}:{nd.layer.name}:grad"] = r.grad.clone()
        for k, v in nd.attrs.items():
            if torch.is_tensor(v):
                d[f"{i}:{nd.layer.name}:{k}"] = v.clone()
    return d


m1, e1 = make()
e1._step_body()
e1._step_body()
a = snap(e1)
m2, e2 = make()
e2._step_body()
e2._capture_safe()
e2.graph.replay()
b = snap(e2)
init_diff = (m1.get_weights()[0] - m2.get_weights()[0])
print("keys", len(a))
for k in a:
    va, vb = a[k].float(), b[k].float()
    dmax = (va - vb).abs().max().item() if va.numel() else 0.0
    scale = va.abs().max().item() if va.numel() else 0.0
    flag = "  <-- DIFF" if dmax > 1e-3 * max(scale, 1e-6) else ""
    print(f"{k:50s} max|a-b| {dmax:.3e}  max|a| {scale:.3e}{flag}")
