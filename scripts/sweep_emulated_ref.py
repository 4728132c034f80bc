"""Seed sweep for tests/test_native_graph_gpu.py::test_small_resnet_step_matches_bf16_emulated_reference:
one plain-SGD step of the small ResNet on the native engine vs the fp32 re-execution with the
plan's bf16 storage points, per init: loss error, worst / median per-layer relative update
error, worst per-layer cosine, head error, whole-vector cos / rel.  GPU box:
    python scripts/sweep_emulated_ref.py [n_inits]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["DAMD_FUSED"] = "0"
import distributed_amd as tf  # noqa: E402
from test_native_graph_gpu import _data, _emulated_reference_grads, _small_resnet  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
x, y = _data(32, (32, 32, 3), 10, seed=4)
lr = 0.1
rows = []
for rep in range(n):
    tf.keras.backend.clear_session()
    m = _small_resnet()
    m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tf.keras.optimizers.SGD(learning_rate=lr), metrics=["accuracy"])
    e = m._get_engine(32, 32)
    e.bind(x, y)
    e.start_epoch(0, False)
    w0 = {id(v): v.value.detach().clone() for v in m.trainable_weights}
    grads, ref_loss = _emulated_reference_grads(e, m, x, y, 32)
    e.run(1)
    e.sync()
    loss = e.metrics()["loss"]
    rels, coss, dn, dr = [], [], [], []
    for v in m.trainable_weights:
        a = (v.value.detach() - w0[id(v)]).double().ravel()
        b = (-lr * grads[id(v)]).double().ravel()
        nb = b.norm().item()
        rels.append((a - b).norm().item() / max(nb, 1e-12))
        coss.append(float(a @ b / max(a.norm().item() * nb, 1e-30)))
        dn.append(a)
        dr.append(b)
    A, Bv = torch.cat(dn), torch.cat(dr)
    wc = float(A @ Bv / (A.norm() * Bv.norm()))
    wr = float((A - Bv).norm() / Bv.norm())
    worst = int(np.argmax(rels))
    rows.append((abs(loss - ref_loss) / abs(ref_loss), max(rels), sorted(rels)[len(rels) // 2], min(coss),
                 rels[-2], wc, wr))
    print(f"init {rep:2d}: loss err {rows[-1][0]:.2e}  worst layer rel {max(rels):.4f} "
          f"({m.trainable_weights[worst].name})  median {rows[-1][2]:.4f}  min cos {min(coss):.4f}  "
          f"head {rels[-2]:.2e}  whole cos {wc:.5f} rel {wr:.4f}", flush=True)
r = np.array(rows)
print("max over inits: loss err %.2e  worst rel %.4f  median %.4f  head %.2e  whole rel %.4f" %
      (r[:, 0].max(), r[:, 1].max(), r[:, 2].max(), r[:, 4].max(), r[:, 6].max()))
print("min over inits: min cos %.4f  whole cos %.5f" % (r[:, 3].min(), r[:, 5].min()))
