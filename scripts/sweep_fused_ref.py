"""Seed sweep for tests/test_fused_convnet_gpu.py::test_one_step_matches_reference: one SGD
step of the fused MNIST engine per unpinned initial draw, relative error of the implied
gradient per tensor vs the bf16-mirrored reference and vs plain fp64.  GPU box:
    python scripts/sweep_fused_ref.py [draws per shape]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["DAMD_GRAPH"] = "0"
from test_fused_convnet_gpu import _data, _engine, _model, _ref_step  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
names = ["wc", "bc", "w1", "b1", "w2", "b2"]
worst_q = {k: 0.0 for k in names}
worst_64 = {k: 0.0 for k in names}
colfrac = {k: 1.0 for k in names}  # min over draws: fraction of output columns within 1e-2 (mirrored)
for B, pp in [(64, 3), (40, 3), (100, 3), (64, 4), (100, 2), (64, 1)]:
    os.environ["DAMD_PP"] = str(pp)
    for d in range(n):
        lr = 0.5
        m = _model(lr=lr, seed=None)
        x, y = _data(300)
        w0 = m.get_weights()
        eng = _engine(m, B)
        eng.bind(x, y)
        eng.start_epoch(0, shuffle=False)
        eng.run(1)
        eng.end_epoch()
        eng.finish()
        w1 = m.get_weights()
        for quant, worst in ((True, worst_q), (False, worst_64)):
            g, _, _ = _ref_step(w0, x[:B], y[:B], B, quant=quant)
            for a, b, gg, k in zip(w0, w1, g, names):
                est = (a - b) / lr
                e = float(np.linalg.norm(est - gg) / (np.linalg.norm(gg) + 1e-12))
                worst[k] = max(worst[k], e)
                if quant:
                    E, G = est.reshape(-1, est.shape[-1]), gg.reshape(-1, gg.shape[-1])
                    ce = np.linalg.norm(E - G, axis=0) / (np.linalg.norm(G, axis=0) + 1e-12)
                    colfrac[k] = min(colfrac[k], float((ce < 1e-2).mean()))
    print(f"B {B} pp {pp}: worst so far vs bf16-mirrored {max(worst_q.values()):.2e}, vs fp64 "
          f"{ {k: round(v, 4) for k, v in worst_64.items()} }", flush=True)
print("vs bf16-mirrored:", {k: f"{v:.2e}" for k, v in worst_q.items()})
print("vs fp64:", {k: f"{v:.3f}" for k, v in worst_64.items()})
print("min fraction of columns within 1e-2 (mirrored):", {k: f"{v:.3f}" for k, v in colfrac.items()})
