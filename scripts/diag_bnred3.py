"""Find a random init where fused (E_BNRED) and unfused BN-backward differ after 2 steps,
then print the per-weight relative update difference after ONE step for that init."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
os.environ["DAMD_CONV3_MIN_WG"] = "1"
from tests.test_native_graph_gpu import _data, _train, tf  # noqa: E402
from distributed_amd.models import resnet18  # noqa: E402


def build():
    return resnet18(classes=10, input_shape=(64, 64, 3), widths=(64, 64, 128, 128), blocks=(1, 1, 1, 1))


def rels(init, wa, wb):
    out = []
    for w0, a, b in zip(init, wa, wb):
        da, db = (a - w0).ravel(), (b - w0).ravel()
        out.append(float(np.linalg.norm(da - db) / (np.linalg.norm(db) + 1e-30)))
    return out


x, y = _data(64, (64, 64, 3), 10, seed=9)
tf.keras.backend.clear_session()
m = build()
names = [getattr(w, "name", str(i)) for i, w in enumerate(m.weights)]
for rep in range(12):
    tf.keras.backend.clear_session()
    init = build().get_weights()
    wf, hf, _ = _train(build, x, y, init, 32, 2, native=True, momentum=0.9)
    wu, hu, _ = _train(build, x, y, init, 32, 2, native=True, momentum=0.9, extra_env={"DAMD_BN_DGRAD_FUSE": "0"})
    r = max(rels(init, wf, wu))
    print(f"rep {rep}: 2-step max rel {r:.3e}", flush=True)
    if r < 1e-2:
        continue
    np.savez("gpurun_out/bad_init.npz", *init)
    for steps in (1,):
        wf, hf, _ = _train(build, x, y, init, 32, steps, native=True, momentum=0.0)
        wu, hu, _ = _train(build, x, y, init, 32, steps, native=True, momentum=0.0,
                           extra_env={"DAMD_BN_DGRAD_FUSE": "0"})
        print(f"  {steps} step(s): loss {hf['loss']} vs {hu['loss']}")
        for nm, v in zip(names, rels(init, wf, wu)):
            print(f"    {nm:48s} {v:.3e}")
    break
