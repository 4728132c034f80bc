"""Distribution of the bf16-vs-fp32 update agreement over many initial draws, for the
tolerance tests whose bounds must hold for ANY init (tests/test_native_layers_gpu.py
test_native_optimizers_track_reference): per optimizer and weight tensor, the min cosine
and max relative error of the native graph engine's 10-step weight update against the
fp32 generic engine over SEEDS draws.  GPU box:
    python scripts/sweep_tolerances.py [seeds] [opt names...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import distributed_amd as tf  # noqa: E402
from test_native_graph_gpu import _data, _mnist, _small_resnet, _train  # noqa: E402
from test_native_layers_gpu import _opt_cases  # noqa: E402


def stats(init, wa, wb):
    out = []
    for w0, a, b in zip(init, wa, wb):
        da, db = (a - w0).ravel().astype(np.float64), (b - w0).ravel().astype(np.float64)
        nb = np.linalg.norm(db)
        cos = float(da @ db / (np.linalg.norm(da) * nb + 1e-30))
        out.append((cos, float(np.linalg.norm(da - db) / max(nb, 1e-30))))
    return out


def main():
    seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    names = sys.argv[2:] or list(_opt_cases())
    names_w = ["k", "b", "k1", "b1", "k2", "b2"]
    x, y = _data(640, (28, 28, 1), 10, seed=3)
    # "track": test_native_graph_gpu.py test_mnist_native_graph_tracks_reference_over_steps
    # (SGD lr 0.05 momentum 0.9 on its seed-1 data)
    cases = dict(_opt_cases(eps=1e-2), track=lambda: tf.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9))
    xt, yt = _data(640, (28, 28, 1), 10, seed=1)
    if names == ["resnet_fp32"]:
        return sweep_resnet_fp32(seeds)
    for name in names:
        rows = []
        for s in range(seeds):
            tf.set_seed(1000 + s)
            tf.keras.backend.clear_session()
            init = _mnist().get_weights()
            opt = cases[name]
            xs, ys = (xt, yt) if name == "track" else (x, y)
            wn, hn, en, _ = _train(_mnist, xs, ys, init, 64, 10, native=True, optimizer=opt)
            wr, hr, er, _ = _train(_mnist, xs, ys, init, 64, 10, native=False, device="cpu", optimizer=opt)
            rows.append(stats(init, wn, wr))
        a = np.array(rows)  # [seed][tensor][cos, rel]
        print(f"{name}: " + "  ".join(f"{nm} cos min {a[:, i, 0].min():.4f} med {np.median(a[:, i, 0]):.4f} "
                                      f"rel max {a[:, i, 1].max():.3f}" for i, nm in enumerate(names_w)), flush=True)


def sweep_resnet_fp32(seeds):
    """test_native_graph_gpu.py test_small_resnet_one_step_matches_fp32_reference: one SGD
    step of the small ResNet, native graph engine (bf16 storage) vs the fp32 generic engine,
    per tensor min cosine / max relative error and the whole-update-vector numbers."""
    x, y = _data(64, (32, 32, 3), 10)
    rows, whole = [], []
    for s in range(seeds):
        tf.set_seed(2000 + s)
        tf.keras.backend.clear_session()
        m0 = _small_resnet()
        init = m0.get_weights()
        names_w = [w.name for w in m0.weights]
        wn, _, _ = _train(_small_resnet, x, y, init, 32, 1, native=True)
        wr, _, _ = _train(_small_resnet, x, y, init, 32, 1, native=False, device="cpu")
        rows.append(stats(init, wn, wr))
        da = np.concatenate([(a - w0).ravel() for w0, a in zip(init, wn)]).astype(np.float64)
        db = np.concatenate([(b - w0).ravel() for w0, b in zip(init, wr)]).astype(np.float64)
        whole.append((float(da @ db / (np.linalg.norm(da) * np.linalg.norm(db))),
                      float(np.linalg.norm(da - db) / np.linalg.norm(db))))
        print(f"draw {s}: worst cos {min(c for c, _ in rows[-1]):.4f} worst rel {max(r for _, r in rows[-1]):.3f} "
              f"whole cos {whole[-1][0]:.4f} rel {whole[-1][1]:.3f}", flush=True)
    a = np.array(rows)
    for i, nm in enumerate(names_w):
        if np.isfinite(a[:, i, 0]).all():
            print(f"{nm}: cos min {a[:, i, 0].min():.4f} rel max {a[:, i, 1].max():.3f}")
    w = np.array(whole)
    print(f"whole: cos min {w[:, 0].min():.4f} rel max {w[:, 1].max():.3f}")


if __name__ == "__main__":
    main()
