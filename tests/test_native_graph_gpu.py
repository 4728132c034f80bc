"""Native graph engine (distributed_amd/engine/native_graph.py): a Keras model lowered to
HIP kernels + HIP graph, checked against the plain-PyTorch fp32 generic engine.

The native path computes activations in bf16 (fp32 accumulation, fp32 master weights),
so the comparison is on the loss and on the weight UPDATES after a step (direction and
magnitude), which is what a bf16 training step must preserve."""
import os

import numpy as np
import pytest
import torch

import distributed_amd as tf
from distributed_amd.models import resnet18

pytestmark = pytest.mark.gpu


def _small_resnet(classes=10):
    return resnet18(classes=classes, input_shape=(32, 32, 3), widths=(16, 32, 32, 64), blocks=(1, 1, 1, 1))


def _mnist():
    return tf.keras.Sequential([
        tf.keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
        tf.keras.layers.MaxPooling2D(),
        tf.keras.layers.Flatten(),
        tf.keras.layers.Dense(64, activation="relu"),
        tf.keras.layers.Dense(10),
    ])


def _train(build, x, y, init, batch, steps, native, lr=0.1, momentum=0.0, graph=True, device=None):
    env = {"DAMD_NATIVE_GRAPH": "1" if native else "0", "DAMD_FUSED": "0", "DAMD_GRAPH": "1" if graph else "0"}
    if device:
        env["DAMD_DEVICE"] = device
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        from distributed_amd.parallel import runtime

        runtime.shutdown()
        tf.keras.backend.clear_session()
        m = build()
        m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tf.keras.optimizers.SGD(learning_rate=lr, momentum=momentum), metrics=["accuracy"])
        m.set_weights(init)
        h = m.fit(x, y, batch_size=batch, epochs=1, steps_per_epoch=steps, shuffle=False, verbose=0)
        eng = m._engine.name
        return m.get_weights(), h.history, eng
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        from distributed_amd.parallel import runtime

        runtime.shutdown()


def _data(n, shape, classes, seed=0):
    rng = np.random.default_rng(seed)
    x = (rng.integers(0, 256, size=(n,) + shape) / 255.0).astype(np.float32)
    y = rng.integers(0, classes, size=n).astype(np.int64)
    return x, y


def _compare_updates(init, wa, wb, names, cos_min=0.98, rel_max=0.08):
    for w0, a, b, nm in zip(init, wa, wb, names):
        da, db = (a - w0).ravel().astype(np.float64), (b - w0).ravel().astype(np.float64)
        nb = np.linalg.norm(db)
        if nb < 1e-7:
            assert np.linalg.norm(da) < 1e-5, nm
            continue
        cos = float(da @ db / (np.linalg.norm(da) * nb + 1e-30))
        rel = float(np.linalg.norm(da - db) / nb)
        assert cos > cos_min and rel < rel_max, f"{nm}: cos {cos:.4f} rel {rel:.4f}"


def test_small_resnet_one_step_matches_fp32_reference():
    tf.keras.backend.clear_session()
    x, y = _data(64, (32, 32, 3), 10)
    m0 = _small_resnet()
    init = m0.get_weights()
    names = [w.name for w in m0.weights]
    wn, hn, en = _train(_small_resnet, x, y, init, 32, 1, native=True)
    wr, hr, er = _train(_small_resnet, x, y, init, 32, 1, native=False, device="cpu")
    assert en == "native_graph" and er == "generic"
    assert abs(hn["loss"][0] - hr["loss"][0]) < 2e-2 * abs(hr["loss"][0])
    _compare_updates(init, wn, wr, names)


def test_mnist_native_graph_tracks_reference_over_steps():
    x, y = _data(640, (28, 28, 1), 10, seed=1)
    tf.keras.backend.clear_session()
    init = _mnist().get_weights()
    wn, hn, en = _train(_mnist, x, y, init, 64, 10, native=True, lr=0.05, momentum=0.9)
    wr, hr, er = _train(_mnist, x, y, init, 64, 10, native=False, device="cpu", lr=0.05, momentum=0.9)
    assert en == "native_graph"
    np.testing.assert_allclose(hn["loss"], hr["loss"], rtol=1e-2)
    _compare_updates(init, wn, wr, ["k", "b", "k1", "b1", "k2", "b2"], cos_min=0.99, rel_max=0.05)


def test_graph_replay_equals_eager():
    x, y = _data(128, (32, 32, 3), 10, seed=2)
    tf.keras.backend.clear_session()
    init = _small_resnet().get_weights()
    wg, hg, _ = _train(_small_resnet, x, y, init, 32, 4, native=True, momentum=0.9, graph=True)
    we, he, _ = _train(_small_resnet, x, y, init, 32, 4, native=True, momentum=0.9, graph=False)
    for a, b in zip(wg, we):
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-4)
    np.testing.assert_allclose(hg["loss"], he["loss"], rtol=1e-4)


def test_resnet18_full_size_trains():
    x, y = _data(64, (224, 224, 3), 1000, seed=3)
    tf.keras.backend.clear_session()
    os.environ["DAMD_FUSED"] = "0"
    try:
        m = resnet18()
        m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tf.keras.optimizers.SGD(learning_rate=0.1, momentum=0.9), metrics=["accuracy"])
        h = m.fit(x, y, batch_size=32, epochs=3, steps_per_epoch=2, verbose=0)
    finally:
        os.environ.pop("DAMD_FUSED", None)
    assert m._engine.name == "native_graph"
    assert all(np.isfinite(h.history["loss"]))
    assert h.history["loss"][-1] < h.history["loss"][0]
