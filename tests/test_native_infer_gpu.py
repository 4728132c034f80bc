"""predict / evaluate through the native forward plan (engine/native_infer.py) against the
PyTorch-ops inference path on the same weights (DAMD_NATIVE_INFER=0)."""
import os

import numpy as np
import pytest
import torch

import distributed_amd as tf
from distributed_amd.engine.native_infer import NativeInference

from test_native_graph_gpu import _data, _mnist, _small_resnet

pytestmark = pytest.mark.gpu


class _Env:
    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kw}
        os.environ.update(self.kw)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _trained(build, x, y, steps=3, batch=32):
    from distributed_amd.parallel import runtime

    runtime.shutdown()
    tf.keras.backend.clear_session()
    m = build()
    m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tf.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9), metrics=["accuracy"])
    m.fit(x, y, batch_size=batch, epochs=1, steps_per_epoch=steps, verbose=0)
    return m


def _both(fn):
    with _Env(DAMD_NATIVE_INFER="0"):
        ref = fn()
    with _Env(DAMD_NATIVE_INFER="1", DAMD_STRICT_NATIVE="1"):
        nat = fn()
    return nat, ref


def test_resnet_predict_uses_moving_statistics():
    x, y = _data(200, (32, 32, 3), 10, seed=2)
    m = _trained(_small_resnet, x, y)
    # the BN moving statistics moved away from their init (0 / 1): inference must use them
    mm = [w for w in m.non_trainable_weights if "moving_mean" in w.name][0]
    assert float(mm.value.abs().sum()) > 0
    nat, ref = _both(lambda: m.predict(x[:77], batch_size=32))  # a short final batch
    assert nat.shape == ref.shape == (77, 10)
    assert any(isinstance(p, NativeInference) for p in m._infer_plans.values())
    err = np.abs(nat - ref).max() / (np.abs(ref).max() + 1e-9)
    assert err < 3e-2, err
    assert (nat.argmax(1) == ref.argmax(1)).mean() > 0.9


def test_mnist_evaluate_matches_reference_path():
    x, y = _data(1000, (28, 28, 1), 10, seed=3)
    m = _trained(_mnist, x, y, steps=10, batch=64)
    nat, ref = _both(lambda: m.evaluate(x, y, batch_size=128, verbose=0, return_dict=True))
    assert abs(nat["loss"] - ref["loss"]) < 1e-2 * ref["loss"]
    assert abs(nat["accuracy"] - ref["accuracy"]) <= 5 / 1000
    # a second call reuses the captured graph and gives the same numbers
    with _Env(DAMD_NATIVE_INFER="1"):
        again = m.evaluate(x, y, batch_size=128, verbose=0, return_dict=True)
    assert again["accuracy"] == nat["accuracy"]
    assert abs(again["loss"] - nat["loss"]) < 1e-5 * nat["loss"]  # per-row loss atomics: order varies


def test_uint8_inputs_are_raw_values_and_dropout_is_identity():
    L = tf.keras.layers
    x, y = _data(128, (28, 28, 1), 10, seed=4)
    xu = (x * 255).round().astype(np.uint8)

    def build():
        return tf.keras.Sequential([
            L.Conv2D(16, 3, activation="relu", input_shape=(28, 28, 1)),
            L.AveragePooling2D(),
            L.Dropout(0.5),
            L.Flatten(),
            L.Dense(32, activation="tanh"),
            L.Dense(10),
        ])

    m = _trained(build, x, y, steps=2)
    with _Env(DAMD_NATIVE_INFER="1", DAMD_STRICT_NATIVE="1"):
        a = m.predict(xu.astype(np.float32), batch_size=64)
        b = m.predict(xu, batch_size=64)
        c = m.predict(xu, batch_size=64)
    np.testing.assert_array_equal(a, b)  # uint8 rows are fed as their raw values
    np.testing.assert_array_equal(b, c)  # no dropout at inference
    # (raw 0..255 inputs drive this [0, 1]-trained net far out of range; the bf16 vs fp32
    # comparison is done on the training scale)
    with _Env(DAMD_NATIVE_INFER="1", DAMD_STRICT_NATIVE="1"):
        a = m.predict(x, batch_size=64)
    with _Env(DAMD_NATIVE_INFER="0"):
        r = m.predict(x, batch_size=64)
    assert np.abs(a - r).max() / (np.abs(r).max() + 1e-9) < 3e-2


def test_validation_split_runs_native_inference():
    x, y = _data(640, (28, 28, 1), 10, seed=5)
    tf.keras.backend.clear_session()
    m = _mnist()
    m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tf.keras.optimizers.Adam(1e-3), metrics=["accuracy"])
    with _Env(DAMD_STRICT_NATIVE="1"):
        h = m.fit(x, y, batch_size=64, epochs=2, validation_split=0.2, verbose=0)
    assert len(h.history["val_loss"]) == 2 and np.isfinite(h.history["val_loss"]).all()
    assert any(isinstance(p, NativeInference) for p in m._infer_plans.values())


def test_frozen_layer_predict_and_fit():
    """A layer frozen with ``trainable = False``: its kernel / bias leave
    ``trainable_weights``, but the inference plan still reads them, and training
    falls back to the generic path (the native training plan holds trainable weights only)."""
    x, y = _data(256, (32, 32, 3), 10, seed=6)
    m = _trained(_small_resnet, x, y, steps=2)
    conv = [l for l in m.layers if type(l).__name__ == "Conv2D"][1]
    dense = [l for l in m.layers if type(l).__name__ == "Dense"][-1]
    conv.trainable = False
    dense.trainable = False
    assert conv.kernel not in m.trainable_weights
    nat, ref = _both(lambda: m.predict(x[:64], batch_size=32))
    assert any(isinstance(p, NativeInference) for p in m._infer_plans.values())
    assert np.abs(nat - ref).max() / (np.abs(ref).max() + 1e-9) < 3e-2
    k0 = conv.kernel.numpy().copy()
    m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tf.keras.optimizers.SGD(learning_rate=0.05), metrics=["accuracy"])
    m.fit(x, y, batch_size=32, epochs=1, steps_per_epoch=2, verbose=0)
    assert m._engine.name == "generic"
    np.testing.assert_array_equal(conv.kernel.numpy(), k0)  # frozen: unchanged
