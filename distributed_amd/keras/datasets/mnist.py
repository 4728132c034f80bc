"""MNIST loader (``tf.keras.datasets.mnist.load_data``, reference README.md:286-287).

There is no network here: if an ``mnist.npz`` exists (``path``,
``$DAMD_MNIST_PATH`` or ``~/.keras/datasets/mnist.npz``) it is read with
``numpy.load(allow_pickle=False)``; otherwise a deterministic **synthetic** MNIST of the
same shapes and dtypes is generated (uint8 28x28 images, uint8 labels 0-9; 60000 train
/ 10000 test).  Synthetic images are noise plus a class-dependent stroke template, so
the task is learnable and "loss goes down" is observable in tests.
"""
from __future__ import annotations

import os

import numpy as np

TRAIN_N, TEST_N = 60000, 10000
_CACHE = {}


def _find(path):
    cands = [path, os.environ.get("DAMD_MNIST_PATH"), os.path.expanduser("~/.keras/datasets/mnist.npz")]
    for c in cands:
        if c and os.path.exists(c):
            return c
    return None


def _templates(rng):
    t = np.zeros((10, 28, 28), dtype=np.float32)
    yy, xx = np.mgrid[0:28, 0:28]
    for k in range(10):
        cy, cx = 8 + (k // 5) * 12, 4 + (k % 5) * 5
        t[k] = np.exp(-(((yy - cy) / 3.0) ** 2 + ((xx - cx) / 2.0) ** 2))
        ang = k * np.pi / 10
        t[k] += 0.8 * np.exp(-(((yy - 14) * np.cos(ang) - (xx - 14) * np.sin(ang)) / 1.5) ** 2) * (
            np.abs((yy - 14) * np.sin(ang) + (xx - 14) * np.cos(ang)) < 10)
    return t / t.max(axis=(1, 2), keepdims=True)


def synthetic(n, seed):
    rng = np.random.default_rng(seed)
    y = rng.integers(0, 10, size=n, dtype=np.int64).astype(np.uint8)
    tmpl = _templates(np.random.default_rng(1234))
    noise = rng.random((n, 28, 28), dtype=np.float32) * 0.6
    x = np.clip(noise + 0.7 * tmpl[y], 0.0, 1.0)
    return (x * 255.0).astype(np.uint8), y


def load_data(path="mnist.npz"):
    """Returns ``(x_train, y_train), (x_test, y_test)`` as uint8 numpy arrays."""
    p = _find(path)
    if p is not None:
        with np.load(p, allow_pickle=False) as f:
            return (f["x_train"], f["y_train"]), (f["x_test"], f["y_test"])
    if "synthetic" not in _CACHE:
        _CACHE["synthetic"] = (synthetic(TRAIN_N, 2020), synthetic(TEST_N, 2021))
    (a, b), (c, d) = _CACHE["synthetic"]
    return (a.copy(), b.copy()), (c.copy(), d.copy())


def is_synthetic(path="mnist.npz") -> bool:
    return _find(path) is None
