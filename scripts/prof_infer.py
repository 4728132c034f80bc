"""fit(validation_split) + evaluate + predict of the MNIST CNN on one GPU: the workload of
the "only damd kernels" rocprof check.  Run under
``rocprofv3 --kernel-trace --stats -- python3 scripts/prof_infer.py``; then
``python scripts/kernel_origin.py <stats csv>`` splits the kernels by library."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_amd as tf  # noqa: E402

rng = np.random.default_rng(0)
x = (rng.integers(0, 256, size=(6400, 28, 28, 1)) / 255.0).astype(np.float32)
y = rng.integers(0, 10, size=6400)
m = tf.keras.Sequential([
    tf.keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
    tf.keras.layers.MaxPooling2D(),
    tf.keras.layers.Flatten(),
    tf.keras.layers.Dense(64, activation="relu"),
    tf.keras.layers.Dense(10),
])
m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
          optimizer=tf.keras.optimizers.SGD(0.01), metrics=["accuracy"])
h = m.fit(x, y, batch_size=64, epochs=2, validation_split=0.2, verbose=0)
print("history", {k: [round(float(v), 4) for v in vs] for k, vs in h.history.items()})
print("evaluate", m.evaluate(x[:2000], y[:2000], batch_size=256, verbose=0))
print("predict", m.predict(x[:1000], batch_size=256).shape)
