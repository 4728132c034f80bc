"""A worker process for the multi-process tests: the README distributed snippet
(README.md:363-392) under TF_CONFIG set by the launcher, on CPU/gloo.  Writes its
weights/history to $DAMD_TEST_OUT/rank<r>.npz."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("DAMD_DEVICE", "cpu")

import numpy as np  # noqa: E402

import distributed_amd as tf  # noqa: E402


def main():
    out = os.environ["DAMD_TEST_OUT"]
    steps = int(os.environ.get("DAMD_TEST_STEPS", "3")) or None  # 0 -> full epochs
    rows = int(os.environ.get("DAMD_TEST_ROWS", "4096"))
    epochs = int(os.environ.get("DAMD_TEST_EPOCHS", "2"))
    per = int(os.environ.get("DAMD_TEST_PER_REPLICA", "16"))
    strategy = tf.distribute.experimental.MultiWorkerMirroredStrategy()
    num_workers = strategy.num_replicas_in_sync
    rank = strategy.rank
    batch_size = per * num_workers
    # different seed per worker: the initial-value broadcast must make replicas equal
    tf.set_seed(100 + rank)
    if os.environ.get("DAMD_TEST_MODEL") == "resnet_small":
        # a small residual net (BN, projection shortcuts): the native graph engine's plan
        # with several gradient buckets (DAMD_BUCKET_MB) reduced while backward runs
        rng = np.random.default_rng(5)
        x_train = (rng.integers(0, 256, size=(rows, 32, 32, 3)) / 255.0).astype(np.float32)
        y_train = rng.integers(0, 10, size=rows).astype(np.int64)
        with strategy.scope():
            model = tf.models.resnet18(classes=10, input_shape=(32, 32, 3), widths=(16, 32, 32, 64),
                                       blocks=(1, 1, 1, 1))
            model.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                          optimizer=tf.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9), metrics=['accuracy'])
    else:
        mnist = tf.keras.datasets.mnist
        (x_train, y_train), _ = mnist.load_data()
        x_train = x_train[:rows].reshape(rows, 28, 28, 1) / 255.0
        y_train = y_train[:rows]
        with strategy.scope():
            model = tf.keras.Sequential([
                tf.keras.layers.Conv2D(32, 3, activation='relu', input_shape=(28, 28, 1)),
                tf.keras.layers.MaxPooling2D(),
                tf.keras.layers.Flatten(),
                tf.keras.layers.Dense(64, activation='relu'),
                tf.keras.layers.Dense(10)
            ])
            model.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                          optimizer=tf.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9), metrics=['accuracy'])
    init = [w.copy() for w in model.get_weights()]
    if os.environ.get("DAMD_TEST_INIT_FROM"):
        init = [a for a in np.load(os.environ["DAMD_TEST_INIT_FROM"]).values()]
        model.set_weights(init)
    h = model.fit(x_train, y_train, batch_size=batch_size, epochs=epochs, steps_per_epoch=steps, verbose=0)
    np.savez(os.path.join(out, f"rank{rank}.npz"), *model.get_weights())
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        eng = getattr(model, "_engine", None)
        json.dump({"history": h.history, "world": num_workers, "rank": rank,
                   "engine": getattr(eng, "name", None),
                   "exchange": getattr(eng, "allreduce_kind", None),
                   "exchange_verified": getattr(eng, "exchange_verified", None),
                   "fallback_from": list(getattr(eng, "exchange_fallback_from", []) or []),
                   "transport_us": dict(getattr(eng, "transport_us", {}) or {}),
                   "iterations": int(model.optimizer.iterations)}, f)
    if rank == 0:
        np.savez(os.path.join(out, "init0.npz"), *init)
    if os.environ.get("DAMD_TEST_DIVERGE"):
        from distributed_amd.utils.debug import MirrorDivergenceError, check_mirrored

        check_mirrored(model)  # equal after training
        if rank == 1:
            w = model.get_weights()
            w[1][0] += 1e-6
            model.set_weights(w)
        try:
            check_mirrored(model)
            verdict = "missed"
        except MirrorDivergenceError:
            verdict = "detected"
        with open(os.path.join(out, f"diverge{rank}.txt"), "w") as f:
            f.write(verdict)
    from distributed_amd.parallel import runtime

    runtime.shutdown()


if __name__ == "__main__":
    main()
