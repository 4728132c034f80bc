"""Fault-tolerance worker: README distributed snippet + BackupAndRestore, optionally with
an injected failure (DAMD_FAIL_AT=rank:step:attempt).  Writes rank<r>.npz / .json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("DAMD_DEVICE", "cpu")

import numpy as np  # noqa: E402

import distributed_amd as tf  # noqa: E402


def main():
    out = os.environ["DAMD_TEST_OUT"]
    strategy = tf.distribute.experimental.MultiWorkerMirroredStrategy()
    rank = strategy.rank
    tf.set_seed(7)
    (x, y), _ = tf.keras.datasets.mnist.load_data()
    x = x[:2048].reshape(2048, 28, 28, 1) / 255.0
    y = y[:2048]
    with strategy.scope():
        model = tf.models.mnist_cnn()
        model.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tf.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9), metrics=["accuracy"])
    cb = [tf.keras.callbacks.BackupAndRestore(os.path.join(out, "backup"))]
    h = model.fit(x, y, batch_size=32 * strategy.num_replicas_in_sync, epochs=4, steps_per_epoch=3, verbose=0,
                  callbacks=cb)
    np.savez(os.path.join(out, f"rank{rank}.npz"), *model.get_weights())
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump({"history": h.history, "iterations": int(model.optimizer.iterations),
                   "attempt": int(os.environ.get("DAMD_RESTART_COUNT", "0"))}, f)
    from distributed_amd.parallel import runtime

    runtime.shutdown()


if __name__ == "__main__":
    main()
