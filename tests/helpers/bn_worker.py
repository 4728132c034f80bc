"""One rank of the BatchNorm-under-MWMS test: a small conv/BN/residual model trained on
per-rank data shards (gloo), then (1) the BN moving statistics must be mirrored after
fit (DAMD_CHECK_MIRRORS inside fit passes), and (2) with the epoch-end sync disabled,
``sync_on_read_variables`` must turn each rank's own statistics into their replica mean."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("DAMD_DEVICE", "cpu")

import numpy as np  # noqa: E402

import distributed_amd as tf  # noqa: E402


def build():
    L = tf.keras.layers
    inp = tf.keras.Input(shape=(12, 12, 3))
    x = L.Conv2D(8, 3, padding="same", use_bias=False)(inp)
    x = L.BatchNormalization()(x)
    x = L.ReLU()(x)
    y = L.Conv2D(8, 3, padding="same", use_bias=False)(x)
    y = L.BatchNormalization()(y)
    x = L.ReLU()(L.Add()([x, y]))
    x = L.GlobalAveragePooling2D()(x)
    out = L.Dense(10)(x)
    return tf.keras.Model(inp, out)


def main():
    out = os.environ["DAMD_TEST_OUT"]
    strategy = tf.distribute.experimental.MultiWorkerMirroredStrategy()
    rank, world = strategy.rank, strategy.num_replicas_in_sync
    tf.set_seed(7 + rank)
    rng = np.random.default_rng(3)
    x = rng.random((256, 12, 12, 3), dtype=np.float32)
    y = rng.integers(0, 10, 256)
    with strategy.scope():
        m = build()
        m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tf.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9), metrics=["accuracy"])
    h = m.fit(x, y, batch_size=16 * world, epochs=2, steps_per_epoch=3, verbose=0)
    stats = [w.numpy() for w in m.weights if w.aggregation == "mean"]
    res = {"history": h.history, "n_stats": len(stats)}
    if os.environ.get("DAMD_BN_SYNC") == "0":
        allstats = strategy.communicator.allgather_object([s.tolist() for s in stats])
        want = [np.mean([np.asarray(a[i], dtype=np.float64) for a in allstats], axis=0) for i in range(len(stats))]
        res["differed"] = any(not np.array_equal(np.asarray(allstats[0][i]), np.asarray(allstats[1][i]))
                              for i in range(len(stats)))
        os.environ["DAMD_BN_SYNC"] = "1"
        m.sync_on_read_variables()
        got = [w.numpy() for w in m.weights if w.aggregation == "mean"]
        res["max_err"] = float(max(np.abs(g - w).max() for g, w in zip(got, want)))
    from distributed_amd.utils.debug import check_mirrored

    res["fingerprint"] = check_mirrored(m)  # raises MirrorDivergenceError on any difference
    np.savez(os.path.join(out, f"bn{rank}.npz"), *m.get_weights())
    with open(os.path.join(out, f"bn{rank}.json"), "w") as f:
        json.dump(res, f)
    from distributed_amd.parallel import runtime

    runtime.shutdown()


if __name__ == "__main__":
    main()
