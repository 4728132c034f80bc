"""Keras-layout HDF5 checkpoints (reference README.md:234-247) via the native _h5 module."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import distributed_amd as tf
from distributed_amd import r_api as k

H5DUMP = "/opt/conda/bin/h5dump"


def _model(momentum=0.0):
    tf.set_seed(1)
    m = tf.models.mnist_cnn()
    m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tf.keras.optimizers.SGD(learning_rate=0.01, momentum=momentum), metrics=["accuracy"])
    return m


def _data(n=256):
    rng = np.random.default_rng(0)
    return rng.random((n, 28, 28, 1), dtype=np.float32), rng.integers(0, 10, n)


def test_roundtrip_weights_config_optimizer(tmp_path):
    m = _model(momentum=0.9)
    x, y = _data()
    m.fit(x, y, batch_size=64, epochs=1, verbose=0)
    p = str(tmp_path / "model.hdf5")
    k.save_model_hdf5(m, p)
    m2 = k.load_model_hdf5(p)
    assert [l.name for l in m2.layers] == [l.name for l in m.layers]
    for a, b in zip(m.get_weights(), m2.get_weights()):
        assert a.dtype == b.dtype and np.array_equal(a, b)
    assert m2.optimizer.momentum == pytest.approx(0.9) and m2.optimizer.learning_rate == pytest.approx(0.01)
    assert m2.optimizer.iterations == m.optimizer.iterations == 4
    np.testing.assert_array_equal(m2.optimizer.slots["momentum"].numpy(), m.optimizer.slots["momentum"].numpy())
    np.testing.assert_allclose(m2.predict(x[:8]), m.predict(x[:8]), rtol=1e-6)
    # training continues identically from the restored state
    h1 = m.fit(x, y, batch_size=64, epochs=1, verbose=0, shuffle=False)
    h2 = m2.fit(x, y, batch_size=64, epochs=1, verbose=0, shuffle=False)
    assert h1.history["loss"] == pytest.approx(h2.history["loss"], rel=1e-6)


@pytest.mark.skipif(not os.path.exists(H5DUMP), reason="h5dump not available")
def test_keras_layout_visible_to_h5dump(tmp_path):
    m = _model()
    p = str(tmp_path / "m.h5")
    m.save(p)
    out = subprocess.run([H5DUMP, "-H", p], capture_output=True, text=True, check=True).stdout
    for token in ('ATTRIBUTE "keras_version"', 'ATTRIBUTE "model_config"', 'ATTRIBUTE "training_config"',
                  'GROUP "model_weights"', 'ATTRIBUTE "layer_names"', 'GROUP "conv2d"', 'DATASET "kernel:0"',
                  'GROUP "dense_1"', 'GROUP "optimizer_weights"', 'H5T_STR_NULLPAD'):
        assert token in out, token
    out = subprocess.run([H5DUMP, "-d", "/model_weights/dense/dense/kernel:0", "-H", p], capture_output=True,
                         text=True, check=True).stdout
    assert "( 5408, 64 )" in out and "H5T_IEEE_F32LE" in out
    from distributed_amd.native import load_h5

    tree = load_h5().read(p)
    cfg = json.loads(tree["attrs"]["model_config"])
    assert cfg["class_name"] == "Sequential"
    assert [l["class_name"] for l in cfg["config"]["layers"]] == ["Conv2D", "MaxPooling2D", "Flatten", "Dense",
                                                                  "Dense"]
    assert cfg["config"]["layers"][0]["config"]["batch_input_shape"] == [None, 28, 28, 1]
    tc = json.loads(tree["attrs"]["training_config"])
    assert tc["loss"]["class_name"] == "SparseCategoricalCrossentropy" and tc["loss"]["config"]["from_logits"]
    assert tc["optimizer_config"]["class_name"] == "SGD"
    assert tree["groups"]["model_weights"]["attrs"]["layer_names"] == ["conv2d", "max_pooling2d", "flatten",
                                                                      "dense", "dense_1"]


def test_save_weights_load_weights(tmp_path):
    m = _model()
    p = str(tmp_path / "w.h5")
    m.save_weights(p)
    m2 = _model()
    m2.set_weights([np.zeros_like(w) for w in m2.get_weights()])
    m2.load_weights(p)
    assert all(np.array_equal(a, b) for a, b in zip(m.get_weights(), m2.get_weights()))


def test_base64_transport(tmp_path):
    """README.md:240-246: chief base64-encodes the file, the driver writes it back."""
    m = _model()
    p = str(tmp_path / "trained-0.hdf5")
    k.save_model_hdf5(m, p)
    payload = k.base64encode(p)
    out = k.write_bytes(k.base64decode(payload), str(tmp_path / "model.hdf5"))
    m2 = k.load_model_hdf5(out)
    assert all(np.array_equal(a, b) for a, b in zip(m.get_weights(), m2.get_weights()))
    # collected barrier rows: chief carries the payload, the others return ""
    rows = [{"address": payload}, {"address": ""}, {"address": ""}]
    out2 = k.save_from_result(rows, str(tmp_path / "model2.hdf5"))
    assert open(out2, "rb").read() == open(p, "rb").read()


def test_model_checkpoint_and_backup_restore(tmp_path):
    x, y = _data(512)
    ck = str(tmp_path / "ck-{epoch:02d}.h5")
    m = _model(momentum=0.5)
    m.fit(x, y, batch_size=64, epochs=2, verbose=0, callbacks=[tf.keras.callbacks.ModelCheckpoint(ck)])
    assert os.path.exists(str(tmp_path / "ck-01.h5")) and os.path.exists(str(tmp_path / "ck-02.h5"))
    # uninterrupted 4 epochs
    ref = _model(momentum=0.5)
    href = ref.fit(x, y, batch_size=64, epochs=4, verbose=0, shuffle=False)
    # interrupted after epoch 2, then resumed by BackupAndRestore
    bdir = str(tmp_path / "backup")

    class Crash(tf.keras.callbacks.Callback):
        def on_epoch_end(self, epoch, logs=None):
            if epoch == 1:
                raise RuntimeError("simulated worker failure")

    m1 = _model(momentum=0.5)
    with pytest.raises(RuntimeError):
        m1.fit(x, y, batch_size=64, epochs=4, verbose=0, shuffle=False,
               callbacks=[tf.keras.callbacks.BackupAndRestore(bdir), Crash()])
    assert os.path.exists(os.path.join(bdir, "chief.h5"))
    m2 = _model(momentum=0.5)  # a fresh process would rebuild the model like this
    h2 = m2.fit(x, y, batch_size=64, epochs=4, verbose=0, shuffle=False,
                callbacks=[tf.keras.callbacks.BackupAndRestore(bdir)])
    assert h2.epoch == [2, 3]
    assert h2.history["loss"] == pytest.approx(href.history["loss"][2:], rel=1e-5)
    for a, b in zip(m2.get_weights(), ref.get_weights()):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-7)
    assert not os.path.exists(os.path.join(bdir, "chief.h5"))  # cleaned after success


def test_functional_resnet_save_load_predict_roundtrip(tmp_path):
    """A functional (residual, BN) model saved as Keras HDF5 carries its graph
    (inbound_nodes / input_layers / output_layers) and reloads to the same predictions."""
    tf.set_seed(4)
    m = tf.models.resnet18(classes=10, input_shape=(16, 16, 3), widths=(8, 16, 16, 16), blocks=(1, 1, 1, 1))
    tf.models.compile_resnet(m, 0.05, 0.9)
    rng = np.random.default_rng(2)
    x = rng.random((64, 16, 16, 3), dtype=np.float32)
    y = rng.integers(0, 10, 64)
    m.fit(x, y, batch_size=32, epochs=1, verbose=0)
    p = str(tmp_path / "resnet.h5")
    m.save(p)
    cfg = json.loads(m.to_json())
    assert cfg["class_name"] == "Model"
    c = cfg["config"]
    assert c["input_layers"] == [["input_1", 0, 0]] and c["output_layers"] == [["predictions", 0, 0]]
    by = {l["name"]: l for l in c["layers"]}
    assert by["input_1"]["inbound_nodes"] == []
    assert by["conv1_conv"]["inbound_nodes"] == [[["input_1", 0, 0, {}]]]
    add = by["conv3_block1_add"]["inbound_nodes"][0]
    assert [e[0] for e in add] == ["conv3_block1_bn2", "conv3_block1_proj_bn"]
    m2 = tf.keras.models.load_model(p)
    assert [l.name for l in m2.layers] == [l.name for l in m.layers]
    for a, b in zip(m.get_weights(), m2.get_weights()):
        assert np.array_equal(a, b)
    np.testing.assert_array_equal(m.predict(x[:16]), m2.predict(x[:16]))
    assert m2.optimizer.momentum == pytest.approx(0.9)
    if shutil.which(H5DUMP) or os.path.exists(H5DUMP):
        out = subprocess.run([H5DUMP, "-a", "/model_config", p], capture_output=True, text=True).stdout
        assert "inbound_nodes" in out and "conv3_block1_add" in out


def test_shared_layer_node_indices():
    """A layer applied twice owns two nodes; its second call is referenced as node 1."""
    L = tf.keras.layers
    inp = tf.keras.Input(shape=(6,))
    d = L.Dense(6, name="shared")
    h = d(d(inp))
    out = L.Dense(2, name="head")(h)
    m = tf.keras.Model(inp, out)
    c = json.loads(m.to_json())["config"]
    by = {l["name"]: l for l in c["layers"]}
    assert by["shared"]["inbound_nodes"] == [[["input_1" if "input_1" in by else c["input_layers"][0][0], 0, 0, {}]],
                                             [["shared", 0, 0, {}]]]
    assert by["head"]["inbound_nodes"] == [[["shared", 1, 0, {}]]]
    m2 = tf.keras.models.model_from_json(m.to_json())
    m2.set_weights(m.get_weights())
    xx = np.random.default_rng(0).random((4, 6), dtype=np.float32)
    np.testing.assert_array_equal(m.predict(xx), m2.predict(xx))


def test_layer_called_outside_the_model_roundtrips():
    """a layer also called outside this model (here by a sub-model built first)
    has global call counters that run past this model's nodes; the config renumbers each
    layer's nodes by position among this model's calls, so the saved graph reloads."""
    L = tf.keras.layers
    d = L.Dense(6, name="shared_outside")
    other_in = tf.keras.Input(shape=(6,))
    tf.keras.Model(other_in, d(other_in))          # call #0 of d belongs to another model
    inp = tf.keras.Input(shape=(6,))
    out = L.Dense(2, name="head2")(d(d(inp)))      # calls #1 and #2 of d
    m = tf.keras.Model(inp, out)
    c = json.loads(m.to_json())["config"]
    by = {l["name"]: l for l in c["layers"]}
    nodes = by["shared_outside"]["inbound_nodes"]
    assert len(nodes) == 2
    assert nodes[1] == [["shared_outside", 0, 0, {}]]   # the second local call eats the first
    assert by["head2"]["inbound_nodes"] == [[["shared_outside", 1, 0, {}]]]
    m2 = tf.keras.models.model_from_config({"class_name": "Model", "config": c})
    x = np.random.default_rng(0).random((4, 6), dtype=np.float32)
    m2.set_weights(m.get_weights())
    np.testing.assert_allclose(m2.predict(x), m.predict(x), rtol=1e-6, atol=1e-7)
