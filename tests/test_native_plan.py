"""Native graph engine planner on CPU: graph lowering, fusion decisions and gradient
buckets for ResNet-18 (BASELINE.json config 4) and the reference CNN — no device needed."""
from distributed_amd import keras
from distributed_amd.engine.native_graph import NativeGraphEngine
from distributed_amd.models import mnist_cnn, resnet18


def test_resnet18_plan_fusions():
    keras.backend.clear_session()
    p = NativeGraphEngine.plan_only(resnet18(), 64).describe_plan()
    # 20 convs, each followed by a BN whose batch statistics come from the conv epilogue
    assert p["conv_bn_stats"] == 20
    # conv1 + the first BN of each of the 8 blocks apply ReLU in the BN pass
    assert p["bn_relu"] == 9
    # 8 residual adds fused into the second BN's apply: 5 identity, 3 projection (BN+BN)
    assert p["add_fused_raw"] == 5 and p["add_fused_bn"] == 3
    assert p["add_relu"] == 8
    # 17 ReLU layers folded away
    assert p["dead"] == 17


def test_resnet18_shapes_and_eligibility_reasons():
    keras.backend.clear_session()
    pl = NativeGraphEngine.plan_only(resnet18(), 8)
    out = {nd.layer.name: nd.out.shape for nd in pl.nodes}
    assert out["conv1_conv"] == (8, 112, 112, 64)
    assert out["pool1_pool"] == (8, 56, 56, 64)
    assert out["conv3_block1_conv1"] == (8, 28, 28, 128)
    assert out["conv5_block2_out"] == (8, 7, 7, 512)
    assert out["avg_pool"] == (8, 512)
    assert out["predictions"] == (8, 1000)
    # RGB stored with 4 channels: the 7x7/2 stem takes the packed-tap kernel (2 pixels x 4
    # channels per 16-byte chunk); without it RGB pads to 8 channels
    assert pl.cin_pad == 4
    assert pl.x0.shape == (8, 224, 224, 4)


def test_mnist_plan():
    keras.backend.clear_session()
    pl = NativeGraphEngine.plan_only(mnist_cnn(), 64)
    kinds = [nd.kind for nd in pl.nodes if not nd.attrs.get("dead")]
    assert kinds == ["Conv2D", "MaxPooling2D", "Dense", "Dense"]  # Flatten is a view


def test_gradient_buckets_tile_the_flat_buffer():
    import numpy as np
    import torch

    keras.backend.clear_session()
    m = resnet18()
    pl = NativeGraphEngine.plan_only(m, 8)
    pl.vars = m.trainable_weights
    pl.sizes = [int(np.prod(v.shape)) for v in pl.vars]
    pl.offsets, off = [], 0
    for sz in pl.sizes:
        pl.offsets.append(off)
        off = -(-(off + sz) // 8) * 8
    pl.G = torch.zeros(off + 8)
    pl._plan_buckets(4.0)  # 4 MB buckets over 46.8 MB of grads
    bs = pl._buckets
    assert 5 <= len(bs) <= 16  # the 3x3x512x512 convs (9.4 MB) are buckets of their own
    assert bs[0]["hi"] == off + 8  # the first bucket (last layers) carries the metric tail
    covered = sorted((b["lo"], b["hi"]) for b in bs)
    assert covered[0][0] == 0 and all(a[1] == b[0] for a, b in zip(covered, covered[1:]))
    ids = [i for b in bs for i in b["vars"]]
    assert sorted(ids) == sorted(id(v) for v in pl.vars)
    # every trainable variable has exactly one writer node in the backward plan
    written = [i for vs in pl._writes.values() for i in vs]
    assert sorted(written) == sorted(id(v) for v in pl.vars)
    # the bucket of the first layers -- written last by backward, so its all-reduce trails
    # the step -- is cut at DAMD_BUCKET_LAST_MB (1 MB): a short exposed tail
    last = [b for b in bs if b["lo"] == 0][0]
    assert (last["hi"] - last["lo"]) * 4 <= 2**20, last["hi"] * 4
    assert bs[-1] is last


class _FakeGPUStrategy:
    import torch as _t

    device = _t.device("cuda")


def _compiled(model, opt):
    model.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=opt,
                  metrics=["accuracy"])
    return model


def test_round3_layers_and_optimizers_are_native_eligible():
    """Dropout, AveragePooling2D, sigmoid / tanh and Adam / RMSprop lower to the native
    engine; what still falls back says why."""
    L = keras.layers
    keras.backend.clear_session()

    def net(units=40, act="tanh"):
        return keras.Sequential([
            L.Conv2D(16, 3, activation=act, input_shape=(16, 16, 3)),
            L.AveragePooling2D(pool_size=3, strides=2, padding="same"),
            L.Dropout(0.25),
            L.Conv2D(16, 3, activation="sigmoid"),
            L.Activation("tanh"),
            L.Flatten(),
            L.Dense(units, activation="sigmoid"),
            L.Dropout(0.0),
            L.Dense(10),
        ])

    for opt in (keras.optimizers.Adam(), keras.optimizers.RMSprop(momentum=0.9, centered=True),
                keras.optimizers.SGD(0.1, momentum=0.9)):
        ok, why = NativeGraphEngine.eligible(_compiled(net(), opt), _FakeGPUStrategy())
        assert ok, why
    ok, why = NativeGraphEngine.eligible(_compiled(net(units=36), "adam"), _FakeGPUStrategy())
    assert not ok and "multiple of 8" in why
    ok, why = NativeGraphEngine.eligible(_compiled(net(act="softplus"), "adam"), _FakeGPUStrategy())
    assert not ok and "softplus" in why
    pl = NativeGraphEngine.plan_only(net(), 8)
    kinds = {nd.layer.name: (nd.kind, nd.attrs.get("dead")) for nd in pl.nodes}
    drops = [nd for nd in pl.nodes if nd.kind == "Dropout"]
    assert [d.attrs["dead"] for d in drops] == [False, True]  # rate 0 is planned away
    assert drops[0].attrs["seed"] != 0
    assert ("Activation", False) in kinds.values()  # tanh is a real node (not an identity)
    pools = [nd for nd in pl.nodes if nd.kind == "AveragePooling2D"]
    assert pools[0].out.shape == (8, 7, 7, 16)


def test_direct_conv3_planner_on_resnet18_shapes():
    """The planner routes the ResNet-18 3x3/stride-1 convs of layers 1-3 (batch 64) to the
    direct kernel (conv3x3.hip) for forward and backprop-input, and keeps the implicit
    GEMM for layer 4 (7x7 images fill 49 of 128 MFMA rows), stride-2 and 1x1 convs; the
    Python mirror of the row planner agrees with the C++ one."""
    from distributed_amd.native import native_status
    from distributed_amd.ops import hip as H

    B = 64
    for h, c, want in ((56, 64, True), (28, 128, True), (14, 256, True), (7, 512, False)):
        f = H.conv_fwd_plan((B, h, h, c), (3, 3, c, c), (1, 1), "same")
        d = H.conv_dgrad_plan((B, h, h, c), (3, 3, c, c), (1, 1), "same")
        assert (f["amode"] == H.A_CONV3) == want and (d["amode"] == H.A_DGRAD3) == want, (h, c)
        if want:
            assert f["splits"] == 1 and f["ws"] == 0
            r = H.conv3_rows(h, h, 64 if c % 128 else 128)
            assert f["stats_T"] == B * -(-h // r)
    assert H.conv_fwd_plan((B, 56, 56, 64), (3, 3, 64, 128), (2, 2), "same")["amode"] != H.A_CONV3
    assert H.conv_fwd_plan((B, 56, 56, 64), (1, 1, 64, 128), (2, 2), "valid")["amode"] != H.A_CONV3
    # small grids keep the split-K implicit GEMM (the default threshold is 256 blocks)
    assert H.conv_fwd_plan((2, 56, 56, 64), (3, 3, 64, 64), (1, 1), "same")["amode"] != H.A_CONV3
    if native_status().get("C"):
        from distributed_amd.native import require_C

        C = require_C()
        for h in (7, 14, 20, 28, 30, 56, 112, 200):
            for bn in (64, 128):
                assert C.conv3_rows(h, h, bn) == H.conv3_rows(h, h, bn), (h, bn)
