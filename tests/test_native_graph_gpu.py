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


def _train(build, x, y, init, batch, steps, native, lr=0.1, momentum=0.0, graph=True, device=None, extra_env=None,
           fused=False, optimizer=None):
    env = {"DAMD_NATIVE_GRAPH": "1" if native else "0", "DAMD_FUSED": "1" if fused else "0",
           "DAMD_GRAPH": "1" if graph else "0"}
    env.update(extra_env or {})
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
                  optimizer=optimizer() if optimizer else tf.keras.optimizers.SGD(learning_rate=lr, momentum=momentum),
                  metrics=["accuracy"])
        m.set_weights(init)
        h = m.fit(x, y, batch_size=batch, epochs=1, steps_per_epoch=steps, shuffle=False, verbose=0)
        eng = m._engine.name
        if optimizer:
            return m.get_weights(), h.history, eng, m.optimizer
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


def _compare_updates(init, wa, wb, names, cos_min=0.98, rel_max=0.08, idx=None):
    if idx is not None:  # compare only the tensors at these positions
        init, wa, wb = [init[i] for i in idx], [wa[i] for i in idx], [wb[i] for i in idx]
    for w0, a, b, nm in zip(init, wa, wb, names):
        da, db = (a - w0).ravel().astype(np.float64), (b - w0).ravel().astype(np.float64)
        nb = np.linalg.norm(db)
        if nb < 1e-7:
            assert np.linalg.norm(da) < 1e-5, nm
            continue
        cos = float(da @ db / (np.linalg.norm(da) * nb + 1e-30))
        rel = float(np.linalg.norm(da - db) / nb)
        assert cos > cos_min and rel < rel_max, f"{nm}: cos {cos:.4f} rel {rel:.4f}"


class _Q(torch.autograd.Function):
    """Round to bf16 in forward AND backward: a tensor the native plan stores in bf16."""

    @staticmethod
    def forward(ctx, x):
        return x.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g.bfloat16().float()


class _QW(torch.autograd.Function):
    """bf16 weight shadow: rounded operand, straight-through gradient."""

    @staticmethod
    def forward(ctx, w):
        return w.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g


class _QG(torch.autograd.Function):
    """fp32 value, bf16-rounded gradient (the logits: fp32 out, bf16 dlogits)."""

    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return g.bfloat16().float()


def _emulated_reference_grads(engine, model, x, y, global_batch):
    """fp32 PyTorch re-execution of the engine's own (fused) plan with bf16 rounding at
    exactly the tensors the plan stores in bf16.  Returns {variable id: grad}."""
    from distributed_amd.ops import reference as ref

    dev = engine.device
    leaves = {}
    for v in model.trainable_weights:
        leaves[id(v)] = v.value.detach().clone().requires_grad_(True)
    relu = torch.relu
    vals = {}
    x0 = torch.from_numpy(x).to(dev).float()
    vals[id(engine.x0.root())] = _Q.apply(x0)
    norm = {}

    def get(t):
        return vals[id(t.root())]

    def bn_norm(nd, xin):
        l = nd.layer
        m = xin.mean(dim=(0, 1, 2))
        v = xin.var(dim=(0, 1, 2), unbiased=False)
        return (xin - m) * torch.rsqrt(v + l.epsilon) * leaves[id(l.gamma)] + leaves[id(l.beta)]

    logits = None
    for nd in engine.nodes:
        if nd.attrs.get("dead"):
            continue
        l, k = nd.layer, nd.kind
        if k == "Conv2D":
            yv = ref.conv2d(get(nd.inputs[0])[..., :l.kernel.shape[2]], _QW.apply(leaves[id(l.kernel)]),
                            leaves[id(l.bias)] if l.use_bias else None, l.strides, l.padding)
            if getattr(l.activation, "__name__", "") == "relu":
                yv = relu(yv)
            vals[id(nd.out.root())] = _Q.apply(yv)
        elif k == "BatchNormalization":
            z = bn_norm(nd, get(nd.inputs[0]))
            if nd.attrs.get("stats_only"):
                norm[id(nd)] = z
            else:
                vals[id(nd.out.root())] = _Q.apply(relu(z) if nd.attrs.get("relu") else z)
        elif k == "Add":
            fused = nd.attrs.get("fused")
            if fused is None:
                z = get(nd.inputs[0]) + get(nd.inputs[1])
            else:
                main, (mode, other) = fused
                z = norm[id(main)] + (get(other) if mode == "raw" else norm[id(other)])
            vals[id(nd.out.root())] = _Q.apply(relu(z) if nd.attrs.get("relu") else z)
        elif k in ("Activation", "ReLU"):
            vals[id(nd.out.root())] = _Q.apply(relu(get(nd.inputs[0])))
        elif k == "MaxPooling2D":
            vals[id(nd.out.root())] = _Q.apply(ref.maxpool2d(get(nd.inputs[0]), l.pool_size, l.strides, l.padding))
        elif k == "GlobalAveragePooling2D":
            vals[id(nd.out.root())] = _Q.apply(get(nd.inputs[0]).mean(dim=(1, 2)))
        elif k == "Dense":
            xin = get(nd.inputs[0]).reshape(x.shape[0], -1)
            z = xin @ _QW.apply(leaves[id(l.kernel)])
            if l.use_bias:
                z = z + leaves[id(l.bias)]
            if nd.attrs.get("logits"):
                logits = _QG.apply(z)
            else:
                vals[id(nd.out.root())] = _Q.apply(relu(z) if getattr(l.activation, "__name__", "") == "relu"
                                                   else z)
    loss = ref.sparse_softmax_xent(logits, torch.from_numpy(y).to(dev)).sum() / global_batch
    ids = list(leaves)
    grads = torch.autograd.grad(loss, [leaves[i] for i in ids], allow_unused=True)
    return {i: g for i, g in zip(ids, grads)}, float(loss)


PINNED_INIT_SEED = 20240521  # the tight-bounds case of the emulated-reference test


def test_small_resnet_step_matches_bf16_emulated_reference():
    """The plan's wiring (fusion, residual fan-in, BN backward, padding, split-K
    accumulation) against an fp32 re-execution with the same bf16 storage points: after
    one plain-SGD step every weight update must agree.

    A 1-ulp fp32 difference (summation order) flips some bf16 roundings and the BN-backward
    cancellation amplifies them, mostly in the BN gamma / beta updates.  Init sweeps
    (scripts/sweep_emulated_ref.py, round 4; 16 + 40 draws): loss error <= 2.2e-3 relative,
    worst layer's relative update error <= 0.262 / cosine >= 0.966 (BN gamma / beta), median
    layer <= 0.145, head <= 1.2e-2, whole update vector cosine >= 0.987 / relative error
    <= 0.160 -- heavy tails, so the bounds below leave margin for any init (three fresh draws
    per run); exact wiring checks are the bitwise fused-vs-unfused tests.  The first case is
    a PINNED init held to the round-3 tight bounds (a reproducible regression detector for
    e.g. BN gamma / beta wiring), the two fresh draws to the sweep-derived ones."""
    x, y = _data(32, (32, 32, 3), 10, seed=4)
    os.environ["DAMD_FUSED"] = "0"
    try:
        for rep in range(3):
            tf.keras.backend.clear_session()
            tight = rep == 0
            # pinned, or a fresh draw printed for replay
            seed = PINNED_INIT_SEED if tight else int.from_bytes(os.urandom(4), "little")
            print(f"init seed {seed} ({'pinned, tight bounds' if tight else 'fresh draw'})")
            tf.set_seed(seed)
            m = _small_resnet()
            lr = 0.1
            m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tf.keras.optimizers.SGD(learning_rate=lr), metrics=["accuracy"])
            e = m._get_engine(32, 32)
            assert e.name == "native_graph"
            e.bind(x, y)
            e.start_epoch(0, False)
            w0 = {id(v): v.value.detach().clone() for v in m.trainable_weights}
            grads, ref_loss = _emulated_reference_grads(e, m, x, y, 32)
            e.run(1)
            e.sync()
            met = e.metrics()
            assert abs(met["loss"] - ref_loss) < 5e-3 * abs(ref_loss)
            rels, dn, dr = [], [], []
            for v in m.trainable_weights:
                d_native = (v.value.detach() - w0[id(v)]).double().ravel()
                d_ref = (-lr * grads[id(v)]).double().ravel()
                nref = d_ref.norm().item()
                rel = (d_native - d_ref).norm().item() / max(nref, 1e-12)
                cos = float(d_native @ d_ref / max(d_native.norm().item() * nref, 1e-30))
                c_min, r_max = (0.97, 0.25) if tight else (0.93, 0.45)
                assert cos > c_min and rel < r_max, f"{v.name}: rel err {rel:.4f} cos {cos:.4f} (|d| {nref:.3e})"
                rels.append(rel)
                dn.append(d_native)
                dr.append(d_ref)
            assert sorted(rels)[len(rels) // 2] < (0.1 if tight else 0.25), rels
            assert rels[-2] < 3e-2, rels  # the head (predictions kernel): no BN below it
            a, b = torch.cat(dn), torch.cat(dr)
            c_all, r_all = (0.99, 0.15) if tight else (0.97, 0.3)
            assert float(a @ b / (a.norm() * b.norm())) > c_all and float((a - b).norm() / b.norm()) < r_all
    finally:
        os.environ.pop("DAMD_FUSED", None)


def test_small_resnet_one_step_matches_fp32_reference():
    """One native step vs a pure fp32 CPU step of the same small ResNet: a SANITY bound,
    deliberately loose for BatchNorm gamma / beta (cos > 0.75, rel < 0.7).  The native step
    stores activations and their gradients in bf16; x-hat amplifies that rounding by
    |mean| / std and the BN backward's cancellation amplifies it again, so BN parameter
    updates drift from fp32 by design (16-draw sweep worst: cos 0.846, rel 0.541).  The
    real numerical checks are the per-op fp32 oracles (test_hip_ops_gpu.py, BN forward /
    backward) and the pinned-seed bf16-EMULATED reference, which rounds at the same storage
    points and is compared tightly (test_small_resnet_step_matches_bf16_emulated_reference)."""
    tf.keras.backend.clear_session()
    x, y = _data(64, (32, 32, 3), 10)
    m0 = _small_resnet()
    init = m0.get_weights()
    names = [w.name for w in m0.weights]
    wn, hn, en = _train(_small_resnet, x, y, init, 32, 1, native=True)
    wr, hr, er = _train(_small_resnet, x, y, init, 32, 1, native=False, device="cpu")
    assert en == "native_graph" and er == "generic"
    assert abs(hn["loss"][0] - hr["loss"][0]) < 2e-2 * abs(hr["loss"][0])
    # bf16 storage of pre-BN activations and gradients vs a pure fp32 run: the head is
    # tight, deep layers drift (|mean|/std of conv outputs amplifies bf16 rounding in
    # x-hat, and BN backward cancellation amplifies it again); wiring is checked
    # exactly by the emulated-reference test above.  Bounds by tensor class from a 16-draw
    # init sweep (scripts/sweep_tolerances.py 16 resnet_fp32, round 4): BN gamma / beta worst
    # cos 0.846 / rel 0.541 (heavy tail: BN-backward cancellation), conv / dense kernels worst
    # cos 0.943 / rel 0.338, whole update vector worst cos 0.956 / rel 0.302
    bn = [i for i, nm in enumerate(names) if "bn" in nm]
    other = [i for i, nm in enumerate(names) if "bn" not in nm]
    _compare_updates(init, wn, wr, [names[i] for i in bn], cos_min=0.75, rel_max=0.7, idx=bn)
    _compare_updates(init, wn, wr, [names[i] for i in other], cos_min=0.9, rel_max=0.45, idx=other)
    da = np.concatenate([(a - w0).ravel() for w0, a in zip(init, wn)]).astype(np.float64)
    db = np.concatenate([(b - w0).ravel() for w0, b in zip(init, wr)]).astype(np.float64)
    assert da @ db / (np.linalg.norm(da) * np.linalg.norm(db)) > 0.93
    assert np.linalg.norm(da - db) / np.linalg.norm(db) < 0.4


def test_mnist_native_graph_tracks_reference_over_steps():
    x, y = _data(640, (28, 28, 1), 10, seed=1)
    tf.keras.backend.clear_session()
    init = _mnist().get_weights()
    wn, hn, en = _train(_mnist, x, y, init, 64, 10, native=True, lr=0.05, momentum=0.9)
    wr, hr, er = _train(_mnist, x, y, init, 64, 10, native=False, device="cpu", lr=0.05, momentum=0.9)
    assert en == "native_graph"
    np.testing.assert_allclose(hn["loss"], hr["loss"], rtol=1e-2)
    # 10 momentum steps amplify the bf16 rounding: over 24 fresh init draws
    # (scripts/sweep_tolerances.py 24 track) the worst tensor reached cos 0.956 / rel 0.317
    # (k2, b2); bounds with margin for any draw
    _compare_updates(init, wn, wr, ["k", "b", "k1", "b1", "k2", "b2"], cos_min=0.90, rel_max=0.45)


def test_short_final_batch_is_masked_like_keras():
    """100 rows at batch 64: the second step has 36 real rows.  The native engine masks the
    28 padding rows (zero gradient, no loss/metric) and scales by 1/36, like the fp32
    generic engine on its real 36-row batch (it used to wrap around)."""
    x, y = _data(100, (28, 28, 1), 10, seed=8)
    tf.keras.backend.clear_session()
    init = _mnist().get_weights()
    wn, hn, en = _train(_mnist, x, y, init, 64, None, native=True, lr=0.05)
    wr, hr, er = _train(_mnist, x, y, init, 64, None, native=False, device="cpu", lr=0.05)
    assert en == "native_graph" and er == "generic"
    np.testing.assert_allclose(hn["loss"], hr["loss"], rtol=1e-2)
    np.testing.assert_allclose(hn["accuracy"], hr["accuracy"], atol=1.5 / 100)
    _compare_updates(init, wn, wr, ["k", "b", "k1", "b1", "k2", "b2"], cos_min=0.97, rel_max=0.25)


def test_set_weights_refreshes_bf16_shadow():
    """set_weights on a model whose native engine is cached: the next step must use the new
    weights (the bf16 shadow the GEMMs read is re-derived), i.e. equal a fresh engine."""
    x, y = _data(128, (32, 32, 3), 10, seed=9)
    os.environ["DAMD_FUSED"] = "0"
    try:
        tf.keras.backend.clear_session()
        init_a = _small_resnet().get_weights()
        init_b = _small_resnet().get_weights()
        res = []
        for warm in (True, False):
            tf.keras.backend.clear_session()
            m = _small_resnet()
            m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tf.keras.optimizers.SGD(learning_rate=0.05), metrics=["accuracy"])
            if warm:
                m.set_weights(init_a)
                m.fit(x, y, batch_size=32, epochs=1, steps_per_epoch=1, shuffle=False, verbose=0)
                assert m._engine is not None
            m.set_weights(init_b)
            h = m.fit(x, y, batch_size=32, epochs=1, steps_per_epoch=1, shuffle=False, verbose=0)
            assert m._engine.name == "native_graph"
            res.append((m.get_weights(), h.history["loss"][0]))
        (wa, la), (wb, lb) = res
        assert abs(la - lb) < 1e-4 * abs(lb)
        for a, b in zip(wa, wb):
            np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)
    finally:
        os.environ.pop("DAMD_FUSED", None)


def test_graph_replay_equals_eager():
    """Replaying the captured step == running it eagerly, BITWISE: every reduction of the
    native step runs in a fixed order (split-K slabs, BN partials, bias column sums, the
    loss / metric sums), so 4 steps (1 eager + 3 replayed vs 4 eager) give the same bits
    -- for any initial draw (three unpinned inits)."""
    x, y = _data(128, (32, 32, 3), 10, seed=2)
    for rep in range(3):
        tf.keras.backend.clear_session()
        init = _small_resnet().get_weights()
        wg, hg, _ = _train(_small_resnet, x, y, init, 32, 4, native=True, momentum=0.9, graph=True)
        we, he, _ = _train(_small_resnet, x, y, init, 32, 4, native=True, momentum=0.9, graph=False)
        for a, b in zip(wg, we):
            np.testing.assert_array_equal(a, b)
        assert hg["loss"] == he["loss"]


def test_native_step_is_run_to_run_reproducible():
    """The same run twice: bitwise equal weights and history (no arrival-order sums)."""
    x, y = _data(128, (32, 32, 3), 10, seed=12)
    tf.keras.backend.clear_session()
    init = _small_resnet().get_weights()
    wa, ha, _ = _train(_small_resnet, x, y, init, 32, 3, native=True, momentum=0.9)
    wb, hb, _ = _train(_small_resnet, x, y, init, 32, 3, native=True, momentum=0.9)
    for a, b in zip(wa, wb):
        np.testing.assert_array_equal(a, b)
    assert ha == hb


def test_stem_fusion_matches_unfused():
    """BN -> ReLU -> MaxPool fused (the BN output never stored; pool routing and ReLU mask
    recomputed in backward) == the three separate passes, one step."""
    from distributed_amd.engine.native_graph import NativeGraphEngine

    x, y = _data(64, (32, 32, 3), 10, seed=6)
    tf.keras.backend.clear_session()
    init = _small_resnet().get_weights()
    plan = NativeGraphEngine.plan_only(_small_resnet(), 32)
    assert sum(1 for nd in plan.nodes if nd.attrs.get("pool") is not None) == 1
    wf, hf, ef = _train(_small_resnet, x, y, init, 32, 1, native=True, momentum=0.9)
    wu, hu, eu = _train(_small_resnet, x, y, init, 32, 1, native=True, momentum=0.9,
                        extra_env={"DAMD_STEM_FUSE": "0"})
    assert ef == eu == "native_graph"
    for a, b in zip(wf, wu):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(hf["loss"], hu["loss"], rtol=1e-6)


def test_bn_backward_reduce_fused_into_dgrad_epilogue(monkeypatch):
    """BN -> ReLU -> Conv2D: the conv's direct backprop-input kernel writes the BN-backward
    partials in its epilogue (DAMD_BN_DGRAD_FUSE, default) == the separate bn_bwd_reduce
    pass: one step of a ResNet whose 64-channel 16x16 stage runs the direct 3x3 kernel
    (DAMD_CONV3_MIN_WG=1 admits the small grid).  One step: the partials differ from
    bn_bwd_reduce's only in fp32 summation order (~1e-6 relative in the updates), but this
    net's bf16 second step amplifies such perturbations (maxpool / ReLU decisions on
    near-ties) to several percent for some random inits, for any two summation orders
    (scripts/diag_bnred3.py); the partials themselves are pinned to an fp32 reference in
    test_conv_gemm_gpu.py::test_direct_conv3_dgrad_bnred."""
    from distributed_amd.ops import hip as H

    def build():
        # two basic blocks on the 16x16 / 64-channel layer: two BN -> ReLU -> direct-conv chains
        # (the 8x8 layers' convs keep the implicit GEMM: an 8x8 image fills 64 of 256 rows)
        return resnet18(classes=10, input_shape=(64, 64, 3), widths=(64, 64, 128, 128), blocks=(2, 1, 1, 1))

    monkeypatch.setenv("DAMD_CONV3_MIN_WG", "1")
    assert H.conv_dgrad_plan((32, 16, 16, 64), (3, 3, 64, 64), (1, 1), "same")["amode"] == H.A_DGRAD3
    x, y = _data(64, (64, 64, 3), 10, seed=9)
    for rep in range(3):  # any initial draw (one step: no bf16 second-step amplification)
        tf.keras.backend.clear_session()
        init = build().get_weights()
        fused, hf, ef = _train(build, x, y, init, 32, 1, native=True)
        unfused, hu, eu = _train(build, x, y, init, 32, 1, native=True, extra_env={"DAMD_BN_DGRAD_FUSE": "0"})
        assert ef == eu == "native_graph"
        for a, b in zip(fused, unfused):
            np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-4)
        np.testing.assert_allclose(hf["loss"], hu["loss"], rtol=1e-5)


@pytest.mark.parametrize("reps", ["1", "8"])
def test_bn_finalize_in_consumer_matches_finalize_kernels(monkeypatch, reps):
    """BatchNorm statistics through int64 fixed-point accumulators (DAMD_BN_FIN=1: producers
    -- conv epilogues, split-K finish, the backprop-input E_BNRED epilogue, bn_bwd_reduce,
    the stem pool -- add per-block partials into `reps` replicas, the apply kernels finalize
    in their prologue) == the per-block partials + finalize launches, one step, three
    initial draws; and two runs with it are bitwise equal (integer sums: the arrival order
    of the producer blocks cannot change them)."""
    from distributed_amd.ops import hip as H

    def build():
        # two basic blocks on the 16x16x64 stage: two BN -> ReLU -> conv chains the direct
        # kernel takes (the deeper stages' 8x8 / 4x4 tiles under-fill its MFMA rows)
        return resnet18(classes=10, input_shape=(64, 64, 3), widths=(64, 64, 128, 128), blocks=(2, 1, 1, 1))

    monkeypatch.setenv("DAMD_CONV3_MIN_WG", "1")
    monkeypatch.setenv("DAMD_BN_REPS", reps)
    # both arms on the split-K finish launch: with fp32 partials (DAMD_BN_FIN=0) the split-K
    # convs cannot finish in-launch (E_FIXUP needs the accumulator), and partials grouped by
    # output tile instead of the finish's row blocks move the statistics by ~1e-8 relative --
    # enough to flip bf16 roundings downstream, not what this test compares
    # (test_splitk_in_launch_finish_matches_finish_kernel covers that path)
    monkeypatch.setenv("DAMD_SPLITK_FIXUP", "0")
    assert H.conv_dgrad_plan((32, 16, 16, 64), (3, 3, 64, 64), (1, 1), "same")["amode"] == H.A_DGRAD3
    x, y = _data(64, (64, 64, 3), 10, seed=9)
    for rep in range(3):
        tf.keras.backend.clear_session()
        init = build().get_weights()
        wf, hf, ef = _train(build, x, y, init, 32, 1, native=True, extra_env={"DAMD_BN_FIN": "1"})
        wk, hk, ek = _train(build, x, y, init, 32, 1, native=True, extra_env={"DAMD_BN_FIN": "0"})
        assert ef == ek == "native_graph"
        for a, b in zip(wf, wk):
            np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-4)
        np.testing.assert_allclose(hf["loss"], hk["loss"], rtol=1e-5)
    w2, h2, _ = _train(build, x, y, init, 32, 2, native=True, momentum=0.9, extra_env={"DAMD_BN_FIN": "1"})
    w3, h3, _ = _train(build, x, y, init, 32, 2, native=True, momentum=0.9, extra_env={"DAMD_BN_FIN": "1"})
    for a, b in zip(w2, w3):
        np.testing.assert_array_equal(a, b)
    assert h2 == h3


def test_bn_applied_inside_direct_conv_is_bitwise(monkeypatch):
    """BN -> ReLU -> Conv2D with a direct 3x3 forward plan: the conv normalises its input on
    load and stores the BN output for its weight gradient (DAMD_BN_CONV_FOLD, default) ==
    the bn_apply launch + the plain conv, bitwise over two momentum steps."""
    from distributed_amd.engine.native_graph import NativeGraphEngine

    def build():
        # two basic blocks on the 16x16x64 stage: two BN -> ReLU -> conv chains the direct
        # kernel takes (the deeper stages' 8x8 / 4x4 tiles under-fill its MFMA rows)
        return resnet18(classes=10, input_shape=(64, 64, 3), widths=(64, 64, 128, 128), blocks=(2, 1, 1, 1))

    monkeypatch.setenv("DAMD_CONV3_MIN_WG", "1")
    x, y = _data(64, (64, 64, 3), 10, seed=7)
    tf.keras.backend.clear_session()
    m = build()
    m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tf.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9))
    e = m._get_engine(32, 32)
    assert e.name == "native_graph" and sum(1 for nd in e.nodes if "bnin" in nd.attrs) >= 2
    init = m.get_weights()
    wf, hf, _ = _train(build, x, y, init, 32, 2, native=True, momentum=0.9)
    wu, hu, _ = _train(build, x, y, init, 32, 2, native=True, momentum=0.9, extra_env={"DAMD_BN_CONV_FOLD": "0"})
    for a, b in zip(wf, wu):
        np.testing.assert_array_equal(a, b)
    assert hf == hu


def test_dual_bn_backward_is_bitwise():
    """The two BatchNorms of every downsampling block's output relu(BN(conv) + BN(shortcut))
    go through ONE reduce and ONE apply launch (bn_bwd_reduce_dual / bn_bwd_apply_dual) ==
    the four single-BN launches (DAMD_BN_DUAL=0), bitwise over two momentum steps; the dual
    path must actually be taken (3 downsampling blocks)."""
    from distributed_amd.engine import native_graph as ng

    calls = []
    orig = ng.NativeGraphEngine._bn_backward_dual

    def spy(self, *a, **k):
        r = orig(self, *a, **k)
        calls.append(r)
        return r

    x, y = _data(64, (32, 32, 3), 10, seed=12)
    tf.keras.backend.clear_session()
    init = _small_resnet().get_weights()
    ng.NativeGraphEngine._bn_backward_dual = spy
    try:
        wd, hd, ed = _train(_small_resnet, x, y, init, 32, 2, native=True, momentum=0.9)
    finally:
        ng.NativeGraphEngine._bn_backward_dual = orig
    assert calls and any(calls), calls
    ws, hs, es = _train(_small_resnet, x, y, init, 32, 2, native=True, momentum=0.9,
                        extra_env={"DAMD_BN_DUAL": "0"})
    assert ed == es == "native_graph"
    for a, b in zip(wd, ws):
        np.testing.assert_array_equal(a, b)
    assert hd == hs


@pytest.mark.parametrize("allreduce", [False, True])
def test_weight_gradients_on_side_stream_are_bitwise(monkeypatch, allreduce):
    """DAMD_WGRAD_STREAM=1: every conv weight gradient (+ split-K reduce) on a side stream
    beside the backprop-input / BN chain (own workspace, joined before the optimizer; with
    DAMD_FORCE_ALLREDUCE each bucket all-reduce also waits on it) == the single-stream
    step, bitwise over two momentum steps (graph replay)."""
    def build():
        return resnet18(classes=10, input_shape=(64, 64, 3), widths=(64, 64, 128, 128), blocks=(2, 1, 1, 1))

    monkeypatch.setenv("DAMD_CONV3_MIN_WG", "1")
    x, y = _data(64, (64, 64, 3), 10, seed=11)
    tf.keras.backend.clear_session()
    init = build().get_weights()
    extra = {"DAMD_FORCE_ALLREDUCE": "1", "DAMD_BUCKET_MB": "0.05"} if allreduce else {}
    ws, hs, es = _train(build, x, y, init, 32, 3, native=True, momentum=0.9,
                        extra_env={**extra, "DAMD_WGRAD_STREAM": "1"})
    w1, h1, e1 = _train(build, x, y, init, 32, 3, native=True, momentum=0.9,
                        extra_env={**extra, "DAMD_WGRAD_STREAM": "0"})
    assert es == e1 == "native_graph"
    for a, b in zip(ws, w1):
        np.testing.assert_array_equal(a, b)
    assert hs == h1


def test_logits_bias_gradient_from_the_loss_launch_is_bitwise(monkeypatch):
    """The logits layer's bias gradient summed in the loss launch's last block (no colsum
    launch, DAMD_XENT_BIAS=1, default) == the colsum launch (DAMD_XENT_BIAS=0), bitwise over
    momentum steps with 1000 classes (the ResNet-18 head width) and with the stem's padded
    weights refreshed in the gather launch."""
    def build():
        return resnet18(classes=1000, input_shape=(64, 64, 3), widths=(64, 64, 128, 128), blocks=(1, 1, 1, 1))

    x, y = _data(64, (64, 64, 3), 1000, seed=12)
    tf.keras.backend.clear_session()
    init = build().get_weights()
    wf, hf, ef = _train(build, x, y, init, 32, 3, native=True, momentum=0.9, extra_env={"DAMD_XENT_BIAS": "1"})
    wc, hc, ec = _train(build, x, y, init, 32, 3, native=True, momentum=0.9, extra_env={"DAMD_XENT_BIAS": "0"})
    assert ef == ec == "native_graph"
    for a, b in zip(wf, wc):
        np.testing.assert_array_equal(a, b)
    assert hf == hc


def test_resnet18_full_size_trains():
    x, y = _data(64, (224, 224, 3), 1000, seed=3)
    tf.keras.backend.clear_session()
    os.environ["DAMD_FUSED"] = "0"
    try:
        m = resnet18()
        m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tf.keras.optimizers.SGD(learning_rate=0.02, momentum=0.9), metrics=["accuracy"])
        # 64 fixed images: memorising them drives the loss down within a few epochs
        h = m.fit(x, y, batch_size=32, epochs=6, steps_per_epoch=2, verbose=0)
    finally:
        os.environ.pop("DAMD_FUSED", None)
    assert m._engine.name == "native_graph"
    assert all(np.isfinite(h.history["loss"]))
    assert min(h.history["loss"][-2:]) < h.history["loss"][0]


@pytest.mark.parametrize("which", ["native_graph", "fused_convnet"])
def test_rccl_allreduce_captured_in_step_graph(which):
    """The multi-GPU step shape on one GPU: DAMD_FORCE_ALLREDUCE keeps the (size-1) RCCL
    all-reduce inside the captured step — for the native engine as many small buckets on
    a side stream (fork/join inside the graph).  Must equal the run without it."""
    if which == "native_graph":
        build, shape, batch, steps = _small_resnet, (32, 32, 3), 32, 2
        x, y = _data(64, shape, 10, seed=5)
    else:
        build, shape, batch, steps = _mnist, (28, 28, 1), 64, 45  # 2 captured graphs of 20 + eager tail
        x, y = _data(64 * 45, shape, 10, seed=5)
    tf.keras.backend.clear_session()
    init = build().get_weights()
    kw = dict(native=which == "native_graph", fused=which == "fused_convnet",
              lr=0.05 if which == "native_graph" else 0.005, momentum=0.9)
    wa, ha, ea = _train(build, x, y, init, batch, steps,
                        extra_env={"DAMD_FORCE_ALLREDUCE": "1", "DAMD_BUCKET_MB": "0.02"}, **kw)
    wb, hb, eb = _train(build, x, y, init, batch, steps, **kw)
    assert ea == eb == which
    # fused engine: F3 adds the conv weight/bias gradient partials with fp32 atomics (order
    # not fixed), and 45 momentum steps amplify that rounding noise on the small conv bias
    tol = dict(rtol=1e-4, atol=1e-5) if which == "native_graph" else dict(rtol=1e-3, atol=5e-4)
    for a, b in zip(wa, wb):
        np.testing.assert_allclose(a, b, **tol)
    np.testing.assert_allclose(ha["loss"], hb["loss"], rtol=1e-4)


def test_u8_batch_gather_matches_float_feed():
    """k/255 inputs kept on the device as uint8 (4-pixel dword gather into the packed
    4-channel stem layout) == the fp32 device copy: one step, same weights and loss."""
    x, y = _data(64, (32, 32, 3), 10, seed=8)
    tf.keras.backend.clear_session()
    init = _small_resnet().get_weights()
    wa, ha, ea = _train(_small_resnet, x, y, init, 32, 2, native=True, momentum=0.9)
    wb, hb, eb = _train(_small_resnet, x, y, init, 32, 2, native=True, momentum=0.9,
                        extra_env={"DAMD_X_U8": "0"})
    assert ea == eb == "native_graph"
    for a, b in zip(wa, wb):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(ha["loss"], hb["loss"], rtol=1e-6)


def test_phase_times_native_graph():
    import numpy as np
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import distributed_amd as tf
    from distributed_amd.utils.profile import step_phases

    tf.set_seed(3)
    m = tf.models.resnet18(classes=10, input_shape=(32, 32, 3), widths=(16, 32, 32, 64), blocks=(1, 1, 1, 1))
    tf.models.compile_resnet(m, 0.05, 0.9)
    rng = np.random.default_rng(0)
    x = rng.random((256, 32, 32, 3), dtype=np.float32)
    y = rng.integers(0, 10, 256)
    ph = step_phases(m, x, y, batch_size=32, steps=4)
    print("native graph phases (ms):", ph)
    assert ph["engine"] == "native_graph"
    for k in ("forward", "backward", "allreduce", "optimizer"):
        assert ph[k] >= 0
    assert ph["forward"] > 0 and ph["backward"] > 0


def _captured_step_nodes(extra_env):
    """(engine, graph nodes) of one captured step of the small ResNet with extra_env."""
    env = {"DAMD_NATIVE_GRAPH": "1", "DAMD_FUSED": "0", **extra_env}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        from distributed_amd.parallel import runtime

        runtime.shutdown()
        tf.keras.backend.clear_session()
        m = _small_resnet()
        m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tf.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9), metrics=["accuracy"])
        x, y = _data(64, (32, 32, 3), 10, seed=5)
        m.fit(x, y, batch_size=32, epochs=1, steps_per_epoch=1, verbose=0)  # eager first step: plan validated
        eng = m._engine
        assert eng.name == "native_graph"
        return eng, eng.graph_nodes()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_bucket_collectives_and_updates_depend_only_on_their_backward():
    """VERDICT r5 task 3: with one RCCL communicator per gradient bucket (DAMD_FORCE_ALLREDUCE
    keeps the size-1 RCCL all-reduces in the captured step on one GPU), no bucket's
    collective or optimizer update waits on another bucket's: in the captured hipGraph
    every RCCL node and every per-bucket opt_step node has exactly ONE dependency (the work
    that wrote the bucket, resp. the bucket's own all-reduce), and no RCCL node depends on
    another RCCL node.  Printed: the node summary, for the round's profile notes."""
    from distributed_amd.parallel import runtime

    try:
        eng, nodes = _captured_step_nodes({"DAMD_FORCE_ALLREDUCE": "1", "DAMD_BUCKET_MB": "0.05"})
        nb = len(eng._buckets)
        assert nb >= 3 and len(eng.bucket_comms) == nb and eng.bucket_opt
        names = [n[1] for n in nodes]
        coll = [i for i, n in enumerate(nodes) if "nccl" in n[1].lower() or "rccl" in n[1].lower()]
        opt = [i for i, n in enumerate(nodes) if "opt_step_k" in n[1]]
        kinds = {}
        for t, nm, _ in nodes:
            k = nm.split("(")[0][-40:] if nm else f"type{t}"
            kinds[k] = kinds.get(k, 0) + 1
        print(f"{len(nodes)} nodes, {nb} buckets, {len(coll)} RCCL nodes, {len(opt)} opt_step nodes")
        print({k: v for k, v in kinds.items() if "damd" not in k})
        assert len(opt) == nb, (len(opt), nb)
        for i in opt:
            assert len(nodes[i][2]) == 1, (names[i], nodes[i][2])
        cset = set(coll)
        for i in coll:
            assert len(nodes[i][2]) == 1, (names[i], [names[d] for d in nodes[i][2]])
            assert not (set(nodes[i][2]) & cset), "an RCCL node depends on another RCCL node (chain)"
        # the round-5 chain for contrast (one shared communicator, one comm stream)
        eng2, nodes2 = _captured_step_nodes({"DAMD_FORCE_ALLREDUCE": "1", "DAMD_BUCKET_MB": "0.05",
                                             "DAMD_BUCKET_COMMS": "0"})
        c2 = [i for i, n in enumerate(nodes2) if "nccl" in n[1].lower() or "rccl" in n[1].lower()]
        print(f"shared communicator: {len(c2)} RCCL nodes, dependencies {[len(nodes2[i][2]) for i in c2]}")
        assert not eng2.bucket_comms
    finally:
        runtime.shutdown()
