"""Fused MNIST-CNN HIP kernels vs a plain PyTorch fp32 reference of the same step."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _model(lr=0.1, momentum=0.0, nesterov=False, seed=3):
    """seed=None: a fresh initial draw from os.urandom, printed so a failure can be replayed
    (the tolerance tests run several of them: their bounds must hold for any draw)."""
    import os

    import distributed_amd as tf

    if seed is None:
        seed = int.from_bytes(os.urandom(4), "little")
        print(f"init seed {seed}")
    tf.set_seed(seed)
    m = tf.models.mnist_cnn()
    m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tf.keras.optimizers.SGD(learning_rate=lr, momentum=momentum, nesterov=nesterov),
              metrics=["accuracy"])
    return m


def _data(n=512, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.random((n, 28, 28, 1), dtype=np.float32)
    y = rng.integers(0, 10, n).astype(np.int64)
    return x, y


def _bf16(t):
    return t.to(torch.bfloat16).to(t.dtype)


def _ref_step(ws, xb, yb, gcount, quant=False):
    """fp64 torch reference of one step: returns (grads, loss_sum, correct).

    ``quant=True`` mirrors the kernels' deliberate bf16 quantisation points (the pooled
    activations and W1 enter the dense-1 MFMAs as bf16, with straight-through
    gradients), so what remains is accumulation-order noise; ``quant=False`` is the
    plain fp64 model."""
    from distributed_amd.ops import reference as R

    ts = [torch.tensor(w, dtype=torch.float64, requires_grad=True) for w in ws]
    x = torch.tensor(xb, dtype=torch.float64)
    h = torch.relu(R.conv2d(x, ts[0], ts[1]))
    p = R.maxpool2d(h)
    f = p.reshape(p.shape[0], -1)
    w1 = ts[2]
    if quant:
        f = f + (_bf16(f) - f).detach()
        w1 = w1 + (_bf16(w1) - w1).detach()
    d = torch.relu(f @ w1 + ts[3])
    z = d @ ts[4] + ts[5]
    ls = torch.nn.functional.cross_entropy(z, torch.tensor(yb), reduction="none")
    (ls.sum() / gcount).backward()
    corr = float((z.argmax(-1) == torch.tensor(yb)).sum())
    return [t.grad.numpy() for t in ts], float(ls.detach().sum()), corr


def _engine(model, B):
    from distributed_amd.parallel.strategy import get_strategy

    eng = model._get_engine(B, B)
    assert eng.name == "fused_convnet", "fused engine must be selected on GPU"
    return eng


@pytest.mark.parametrize("B,pp", [(64, 3), (40, 3), (100, 3), (64, 4), (100, 2), (64, 1)])
def test_one_step_matches_reference(B, pp, monkeypatch):
    """pp = pooled positions per fused slice (DAMD_PP; 3 is the default: 57 slices, the
    last one partial).  Two unpinned initial draws per shape: the bounds hold for any."""
    _need_gpu()
    monkeypatch.setenv("DAMD_GRAPH", "0")
    monkeypatch.setenv("DAMD_PP", str(pp))
    for _ in range(2):
        _one_step_vs_reference(B)


def _one_step_vs_reference(B):
    lr = 0.5
    m = _model(lr=lr, seed=None)
    x, y = _data(300)
    w0 = m.get_weights()
    eng = _engine(m, B)
    eng.bind(x, y)
    eng.start_epoch(0, shuffle=False)
    eng.run(1)
    met = eng.end_epoch()
    eng.finish()
    w1 = m.get_weights()
    names = ["wc", "bc", "w1", "b1", "w2", "b2"]

    def rel_errs(grads):
        out, cols = {}, {}
        for a, b, g, name in zip(w0, w1, grads, names):
            est = (a - b) / lr
            out[name] = float(np.linalg.norm(est - g) / (np.linalg.norm(g) + 1e-12))
            E, G = est.reshape(-1, est.shape[-1]), g.reshape(-1, g.shape[-1])
            ce = np.linalg.norm(E - G, axis=0) / (np.linalg.norm(G, axis=0) + 1e-12)
            cols[name] = float((ce < 1e-2).mean())  # fraction of output columns within 1e-2
        return out, cols

    # Bounds from a 60-draw sweep (scripts/sweep_fused_ref.py, round 4).  For most draws
    # every tensor agrees with the bf16-mirrored reference to ~1e-3, but a dense-1
    # pre-activation within rounding distance of 0 flips its ReLU between the kernels'
    # fp32 sums and the fp64 reference: that hidden unit's column of dW1 / db1 differs
    # (worst draw: 1 of 64 columns, whole tensor 4.9e-2), and through dh the conv
    # gradient shifts as a whole (4.5e-2).  So: dW1 / db1 column-wise (>= 95 % of the 64
    # hidden units within 1e-2 -- a wiring error moves every column), W2 / b2 (downstream
    # of no flip-prone decision but the argmax-free softmax) tightly, the conv gradient
    # and the whole tensors loosely; vs plain fp64 (the cost of bf16 dense compute) the
    # sweep's worst tensor is 0.104.
    gq, lsum, corr = _ref_step(w0, x[:B], y[:B], B, quant=True)
    eq, cq = rel_errs(gq)
    print("vs bf16-mirrored reference:", {k: f"{v:.2e}" for k, v in eq.items()}, "columns within 1e-2:", cq)
    assert cq["w1"] >= 0.95 and cq["b1"] >= 0.95, cq
    assert eq["w2"] < 5e-3 and eq["b2"] < 5e-3, eq
    assert max(eq.values()) < 0.1, eq
    g64, _, _ = _ref_step(w0, x[:B], y[:B], B, quant=False)
    e64, _ = rel_errs(g64)
    print("vs fp64 reference:", {k: f"{v:.2e}" for k, v in e64.items()})
    assert max(e64.values()) < 0.2, e64
    assert abs(met["loss"] - lsum / B) < 2e-2
    assert abs(met["accuracy"] - corr / B) < 1.5 / B


def test_graph_replay_bitwise_equals_eager(monkeypatch):
    _need_gpu()
    x, y = _data(2000)
    res = []
    for graph in ("0", "1"):
        monkeypatch.setenv("DAMD_GRAPH", graph)
        monkeypatch.setenv("DAMD_GRAPH_STEPS", "4")
        m = _model(lr=0.05, momentum=0.9, seed=11)
        eng = _engine(m, 64)
        eng.bind(x, y)
        eng.start_epoch(0, shuffle=True)
        eng.run(10)
        met = eng.end_epoch()
        eng.finish()
        res.append((np.concatenate([w.ravel() for w in m.get_weights()]), met))
    # the 2-launch step combines every cross-block sum as int64 fixed point: graph replay
    # and eager launches give the same bits
    np.testing.assert_array_equal(res[0][0], res[1][0])
    assert res[0][1]["loss"] == res[1][1]["loss"]


_DRAWS = range(int(os.environ.get("DAMD_TEST_DRAWS", "3")))  # fresh initial draws per test


def _check_updates(w0, got, ref, what):
    """Momentum-mechanics tests: the engine's total update (got - w0) against the fp64
    reference's (ref - w0).  A dense-1 ReLU decision within rounding distance of 0 flips for
    some draws and perturbs the later steps (the bias vectors, starting at 0, carry the
    largest relative share), so the check is on the concatenated update vector plus loose
    per-kernel bounds.  30-draw sweeps (round 4, DAMD_TEST_DRAWS=30): 3 Nesterov steps
    whole-update cos >= 0.9985, rel <= 0.055, kernels <= 0.056; 2 + 2 steps across a flush
    cos >= 0.975, rel <= 0.222, kernels <= 0.22 -- the bounds below hold for any draw, and
    the mechanics themselves are pinned exactly (bitwise) where the test can do so."""
    du = [(a - b0).ravel() for a, b0 in zip(got, w0)]
    dr = [(b - b0).ravel() for b, b0 in zip(ref, w0)]
    A, B = np.concatenate(du), np.concatenate(dr)
    cos = float(A @ B / (np.linalg.norm(A) * np.linalg.norm(B)))
    rel = float(np.linalg.norm(A - B) / np.linalg.norm(B))
    per = [float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-12)) for a, b in zip(du, dr)]
    print(f"{what}: whole-update cos {cos:.5f} rel {rel:.4f}; per tensor", [f"{e:.1e}" for e in per])
    assert cos > 0.95 and rel < 0.35, (cos, rel)
    assert max(per[0], per[2], per[4]) < 0.35, per  # the kernels wc, W1, W2


@pytest.mark.parametrize("draw", _DRAWS)
def test_momentum_three_steps(monkeypatch, draw):
    _need_gpu()
    monkeypatch.setenv("DAMD_GRAPH", "0")
    lr, mom = 0.1, 0.9
    m = _model(lr=lr, momentum=mom, nesterov=True, seed=None)
    x, y = _data(256)
    w = [a.astype(np.float64) for a in m.get_weights()]
    v = [np.zeros_like(a) for a in w]
    eng = _engine(m, 64)
    eng.bind(x, y)
    eng.start_epoch(0, shuffle=False)
    eng.run(3)
    eng.end_epoch()
    eng.finish()
    w0 = [a.copy() for a in w]
    for s in range(3):
        g, _, _ = _ref_step(w, x[s * 64:(s + 1) * 64], y[s * 64:(s + 1) * 64], 64, quant=True)
        for i in range(6):
            v[i] = mom * v[i] - lr * g[i]
            w[i] = w[i] + mom * v[i] - lr * g[i]
    _check_updates(w0, m.get_weights(), w, "nesterov, 3 steps")


def test_fit_reference_script_on_gpu(capsys):
    _need_gpu()
    import distributed_amd as tf

    (x, y), _ = tf.keras.datasets.mnist.load_data()
    x = x.reshape(len(x), 28, 28, 1) / 255.0
    m = _model(lr=0.001)
    h = m.fit(x, y, batch_size=64, epochs=3, steps_per_epoch=5)
    assert m._engine.name == "fused_convnet"
    assert len(h.history["loss"]) == 3
    assert all(abs(l - 2.30) < 0.1 for l in h.history["loss"])
    out = capsys.readouterr().out
    assert "Train on 60000 samples" in out and "320/60000" in out


def test_fit_learns_synthetic(monkeypatch):
    _need_gpu()
    import distributed_amd as tf

    (x, y), _ = tf.keras.datasets.mnist.load_data()
    x = x.reshape(len(x), 28, 28, 1) / 255.0
    m = _model(lr=0.05, momentum=0.9)
    h = m.fit(x, y, batch_size=64, epochs=2, steps_per_epoch=300, verbose=0)
    assert h.history["loss"][-1] < 1.0
    assert h.history["accuracy"][-1] > 0.6
    ev = m.evaluate(x[:2000], y[:2000], verbose=0)
    assert ev[1] > 0.6


def test_native_module_loaded():
    _need_gpu()
    import sys

    import distributed_amd.native as n

    C = n.require_C()
    assert C.__file__.endswith(".so")
    assert any(k.startswith("distributed_amd._C") for k in sys.modules)


def test_uint8_dataset_path_matches_fp32(monkeypatch):
    """Inputs that are exactly k/255 are kept as uint8 on device; results must equal the fp32
    path bitwise (k/255.f is formed exactly as the fp32 dataset holds it)."""
    _need_gpu()
    monkeypatch.setenv("DAMD_GRAPH", "0")
    rng = np.random.default_rng(7)
    x = rng.integers(0, 256, (512, 28, 28, 1)).astype(np.uint8) / 255.0
    y = rng.integers(0, 10, 512)
    out = []
    for u8 in ("1", "0"):
        monkeypatch.setenv("DAMD_X_U8", u8)
        m = _model(lr=0.1, seed=21)
        eng = _engine(m, 64)
        eng.bind(x, y)
        assert eng.feed.x_u8 == (u8 == "1")
        eng.start_epoch(0, shuffle=False)
        eng.run(3)
        eng.end_epoch()
        eng.finish()
        out.append(np.concatenate([w.ravel() for w in m.get_weights()]))
    np.testing.assert_array_equal(out[0], out[1])


@pytest.mark.parametrize("draw", _DRAWS)
def test_momentum_across_epoch_flushes(monkeypatch, draw):
    """An epoch end applies the pending (deferred) update; the first step of the next
    epoch must then apply none -- with momentum a zero-gradient update would still move
    the weights (v <- m v; w += v).  Exact: 2 epochs x 2 steps over 128 rows == one epoch
    of 4 steps over the same rows twice (the same updates, only the epoch boundary and its
    flush differ); loose: against the fp64 reference (flip-prone, see _check_updates)."""
    _need_gpu()
    monkeypatch.setenv("DAMD_GRAPH", "0")
    lr, mom = 0.1, 0.9
    seed = int.from_bytes(os.urandom(4), "little")
    print(f"init seed {seed}")
    x, y = _data(128)
    outs = []
    for split in (True, False):
        m = _model(lr=lr, momentum=mom, seed=seed)
        eng = _engine(m, 64)
        if split:
            eng.bind(x, y)
            w_init = m.get_weights()
            for ep in range(2):
                eng.start_epoch(ep, shuffle=False)
                eng.run(2)
                eng.end_epoch()
        else:
            eng.bind(np.concatenate([x, x]), np.concatenate([y, y]))
            eng.start_epoch(0, shuffle=False)
            eng.run(4)
            eng.end_epoch()
        eng.finish()
        outs.append(m.get_weights())
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)
    w = [a.astype(np.float64) for a in w_init]
    v = [np.zeros_like(a) for a in w]
    w0 = [a.copy() for a in w]
    for s in range(4):
        lo = (s % 2) * 64
        g, _, _ = _ref_step(w, x[lo:lo + 64], y[lo:lo + 64], 64, quant=True)
        for i in range(6):
            v[i] = mom * v[i] - lr * g[i]
            w[i] = w[i] + v[i]
    _check_updates(w0, m.get_weights(), w, "momentum across flushes")


def test_training_is_bitwise_reproducible(monkeypatch):
    """Same seed, same data -> the same bits after 12 steps (no order-dependent sums)."""
    _need_gpu()
    x, y = _data(1024)
    outs = []
    for _ in range(2):
        m = _model(lr=0.05, momentum=0.9, seed=13)
        eng = _engine(m, 64)
        eng.bind(x, y)
        eng.start_epoch(0, shuffle=True)
        eng.run(12)
        met = eng.end_epoch()
        eng.finish()
        outs.append((np.concatenate([w.ravel() for w in m.get_weights()]), met["loss"]))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]


def test_phase_times_fused_step():
    """HIP-event phase split of the 2-launch step: forward, backward, all-reduce (world 1:
    none) -- and the steps it ran are real training steps."""
    _need_gpu()
    m = _model(lr=0.05)
    x, y = _data(1024)
    eng = _engine(m, 64)
    eng.bind(x, y)
    eng.start_epoch(0, shuffle=False)
    it0 = int(m.optimizer.iterations)
    ph = eng.phase_times(5)
    eng.end_epoch()
    print("fused step phases (ms):", ph)
    assert ph["forward"] > 0 and ph["backward"] > 0 and ph["allreduce"] >= 0
    assert int(m.optimizer.iterations) == it0 + 5


@pytest.mark.parametrize("nesterov", [False, True])
def test_eager_w1_update_bitwise_equals_deferred(nesterov, monkeypatch):
    """World 1: bwd applies the W1 update as soon as it has the slice's gradient and fwd
    reads only the bf16 copy (DAMD_EAGER_W1, default); the same arithmetic as the deferred
    update in the next fwd, so the runs agree bitwise -- across graph replays, an epoch
    flush and a host-side set_weights (which must refresh the bf16 copy)."""
    _need_gpu()
    monkeypatch.setenv("DAMD_GRAPH_STEPS", "4")
    x, y = _data(1024)
    res = []
    for eager in ("1", "0"):
        monkeypatch.setenv("DAMD_EAGER_W1", eager)
        m = _model(lr=0.05, momentum=0.9, nesterov=nesterov, seed=5)
        eng = _engine(m, 64)
        assert eng.eager_w1 == (eager == "1")
        eng.bind(x, y)
        eng.start_epoch(0, shuffle=True)
        eng.run(9)
        met0 = eng.end_epoch()
        w = m.get_weights()
        w[2] = w[2] * 0.5  # host write of W1 between epochs
        m.set_weights(w)
        eng.start_epoch(1, shuffle=True)
        eng.run(7)
        met1 = eng.end_epoch()
        eng.finish()
        res.append((np.concatenate([v.ravel() for v in m.get_weights()]), met0, met1))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1] and res[0][2] == res[1][2]


def test_final_graph_equals_run_then_flush(monkeypatch):
    """prepare_final / run_and_flush (k steps + the flush of the last deferred update in
    one captured graph, bench.py's timed region) == run(k) then the eager flush, bitwise,
    weights and epoch metrics; a count without a final graph falls back to run + flush."""
    _need_gpu()
    monkeypatch.setenv("DAMD_GRAPH_STEPS", "5")
    x, y = _data(2000)
    res = []
    for final in (True, False):
        m = _model(lr=0.05, momentum=0.9, seed=29)
        eng = _engine(m, 64)
        eng.bind(x, y)
        eng.start_epoch(0, shuffle=True)
        eng.prepare(5)
        if final:
            assert eng.prepare_final(12)
        eng.run(5)
        if final:
            eng.run_and_flush(12)
            assert not eng._pending
            eng.run_and_flush(3)  # no 3-step final graph: run + flush
        else:
            eng.run(12)
            eng._flush()
            eng.run(3)
            eng._flush()
        met = eng.end_epoch()
        eng.finish()
        res.append((np.concatenate([w.ravel() for w in m.get_weights()]), met))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    assert res[0][1]["loss"] == res[1][1]["loss"] and res[0][1]["accuracy"] == res[1][1]["accuracy"]


@pytest.mark.parametrize("where", ["w1", "conv", "b1"])
def test_nonfinite_weight_reports_nan_loss(where, monkeypatch):
    """the fixed-point cross-block sums cannot carry NaN / inf, so a non-finite
    value raises the sticky ctrl.bad flag and the loss reads NaN (as the fp32 engines show
    it) instead of finite garbage; TerminateOnNaN then stops fit.  New weights clear it."""
    _need_gpu()
    import distributed_amd as tf

    x, y = _data(512)
    m = _model(lr=0.1)
    ws = m.get_weights()
    if where == "w1":
        ws[2][7, 3] = np.nan
    elif where == "conv":
        ws[0][1, 1, 0, 5] = np.inf  # the conv's ReLU (fmaxf) alone would map the NaN products to 0
    else:
        ws[3][5] = np.nan           # as would the head's ReLU for a NaN b1
    m.set_weights(ws)
    h = m.fit(x, y, batch_size=64, epochs=2, steps_per_epoch=2, verbose=0,
              callbacks=[tf.keras.callbacks.TerminateOnNaN()])
    assert m._engine.name == "fused_convnet"
    assert np.isnan(h.history["loss"][0])
    assert len(h.history["loss"]) == 1  # TerminateOnNaN stopped training after epoch 1
    m.set_weights(_model(lr=0.1).get_weights())
    h = m.fit(x, y, batch_size=64, epochs=1, steps_per_epoch=2, verbose=0)
    assert np.isfinite(h.history["loss"][0])


@pytest.mark.parametrize("B", [64, 40])
def test_prefetch_and_parity_hints_are_bitwise_neutral(B, monkeypatch):
    """The next-batch prefetch (bwd copies the next step's rows, tagged; the fwd stages this
    step's rows / labels for the bwd) and the host-known step parity passed to the kernels
    (graphs captured per parity) change only WHERE loads come from: the same bits as the
    plain path (DAMD_XPREFETCH=0 DAMD_PAR_HINT=0), over odd-length graph replays, eager
    steps, an epoch change (new rows: the prefetch must miss) and the final-graph path; and
    no parity mismatch is ever flagged (ctrl.bad stays 0: the loss is finite)."""
    _need_gpu()
    x, y = _data(1000)  # 1000 / B: a short last batch at B = 64
    outs = []
    for plain in (False, True):
        monkeypatch.setenv("DAMD_XPREFETCH", "0" if plain else "1")
        monkeypatch.setenv("DAMD_PAR_HINT", "0" if plain else "1")
        monkeypatch.setenv("DAMD_GRAPH_STEPS", "3")
        m = _model(lr=0.05, momentum=0.9, seed=17)
        eng = _engine(m, B)
        eng.bind(x, y)
        mets = []
        for ep in range(2):
            eng.start_epoch(ep, shuffle=True)
            eng.prepare(3)
            eng.run(7)        # 2 replays of the 3-step graph (parities 0 / 1) + 1 eager step
            eng.trainer.step(2)
            eng._pending = True
            mets.append(eng.end_epoch())
        eng.start_epoch(2, shuffle=True)
        if eng.prepare_final(5):
            eng.run_and_flush(5)
        mets.append(eng.metrics())
        eng.finish()
        assert all(np.isfinite(mt["loss"]) for mt in mets), mets
        outs.append((np.concatenate([w.ravel() for w in m.get_weights()]), [mt["loss"] for mt in mets]))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]
