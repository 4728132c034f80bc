"""Native-engine coverage beyond the ResNet/MNIST layer set: Adam and
RMSprop in the flat opt_step kernel, sigmoid / tanh activations, AveragePooling2D and
Dropout -- kernel numerics against plain PyTorch fp32, and whole training runs of the
native graph engine against the fp32 generic engine on the CPU."""
import numpy as np
import pytest
import torch

import distributed_amd as tf
from distributed_amd.ops import hip as H
from distributed_amd.ops import reference as R

from test_native_graph_gpu import _compare_updates, _data, _mnist, _train

pytestmark = pytest.mark.gpu
dev = "cuda"


def _bf(t):
    return t.to(dev).bfloat16().contiguous()


@pytest.mark.parametrize("kind", ["relu", "sigmoid", "tanh"])
def test_act_kernels_match_torch(kind):
    torch.manual_seed(0)
    n = 8 * 1000 + 5  # a partial last group of 8
    x = torch.randn(n) * 3
    xb = _bf(x)
    y = torch.empty_like(xb)
    H.act_fwd(xb, y, kind)
    f = {"relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh}[kind]
    ref = f(xb.float())
    torch.testing.assert_close(y.float(), ref, atol=1e-2, rtol=1e-2)
    dy = _bf(torch.randn(n))
    dx = torch.empty_like(dy)
    H.act_bwd(dy, y, dx, kind)
    yf = y.float()
    d = {"relu": (yf > 0).float(), "sigmoid": yf * (1 - yf), "tanh": 1 - yf * yf}[kind]
    torch.testing.assert_close(dx.float(), dy.float() * d, atol=1e-2, rtol=1e-2)
    # in place (the Conv2D / Dense epilogue use)
    z = xb.clone()
    H.act_fwd(z, z, kind)
    assert torch.equal(z, y)


@pytest.mark.parametrize("pool,strides,padding", [((2, 2), (2, 2), "valid"), ((3, 3), (2, 2), "same"),
                                                  ((3, 3), (1, 1), "same"), ((2, 2), (1, 1), "valid")])
def test_avgpool_kernels_match_torch(pool, strides, padding):
    torch.manual_seed(1)
    x = torch.randn(3, 11, 13, 16)
    xb = _bf(x)
    g = H.pool_geo(xb.shape, pool, strides, padding)
    y = torch.empty(3, g[10], g[11], 16, device=dev, dtype=torch.bfloat16)
    H.avgpool_fwd(xb, y, pool, strides, padding)
    xr = xb.float().cpu().requires_grad_(True)
    yr = R.avgpool2d(xr, pool, strides, padding)
    torch.testing.assert_close(y.float().cpu(), yr.detach(), atol=2e-2, rtol=1e-2)
    dy = torch.randn_like(yr)
    yr.backward(dy)
    dx = torch.empty_like(xb)
    H.avgpool_bwd(_bf(dy), dx, pool, strides, padding)
    dyq = _bf(dy).float().cpu()
    xr2 = xb.float().cpu().requires_grad_(True)
    R.avgpool2d(xr2, pool, strides, padding).backward(dyq)
    torch.testing.assert_close(dx.float().cpu(), xr2.grad, atol=2e-2, rtol=1e-2)


def test_dropout_kernel_matches_host_mask():
    n, rate, seed = 8 * 4096 + 3, 0.3, 1234
    x = _bf(torch.randn(n))
    ctrl = torch.zeros(32, dtype=torch.int32, device=dev)
    outs = []
    for t in (1, 2):
        ctrl[15] = t  # Ctrl::cur3, the step's iteration
        y = torch.empty_like(x)
        H.dropout(x, y, ctrl, seed, rate)
        keep = torch.from_numpy(H.dropout_mask_reference(n, seed, t, rate)).to(dev)
        ref = torch.where(keep, (x.float() * (1 / (1 - rate))).bfloat16(), torch.zeros_like(x))
        assert torch.equal(y, ref)
        assert abs(keep.float().mean().item() - (1 - rate)) < 0.01
        outs.append(keep)
    assert (outs[0] != outs[1]).float().mean().item() > 0.3  # a fresh mask per step


@pytest.mark.parametrize("name", ["adam", "adam_amsgrad", "rmsprop", "rmsprop_momentum", "rmsprop_centered_momentum",
                                  "sgd_nesterov"])
def test_opt_step_kernel_matches_apply_flat(name):
    """The flat opt_step kernel against the Keras optimizer's own fp32 apply_flat, three
    consecutive steps from the same P / G / slots (exact up to fp32 rounding)."""
    import struct

    from distributed_amd.engine.native_graph import _opt_kernel_slots
    from distributed_amd.native import require_C

    C = require_C()
    n = 10007
    torch.manual_seed(2)
    opt_d, opt_h = _opt_cases()[name](), _opt_cases()[name]()
    kind, names = _opt_kernel_slots(opt_d)
    p0 = torch.randn(n)
    ph = p0.clone()
    opt_h.ensure_slots(n, torch.device("cpu"))
    P = p0.clone().to(dev)
    Pb = torch.empty(n, dtype=torch.bfloat16, device=dev)
    S = [torch.zeros(n, device=dev) for _ in range(3)]
    ctrl = torch.zeros(32, dtype=torch.int32, device=dev)
    ctrl[0] = struct.unpack("<i", struct.pack("<f", opt_h.learning_rate))[0]
    tail = torch.zeros(8, device=dev)
    if kind == 1:
        args = (opt_h.beta_1, opt_h.beta_2, opt_h.epsilon, 0.0, 0.0, int(opt_h.amsgrad))
    elif kind == 2:
        args = (0.0, 0.0, opt_h.epsilon, opt_h.rho, opt_h.momentum, int(opt_h.centered))
    else:
        args = (0.0, 0.0, 0.0, 0.0, opt_h.momentum, int(opt_h.nesterov))
    for t in range(1, 4):
        g = torch.randn(n) * (0.1 if t % 2 else 1.0) + 0.05
        ctrl[15] = t  # what gather_batch writes at the start of the step
        C.opt_step(P.data_ptr(), g.to(dev).data_ptr(), S[0].data_ptr(), S[1].data_ptr(), S[2].data_ptr(),
                   Pb.data_ptr(), n, ctrl.data_ptr(), tail.data_ptr(), kind, *map(float, args[:5]), args[5],
                   torch.cuda.current_stream().cuda_stream)
        opt_h.apply_flat(ph, g)
        torch.testing.assert_close(P.cpu(), ph, rtol=1e-5, atol=1e-6)
        assert int(ctrl[7]) == t  # iterations
        for i, nm in enumerate(names):
            if nm:
                torch.testing.assert_close(S[i].cpu(), opt_h.slots[nm], rtol=1e-5, atol=1e-7)
    assert torch.equal(Pb, P.bfloat16())


def _opt_cases(eps=1e-7):
    O = tf.keras.optimizers
    return {
        "adam": lambda: O.Adam(learning_rate=1e-3, epsilon=eps),
        "adam_amsgrad": lambda: O.Adam(learning_rate=1e-3, amsgrad=True, epsilon=eps),
        "rmsprop": lambda: O.RMSprop(learning_rate=1e-3, epsilon=eps),
        "rmsprop_momentum": lambda: O.RMSprop(learning_rate=5e-4, momentum=0.9, epsilon=eps),
        "rmsprop_centered_momentum": lambda: O.RMSprop(learning_rate=5e-4, momentum=0.9, centered=True, epsilon=eps),
        "sgd_nesterov": lambda: O.SGD(learning_rate=0.05, momentum=0.9, nesterov=True),
    }


@pytest.mark.parametrize("name", list(_opt_cases()))
def test_native_optimizers_track_reference(name):
    # This checks the engine's wiring (slots, step t, hyper-parameters, write-back); the
    # update rules themselves are pinned at the default epsilon by the kernel oracle
    # above.  epsilon 1e-2, not 1e-7: with a tiny epsilon Adam / RMSprop move every weight
    # by ~lr * sign(g), so weights whose gradient is ~0 follow the sign of the bf16 vs fp32
    # rounding noise (measured cos 0.885 at 1e-7, 0.926 at 1e-3 after 10 steps)
    # the bounds must hold for any initial draw: three unpinned inits in one process
    x, y = _data(640, (28, 28, 1), 10, seed=3)
    for rep in range(3):
        opt = _opt_cases(eps=1e-2)[name]
        tf.keras.backend.clear_session()
        init = _mnist().get_weights()
        wn, hn, en, on = _train(_mnist, x, y, init, 64, 10, native=True, optimizer=opt)
        wr, hr, er, orf = _train(_mnist, x, y, init, 64, 10, native=False, device="cpu", optimizer=opt)
        assert en == "native_graph" and er == "generic"
        assert on.iterations == orf.iterations == 10
        np.testing.assert_allclose(hn["loss"], hr["loss"], rtol=2e-2)
        # kernels 0.9 / 0.45; the 32-/64-/10-entry bias vectors are where the rounding-noise
        # share is largest (a bias gradient is a column sum of the bf16 dz: the adaptive
        # denominators turn its noise into O(lr) steps) -- measured down to cos 0.8998 on one
        # draw, so they get 0.8 / 0.65; the whole update vector (dominated by the 5408 x 64
        # dense kernel, so no tighter than the kernels' bound: RMSprop measured 0.926 on one
        # draw) to cos 0.9
        _compare_updates(init, wn, wr, ["k", "k1", "k2"], cos_min=0.9, rel_max=0.45,
                         idx=[0, 2, 4])
        _compare_updates(init, wn, wr, ["b", "b1", "b2"], cos_min=0.8, rel_max=0.65, idx=[1, 3, 5])
        da = np.concatenate([(a - w0).ravel() for a, w0 in zip(wn, init)]).astype(np.float64)
        db = np.concatenate([(b - w0).ravel() for b, w0 in zip(wr, init)]).astype(np.float64)
        assert float(da @ db / (np.linalg.norm(da) * np.linalg.norm(db))) > 0.9
        # the slots come back to the Keras optimizer in its dense (unpadded) layout
        for s in orf.slot_names():
            a, b = on.slots[s].cpu().double(), orf.slots[s].cpu().double()
            assert a.shape == b.shape
            assert float(a @ b / (a.norm() * b.norm() + 1e-30)) > 0.85, s


def _act_pool_model():
    L = tf.keras.layers
    return tf.keras.Sequential([
        L.Conv2D(16, 3, activation="tanh", input_shape=(16, 16, 3)),
        L.AveragePooling2D(pool_size=3, strides=2, padding="same"),
        L.Conv2D(16, 3, activation="sigmoid", padding="same"),
        L.Activation("tanh"),
        L.AveragePooling2D(),
        L.Flatten(),
        L.Dense(40, activation="sigmoid"),
        L.Dense(10),
    ])


def test_native_sigmoid_tanh_avgpool_track_reference():
    x, y = _data(256, (16, 16, 3), 10, seed=4)
    tf.keras.backend.clear_session()
    init = _act_pool_model().get_weights()
    wn, hn, en = _train(_act_pool_model, x, y, init, 32, 6, native=True, lr=0.2, momentum=0.9)
    wr, hr, er = _train(_act_pool_model, x, y, init, 32, 6, native=False, device="cpu", lr=0.2, momentum=0.9)
    assert en == "native_graph" and er == "generic"
    np.testing.assert_allclose(hn["loss"], hr["loss"], rtol=2e-2)
    _compare_updates(init, wn, wr, ["k", "b", "k1", "b1", "k2", "b2", "k3", "b3"], cos_min=0.95, rel_max=0.3)


def _dropout_model(rate):
    L = tf.keras.layers
    return tf.keras.Sequential([
        L.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
        L.MaxPooling2D(),
        L.Dropout(rate),
        L.Flatten(),
        L.Dense(64, activation="relu"),
        L.Dropout(rate, seed=7),
        L.Dense(10),
    ])


def test_native_dropout_trains_and_rate0_is_identity():
    x, y = _data(640, (28, 28, 1), 10, seed=5)
    tf.keras.backend.clear_session()
    init = _dropout_model(0.0).get_weights()
    # rate 0: the node is planned away; the run equals the dropout-free MNIST model's
    w0, h0, e0 = _train(lambda: _dropout_model(0.0), x, y, init, 64, 5, native=True, lr=0.05)
    w1, h1, e1 = _train(_mnist, x, y, init, 64, 5, native=True, lr=0.05)
    assert e0 == e1 == "native_graph"
    # identical plans, and every reduction of the native step is in a fixed order (the
    # bias column sums and the loss / metric sums included): bitwise the same run
    for a, b in zip(w0, w1):
        np.testing.assert_array_equal(a, b)
    assert h0["loss"] == h1["loss"]
    # rate 0.4: trains (loss falls over two epochs' worth of steps), differs from rate 0
    w2, h2, e2 = _train(lambda: _dropout_model(0.4), x, y, init, 64, 10, native=True, lr=0.05, momentum=0.9)
    assert e2 == "native_graph"
    assert np.isfinite(h2["loss"][0])
    assert not np.array_equal(w2[0], w0[0])
    # the native run stays close to the fp32 reference in expectation: same loss scale
    wr, hr, er = _train(lambda: _dropout_model(0.4), x, y, init, 64, 10, native=False, device="cpu", lr=0.05,
                        momentum=0.9)
    assert abs(h2["loss"][0] - hr["loss"][0]) < 0.25 * hr["loss"][0]
