"""The LDS-DMA (global_load_lds) implicit-GEMM conv kernels (csrc/kernels/conv_gemm.hip):
forward for any conv whose input has C % 64 == 0, backprop-input for stride-1 convs
whose output has C % 64 == 0.

Checked two ways: against the plain PyTorch fp32 conv (same bf16-rounded operands), and
BITWISE against the register-staged kernel (csrc/kernels/gemm.hip, DAMD_CONV_GLDS=0): with
no K split both accumulate the same 32-deep MFMA chunks in the same k order, so any
difference is a staging / swizzle / padding bug, not rounding.  Shapes are ragged (M and
N not multiples of the tiles, odd image sizes, zero padding on every side)."""
import pytest
import numpy as np
import torch

from distributed_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

dev = torch.device("cuda:0") if torch.cuda.is_available() else None


@pytest.fixture(scope="module")
def H():
    from distributed_amd.ops import hip

    return hip


def rb(t):
    return t.to(torch.bfloat16).float()


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dev)


def close(a, b, rtol, atol_frac):
    a, b = a.float(), b.float()
    atol = atol_frac * b.abs().max().item() + 1e-12
    err = (a - b).abs().max().item()
    assert torch.allclose(a, b, rtol=rtol, atol=atol), f"max abs err {err:.3e} (atol {atol:.3e})"


CASES = [
    # n, h, cin, cout, k, s, padding
    (2, 9, 64, 64, 3, 1, "same"),      # 256x64 tiles, ragged M
    (3, 11, 64, 200, 3, 1, "same"),    # 128x128 tiles, ragged N (200 = 128 + 72)
    (2, 10, 128, 128, 3, 2, "same"),   # stride 2 (forward only on the DMA path)
    (3, 7, 64, 128, 1, 2, "valid"),    # 1x1 projection
    (2, 12, 192, 64, 3, 1, "valid"),   # valid padding, Cin = 3 x 64
    (1, 7, 512, 512, 3, 1, "same"),    # ResNet layer4 shape
]


@pytest.mark.parametrize("n,h,cin,cout,k,s,padding", CASES)
def test_glds_conv_matches_reference_and_regstaged_kernel(H, monkeypatch, n, h, cin, cout, k, s, padding):
    monkeypatch.setattr(H, "SPLIT_MIN_TILES", 0)  # fused epilogue (split-K: the test below)
    x = rb(rnd(n, h, h, cin, seed=1)).requires_grad_(True)
    w = rb(rnd(k, k, cin, cout, scale=0.1, seed=2)).requires_grad_(True)
    y = ref.conv2d(x, w, None, (s, s), padding)
    dy = rb(rnd(*y.shape, seed=3))
    gx, = torch.autograd.grad(y, (x,), dy)
    xb, wb, dyb = x.detach().bfloat16(), w.detach().bfloat16(), dy.bfloat16()

    fplan = H.conv_fwd_plan(x.shape, w.shape, (s, s), padding)
    assert fplan["amode"] == H.A_CONV64
    out = torch.empty(y.shape, device=dev, dtype=torch.bfloat16)
    H.conv_fwd(xb, wb, out, (s, s), padding)
    close(out, y.detach(), 1e-2, 4e-3)
    dplan = H.conv_dgrad_plan(x.shape, w.shape, (s, s), padding)
    assert (dplan["amode"] == H.A_DGRAD64) == ((s == 1 or h % 2 == 0) and cout % 64 == 0)
    dx = torch.empty(x.shape, device=dev, dtype=torch.bfloat16)
    H.conv_dgrad(dyb, wb, dx, (s, s), padding)
    close(dx, gx, 1e-2, 4e-3)

    monkeypatch.setenv("DAMD_CONV_GLDS", "0")
    assert H.conv_fwd_plan(x.shape, w.shape, (s, s), padding)["amode"] == H.A_IM2COL
    assert fplan["splits"] == 1 and dplan["splits"] == 1
    out0 = torch.empty_like(out)
    H.conv_fwd(xb, wb, out0, (s, s), padding)
    assert torch.equal(out, out0)
    dx0 = torch.empty_like(dx)
    H.conv_dgrad(dyb, wb, dx0, (s, s), padding)
    if s == 1:
        assert torch.equal(dx, dx0)
    else:  # sub-pixel classes sum the taps in another order than the dilated formulation
        close(dx, dx0, 1e-2, 4e-3)


WGRAD_CASES = CASES + [
    (2, 30, 8, 64, 7, 2, "same"),      # ResNet stem geometry (Wo = 15: 4 virtual rows per k-step)
    (1, 140, 8, 16, 3, 1, "same"),     # Wo = 140 > 64: 3 segments of 47 per output row
]


@pytest.mark.parametrize("n,h,cin,cout,k,s,padding", WGRAD_CASES)
@pytest.mark.parametrize("target_wg", [1, 512])
def test_glds_wgrad(H, monkeypatch, n, h, cin, cout, k, s, padding, target_wg):
    """Weight gradient over virtual rows (one split: atomic epilogue; many: slabs +
    fixed-order reduce) against the fp32 reference and the register-staged kernel."""
    monkeypatch.setattr(H, "WGRAD_TARGET_WG", target_wg)
    monkeypatch.setenv("DAMD_WGRAD_KERNEL", "glds")  # also the N <= 64 layers the planner keeps off it
    x = rb(rnd(n, h, h, cin, seed=11)).requires_grad_(True)
    w = rb(rnd(k, k, cin, cout, scale=0.1, seed=12)).requires_grad_(True)
    y = ref.conv2d(x, w, None, (s, s), padding)
    dy = rb(rnd(*y.shape, seed=13))
    gw, = torch.autograd.grad(y, (w,), dy)
    plan = H.conv_wgrad_plan(x.shape, w.shape, (s, s), padding)
    assert plan["amode"] == H.A_WGRAD64
    assert plan["splits"] == 1 or target_wg > 1
    dw = torch.zeros(w.shape, device=dev)
    H.conv_wgrad(x.detach().bfloat16(), dy.bfloat16(), dw, (s, s), padding)
    close(dw, gw, 1e-4, 2e-5)
    monkeypatch.setenv("DAMD_WGRAD_KERNEL", "reg")
    assert H.conv_wgrad_plan(x.shape, w.shape, (s, s), padding)["amode"] == H.A_WGRAD
    dw0 = torch.zeros(w.shape, device=dev)
    H.conv_wgrad(x.detach().bfloat16(), dy.bfloat16(), dw0, (s, s), padding)
    close(dw, dw0, 1e-4, 2e-5)


@pytest.mark.parametrize("kb", [32, 64])
@pytest.mark.parametrize("n,h,cin,cout,k,s,padding", [CASES[0], CASES[1], CASES[4], WGRAD_CASES[-2]])
def test_glds_kstep_variants_deterministic(H, monkeypatch, kb, n, h, cin, cout, k, s, padding):
    """Both k-step depths of the LDS-DMA kernels (DAMD_CONV_KB) are exercised on every
    operand path and each is run repeatedly: outputs must be bitwise identical run to run
    (a staging race shows up as a mismatch) and match the reference."""
    monkeypatch.setenv("DAMD_CONV_KB", str(kb))
    monkeypatch.setenv("DAMD_WGRAD_KERNEL", "glds")
    x = rb(rnd(n, h, h, cin, seed=21)).bfloat16()
    w = rb(rnd(k, k, cin, cout, scale=0.1, seed=22)).bfloat16()
    ho, _ = H.conv_out(h, k, s, padding)
    dy = rb(rnd(n, ho, ho, cout, seed=23)).bfloat16()

    def run():
        outs = []
        if cin % 64 == 0:
            y = torch.empty(n, ho, ho, cout, device=dev, dtype=torch.bfloat16)
            H.conv_fwd(x, w, y, (s, s), padding)
            outs.append(y)
        if s == 1 and cout % 64 == 0:
            dx = torch.empty(n, h, h, cin, device=dev, dtype=torch.bfloat16)
            H.conv_dgrad(dy, w, dx, (s, s), padding)
            outs.append(dx)
        dw = torch.zeros(k, k, cin, cout, device=dev)
        H.conv_wgrad(x, dy, dw, (s, s), padding)
        outs.append(dw)
        return outs

    ref2 = run()
    for _ in range(3):
        for a, b in zip(run(), ref2):
            assert torch.equal(a, b)
    xr, wr, dyr = x.float().requires_grad_(True), w.float().requires_grad_(True), dy.float()
    y = ref.conv2d(xr, wr, None, (s, s), padding)
    gx, gw = torch.autograd.grad(y, (xr, wr), dyr)
    close(ref2[-1], gw, 1e-4, 2e-5)
    if cin % kb == 0:
        close(ref2[0], y.detach(), 1e-2, 4e-3)


@pytest.mark.parametrize("n,h,c", [(2, 16, 16), (3, 11, 64), (2, 20, 64)])
def test_stem_fused_kernels_match_unfused(H, n, h, c):
    """bn_relu_maxpool_fwd / pool_bn_bwd == bn_apply(relu) + maxpool_fwd and maxpool_bwd +
    BN backward (relu mask): bitwise on the pooled output and argmax.  Odd h takes the
    pixel-centric backward kernels (bitwise equal partials, dgamma/dbeta and dx); even h
    the 2x2-quad kernels (same routed gradient, partial sums grouped by quad: fp32 sums
    in another order, so the statistics and dx agree to rounding)."""
    C_ = H._C()
    x = rb(rnd(n, h, h, c, scale=2.0, seed=31)).bfloat16()
    M = n * h * h
    g = (rnd(c, seed=32).abs() + 0.5).float()
    b = rnd(c, seed=33).float()
    st = torch.stack([rnd(c, seed=34) * 0.1, rnd(c, seed=35).abs() + 0.5, g, b])  # mean, inv, sc, sh
    pool, strides, pad = (3, 3), (2, 2), "same"
    geo = H.pool_geo(x.shape, pool, strides, pad)
    ho, wo = geo[10], geo[11]
    # forward
    yb = torch.empty_like(x)
    H.bn_apply(x, st, yb, relu=True)
    p0 = torch.empty(n, ho, wo, c, device=dev, dtype=torch.bfloat16)
    a0 = torch.empty(n, ho, wo, c, device=dev, dtype=torch.uint8)
    H.maxpool_fwd(yb, p0, a0, pool, strides, pad)
    p1, a1 = torch.empty_like(p0), torch.empty_like(a0)
    H.bn_relu_maxpool_fwd(x, st, p1, a1, pool, strides, pad)
    assert torch.equal(p0, p1) and torch.equal(a0, a1)
    # backward
    dp = rb(rnd(n, ho, wo, c, seed=36)).bfloat16()
    T = C_.bn_bwd_blocks(M, c)
    part0, part1 = torch.zeros(T, 2, c, device=dev), torch.zeros(T, 2, c, device=dev)
    co0, co1 = torch.zeros(3, c, device=dev), torch.zeros(3, c, device=dev)
    dg0, db0, dg1, db1 = (torch.zeros(c, device=dev) for _ in range(4))
    dyb = torch.empty_like(x)
    H.maxpool_bwd(dp, a0, dyb, pool, strides, pad)
    dx0 = torch.empty_like(x)
    H.bn_bwd(dyb, yb, True, x, st, part0, co0, dx0, dgamma=dg0, dbeta=db0)
    dx1 = torch.empty_like(x)
    H.pool_bn_bwd(dp, a1, x, st, part1, co1, dx1, pool, strides, pad, dgamma=dg1, dbeta=db1)
    if h % 2:
        assert torch.equal(part0, part1)
        assert torch.equal(dg0, dg1) and torch.equal(db0, db1)
        assert torch.equal(dx0, dx1)
    else:
        close(part1.sum(0), part0.sum(0), 1e-5, 1e-6)
        close(dg1, dg0, 1e-5, 1e-6)
        close(db1, db0, 1e-5, 1e-6)
        close(dx1, dx0, 1e-2, 1e-2)
        # the quad kernel with the unfused kernel's own coefficients: bitwise dx
        dx2 = torch.empty_like(x)
        g_ = H.pool_geo(x.shape, pool, strides, pad)
        C_.pool_bn_bwd_apply(H._ptr(dp), H._ptr(a1), g_, H._ptr(x), H._ptr(st), H._ptr(co0), H._ptr(dx2),
                             H.stream_handle())
        assert torch.equal(dx2, dx0)


@pytest.mark.parametrize("split", [False, True])
def test_glds_conv_epilogues(H, monkeypatch, split):
    """bias + ReLU, BN statistics, dgrad accumulation; fused epilogue and split-K slabs
    (k_per_split a multiple of the 64-deep k-step) + the finishing kernel."""
    monkeypatch.setattr(H, "SPLIT_MIN_TILES", 1 << 30 if split else 0)
    n, h, cin, cout = 2, 7, 128, 64
    plan = H.conv_fwd_plan((n, h, h, cin), (3, 3, cin, cout), (1, 1), "same")
    assert plan["amode"] == H.A_CONV64 and (plan["splits"] > 1) == split
    assert plan["kps"] % H.conv_kstep() == 0
    x = rb(rnd(n, h, h, cin, seed=40))
    w = rb(rnd(3, 3, cin, cout, scale=0.1, seed=41))
    b = rnd(cout, seed=42)
    y = ref.conv2d(x, w, b, (1, 1), "same")
    out = torch.empty(y.shape, device=dev, dtype=torch.bfloat16)
    st = torch.zeros(plan["stats_T"], 2, cout, device=dev)
    H.conv_fwd(x.bfloat16(), w.bfloat16(), out, (1, 1), "same", bias=b, stats=st)
    close(out, y, 1e-2, 4e-3)
    yb = out.float().reshape(-1, cout)
    close(st[:, 0].sum(0), yb.sum(0), 1e-4, 1e-5)
    close(st[:, 1].sum(0), (yb * yb).sum(0), 1e-4, 1e-5)
    H.conv_fwd(x.bfloat16(), w.bfloat16(), out, (1, 1), "same", bias=b, relu=True)
    close(out, y.relu(), 1e-2, 4e-3)
    # dgrad of a conv with 64 output channels: gathered tensor dy has C = 64
    dy = rb(rnd(n, h, h, cout, seed=43))
    xx = x.clone().requires_grad_(True)
    gx, = torch.autograd.grad(ref.conv2d(xx, w, None, (1, 1), "same"), (xx,), dy)
    dplan = H.conv_dgrad_plan(x.shape, w.shape, (1, 1), "same")
    assert dplan["amode"] == H.A_DGRAD64 and (dplan["splits"] > 1) == split
    dx = torch.empty(x.shape, device=dev, dtype=torch.bfloat16)
    H.conv_dgrad(dy.bfloat16(), w.bfloat16(), dx, (1, 1), "same")
    close(dx, gx, 1e-2, 4e-3)
    H.conv_dgrad(dy.bfloat16(), w.bfloat16(), dx, (1, 1), "same", accumulate=True)
    close(dx, 2 * gx, 1e-2, 8e-3)


WGRAD3_CASES = [
    # n, h, cin, cout: every ResNet-18 3x3/s1 width class plus ragged / small images
    (2, 56, 64, 64),     # layer1 (pitch 57: two look-back blocks, 8-block x ring)
    (3, 28, 128, 64),    # layer2-like, 2 ci tiles
    (2, 14, 64, 256),    # layer3-like, 4 co tiles
    (3, 7, 128, 128),    # layer4 geometry (pitch 8: 4 rows per k-step)
    (1, 5, 64, 64),      # image smaller than one k-step
    (2, 30, 64, 128),    # pitch 31 = exactly one look-back block
]


@pytest.mark.parametrize("n,h,cin,cout", WGRAD3_CASES)
@pytest.mark.parametrize("target_wg", ["1", "4096"])
def test_direct_wgrad3(H, monkeypatch, n, h, cin, cout, target_wg):
    """Direct 3x3/s1/p1 weight gradient (csrc/kernels/conv_wgrad3.hip: sliding x window,
    nine shifted taps) against the fp32 reference and the LDS-DMA GEMM kernel; one split
    (atomic epilogue) and many (slabs, fixed-order reduce); repeat runs bitwise equal."""
    monkeypatch.setenv("DAMD_WGRAD3_WG", target_wg)
    x = rb(rnd(n, h, h, cin, seed=51)).requires_grad_(True)
    w = rb(rnd(3, 3, cin, cout, scale=0.1, seed=52)).requires_grad_(True)
    y = ref.conv2d(x, w, None, (1, 1), "same")
    dy = rb(rnd(*y.shape, seed=53))
    gw, = torch.autograd.grad(y, (w,), dy)
    plan = H.conv_wgrad_plan(x.shape, w.shape, (1, 1), "same")
    assert plan["amode"] == H.A_WGRAD3
    assert plan["splits"] == 1 or target_wg != "1"
    xb, dyb = x.detach().bfloat16(), dy.bfloat16()
    dw = torch.zeros(w.shape, device=dev)
    H.conv_wgrad(xb, dyb, dw, (1, 1), "same")
    close(dw, gw, 1e-4, 2e-5)
    if plan["splits"] > 1:
        for _ in range(2):
            dw2 = torch.zeros(w.shape, device=dev)
            H.conv_wgrad(xb, dyb, dw2, (1, 1), "same")
            assert torch.equal(dw, dw2)
    monkeypatch.setenv("DAMD_WGRAD_KERNEL", "glds")
    assert H.conv_wgrad_plan(x.shape, w.shape, (1, 1), "same")["amode"] == H.A_WGRAD64
    dw0 = torch.zeros(w.shape, device=dev)
    H.conv_wgrad(xb, dyb, dw0, (1, 1), "same")
    close(dw, dw0, 1e-4, 2e-5)


@pytest.mark.parametrize("n,h,cin,cout,k,padding", [
    (2, 10, 64, 128, 3, "same"),    # ResNet downsample 3x3/s2 (TF "same": pad 0 top/left)
    (3, 14, 128, 64, 3, "same"),    # 256x64 tiles, ragged class grid (7x7)
    (2, 12, 64, 128, 1, "valid"),   # 1x1/s2 projection: one class has the tap, three are zero
])
@pytest.mark.parametrize("accumulate", [False, True])
def test_subpixel_dgrad_stride2(H, n, h, cin, cout, k, padding, accumulate):
    """Stride-2 backprop-input as four parity-class convolutions (conv_gemm.hip, grid z =
    class, scattered epilogue rows) against the fp32 reference; accumulate adds onto dx."""
    plan = H.conv_dgrad_plan((n, h, h, cin), (k, k, cin, cout), (2, 2), padding)
    assert plan["amode"] == H.A_DGRAD64 and plan["splits"] == 1
    x = rb(rnd(n, h, h, cin, seed=61)).requires_grad_(True)
    w = rb(rnd(k, k, cin, cout, scale=0.1, seed=62))
    y = ref.conv2d(x, w, None, (2, 2), padding)
    dy = rb(rnd(*y.shape, seed=63))
    gx, = torch.autograd.grad(y, (x,), dy)
    base = rb(rnd(n, h, h, cin, seed=64)) if accumulate else torch.zeros(n, h, h, cin, device=dev)
    dx = base.bfloat16().clone()
    H.conv_dgrad(dy.bfloat16(), w.bfloat16(), dx, (2, 2), padding, accumulate=accumulate)
    close(dx, base + gx, 1e-2, 4e-3)


@pytest.mark.parametrize("n,h,cin,cout,k,padding", [(2, 32, 3, 64, 7, "same"), (3, 18, 4, 32, 5, "valid"),
                                                     (1, 24, 1, 64, 3, "same")])
def test_packed_tap_stem(H, n, h, cin, cout, k, padding):
    """Packed-tap stem (conv_gemm.hip, 4-channel input, K = KH x 8 pixels x 4 channels):
    forward (+BN statistics) and weight gradient against the fp32 reference of the true
    KxK x cin conv; the layout's padding taps/channels come back as zero-input junk only."""
    x = rb(rnd(n, h, h, cin, seed=71))
    w = rb(rnd(k, k, cin, cout, scale=0.1, seed=72))
    x4 = torch.zeros(n, h, h, 4, device=dev)
    x4[..., :cin] = x
    wshape = (k, k, 4, cout)
    assert H.stem4_ok(x4.shape, wshape, (2, 2), padding)
    w8 = torch.zeros(H.stem4_weight_shape(wshape), device=dev, dtype=torch.bfloat16)
    w8[:, :k, :cin] = w.bfloat16()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y = ref.conv2d(xr, wr, None, (2, 2), padding)
    plan = H.conv_fwd_plan(x4.shape, wshape, (2, 2), padding)
    out = torch.empty(y.shape, device=dev, dtype=torch.bfloat16)
    st = torch.zeros(plan["stats_T"], 2, cout, device=dev)
    H.conv_fwd_stem4(x4.bfloat16(), w8, out, k, (2, 2), padding, stats=st)
    close(out, y.detach(), 1e-2, 4e-3)
    yb = out.float().reshape(-1, cout)
    close(st[:, 0].sum(0), yb.sum(0), 1e-4, 1e-5)
    dy = rb(rnd(*y.shape, seed=73))
    gw, = torch.autograd.grad(y, (wr,), dy)
    dw8 = torch.zeros(H.stem4_weight_shape(wshape), device=dev)
    H.conv_wgrad_stem4(x4.bfloat16(), dy.bfloat16(), dw8, k, (2, 2), padding)
    close(dw8[:, :k, :cin], gw, 1e-4, 2e-5)


def test_packed_tap_stem_wgrad_reduces_into_true_layout(H):
    """The stem's split-K weight gradient reduced straight into the true [7][7][3][64]
    gradient (splitk_reduce_unpad: the junk taps / channel dropped in the reduce) == the
    padded reduce + unpad: bitwise onto zeros (both 0 + the same fixed-order sum), within
    rounding onto a non-zero buffer, and against the fp32 reference."""
    n, h, cin, cout, k = 8, 64, 3, 64, 7
    x = rb(rnd(n, h, h, cin, seed=74))
    x4 = torch.zeros(n, h, h, 4, device=dev)
    x4[..., :cin] = x
    wshape = (k, k, 4, cout)
    plan = H.conv_wgrad_plan(x4.shape, wshape, (2, 2), "same")
    assert plan["splits"] > 1, plan
    w = rb(rnd(k, k, cin, cout, scale=0.1, seed=75)).requires_grad_(True)
    y = ref.conv2d(x, w, None, (2, 2), "same")
    dy = rb(rnd(*y.shape, seed=76))
    gw, = torch.autograd.grad(y, (w,), dy)
    dw8 = torch.zeros(H.stem4_weight_shape(wshape), device=dev)
    assert not H.conv_wgrad_stem4(x4.bfloat16(), dy.bfloat16(), dw8, k, (2, 2), "same", accumulate=False)
    dw = torch.zeros(k, k, cin, cout, device=dev)
    junk = torch.full(H.stem4_weight_shape(wshape), 7.0, device=dev)
    assert H.conv_wgrad_stem4(x4.bfloat16(), dy.bfloat16(), junk, k, (2, 2), "same", accumulate=False, dw=dw)
    assert torch.equal(dw, dw8[:, :k, :cin])
    assert torch.equal(junk, torch.full_like(junk, 7.0))  # the padded buffer is not touched
    close(dw, gw, 1e-4, 2e-5)
    base = rnd(k, k, cin, cout, seed=77)
    dwb = base.clone()
    H.conv_wgrad_stem4(x4.bfloat16(), dy.bfloat16(), dw8, k, (2, 2), "same", accumulate=False, dw=dwb)
    close(dwb, base + gw, 1e-4, 2e-5)


@pytest.mark.parametrize("shape", [(8, 7, 512, 512), (4, 7, 256, 256), (2, 7, 256, 128)])
def test_splitk_in_launch_finish_matches_finish_kernel(H, shape, monkeypatch):
    """Split-K conv GEMMs finished inside the launch (E_FIXUP: per-tile ticket, the last split
    sums the slabs in split order and runs the epilogue) == the slab GEMM + splitk_finish
    launch (DAMD_SPLITK_FIXUP=0): forward output and backprop-input (also accumulating onto
    dx) bitwise; the BN statistics accumulator within fp32 rounding of the regrouped
    partials; both against the fp32 reference.  Three launches each, so the self-resetting
    tickets are exercised."""
    n, h, cin, cout = shape
    x = rb(rnd(n, h, h, cin, seed=91))
    w = rb(rnd(3, 3, cin, cout, scale=0.05, seed=92))
    plan = H.conv_fwd_plan(x.shape, w.shape, (1, 1), "same")
    assert plan["splits"] > 1 and plan["amode"] == H.A_CONV64, plan
    y = ref.conv2d(x, w, None, (1, 1), "same")
    outs, accs = [], []
    for fix in ("1", "0"):
        monkeypatch.setenv("DAMD_SPLITK_FIXUP", fix)
        for _ in range(3):
            out = torch.empty(y.shape, device=dev, dtype=torch.bfloat16)
            acc = H.acc_zeros(8, 2 * cout, dev)
            H.conv_fwd(x.bfloat16(), w.bfloat16(), out, (1, 1), "same", stats=acc)
        torch.cuda.synchronize()
        outs.append(out)
        accs.append(H.bn_acc_decode(acc))
    assert torch.equal(outs[0], outs[1])
    close(outs[0], y, 1e-2, 4e-3)
    np.testing.assert_allclose(accs[0].numpy(), accs[1].numpy(), rtol=1e-5, atol=1e-2)
    dplan = H.conv_dgrad_plan(x.shape, w.shape, (1, 1), "same")
    dy = rb(rnd(*y.shape, seed=93))
    base = rb(rnd(*x.shape, seed=94)).bfloat16()
    for accumulate in (False, True):
        res = []
        for fix in ("1", "0"):
            monkeypatch.setenv("DAMD_SPLITK_FIXUP", fix)
            for _ in range(3):
                dx = base.clone()
                H.conv_dgrad(dy.bfloat16(), w.bfloat16(), dx, (1, 1), "same", accumulate=accumulate)
            torch.cuda.synchronize()
            res.append(dx)
        if dplan["splits"] > 1:
            assert torch.equal(res[0], res[1]), accumulate


@pytest.mark.parametrize("n,relu,bias", [(2, False, False), (3, False, True)])
def test_stem_direct_bitwise_equals_implicit_gemm(H, n, relu, bias, monkeypatch):
    """The direct stem forward (conv_stem.hip: input rows staged once per 256-pixel tile,
    A fragments read from them) == the implicit-GEMM packed-tap kernel (DAMD_STEM_DIRECT=0),
    bitwise: output and the fixed-point BN statistics accumulator (same tiles, fragments,
    MFMA order and replica assignment); the ResNet-18 stem shape (224 x 224, 7x7 / 2, 64
    outputs) and the true KxK conv as the fp32 oracle."""
    k, cout, h = 7, 64, 224
    x = rb(rnd(n, h, h, 3, seed=81))
    w = rb(rnd(k, k, 3, cout, scale=0.1, seed=82))
    x4 = torch.zeros(n, h, h, 4, device=dev)
    x4[..., :3] = x
    wshape = (k, k, 4, cout)
    w8 = torch.zeros(H.stem4_weight_shape(wshape), device=dev, dtype=torch.bfloat16)
    w8[:, :k, :3] = w.bfloat16()
    b = rnd(cout, seed=83) if bias else None
    y = ref.conv2d(x, w, b, (2, 2), "same")
    if relu:
        y = torch.relu(y)
    outs, accs = [], []
    for direct in ("1", "0"):
        monkeypatch.setenv("DAMD_STEM_DIRECT", direct)
        out = torch.empty(y.shape, device=dev, dtype=torch.bfloat16)
        acc = H.acc_zeros(8, 2 * cout, dev)
        H.conv_fwd_stem4(x4.bfloat16(), w8, out, k, (2, 2), "same", bias=b, relu=relu, stats=acc)
        torch.cuda.synchronize()
        outs.append(out)
        accs.append(acc)
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(accs[0], accs[1])
    close(outs[0], y, 1e-2, 4e-3)


@pytest.mark.parametrize("splits,n", [(3, 1 << 16), (16, 3 << 14), (3, 4096), (40, 1 << 15)])
def test_splitk_reduce_paths(H, splits, n):
    """dst += sum of the split slabs in split order: the flat kernel (<= 16 splits, large n)
    and the split-group kernel (small n, or many splits) against a sequential torch sum."""
    slab = torch.randn(splits, n, device=dev)
    dst = torch.randn(n, device=dev)
    want = dst.clone()
    for sp in range(splits):
        want = want + slab[sp]
    H._C().splitk_reduce(H._ptr(slab), splits, n, H._ptr(dst), H.stream_handle())
    torch.cuda.synchronize()
    if splits <= 16:
        assert torch.equal(dst, want)  # same order: bitwise
    else:
        close(dst, want, 1e-5, 1e-6)


@pytest.mark.parametrize("M,c", [(3000, 64), (1000, 256)])
def test_bn_bwd_relu_mask_from_x(H, M, c):
    """relu_mask 2 (mask recomputed from x and the BN scale/shift) == relu_mask 1 reading
    y = bn_apply(x, relu): bitwise partials, dgamma/dbeta and dx."""
    C_ = H._C()
    x = rb(rnd(M, c, scale=2.0, seed=51)).bfloat16()
    st = torch.stack([rnd(c, seed=52) * 0.1, rnd(c, seed=53).abs() + 0.5,
                      rnd(c, seed=54).abs() + 0.5, rnd(c, seed=55)]).float()
    y = torch.empty_like(x)
    H.bn_apply(x, st, y, relu=True)
    dy = rb(rnd(M, c, seed=56)).bfloat16()
    T = C_.bn_bwd_blocks(M, c)
    out = []
    for mode in (1, 2):
        part, co = torch.zeros(T, 2, c, device=dev), torch.zeros(3, c, device=dev)
        dg, db, dx = torch.zeros(c, device=dev), torch.zeros(c, device=dev), torch.empty_like(x)
        H.bn_bwd(dy, y if mode == 1 else None, mode, x, st, part, co, dx, dgamma=dg, dbeta=db)
        out.append((part, dg, db, dx))
    for a, b in zip(*out):
        assert torch.equal(a, b)


CONV3_CASES = [
    # n, h, cin, cout: tile BN 64 (256 x 64) / 128 (128 x 128), R output rows per block
    (2, 56, 64, 64),     # ResNet layer 1: BN 64, R 4 (224 of 256 rows)
    (2, 28, 128, 128),   # layer 2: BN 128, R 4
    (2, 14, 256, 256),   # BN 128, R 9: row blocks of 9 + 5 rows (ragged last block)
    (3, 20, 64, 128),    # R 6 over 20 rows (6, 6, 6, 2)
    (2, 30, 128, 64),    # BN 64, R 8 over 30 rows; 2 ci-chunks
    (3, 28, 64, 64),     # 64 -> 64 at R 9 (28 = 9 + 9 + 9 + 1 rows)
]


@pytest.mark.parametrize("n,h,cin,cout", CONV3_CASES)
def test_direct_conv3(H, monkeypatch, n, h, cin, cout):
    """The direct 3x3/s1/p1 kernel (csrc/kernels/conv3x3.hip: input halo resident in LDS,
    weights streamed per tap) against the fp32 conv and the implicit-GEMM kernel, forward
    with bias + ReLU and with the BN-statistics epilogue, backprop-input plain and
    accumulating."""
    monkeypatch.setenv("DAMD_CONV3_MIN_WG", "1")
    x = rb(rnd(n, h, h, cin, seed=11)).requires_grad_(True)
    w = rb(rnd(3, 3, cin, cout, scale=0.05, seed=12)).requires_grad_(True)
    bias = rnd(cout, scale=0.1, seed=13)
    y = ref.conv2d(x, w, None, (1, 1), "same")
    dy = rb(rnd(*y.shape, seed=14))
    gx, = torch.autograd.grad(y, (x,), dy)
    xb, wb, dyb = x.detach().bfloat16(), w.detach().bfloat16(), dy.bfloat16()
    fplan = H.conv_fwd_plan(x.shape, w.shape, (1, 1), "same")
    dplan = H.conv_dgrad_plan(x.shape, w.shape, (1, 1), "same")
    assert fplan["amode"] == H.A_CONV3 and dplan["amode"] == H.A_DGRAD3
    # forward, bias + ReLU epilogue
    out = torch.empty(y.shape, device=dev, dtype=torch.bfloat16)
    H.conv_fwd(xb, wb, out, (1, 1), "same", bias=bias, relu=True)
    close(out, torch.relu(y.detach() + bias), 1e-2, 4e-3)
    # forward with BN statistics: per-tile partials summing to the stored values' moments
    st = torch.zeros(fplan["stats_T"], 2, cout, device=dev)
    out2 = torch.empty_like(out)
    H.conv_fwd(xb, wb, out2, (1, 1), "same", stats=st)
    close(out2, y.detach(), 1e-2, 4e-3)
    y32 = out2.float().reshape(-1, cout)
    close(st[:, 0].sum(0), y32.sum(0), 1e-3, 1e-4)
    close(st[:, 1].sum(0), (y32 * y32).sum(0), 1e-3, 1e-4)
    # the implicit-GEMM kernel: same products, another summation order
    monkeypatch.setenv("DAMD_CONV3", "0")
    assert H.conv_fwd_plan(x.shape, w.shape, (1, 1), "same")["amode"] != H.A_CONV3
    out0 = torch.empty_like(out)
    H.conv_fwd(xb, wb, out0, (1, 1), "same")
    close(out2, out0, 1e-2, 2e-3)
    monkeypatch.setenv("DAMD_CONV3", "1")
    # backprop-input, then accumulating onto it
    dx = torch.empty(x.shape, device=dev, dtype=torch.bfloat16)
    H.conv_dgrad(dyb, wb, dx, (1, 1), "same")
    close(dx, gx, 1e-2, 4e-3)
    base = rb(rnd(*x.shape, seed=15))
    dx2 = base.bfloat16().contiguous()
    H.conv_dgrad(dyb, wb, dx2, (1, 1), "same", accumulate=True)
    close(dx2, gx + base, 1e-2, 4e-3)


@pytest.mark.parametrize("n,h,cin,cout", [(2, 56, 64, 64), (2, 28, 128, 128), (2, 14, 256, 256), (32, 16, 64, 64)])
def test_direct_conv3_dgrad_bnred(H, monkeypatch, n, h, cin, cout):
    """Backprop-input with the BN-backward epilogue (E_BNRED): dx bitwise == the plain
    direct kernel's, and the per-tile partials sum to sum(dz), sum(dz * xhat) with
    dz = bf16(dx) * [bf16(relu(x sc + sh)) > 0] (fp32 reference)."""
    monkeypatch.setenv("DAMD_CONV3_MIN_WG", "1")
    shape = (n, h, h, cin)
    dplan = H.conv_dgrad_plan(shape, (3, 3, cin, cout), (1, 1), "same")
    assert dplan["amode"] == H.A_DGRAD3
    wb = rb(rnd(3, 3, cin, cout, scale=0.05, seed=21)).bfloat16()
    dyb = rb(rnd(n, h, h, cout, seed=22)).bfloat16()
    xb = rb(rnd(*shape, scale=2.0, seed=23)).bfloat16()
    st = torch.stack([rnd(cin, seed=24) * 0.1, rnd(cin, seed=25).abs() + 0.5,
                      rnd(cin, seed=26).abs() + 0.5, rnd(cin, seed=27)]).float().contiguous()
    dx0 = torch.empty(shape, device=dev, dtype=torch.bfloat16)
    assert not H.conv_dgrad(dyb, wb, dx0, (1, 1), "same")
    dx = torch.empty_like(dx0)
    part = torch.full((dplan["stats_T"], 2, cin), float("nan"), device=dev)
    assert H.conv_dgrad(dyb, wb, dx, (1, 1), "same", bnred=(xb, st, part))
    assert torch.equal(dx, dx0)
    assert not torch.isnan(part).any()
    x32 = xb.float().reshape(-1, cin)
    mask = rb(torch.relu(x32 * st[2] + st[3])) > 0
    dz = dx.float().reshape(-1, cin) * mask
    xhat = (x32 - st[0]) * st[1]
    close(part[:, 0].sum(0), dz.sum(0), 1e-3, 1e-4)
    close(part[:, 1].sum(0), (dz * xhat).sum(0), 1e-3, 1e-4)


@pytest.mark.parametrize("n,h,cin,cout", [(2, 56, 64, 64), (2, 28, 128, 128), (2, 14, 256, 256), (2, 30, 128, 64)])
@pytest.mark.parametrize("reps", [1, 8])
def test_direct_conv3_bn_input(H, monkeypatch, n, h, cin, cout, reps):
    """Direct forward conv on a BatchNorm's INPUT (GemmArgs::bnin: statistics finalized from
    the fp64 accumulator replicas in the kernel, BN + ReLU applied to the staged halo) ==
    bn_apply_fin + the plain direct conv, bitwise: the stored y, the conv output and its
    statistics epilogue, the published st and the moving statistics; padding stays zero."""
    monkeypatch.setenv("DAMD_CONV3_MIN_WG", "1")
    shape = (n, h, h, cin)
    assert H.conv_fwd_plan(shape, (3, 3, cin, cout), (1, 1), "same")["amode"] == H.A_CONV3
    xb = rb(rnd(*shape, scale=2.0, seed=31) + 0.3).bfloat16()
    wb = rb(rnd(3, 3, cin, cout, scale=0.05, seed=32)).bfloat16()
    gamma, beta = rnd(cin, seed=33).abs() + 0.5, rnd(cin, seed=34) * 0.2
    x64 = xb.double().reshape(-1, cin)
    sums = torch.cat([x64.sum(0), (x64 * x64).sum(0)])
    # split the sums over the replicas (the consumers add the replicas' integer words)
    acc = torch.stack([H.bn_acc_encode(sums * (0.5 ** (r + 1) if r < reps - 1 else 0.5 ** (reps - 1)))
                       for r in range(reps)] + [torch.zeros(2 * cin, dtype=torch.int64)]).to(dev)  # + flag plane
    M = n * h * h
    res = []
    for fold in (True, False):
        st = torch.zeros(4, cin, device=dev)
        rm, rv = torch.zeros(cin, device=dev), torch.ones(cin, device=dev)
        fin = H.BNFin(acc, gamma, beta, st, rm, rv, M, 1e-3, 0.99)
        y = torch.full(shape, float("nan"), device=dev, dtype=torch.bfloat16)
        out = torch.empty(n, h, h, cout, device=dev, dtype=torch.bfloat16)
        ostat = torch.zeros(2 * 2 * cout, dtype=torch.int64, device=dev)  # one replica + flag plane
        if fold:
            H.conv_fwd(xb, wb, out, (1, 1), "same", stats=ostat, bnin=(fin, y))
        else:
            H.bn_apply_fin(xb, y, fin, relu=True)
            H.conv_fwd(y, wb, out, (1, 1), "same", stats=ostat)
        res.append((y, out, ostat, st, rm, rv))
    for a, b in zip(*res):
        assert torch.equal(a, b)
    # and the values are BN -> ReLU of x (fp32 reference of the normalisation)
    y = res[0][0].float().reshape(-1, cin)
    mean = x64.mean(0)
    var = (x64 * x64).mean(0) - mean * mean
    ref_y = torch.relu((xb.float().reshape(-1, cin) - mean.float()) * torch.rsqrt(var.float() + 1e-3) * gamma + beta)
    close(y, ref_y, 1e-2, 4e-3)


@pytest.mark.parametrize("n", [2, 20, 64])
def test_direct_conv3r_bitwise_equals_general_kernel(H, monkeypatch, n):
    """The persistent weight-stationary 64 -> 64 kernel (csrc/kernels/conv3r.hip: one strip
    of 4-row tiles per CU, a ring of halo rows, a loader wave) == the general direct kernel
    (conv3x3.hip, DAMD_CONV3R=0), BITWISE -- same tiles, fragment layouts and MFMA order:
    forward with bias + ReLU, with fixed-point BN statistics, on a BatchNorm input (y, the
    conv output, the statistics, the published st / moving statistics); backprop-input
    plain, accumulating, and with the BN-backward epilogue.  n = 2: one tile per strip;
    20: strips of one or two tiles; 64: the ResNet-18 batch, strips of 3-4 tiles (the ring
    reuses slots)."""
    monkeypatch.setenv("DAMD_CONV3_MIN_WG", "1")
    h, c = 56, 64
    shape = (n, h, h, c)
    xb = rb(rnd(*shape, scale=2.0, seed=61) + 0.3).bfloat16()
    wb = rb(rnd(3, 3, c, c, scale=0.05, seed=62)).bfloat16()
    dyb = rb(rnd(*shape, seed=63)).bfloat16()
    bias = rnd(c, scale=0.1, seed=64)
    gamma, beta = rnd(c, seed=65).abs() + 0.5, rnd(c, seed=66) * 0.2
    x64 = xb.double().reshape(-1, c)
    sums = torch.cat([x64.sum(0), (x64 * x64).sum(0)])
    accin = torch.stack([H.bn_acc_encode(sums * 0.5), H.bn_acc_encode(sums * 0.5),
                         torch.zeros(2 * c, dtype=torch.int64)]).to(dev)
    st_bw = torch.stack([rnd(c, seed=67) * 0.1, rnd(c, seed=68).abs() + 0.5,
                         rnd(c, seed=69).abs() + 0.5, rnd(c, seed=70)]).float().contiguous()
    base = rb(rnd(*shape, seed=71)).bfloat16()

    def run():
        out = {}
        o = torch.empty(shape, device=dev, dtype=torch.bfloat16)
        H.conv_fwd(xb, wb, o, (1, 1), "same", bias=bias, relu=True)
        out["fwd_bias_relu"] = o
        o2, acc = torch.empty_like(o), H.acc_zeros(8, 2 * c, dev)
        H.conv_fwd(xb, wb, o2, (1, 1), "same", stats=acc)
        out["fwd_stats"], out["fwd_stats_acc"] = o2, acc
        st, rm, rv = torch.zeros(4, c, device=dev), torch.zeros(c, device=dev), torch.ones(c, device=dev)
        fin = H.BNFin(accin, gamma, beta, st, rm, rv, n * h * h, 1e-3, 0.99)
        y = torch.full(shape, float("nan"), device=dev, dtype=torch.bfloat16)
        o3, acc3 = torch.empty_like(o), H.acc_zeros(8, 2 * c, dev)
        H.conv_fwd(xb, wb, o3, (1, 1), "same", stats=acc3, bnin=(fin, y))
        out.update(bnin_y=y, bnin_out=o3, bnin_acc=acc3, bnin_st=st, bnin_rm=rm, bnin_rv=rv)
        dx = torch.empty_like(o)
        H.conv_dgrad(dyb, wb, dx, (1, 1), "same")
        out["dgrad"] = dx
        dx2 = base.clone()
        H.conv_dgrad(dyb, wb, dx2, (1, 1), "same", accumulate=True)
        out["dgrad_acc"] = dx2
        dx3, part = torch.empty_like(o), H.acc_zeros(8, 4 * c, dev)
        assert H.conv_dgrad(dyb, wb, dx3, (1, 1), "same", bnred=(xb, st_bw, part))
        out["dgrad_bnred"], out["dgrad_bnred_acc"] = dx3, part
        torch.cuda.synchronize()
        return out

    monkeypatch.setenv("DAMD_CONV3R", "1")
    new = run()
    monkeypatch.setenv("DAMD_CONV3R", "0")
    old = run()
    for k in new:
        assert torch.equal(new[k], old[k]), k
    # and against the fp32 reference (guards a shared bug)
    y = ref.conv2d(xb.float(), wb.float(), None, (1, 1), "same")
    close(new["fwd_stats"], y, 1e-2, 4e-3)
