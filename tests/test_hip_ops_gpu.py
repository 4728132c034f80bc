"""Numerics of the generic-path HIP kernels (csrc/kernels/gemm.hip, layer_ops.hip)
against plain PyTorch fp32 references of the same ops (distributed_amd/ops/reference.py).

bf16 operands are rounded once and then fed to BOTH sides, so the only differences are
fp32 accumulation order (and the bf16 rounding of bf16 outputs).  Matrices are
asymmetric and shapes ragged (M, N, K not multiples of the tiles) so transposed /
swapped operand maps and tail handling are exercised (cdna_hip_programming.md §3)."""
import pytest
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


@pytest.mark.parametrize("M,K,N", [(64, 512, 1000), (100, 72, 24), (300, 5408, 64), (1, 8, 8), (257, 96, 136)])
@pytest.mark.parametrize("relu,bias,out_bf16", [(False, False, False), (True, True, True), (False, True, False)])
def test_dense_fwd(H, M, K, N, relu, bias, out_bf16):
    x = rb(rnd(M, K, seed=1))
    w = rb(rnd(K, N, scale=0.1, seed=2))
    b = rnd(N, seed=3) if bias else None
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16 if out_bf16 else torch.float32)
    H.dense_fwd(x.bfloat16(), w.bfloat16(), out, bias=b, relu=relu)
    r = x @ w
    if bias:
        r = r + b
    if relu:
        r = r.relu()
    close(out, r, 1e-2 if out_bf16 else 1e-4, 4e-3 if out_bf16 else 1e-5)


@pytest.mark.parametrize("M,K,N", [(64, 512, 1000), (64, 5408, 64), (37, 24, 40)])
def test_dense_backward(H, M, K, N):
    x = rb(rnd(M, K, seed=4))
    w = rb(rnd(K, N, scale=0.1, seed=5))
    dy = rb(rnd(M, N, seed=6))
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    H.dense_dgrad(dy.bfloat16(), w.bfloat16(), dx)
    close(dx, dy @ w.t(), 1e-2, 4e-3)
    # accumulate mode adds onto what dx already holds
    H.dense_dgrad(dy.bfloat16(), w.bfloat16(), dx, accumulate=True)
    close(dx, 2 * (dy @ w.t()), 1e-2, 8e-3)
    dw = torch.zeros(K, N, device=dev)
    H.dense_wgrad(x.bfloat16(), dy.bfloat16(), dw)
    close(dw, x.t() @ dy, 1e-4, 1e-5)


CONV_CASES = [
    # n, h, cin, cout, k, s, padding
    (2, 9, 8, 16, 3, 1, "same"),
    (2, 10, 16, 64, 3, 2, "same"),
    (2, 14, 8, 64, 7, 2, "same"),
    (3, 7, 64, 128, 1, 2, "valid"),
    (2, 12, 24, 40, 3, 1, "valid"),
    (1, 8, 128, 256, 3, 2, "same"),
]


@pytest.mark.parametrize("n,h,cin,cout,k,s,padding", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(H, n, h, cin, cout, k, s, padding):
    x = rb(rnd(n, h, h, cin, seed=7)).requires_grad_(True)
    w = rb(rnd(k, k, cin, cout, scale=0.2, seed=8)).requires_grad_(True)
    y = ref.conv2d(x, w, None, (s, s), padding)
    dy = rb(rnd(*y.shape, seed=9))
    gx, gw = torch.autograd.grad(y, (x, w), dy)
    out = torch.empty(y.shape, device=dev, dtype=torch.bfloat16)
    H.conv_fwd(x.detach().bfloat16(), w.detach().bfloat16(), out, (s, s), padding)
    close(out, y.detach(), 1e-2, 4e-3)
    dx = torch.empty(x.shape, device=dev, dtype=torch.bfloat16)
    H.conv_dgrad(dy.bfloat16(), w.detach().bfloat16(), dx, (s, s), padding)
    close(dx, gx, 1e-2, 4e-3)
    dw = torch.zeros(w.shape, device=dev)
    H.conv_wgrad(x.detach().bfloat16(), dy.bfloat16(), dw, (s, s), padding)
    close(dw, gw, 1e-4, 2e-5)


def test_conv_bias_relu_and_stats(H):
    n, h, cin, cout = 4, 11, 16, 72
    x = rb(rnd(n, h, h, cin, seed=10))
    w = rb(rnd(3, 3, cin, cout, scale=0.2, seed=11))
    b = rnd(cout, seed=12)
    y = ref.conv2d(x, w, b, (1, 1), "same")
    out = torch.empty(y.shape, device=dev, dtype=torch.bfloat16)
    H.conv_fwd(x.bfloat16(), w.bfloat16(), out, (1, 1), "same", bias=b, relu=True)
    close(out, y.relu(), 1e-2, 4e-3)
    # BN statistics in the epilogue: per-M-tile partial column sums of the stored values
    T = H.conv_fwd_plan(x.shape, w.shape, (1, 1), "same")["stats_T"]
    st = torch.zeros(T, 2, cout, device=dev)
    H.conv_fwd(x.bfloat16(), w.bfloat16(), out, (1, 1), "same", stats=st)
    yb = out.float().reshape(-1, cout)
    close(st[:, 0].sum(0), yb.sum(0), 1e-4, 1e-5)
    close(st[:, 1].sum(0), (yb * yb).sum(0), 1e-4, 1e-5)


@pytest.mark.parametrize("split", [False, True])
def test_conv_split_k_epilogues(H, monkeypatch, split):
    """Both bf16-output GEMM paths: fused epilogue (no split) and split-K slabs + the
    finishing kernel (bias / ReLU / BN statistics / dgrad accumulation)."""
    monkeypatch.setattr(H, "SPLIT_MIN_TILES", 1 << 30 if split else 0)
    n, h, cin, cout = 2, 7, 128, 64
    plan = H.conv_fwd_plan((n, h, h, cin), (3, 3, cin, cout), (1, 1), "same")
    assert (plan["splits"] > 1) == split
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
    # dgrad (+accumulate) through the same two paths (dx has Cin = 128 columns)
    dy = rb(rnd(n, h, h, cout, seed=43)).requires_grad_(False)
    xx = x.clone().requires_grad_(True)
    gx, = torch.autograd.grad(ref.conv2d(xx, w, None, (1, 1), "same"), (xx,), dy)
    assert (H.conv_dgrad_plan(x.shape, w.shape, (1, 1), "same")["splits"] > 1) == split
    dx = torch.empty(x.shape, device=dev, dtype=torch.bfloat16)
    H.conv_dgrad(dy.bfloat16(), w.bfloat16(), dx, (1, 1), "same")
    close(dx, gx, 1e-2, 4e-3)
    H.conv_dgrad(dy.bfloat16(), w.bfloat16(), dx, (1, 1), "same", accumulate=True)
    close(dx, 2 * gx, 1e-2, 8e-3)


@pytest.mark.parametrize("relu,res", [(False, None), (True, None), (True, "raw"), (True, "bn")])
def test_batchnorm_train_fwd_bwd(H, relu, res):
    n, h, C = 4, 6, 48
    M = n * h * h
    x = rb(rnd(n, h, h, C, scale=2.0, seed=13) + 0.5)
    g = rnd(C, seed=14).abs() + 0.5
    be = rnd(C, seed=15)
    r = rb(rnd(n, h, h, C, seed=16))
    g2, be2 = rnd(C, seed=17).abs() + 0.5, rnd(C, seed=18)
    eps, mom = 1e-3, 0.99
    # torch reference
    xr = x.clone().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), be.clone().requires_grad_(True)
    rr = r.clone().requires_grad_(True)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    yr = ref.batchnorm(xr, gr, br, rm, rv, True, mom, eps)
    if res == "raw":
        yr = yr + rr
    elif res == "bn":
        yr = yr + ref.batchnorm(rr, g2, be2, torch.zeros(C, device=dev), torch.ones(C, device=dev), True, mom, eps)
    if relu:
        yr = yr.relu()
    dy = rb(rnd(*yr.shape, seed=19))
    grads = torch.autograd.grad(yr, (xr, gr, br, rr) if res else (xr, gr, br), dy)
    # HIP: stats from a plain column-sum pass (as the GEMM epilogue would give)
    xf = x.reshape(M, C)
    part = torch.stack([xf.sum(0), (xf * xf).sum(0)]).unsqueeze(0).contiguous()
    st = torch.empty(4, C, device=dev)
    mean = torch.zeros(C, device=dev)
    var = torch.ones(C, device=dev)
    H.bn_finalize(part, 1, C, M, g, be, eps, mom, mean, var, st)
    close(mean, rm, 1e-5, 1e-6)
    close(var, rv, 1e-5, 1e-6)
    st2 = None
    if res == "bn":
        rf = r.reshape(M, C)
        p2 = torch.stack([rf.sum(0), (rf * rf).sum(0)]).unsqueeze(0).contiguous()
        st2 = torch.empty(4, C, device=dev)
        H.bn_finalize(p2, 1, C, M, g2, be2, eps, mom, None, None, st2)
    y = torch.empty(x.shape, device=dev, dtype=torch.bfloat16)
    H.bn_apply(x.bfloat16(), st, y, relu=relu, r=r.bfloat16() if res else None, st2=st2)
    close(y, yr.detach(), 1e-2, 5e-3)
    from distributed_amd.native import require_C

    T = require_C().bn_bwd_blocks(M, C)
    bpart = torch.empty(T, 2, C, device=dev)
    co = torch.empty(3, C, device=dev)
    dx = torch.empty(x.shape, device=dev, dtype=torch.bfloat16)
    dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    dz = torch.empty(x.shape, device=dev, dtype=torch.bfloat16) if res else None
    # the HIP backward takes the relu mask from the bf16 block output y
    H.bn_bwd(dy.bfloat16(), y, relu, x.bfloat16(), st, bpart, co, dx, dg, db, dz_out=dz)
    if relu and res is None:
        # mask from the kernel's own output (a bf16-rounded 0 can differ from fp32 sign)
        pass
    close(dx, grads[0], 2e-2, 1e-2)
    close(dg, grads[1], 1e-3, 1e-3)
    close(db, grads[2], 1e-3, 1e-3)
    if res == "raw":
        close(dz, grads[3], 1e-2, 4e-3)


@pytest.mark.parametrize("pool,strides,padding,h", [((3, 3), (2, 2), "same", 12), ((2, 2), (2, 2), "valid", 26),
                                                    ((3, 3), (2, 2), "same", 7)])
def test_maxpool(H, pool, strides, padding, h):
    C = 32
    x = rb(rnd(2, h, h, C, seed=20)).requires_grad_(True)
    y = ref.maxpool2d(x, pool, strides, padding)
    dy = rb(rnd(*y.shape, seed=21))
    (gx,) = torch.autograd.grad(y, (x,), dy)
    out = torch.empty(y.shape, device=dev, dtype=torch.bfloat16)
    arg = torch.empty(y.shape, device=dev, dtype=torch.uint8)
    H.maxpool_fwd(x.detach().bfloat16(), out, arg, pool, strides, padding)
    close(out, y.detach(), 0, 0)
    dx = torch.empty(x.shape, device=dev, dtype=torch.bfloat16)
    H.maxpool_bwd(dy.bfloat16(), arg, dx, pool, strides, padding)
    close(dx, gx, 1e-2, 4e-3)


def test_gap_xent_colsum_sgd(H):
    x = rb(rnd(3, 7, 7, 64, seed=22))
    y32 = torch.empty(3, 64, device=dev)
    H.gap_fwd(x.bfloat16(), y32)
    close(y32, x.mean(dim=(1, 2)), 1e-4, 1e-5)
    dy = rnd(3, 64, seed=23)
    dx = torch.empty(x.shape, device=dev, dtype=torch.bfloat16)
    H.gap_bwd(dy, dx)
    close(dx, (dy / 49)[:, None, None, :].expand(x.shape), 1e-2, 4e-3)
    # softmax xent over a padded row pitch
    B, K, ld = 5, 10, 16
    z = rnd(B, ld, seed=24)
    lab = torch.tensor([0, 3, 9, 9, 1], device=dev, dtype=torch.int32)
    dl = torch.zeros(B, ld, device=dev, dtype=torch.bfloat16)
    tail = torch.zeros(3, device=dev)
    H.softmax_xent(z, lab, K, 0.5, dl, tail)
    zz = z[:, :K].clone().requires_grad_(True)
    loss = ref.sparse_softmax_xent(zz, lab)
    (gz,) = torch.autograd.grad(loss.sum() * 0.5, (zz,))
    close(dl[:, :K], gz, 1e-2, 4e-3)
    assert dl[:, K:].abs().max().item() == 0
    close(tail[0], loss.sum(), 1e-5, 1e-6)
    assert tail[1].item() == ref.sparse_accuracy(z[:, :K], lab).sum().item()
    assert tail[2].item() == B
    # a label < 0 masks its row: zero gradient, no loss / metric contribution
    lab2 = lab.clone()
    lab2[2] = -1
    dl2 = torch.ones(B, ld, device=dev, dtype=torch.bfloat16)
    tail2 = torch.zeros(3, device=dev)
    H.softmax_xent(z, lab2, K, 0.5, dl2, tail2)
    keep = torch.tensor([0, 1, 3, 4], device=dev)
    close(dl2[keep, :K], gz[keep], 1e-2, 4e-3)
    assert dl2[2, :K].abs().max().item() == 0
    close(tail2[0], loss[keep].sum(), 1e-5, 1e-6)
    assert tail2[2].item() == B - 1
    # column sums (bias grads)
    a = rb(rnd(300, 24, seed=25))
    cs = torch.zeros(24, device=dev)
    H.colsum(a.bfloat16(), cs)
    close(cs, a.sum(0), 1e-4, 1e-5)
    # flat SGD (+momentum, nesterov) with the bf16 shadow
    n = 1001
    P, G, V = rnd(n, seed=26), rnd(n, seed=27), rnd(n, seed=28)
    Pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
    p0, v0 = P.clone(), V.clone()
    H.sgd_flat(P, G, V, Pb, 0.1, 0.9, True)
    vn = 0.9 * v0 - 0.1 * G
    close(V, vn, 1e-6, 1e-7)
    close(P, p0 + 0.9 * vn - 0.1 * G, 1e-6, 1e-7)
    assert torch.equal(Pb, P.bfloat16())


@pytest.mark.parametrize("M,K,N", [(64, 512, 1008), (64, 5408, 64), (64, 64, 16), (64, 256, 4096), (64, 4096, 256)])
@pytest.mark.parametrize("out_bf16", [False, True])
def test_dense_split_k(H, M, K, N, out_bf16):
    """Split-K dense forward / backprop-input (workspace given, small-M shapes) against the
    fp32 reference, including the bias/ReLU and accumulate epilogues of the finish kernels.
    N or K = 4096: the finish kernel's column bands (more than 2048 columns per row)."""
    splits, _ = H.dense_split_plan(M, N, K)
    assert splits > 1
    ws = torch.empty(H.dense_workspace_elems(M, N, K), device=dev)
    x = rb(rnd(M, K, seed=11))
    w = rb(rnd(K, N, scale=0.1, seed=12))
    b = rnd(N, seed=13)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16 if out_bf16 else torch.float32)
    H.dense_fwd(x.bfloat16(), w.bfloat16(), out, bias=b, relu=True, workspace=ws)
    close(out, (x @ w + b).relu(), 1e-2 if out_bf16 else 1e-4, 4e-3 if out_bf16 else 1e-5)
    dy = rb(rnd(M, N, seed=14))
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    H.dense_dgrad(dy.bfloat16(), w.bfloat16(), dx, workspace=ws)
    close(dx, dy @ w.t(), 1e-2, 4e-3)
    H.dense_dgrad(dy.bfloat16(), w.bfloat16(), dx, accumulate=True, workspace=ws)
    close(dx, 2 * (dy @ w.t()), 1e-2, 8e-3)


@pytest.mark.parametrize("B,K,ld", [(64, 1000, 1024), (7, 1024, 1024), (3, 1500, 1504), (4, 300, 300)])
def test_softmax_xent_wide_rows(H, B, K, ld):
    """softmax_xent_k at the ResNet-18 head's width (64 x 1000) and around its register
    path's limit (4 x 256 values per row; 1500 takes the re-reading loop): gradient, loss,
    accuracy and count against the fp32 reference, ties of the max resolved to the smallest
    index as the reference's argmax does, and two runs bitwise equal."""
    z = rnd(B, ld, seed=31)
    z[0, 5] = z[0, 9] = z[0, :K].max() + 1.0  # a tie for the max: class 5 wins
    lab = torch.randint(0, K, (B,), device=dev, dtype=torch.int32)
    lab[0] = 5
    dl = torch.zeros(B, ld, device=dev, dtype=torch.bfloat16)
    tail = torch.zeros(3, device=dev)
    H.softmax_xent(z, lab, K, 1.0 / B, dl, tail)
    zz = z[:, :K].clone().requires_grad_(True)
    loss = ref.sparse_softmax_xent(zz, lab)
    (gz,) = torch.autograd.grad(loss.sum() / B, (zz,))
    close(dl[:, :K], gz, 1e-2, 4e-3)
    assert ld == K or dl[:, K:].abs().max().item() == 0
    close(tail[0], loss.sum(), 1e-5, 1e-6)
    assert tail[1].item() == ref.sparse_accuracy(z[:, :K], lab).sum().item()
    assert tail[1].item() >= 1  # row 0: the tie resolved to its label
    assert tail[2].item() == B
    dl2 = torch.zeros_like(dl)
    tail2 = torch.zeros(3, device=dev)
    H.softmax_xent(z, lab, K, 1.0 / B, dl2, tail2)
    assert torch.equal(dl, dl2) and torch.equal(tail, tail2)
    # the bias-gradient fold (vectorised path for ld % 8 == 0 and K <= 1024, else the
    # per-column loop) adds exactly what colsum adds
    if H.softmax_bias_fold_ok(B, K):
        base = rnd(K, seed=32)
        bg, bc = base.clone(), base.clone()
        dl3 = torch.zeros_like(dl)
        H.softmax_xent(z, lab, K, 1.0 / B, dl3, torch.zeros(3, device=dev), bias_grad=bg)
        H.colsum(dl3, bc, M=B, N=K, ld=ld)
        assert torch.equal(bg, bc)


@pytest.mark.parametrize("n,hw,c,f32", [(64, 7, 512, True), (5, 7, 2048, False), (3, 2, 64, False), (2, 14, 8, True)])
def test_gap_fwd_paths(H, n, hw, c, f32):
    """Global average pool: per-image split kernel (C/8 <= 128, HW >= 8) and the
    per-channel-group kernel, fp32 and bf16 outputs."""
    x = rb(rnd(n, hw, hw, c, seed=60))
    y = torch.empty(n, c, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
    H.gap_fwd(x.bfloat16(), y)
    close(y, x.mean(dim=(1, 2)), 1e-4 if f32 else 1e-2, 1e-5 if f32 else 4e-3)


def test_bn_statistics_accumulators_are_order_independent(H):
    """BatchNorm statistics through the int64 fixed-point accumulators (damd_common.h
    bnacc_add1 / bnacc_add2): the sums do not depend on the order in which producer blocks
    arrive nor on how they are spread over replicas -- bitwise.  Backward (two words per
    value): bn_bwd_reduce with 8 replicas, with its grid launched in REVERSED block order
    (block b reduces the rows of block G-1-b) and with 1 replica.  Forward (one word): a
    conv epilogue's statistics into 1 and 8 replicas.  Both agree with an fp64 reference."""
    from distributed_amd.native import require_C

    C_ = require_C()
    M, C = 4096 + 37, 64
    dy = rb(rnd(M, C, scale=1e-4, seed=41)).bfloat16()
    x = rb(rnd(M, C, seed=42) * 2 + 0.5).bfloat16()
    st = torch.stack([x.float().mean(0), torch.rsqrt(x.float().var(0) + 1e-3),
                      torch.ones(C, device=dev), torch.zeros(C, device=dev)]).contiguous()
    T = C_.bn_bwd_blocks(M, C)
    s = torch.cuda.current_stream().cuda_stream
    outs = []
    for reps, rev in ((8, False), (8, True), (1, False)):
        acc = H.acc_zeros(reps, 4 * C, dev)
        C_.bn_reduce_reverse(rev)
        try:
            C_.bn_bwd_reduce_acc(dy.data_ptr(), 0, 0, x.data_ptr(), st.data_ptr(), 0, acc.data_ptr(), T, M, C, s, reps)
            torch.cuda.synchronize()
        finally:
            C_.bn_reduce_reverse(False)
        assert not acc[-1].any(), "finite partials set the non-finite flag"
        words = acc.cpu()[:-1].sum(0)
        outs.append(words)
    assert torch.equal(outs[0], outs[1]), "reversed block order changed the backward sums"
    assert torch.equal(outs[0], outs[2]), "the replica count changed the backward sums"
    got = H.bn_acc_decode(torch.stack([outs[0], torch.zeros_like(outs[0])]), words=2)
    d, xh = dy.double(), (x.double() - st[0].double()) * st[1].double()
    want = torch.cat([d.sum(0), (d * xh).sum(0)]).cpu()
    assert torch.allclose(got, want, rtol=1e-5, atol=1e-12), (got - want).abs().max()

    # forward statistics (one word per value) from a conv epilogue, 1 vs 8 replicas
    n, h, cin, cout = 8, 16, 64, 64
    xb = rb(rnd(n, h, h, cin, seed=43)).bfloat16()
    wb = rb(rnd(3, 3, cin, cout, scale=0.05, seed=44)).bfloat16()
    sums = []
    for reps in (1, 8):
        acc = H.acc_zeros(reps, 2 * cout, dev)
        out = torch.empty(n, h, h, cout, device=dev, dtype=torch.bfloat16)
        # (reps 1: the 1-D form, one replica then its flag plane)
        H.conv_fwd(xb, wb, out, (1, 1), "same", stats=acc if reps > 1 else acc.view(-1))
        torch.cuda.synchronize()
        sums.append(acc.cpu()[:-1].sum(0))
    assert torch.equal(sums[0], sums[1]), "the replica count changed the forward statistics"
    o = out.double().reshape(-1, cout)
    want = torch.cat([o.sum(0), (o * o).sum(0)]).cpu()
    got = H.bn_acc_decode(torch.stack([sums[0], torch.zeros_like(sums[0])]), words=1)
    assert torch.allclose(got, want, rtol=1e-5, atol=1e-3), (got - want).abs().max()


def test_bn_accumulators_large_sums_and_sticky_nonfinite_flag(H):
    """(a) a FINITE sum above 2^33 (sum of squares of a conv output with mean
    square ~5e5 over 65,536 positions ~ 3e10) decodes finite and right -- round 5's in-word
    poison read every |word| >= 2^57 (sums >= 2^33) as NaN; (b) non-finite partials set a
    sticky per-channel flag: channel 3 NaN in EVERY block (a block count that is a multiple
    of 64 wrapped the additive poison to 0) and channel 5 with +inf in one block and -inf
    in another (they cancelled) both decode NaN; the other channels stay exact."""
    from distributed_amd.native import require_C

    C_ = require_C()
    n, h, cin, cout = 64, 32, 64, 64
    xb = rb(rnd(n, h, h, cin, seed=51) * 60).bfloat16()
    wb = rb(rnd(3, 3, cin, cout, scale=0.5, seed=52)).bfloat16()
    acc = H.acc_zeros(8, 2 * cout, dev)
    out = torch.empty(n, h, h, cout, device=dev, dtype=torch.bfloat16)
    H.conv_fwd(xb, wb, out, (1, 1), "same", stats=acc)
    torch.cuda.synchronize()
    o = out.double().reshape(-1, cout)
    want = torch.cat([o.sum(0), (o * o).sum(0)]).cpu()
    assert want[cout:].min() > 2.0 ** 33, want[cout:].min()
    got = H.bn_acc_decode(acc, words=1)
    assert torch.isfinite(got).all()
    assert torch.allclose(got, want, rtol=1e-5, atol=1e-3), (got - want).abs().max()

    M, C = 64 * 1024, 64
    T = C_.bn_bwd_blocks(M, C)
    dy = rb(rnd(M, C, scale=1e-3, seed=53))
    dy[:, 3] = float("nan")
    dy[7, 5] = float("inf")
    dy[M - 9, 5] = float("-inf")
    dy = dy.bfloat16()
    x = rb(rnd(M, C, seed=54)).bfloat16()
    st = torch.stack([x.float().mean(0), torch.rsqrt(x.float().var(0) + 1e-3),
                      torch.ones(C, device=dev), torch.zeros(C, device=dev)]).contiguous()
    acc = H.acc_zeros(8, 4 * C, dev)
    s = torch.cuda.current_stream().cuda_stream
    C_.bn_bwd_reduce_acc(dy.data_ptr(), 0, 0, x.data_ptr(), st.data_ptr(), 0, acc.data_ptr(), T, M, C, s, 8)
    torch.cuda.synchronize()
    got = H.bn_acc_decode(acc, words=2)
    bad = torch.zeros(2 * C, dtype=torch.bool)
    for c in (3, 5):
        bad[c] = bad[C + c] = True
    assert torch.isnan(got[bad]).all(), got[bad]
    assert torch.isfinite(got[~bad]).all()
    d, xh = dy.double(), (x.double() - st[0].double()) * st[1].double()
    want = torch.cat([d.sum(0), (d * xh).sum(0)]).cpu()
    assert torch.allclose(got[~bad], want[~bad], rtol=1e-5, atol=1e-12)
