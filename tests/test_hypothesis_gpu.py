"""Property tests of the HIP GEMM / conv kernels over hypothesis-drawn shapes (SURVEY.md
§4.2 "kernel (GPU)": ragged M/N/K, tails, both tile shapes, split-K and the LDS-DMA conv
paths), each against the plain PyTorch fp32 reference of the same op.  Derandomized, so a
run is reproducible; bf16 operands are rounded once and fed to both sides."""
import pytest
import torch

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from distributed_amd.ops import reference as ref  # noqa: E402

pytestmark = pytest.mark.gpu

dev = torch.device("cuda:0") if torch.cuda.is_available() else None
SETTINGS = dict(deadline=None, derandomize=True, suppress_health_check=[HealthCheck.too_slow],
                database=None)


def _H():
    from distributed_amd.ops import hip

    return hip


def rb(t):
    return t.to(torch.bfloat16).float()


def rnd(shape, scale, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dev)


def close(a, b, rtol, atol_frac):
    a, b = a.float(), b.float()
    atol = atol_frac * b.abs().max().item() + 1e-12
    err = (a - b).abs().max().item()
    assert torch.allclose(a, b, rtol=rtol, atol=atol), f"max abs err {err:.3e} (atol {atol:.3e})"


@settings(max_examples=30, **SETTINGS)
@given(M=st.integers(1, 300), K8=st.integers(1, 96), N8=st.integers(1, 64), bias=st.booleans(),
       relu=st.booleans(), out_bf16=st.booleans(), split=st.booleans(), seed=st.integers(0, 1000))
def test_dense_shapes(M, K8, N8, bias, relu, out_bf16, split, seed):
    H = _H()
    K, N = 8 * K8, 8 * N8
    x = rb(rnd((M, K), 1.0, seed))
    w = rb(rnd((K, N), 0.1, seed + 1))
    b = rnd((N,), 1.0, seed + 2) if bias else None
    ws = torch.empty(max(H.dense_workspace_elems(M, N, K), 4), device=dev) if split else None
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16 if out_bf16 else torch.float32)
    H.dense_fwd(x.bfloat16(), w.bfloat16(), out, bias=b, relu=relu, workspace=ws)
    r = x @ w + (b if bias else 0)
    r = r.relu() if relu else r
    close(out, r, 1e-2 if out_bf16 else 1e-4, 4e-3 if out_bf16 else 1e-5)
    dy = rb(rnd((M, N), 1.0, seed + 3))
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    H.dense_dgrad(dy.bfloat16(), w.bfloat16(), dx, workspace=ws)
    close(dx, dy @ w.t(), 1e-2, 4e-3)
    dw = torch.zeros(K, N, device=dev)
    H.dense_wgrad(x.bfloat16(), dy.bfloat16(), dw)
    close(dw, x.t() @ dy, 1e-4, 1e-5)


@settings(max_examples=25, **SETTINGS)
@given(n=st.integers(1, 3), h=st.integers(4, 18), cin=st.sampled_from([8, 16, 64, 128]),
       cout=st.sampled_from([8, 16, 64, 128]), k=st.sampled_from([1, 3]), s=st.sampled_from([1, 2]),
       padding=st.sampled_from(["same", "valid"]), bias=st.booleans(), relu=st.booleans(),
       seed=st.integers(0, 1000))
def test_conv_shapes(n, h, cin, cout, k, s, padding, bias, relu, seed):
    H = _H()
    if padding == "valid" and h < k:
        return
    x = rb(rnd((n, h, h, cin), 1.0, seed)).requires_grad_(True)
    w = rb(rnd((k, k, cin, cout), 0.2, seed + 1)).requires_grad_(True)
    y = ref.conv2d(x, w, None, (s, s), padding)
    dy = rb(rnd(tuple(y.shape), 1.0, seed + 2))
    gx, gw = torch.autograd.grad(y, (x, w), dy)
    ws = torch.empty(max(H.conv_fwd_plan(x.shape, w.shape, (s, s), padding)["ws"],
                         H.conv_dgrad_plan(x.shape, w.shape, (s, s), padding)["ws"],
                         H.conv_wgrad_workspace_elems(x.shape, w.shape, (s, s), padding), 4), device=dev)
    out = torch.empty(y.shape, device=dev, dtype=torch.bfloat16)
    b = rnd((cout,), 1.0, seed + 3) if bias else None
    H.conv_fwd(x.detach().bfloat16(), w.detach().bfloat16(), out, (s, s), padding, bias=b, relu=relu, workspace=ws)
    yr = y.detach() + (b if bias else 0)
    close(out, yr.relu() if relu else yr, 1e-2, 4e-3)
    dx = torch.empty(x.shape, device=dev, dtype=torch.bfloat16)
    H.conv_dgrad(dy.bfloat16(), w.detach().bfloat16(), dx, (s, s), padding, workspace=ws)
    close(dx, gx, 1e-2, 4e-3)
    dw = torch.zeros(w.shape, device=dev)
    H.conv_wgrad(x.detach().bfloat16(), dy.bfloat16(), dw, (s, s), padding, workspace=ws)
    close(dw, gw, 1e-4, 2e-5)
