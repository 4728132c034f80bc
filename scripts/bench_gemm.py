"""Micro-benchmark of the generic-path MFMA kernels on the ResNet-18 conv shapes
(batch 64, bf16): our implicit-GEMM fwd / dgrad / wgrad -- the LDS-DMA kernels
(conv_gemm.hip) where they apply and the register-staged ones (gemm.hip,
DAMD_CONV_GLDS=0) -- vs torch's (MIOpen) conv in channels_last bf16, in ms / TFLOP/s.
Usage: python scripts/bench_gemm.py [B]"""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.ops import hip as H  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda:0")
SHAPES = [  # h, cin, cout, k, s
    (224, 8, 64, 7, 2),
    (56, 64, 64, 3, 1),
    (56, 64, 128, 3, 2),
    (56, 64, 128, 1, 2),
    (28, 128, 128, 3, 1),
    (28, 128, 256, 3, 2),
    (28, 128, 256, 1, 2),
    (14, 256, 256, 3, 1),
    (14, 256, 512, 3, 2),
    (14, 256, 512, 1, 2),
    (7, 512, 512, 3, 1),
]
# instances of each shape in one ResNet-18 step (for the weighted sum)
COUNT = [1, 4, 1, 1, 3, 1, 1, 3, 1, 1, 3]


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def ours(x, w, y, dy, dx, dw, s, pad, glds, cfg="32:2"):
    os.environ["DAMD_CONV_GLDS"] = "1" if glds else "0"
    os.environ["DAMD_CONV_KB"], os.environ["DAMD_CONV_STAGES"] = cfg.split(":")
    ws = torch.empty(max(H.conv_fwd_plan(x.shape, w.shape, (s, s), pad)["ws"],
                         H.conv_dgrad_plan(x.shape, w.shape, (s, s), pad)["ws"],
                         H.conv_wgrad_workspace_elems(x.shape, w.shape, (s, s), pad), 4), device=dev)
    tf = timeit(lambda: H.conv_fwd(x, w, y, (s, s), pad, workspace=ws))
    td = timeit(lambda: H.conv_dgrad(dy, w, dx, (s, s), pad, workspace=ws)) if x.shape[1] != 224 else float("nan")
    tw = timeit(lambda: H.conv_wgrad(x, dy, dw, (s, s), pad, workspace=ws))
    return [tf, td, tw]


CFGS = os.environ.get("BENCH_CFG", "32:2").split(",")  # LDS-DMA kernels: kstep:stages
print(f"B={B}  (ms / TFLOP/s)  fwd dgrad wgrad:  glds {CFGS} | register-staged | torch channels_last",
      flush=True)
tot = {f"glds{c}": 0.0 for c in CFGS}
tot.update({"reg": 0.0, "torch": 0.0})
for (h, cin, cout, k, s), cnt in zip(SHAPES, COUNT):
    pad = "same" if k > 1 else "valid"
    ho, p = H.conv_out(h, k, s, pad)
    x = torch.randn(B, h, h, cin, device=dev).bfloat16()
    w = (torch.randn(k, k, cin, cout, device=dev) * 0.05).bfloat16()
    y = torch.empty(B, ho, ho, cout, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(B, ho, ho, cout, device=dev).bfloat16()
    dx = torch.empty_like(x)
    dw = torch.zeros(k, k, cin, cout, device=dev)
    flop = 2.0 * B * ho * ho * cout * k * k * cin
    gs = [ours(x, w, y, dy, dx, dw, s, pad, True, c) for c in CFGS]
    r = ours(x, w, y, dy, dx, dw, s, pad, False)
    xc = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wc = w.permute(3, 2, 0, 1).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    tp = (k - 1) // 2 if k > 1 else 0
    yc = F.conv2d(xc, wc, stride=s, padding=tp)
    dyc = torch.randn_like(yc)
    rf = timeit(lambda: F.conv2d(xc, wc, stride=s, padding=tp))
    rd = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [s, s], [tp, tp], [1, 1], False,
                                                              [0, 0], 1, [True, False, False]))
    rw = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [s, s], [tp, tp], [1, 1], False,
                                                              [0, 0], 1, [False, True, False]))
    t_ = [rf, rd, rw]
    rows = [(f"glds{c}", g) for c, g in zip(CFGS, gs)] + [("reg", r), ("torch", t_)]
    for key, v in rows:
        tot[key] += cnt * sum(t for t in v if t == t)
    fmt = lambda t: f"{t * 1e3:6.3f}/{flop / t / 1e12:4.0f}" if t == t else "  n/a      "
    print(f"{h:3d}x{h:<3d} {cin:3d}->{cout:3d} k{k} s{s} x{cnt}: " +
          " | ".join(" ".join(fmt(t) for t in v) for _, v in rows), flush=True)
print("ResNet-18 step-weighted sum of conv GEMMs: " +
      ", ".join(f"{k} {v * 1e3:.3f} ms" for k, v in tot.items()), flush=True)
