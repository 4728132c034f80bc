"""Micro-benchmark of the generic-path MFMA kernels on the ResNet-18 conv shapes
(batch 64, bf16): our implicit-GEMM fwd / dgrad / wgrad vs torch's (MIOpen) conv in
channels_last bf16, reported in TFLOP/s.  Usage: python scripts/bench_gemm.py [B]"""
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
    (14, 256, 256, 3, 1),
    (14, 256, 512, 3, 2),
    (7, 512, 512, 3, 1),
]


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


print(f"B={B}  (ms / TFLOP/s)   ours: fwd dgrad wgrad | torch channels_last: fwd dgrad wgrad")
tot = [0.0, 0.0]
for h, cin, cout, k, s in SHAPES:
    pad = "same" if k > 1 else "valid"
    ho, p = H.conv_out(h, k, s, pad)
    x = torch.randn(B, h, h, cin, device=dev).bfloat16()
    w = (torch.randn(k, k, cin, cout, device=dev) * 0.05).bfloat16()
    y = torch.empty(B, ho, ho, cout, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(B, ho, ho, cout, device=dev).bfloat16()
    dx = torch.empty_like(x)
    dw = torch.zeros(k, k, cin, cout, device=dev)
    flop = 2.0 * B * ho * ho * cout * k * k * cin
    tf = timeit(lambda: H.conv_fwd(x, w, y, (s, s), pad))
    td = timeit(lambda: H.conv_dgrad(dy, w, dx, (s, s), pad)) if cin % 8 == 0 and h != 224 else float("nan")
    tw = timeit(lambda: H.conv_wgrad(x, dy, dw, (s, s), pad))
    # torch reference (NCHW logical, channels_last memory)
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
    ours = [tf, td, tw]
    ref = [rf, rd, rw]
    tot[0] += sum(t for t in ours if t == t)
    tot[1] += sum(ref)
    fmt = lambda t: f"{t * 1e3:7.3f}/{flop / t / 1e12:6.1f}" if t == t else "    n/a       "
    print(f"{h:3d}x{h:<3d} {cin:3d}->{cout:3d} k{k} s{s}: " + " ".join(fmt(t) for t in ours) + " | " +
          " ".join(fmt(t) for t in ref), flush=True)
print(f"sum of layers (one instance each): ours {tot[0] * 1e3:.3f} ms, torch {tot[1] * 1e3:.3f} ms")
