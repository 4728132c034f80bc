"""Direct 3x3 conv (conv3x3.hip) on the ResNet-18 shapes: kernel time (hipEvent over 50
back-to-back launches) and per-block in-kernel phases from s_memrealtime stamps (start,
first tap's operands landed, taps done, epilogue done), to see where a block's lifetime
goes; forward also on a BatchNorm input (bnin).  GPU box:  python scripts/conv3_probe.py [B]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.native import require_C  # noqa: E402
from distributed_amd.ops import hip as H  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda:0")
C = require_C()


def timeit(fn, n=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3  # us


def phases(fn, nblk):
    C.conv3_stamps_enable(1)
    fn()
    torch.cuda.synchronize()
    st = np.array(C.conv3_stamps_read(min(nblk, 4096)), dtype=np.float64).reshape(-1, 4)
    C.conv3_stamps_enable(0)
    st = st[st[:, 0] > 0]
    if len(st) == 0:  # a kernel without stamps (conv3r.hip)
        print("    (no phase stamps: persistent conv3r kernel)")
        return
    t0 = st[:, 0].min()
    rel = (st - t0) / 100.0  # 100 MHz -> us
    land, taps, epi = rel[:, 1] - rel[:, 0], rel[:, 2] - rel[:, 1], rel[:, 3] - rel[:, 2]  # (persistent: first
    # tile's landing, all tiles' taps + epilogues but the last, the last epilogue + BN tail)
    life = rel[:, 3] - rel[:, 0]
    q = lambda v: f"{np.median(v):6.2f} [{np.percentile(v, 10):5.2f}, {np.percentile(v, 90):5.2f}]"
    # (s_memrealtime is not synchronised across the two halves of the chip: the spreads
    # below mix clocks; per-block durations are exact)
    print(f"    blocks {len(st)}: start spread {rel[:, 0].max():.2f} us, end {rel[:, 3].max():.2f} us")
    print(f"    landed {q(land)}  taps {q(taps)}  epilogue {q(epi)}  lifetime {q(life)}  (median [p10, p90] us)")
    # start-time histogram: how many rounds of blocks
    h, e = np.histogram(rel[:, 0], bins=8)
    print("    start histogram:", " ".join(f"{int(c)}@{x:.1f}" for c, x in zip(h, e)))


SHAPES = [(56, 64, 64), (28, 128, 128), (14, 256, 256)]
for h, cin, cout in SHAPES:
    x = torch.randn(B, h, h, cin, device=dev).bfloat16()
    w = (torch.randn(3, 3, cin, cout, device=dev) * 0.05).bfloat16()
    y = torch.empty(B, h, h, cout, device=dev, dtype=torch.bfloat16)
    plan = H.conv_fwd_plan(x.shape, w.shape, (1, 1), "same")
    st = H.acc_zeros(8, 2 * cout, dev)  # fixed-point statistics accumulators (as the engine)
    flop = 2.0 * B * h * h * cout * 9 * cin
    f = lambda: H.conv_fwd(x, w, y, (1, 1), "same", stats=st)
    t = timeit(f)
    print(f"fwd  {h}x{h} {cin}->{cout}: {t:7.2f} us  {flop / t / 1e6:6.1f} TFLOP/s  plan {plan['amode']} tile {plan['tile']}")
    phases(f, 4096)
    # the same conv on a BatchNorm's input (GemmArgs::bnin: finalize + BN/ReLU on load + y store)
    acc = torch.zeros(8 + 1, 2 * cin, dtype=torch.int64, device=dev)  # 8 replicas + the flag plane
    acc[0, cin:] = (B * h * h) << 24  # sum of squares = count (fixed point, 2^-24 units)
    bst = torch.zeros(4, cin, device=dev)
    fin = H.BNFin(acc, None, None, bst, None, None, B * h * h, 1e-3, 0.99)
    yb = torch.empty_like(x)
    fb = lambda: H.conv_fwd(x, w, y, (1, 1), "same", stats=st, bnin=(fin, yb))
    t = timeit(fb)
    print(f"fwd+bn {h}x{h} {cin}->{cout}: {t:7.2f} us  (BN input: finalize, normalise on load, store y)")
    phases(fb, 4096)
    dy = torch.randn(B, h, h, cout, device=dev).bfloat16()
    dx = torch.empty_like(x)
    g = lambda: H.conv_dgrad(dy, w, dx, (1, 1), "same")
    t = timeit(g)
    print(f"dgrad {h}x{h} {cin}<-{cout}: {t:7.2f} us  {flop / t / 1e6:6.1f} TFLOP/s")
    phases(g, 4096)
