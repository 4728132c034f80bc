"""Direct 3x3 weight gradient (conv_wgrad3.hip) on the ResNet-18 shapes: time of the
wgrad3 launch alone and of conv_wgrad (+ the split-K reduce), per pipeline depth
DAMD_WGRAD3_STAGES, and per-block phases from s_memrealtime stamps (start, first k-step's
operands landed, k-loop done, slab stores done).  GPU box:
    python scripts/wgrad3_probe.py [stages ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.native import require_C  # noqa: E402
from distributed_amd.ops import hip as H  # noqa: E402

dev = torch.device("cuda:0")
C = require_C()
STAGES = [int(a) for a in sys.argv[1:]] or [3, 4, 6]


def timeit(fn, n=30):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def phases(fn, nblk):
    C.wgrad3_stamps_enable(1)
    fn()
    torch.cuda.synchronize()
    st = np.array(C.wgrad3_stamps_read(min(nblk, 4096)), dtype=np.float64).reshape(-1, 4)
    C.wgrad3_stamps_enable(0)
    st = st[st[:, 0] > 0]
    rel = (st - st[:, :1]) / 100.0  # per-block durations (the clock differs across the chip halves)
    q = lambda v: f"{np.median(v):6.2f} [{np.percentile(v, 10):5.2f}, {np.percentile(v, 90):5.2f}]"
    print(f"      blocks {len(st)}: landed {q(rel[:, 1])}  k-loop {q(rel[:, 2] - rel[:, 1])}  "
          f"slab stores {q(rel[:, 3] - rel[:, 2])}  lifetime {q(rel[:, 3])}  (median [p10, p90] us)")


B = 64
for h, c in [(56, 64), (28, 128), (14, 256)]:
    x = torch.randn(B, h, h, c, device=dev).bfloat16()
    dy = torch.randn(B, h, h, c, device=dev).bfloat16()
    dw = torch.zeros(3, 3, c, c, device=dev)
    plan = H.conv_wgrad_plan(x.shape, dw.shape, (1, 1), "same")
    assert plan["amode"] == H.A_WGRAD3
    ws = torch.empty(plan["ws"], device=dev)
    geo = (h, h, c, h, h, 3, 3, 1, 1)
    flop = 2.0 * B * h * h * c * 9 * c
    kern = lambda: H.gemm(x, dy, ws, amode=H.A_WGRAD3, bmode=H.B_NC, M=plan["M"], N=plan["N"], K=plan["K"],
                          ldb=c, ldc=plan["N"], epi=H.E_SLAB, splits=plan["splits"], k_per_split=plan["kps"],
                          tile=0, geo=geo)
    full = lambda: H.conv_wgrad(x, dy, dw, (1, 1), "same", workspace=ws, accumulate=False)
    print(f"{h}x{h} {c}->{c}: splits {plan['splits']}  slab {plan['ws'] * 4 / 2**20:.1f} MB")
    for s in STAGES:
        os.environ["DAMD_WGRAD3_STAGES"] = str(s)
        tk, tf = timeit(kern), timeit(full)
        print(f"   S={s}: wgrad3 {tk:7.2f} us ({flop / tk / 1e6:6.1f} TFLOP/s)   + reduce {tf:7.2f} us")
        phases(kern, plan["splits"] * (c // 64) ** 2)
