"""Sweep of the direct 3x3 weight-gradient kernel (csrc/kernels/conv_wgrad3.hip) on the
ResNet-18 3x3/stride-1 shapes: pipeline stages and target workgroups,
vs the LDS-DMA GEMM weight gradient; ms per call including the split-K slab reduce.
Usage: python scripts/bench_wgrad3.py [B]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.ops import hip as H  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda:0")
SHAPES = [(56, 64, 64, 4), (28, 128, 128, 3), (14, 256, 256, 3), (7, 512, 512, 3)]  # h, cin, cout, count
VARIANTS = [("glds", {"DAMD_WGRAD_KERNEL": "glds"})]
for st in ("2", "3", "4"):
    for wg in ("192", "256", "512"):
        VARIANTS.append((f"s{st}w{wg}", {"DAMD_WGRAD_KERNEL": "direct", "DAMD_WGRAD3_STAGES": st,
                                         "DAMD_WGRAD3_WG": wg}))


ONLY = os.environ.get("BENCH_W3_ONLY")  # comma-separated variant names
if ONLY:
    VARIANTS = [v for v in VARIANTS if v[0] in ONLY.split(",")]


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


tot = {}
for h, cin, cout, cnt in SHAPES:
    x = torch.randn(B, h, h, cin, device=dev).bfloat16()
    dy = torch.randn(B, h, h, cout, device=dev).bfloat16()
    dw = torch.zeros(3, 3, cin, cout, device=dev)
    flop = 2.0 * B * h * h * cout * 9 * cin
    line = []
    for name, env in VARIANTS:
        os.environ.update(env)
        plan = H.conv_wgrad_plan(x.shape, dw.shape, (1, 1), "same")
        ws = torch.empty(max(plan["ws"], 4), device=dev)
        t = timeit(lambda: H.conv_wgrad(x, dy, dw, (1, 1), "same", workspace=ws))
        tot[name] = tot.get(name, 0.0) + cnt * t
        line.append(f"{name} {t * 1e3:.4f}/{flop / t / 1e12:.0f}/{plan['splits']}")
    print(f"{h}x{h} {cin}->{cout}: " + "  ".join(line), flush=True)
best = sorted(tot.items(), key=lambda kv: kv[1])
print("step-weighted 3x3/s1 wgrad (ms): " + ", ".join(f"{k} {v * 1e3:.3f}" for k, v in best), flush=True)
