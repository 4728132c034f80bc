"""Time the ResNet-18 stem forward (B = 64, 224 x 224 x 4 -> 112 x 112 x 64) through the
direct kernel (conv_stem.hip) and the implicit GEMM (DAMD_STEM_DIRECT=0), with and without
the BN-statistics epilogue: python scripts/stem_probe.py [batch]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from distributed_amd.ops import hip as H

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
k, cout = 7, 64
x4 = (torch.rand(n, 224, 224, 4, device=dev) * (torch.arange(4, device=dev) < 3)).bfloat16()
w8 = (torch.randn(H.stem4_weight_shape((k, k, 4, cout)), device=dev) * 0.1).bfloat16()
out = torch.empty(n, 112, 112, cout, device=dev, dtype=torch.bfloat16)
acc = H.acc_zeros(8, 2 * cout, dev)
for direct in ("1", "0"):
    os.environ["DAMD_STEM_DIRECT"] = direct
    for stats in (acc, None):
        for _ in range(3):
            H.conv_fwd_stem4(x4, w8, out, k, (2, 2), "same", stats=stats)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            H.conv_fwd_stem4(x4, w8, out, k, (2, 2), "same", stats=stats)
        e1.record()
        torch.cuda.synchronize()
        print(f"direct={direct} stats={'acc' if stats is not None else 'none'}: {e0.elapsed_time(e1) / reps * 1000:.1f} us")

# in-kernel phases of the direct kernel (s_memrealtime, 100 MHz): medians over blocks
import numpy as np  # noqa: E402

C = H._C()
os.environ["DAMD_STEM_DIRECT"] = "1"
H.conv_fwd_stem4(x4, w8, out, k, (2, 2), "same", stats=acc)
torch.cuda.synchronize()
C.stem_stamps_enable(1)
H.conv_fwd_stem4(x4, w8, out, k, (2, 2), "same", stats=acc)
torch.cuda.synchronize()
st = np.array(C.stem_stamps_read(512), dtype=np.float64).reshape(-1, 8)
C.stem_stamps_enable(0)
st = st[st[:, 0] > 0]
t0 = st[:, 0].min()
us = (st - t0) / 100.0  # 10 ns ticks -> us
names = ["start", "filter staged", "t0 rows landed", "t0 mfma done", "t0 epilogue done", "t1 rows landed",
         "t1 mfma done", "t1 epilogue done"]
for i, nm in enumerate(names):
    col = us[:, i]
    print(f"{nm:18s} median {np.median(col):7.2f} us  [p10 {np.percentile(col, 10):7.2f}, p90 {np.percentile(col, 90):7.2f}]")
