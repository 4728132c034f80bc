"""Phase stamps of the direct 3x3 conv kernel (csrc/kernels/conv3x3.hip) on one ResNet-18
layer: per block s_memrealtime at start, when the first tap's operands have landed, after
the nine taps, after the epilogue (100 MHz ticks).  usage: stamps_conv3.py h cin cout [dgrad]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.ops import hip as H  # noqa: E402

h, cin, cout = (int(v) for v in sys.argv[1:4])
dgrad = len(sys.argv) > 4 and sys.argv[4] == "dgrad"
B = 64
dev = torch.device("cuda:0")
x = torch.randn(B, h, h, cin, device=dev).bfloat16()
w = (torch.randn(3, 3, cin, cout, device=dev) * 0.05).bfloat16()
y = torch.empty(B, h, h, cout, device=dev, dtype=torch.bfloat16)
dy = torch.randn(B, h, h, cout, device=dev).bfloat16()
dx = torch.empty_like(x)
plan = (H.conv_dgrad_plan if dgrad else H.conv_fwd_plan)(x.shape, w.shape, (1, 1), "same")
assert plan["amode"] in (H.A_CONV3, H.A_DGRAD3), plan
st = torch.zeros(plan.get("stats_T", 1), 2, cout, device=dev)


def run():
    if dgrad:
        H.conv_dgrad(dy, w, dx, (1, 1), "same")
    else:
        H.conv_fwd(x, w, y, (1, 1), "same", stats=st)


for _ in range(10):
    run()
torch.cuda.synchronize()
C = H._C()
C.conv3_stamps_enable(1)
run()
torch.cuda.synchronize()
C.conv3_stamps_enable(0)
bn = 64 if (cin if dgrad else cout) % 128 else 128
r = H.conv3_rows(h, h, bn)
nb = ((cin if dgrad else cout) // bn) * B * -(-h // r)
s = np.array(C.conv3_stamps_read(nb), dtype=np.int64).reshape(nb, 4)
t0 = s[:, 0].min()
rel = (s - t0) / 100.0  # us
print(f"{'dgrad' if dgrad else 'fwd'} {h}x{h} {cin}->{cout}: {nb} blocks, span {rel[:, 3].max():.2f} us")
for name, v in (("start", rel[:, 0]), ("operands landed", rel[:, 1] - rel[:, 0]), ("taps", rel[:, 2] - rel[:, 1]),
                ("epilogue", rel[:, 3] - rel[:, 2]), ("block total", rel[:, 3] - rel[:, 0])):
    print(f"  {name:16s} median {np.median(v):7.2f}  min {v.min():7.2f}  max {v.max():7.2f} us")
