"""Run one ResNet-18 conv layer's fwd / dgrad / wgrad HIP GEMMs N times (for rocprofv3
--pmc passes on isolated kernels).  usage: gemm_one.py h cin cout k s [iters] [B]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.ops import hip as H  # noqa: E402

h, cin, cout, k, s = (int(v) for v in sys.argv[1:6])
it = int(sys.argv[6]) if len(sys.argv) > 6 else 20
B = int(sys.argv[7]) if len(sys.argv) > 7 else 64
dev = torch.device("cuda:0")
pad = "same" if k > 1 else "valid"
ho, _ = H.conv_out(h, k, s, pad)
x = torch.randn(B, h, h, cin, device=dev).bfloat16()
w = (torch.randn(k, k, cin, cout, device=dev) * 0.05).bfloat16()
y = torch.empty(B, ho, ho, cout, device=dev, dtype=torch.bfloat16)
dy = torch.randn(B, ho, ho, cout, device=dev).bfloat16()
dx = torch.empty_like(x)
dw = torch.zeros(k, k, cin, cout, device=dev)
ws = torch.empty(max(H.conv_fwd_plan(x.shape, w.shape, (s, s), pad)["ws"],
                     H.conv_dgrad_plan(x.shape, w.shape, (s, s), pad)["ws"],
                     H.conv_wgrad_workspace_elems(x.shape, w.shape, (s, s), pad), 4), device=dev)
for _ in range(it):
    H.conv_fwd(x, w, y, (s, s), pad, workspace=ws)
    H.conv_dgrad(dy, w, dx, (s, s), pad, workspace=ws)
    H.conv_wgrad(x, dy, dw, (s, s), pad, workspace=ws)
torch.cuda.synchronize()
print("ok")
