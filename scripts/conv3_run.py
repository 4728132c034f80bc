"""Run one direct 3x3 conv of a ResNet-18 shape N times (for rocprofv3 PMC passes):
    python scripts/conv3_run.py H CIN COUT [fwd|fwdbn|dgrad|wgrad] [B] [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.ops import hip as H  # noqa: E402

h, cin, cout = (int(v) for v in sys.argv[1:4])
mode = sys.argv[4] if len(sys.argv) > 4 else "fwd"
B = int(sys.argv[5]) if len(sys.argv) > 5 else 64
n = int(sys.argv[6]) if len(sys.argv) > 6 else 11
dev = torch.device("cuda:0")
x = torch.randn(B, h, h, cin, device=dev).bfloat16()
w = (torch.randn(3, 3, cin, cout, device=dev) * 0.05).bfloat16()
y = torch.empty(B, h, h, cout, device=dev, dtype=torch.bfloat16)
dy = torch.randn(B, h, h, cout, device=dev).bfloat16()
acc = H.acc_zeros(8, 2 * cout, dev)
if mode == "fwdbn":
    ain = H.acc_zeros(8, 2 * cin, dev)
    ain[0, cin:] = (B * h * h) << 24
    fin = H.BNFin(ain, None, None, torch.zeros(4, cin, device=dev), None, None, B * h * h, 1e-3, 0.99)
    yb = torch.empty_like(x)
if mode == "wgrad":
    dw = torch.zeros(3, 3, cin, cout, device=dev)
    ws = torch.empty(H.conv_wgrad_workspace_elems(x.shape, w.shape, (1, 1), "same") or 1, device=dev)
for _ in range(n):
    if mode == "fwd":
        H.conv_fwd(x, w, y, (1, 1), "same", stats=acc)
    elif mode == "fwdbn":
        H.conv_fwd(x, w, y, (1, 1), "same", stats=acc, bnin=(fin, yb))
    elif mode == "dgrad":
        H.conv_dgrad(dy, w, x, (1, 1), "same")
    else:
        H.conv_wgrad(x, dy, dw, (1, 1), "same", workspace=ws, accumulate=False)
torch.cuda.synchronize()
print("done", mode, h, cin, cout)
