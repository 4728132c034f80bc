"""In-launch split-K finish vs the finish kernel on the small-ResNet conv shapes: forward
output / BN statistics and backprop-input, printing the max differences."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from distributed_amd.ops import hip as H  # noqa: E402
from distributed_amd.ops import reference as ref  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
for (n, h, cin, cout, s) in [(32, 8, 128, 128, 1), (32, 4, 128, 128, 1), (32, 2, 128, 128, 1), (32, 16, 64, 128, 2),
                             (32, 8, 128, 128, 2), (8, 7, 512, 512, 1)]:
    x = (torch.randn(n, h, h, cin, generator=g) * 0.5).to(dev).bfloat16()
    w = (torch.randn(3, 3, cin, cout, generator=g) * 0.05).to(dev).bfloat16()
    plan = H.conv_fwd_plan(x.shape, w.shape, (s, s), "same")
    res = {}
    for fix in ("1", "0"):
        os.environ["DAMD_SPLITK_FIXUP"] = fix
        ho = plan["M"] // n
        out = torch.empty(n, int(ho ** 0.5), int(ho ** 0.5), cout, device=dev, dtype=torch.bfloat16)
        acc = H.acc_zeros(8, 2 * cout, dev)
        H.conv_fwd(x, w, out, (s, s), "same", stats=acc)
        torch.cuda.synchronize()
        res[fix] = (out.float(), H.bn_acc_decode(acc))
    yref = ref.conv2d(x.float(), w.float(), None, (s, s), "same")
    d_out = (res["1"][0] - res["0"][0]).abs().max().item()
    d_st = (res["1"][1] - res["0"][1]).abs().max().item()
    st_true = torch.cat([yref.reshape(-1, cout).sum(0), (yref.reshape(-1, cout) ** 2).sum(0)]).double().cpu()
    print(f"{(n, h, cin, cout, s)} amode {plan['amode']} splits {plan['splits']}: out diff {d_out:.3e}, "
          f"stats diff {d_st:.3e} (|stats| max {res['0'][1].abs().max().item():.3e}), "
          f"vs fp32 ref {(res['1'][1] - st_true).abs().max().item():.3e} / {(res['0'][1] - st_true).abs().max().item():.3e}")
