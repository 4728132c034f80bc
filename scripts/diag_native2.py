"""Check the first conv + BN of the native plan against torch after one step."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_amd as tf  # noqa: E402
from distributed_amd.ops import reference as ref  # noqa: E402
from tests.test_native_graph_gpu import _data, _small_resnet  # noqa: E402

x, y = _data(64, (32, 32, 3), 10)
os.environ["DAMD_FUSED"] = "0"
m = _small_resnet()
m.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
          optimizer=tf.keras.optimizers.SGD(learning_rate=0.0), metrics=["accuracy"])
w_init = m.get_weights()
h = m.fit(x, y, batch_size=32, epochs=1, steps_per_epoch=1, shuffle=False, verbose=0)
e = m._engine
torch.cuda.synchronize()
print("engine", e.name, "loss", h.history["loss"])
for nd in e.nodes:
    print(nd.kind, nd.layer.name, "dead" if nd.attrs.get("dead") else "", {k: (tuple(v.shape) if torch.is_tensor(v) else v)
          for k, v in nd.attrs.items() if k not in ("dead",) and not isinstance(v, tuple)})
conv = e.nodes[0]
bn = e.nodes[1]
x0 = e.x0.buf.float()
print("x0", tuple(x0.shape), "pad channels max", x0[..., 3:].abs().max().item(), "x0 vs data", (x0[..., :3].cpu() - torch.from_numpy(x[:32]).bfloat16().float()).abs().max().item())
wp = conv.attrs["w_pad"].float()
yref = ref.conv2d(x0, wp, None, conv.layer.strides, conv.layer.padding)
yk = conv.out.buf.float()
print("conv out err", (yk - yref).abs().max().item(), "ref max", yref.abs().max().item())
sb = conv.attrs["stats_buf"]
yr2 = yk.reshape(-1, yk.shape[-1])
print("stats sum err", (sb[:, 0].sum(0) - yr2.sum(0)).abs().max().item(), (sb[:, 1].sum(0) - (yr2 * yr2).sum(0)).abs().max().item())
st = bn.attrs["st"]
print("mean err", (st[0] - yr2.mean(0)).abs().max().item(), "inv err", (st[1] - torch.rsqrt(yr2.var(0, unbiased=False) + 1.001e-5)).abs().max().item())
mm = bn.layer.moving_mean.value
print("moving mean", mm[:4].tolist(), "expected", (0.01 * yr2.mean(0))[:4].tolist())
print("stats T", sb.shape, "part rows", [float(v) for v in sb[:, 0, 0][:8]])
