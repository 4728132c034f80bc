"""Yardstick for the ResNet-18 config (BASELINE.json config 4): the same network and
training step written in plain PyTorch eager (MIOpen convs, channels_last, bf16 autocast,
fp32 master weights, SGD momentum 0.9), timed the way bench.py times ours.  The
reference publishes no ResNet number, so this is the on-hardware comparison point.

usage: python scripts/torch_resnet_ref.py [batch] [steps] [warmup] [--graph]"""
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Block(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.b1 = nn.BatchNorm2d(cout, eps=1.001e-5)
        self.c2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.b2 = nn.BatchNorm2d(cout, eps=1.001e-5)
        self.proj = None
        if stride != 1 or cin != cout:
            self.proj = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout, eps=1.001e-5))

    def forward(self, x):
        y = F.relu(self.b1(self.c1(x)))
        y = self.b2(self.c2(y))
        s = x if self.proj is None else self.proj(x)
        return F.relu(y + s)


class ResNet18(nn.Module):
    def __init__(self, classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64, eps=1.001e-5), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        blocks, cin = [], 64
        for i, w in enumerate((64, 128, 256, 512)):
            for j in range(2):
                blocks.append(Block(cin, w, 2 if (i > 0 and j == 0) else 1))
                cin = w
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(512, classes)

    def forward(self, x):
        x = self.blocks(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    B = int(args[0]) if args else 64
    steps = int(args[1]) if len(args) > 1 else 30
    warm = int(args[2]) if len(args) > 2 else 5
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = True
    m = ResNet18().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    x = torch.rand(B, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    print(f'{{"torch_eager_resnet18": {{"batch": {B}, "ms_per_step": {dt * 1e3:.3f}, '
          f'"images_per_s": {B / dt:.1f}, "loss": {float(loss):.4f}}}}}', flush=True)


if __name__ == "__main__":
    main()
