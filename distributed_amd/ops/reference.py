"""Plain PyTorch reference ops in Keras (NHWC / HWIO) conventions.

Keras conventions reproduced (tf.keras 2.0 defaults, exercised by reference
README.md:58-73): channels_last activations ``[N,H,W,C]``, conv kernels ``[kh,kw,cin,cout]``,
dense kernels ``[in,out]``, 'valid'/'same' padding (TF 'same' pads the extra pixel at
the bottom/right), MaxPool ties resolved to the first max in row-major window order.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _same_pad(in_size: int, k: int, s: int, d: int = 1):
    eff = (k - 1) * d + 1
    out = math.ceil(in_size / s)
    total = max((out - 1) * s + eff - in_size, 0)
    return total // 2, total - total // 2


def conv2d(x, w, b=None, strides=(1, 1), padding="valid", dilation=(1, 1)):
    """x [N,H,W,Cin], w [kh,kw,Cin,Cout] -> [N,Ho,Wo,Cout]."""
    xc = x.permute(0, 3, 1, 2)
    wc = w.permute(3, 2, 0, 1)
    if padding == "same":
        pt, pb = _same_pad(x.shape[1], w.shape[0], strides[0], dilation[0])
        pl, pr = _same_pad(x.shape[2], w.shape[1], strides[1], dilation[1])
        xc = F.pad(xc, (pl, pr, pt, pb))
    elif padding != "valid":
        raise ValueError(f"padding {padding!r}")
    y = F.conv2d(xc, wc, b, stride=tuple(strides), dilation=tuple(dilation))
    return y.permute(0, 2, 3, 1)


def maxpool2d(x, pool=(2, 2), strides=None, padding="valid"):
    strides = strides or pool
    xc = x.permute(0, 3, 1, 2)
    if padding == "same":
        pt, pb = _same_pad(x.shape[1], pool[0], strides[0])
        pl, pr = _same_pad(x.shape[2], pool[1], strides[1])
        xc = F.pad(xc, (pl, pr, pt, pb), value=float("-inf"))
    y = F.max_pool2d(xc, tuple(pool), tuple(strides))
    return y.permute(0, 2, 3, 1)


def avgpool2d(x, pool=(2, 2), strides=None, padding="valid"):
    strides = strides or pool
    xc = x.permute(0, 3, 1, 2)
    if padding == "same":
        # TF 'same' average pooling excludes the padding from the divisor
        pt, pb = _same_pad(x.shape[1], pool[0], strides[0])
        pl, pr = _same_pad(x.shape[2], pool[1], strides[1])
        ones = torch.ones_like(xc[:, :1])
        num = F.avg_pool2d(F.pad(xc, (pl, pr, pt, pb)), tuple(pool), tuple(strides), divisor_override=1)
        den = F.avg_pool2d(F.pad(ones, (pl, pr, pt, pb)), tuple(pool), tuple(strides), divisor_override=1)
        y = num / den
    else:
        y = F.avg_pool2d(xc, tuple(pool), tuple(strides))
    return y.permute(0, 2, 3, 1)


def dense(x, w, b=None):
    y = x.matmul(w)
    return y + b if b is not None else y


def batchnorm(x, gamma, beta, mean, var, training, momentum=0.99, eps=1e-3):
    """Keras BatchNormalization over the last axis; updates moving stats in place."""
    if training:
        dims = tuple(range(x.dim() - 1))
        bm = x.mean(dim=dims)
        bv = x.var(dim=dims, unbiased=False)
        with torch.no_grad():
            mean.mul_(momentum).add_(bm.detach(), alpha=1 - momentum)
            var.mul_(momentum).add_(bv.detach(), alpha=1 - momentum)
        m, v = bm, bv
    else:
        m, v = mean, var
    return (x - m) * torch.rsqrt(v + eps) * gamma + beta


def sparse_softmax_xent(logits, labels):
    """Per-sample loss of SparseCategoricalCrossentropy(from_logits=True)."""
    return F.cross_entropy(logits.float(), labels.long(), reduction="none")


def sparse_accuracy(logits, labels):
    """Per-sample 0/1 of sparse categorical accuracy (argmax ties -> first index)."""
    return (logits.argmax(dim=-1) == labels.long()).float()
