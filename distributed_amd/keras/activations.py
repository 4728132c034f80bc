"""Keras activations by name (``activation='relu'`` etc.)."""
from __future__ import annotations

import torch
import torch.nn.functional as F


def linear(x):
    return x


def relu(x):
    return torch.relu(x)


def softmax(x):
    return torch.softmax(x, dim=-1)


def sigmoid(x):
    return torch.sigmoid(x)


def tanh(x):
    return torch.tanh(x)


def elu(x):
    return F.elu(x)


def selu(x):
    return F.selu(x)


def softplus(x):
    return F.softplus(x)


_BY_NAME = {f.__name__: f for f in (linear, relu, softmax, sigmoid, tanh, elu, selu, softplus)}


def get(identifier):
    if identifier is None:
        return linear
    if callable(identifier):
        return identifier
    if identifier in _BY_NAME:
        return _BY_NAME[identifier]
    raise ValueError(f"unknown activation {identifier!r}")


def serialize(fn) -> str:
    for k, v in _BY_NAME.items():
        if v is fn:
            return k
    return getattr(fn, "__name__", "custom")
