"""Keras initializers (tf.keras 2.0 defaults: kernels glorot_uniform, biases zeros)."""
from __future__ import annotations

import math

import numpy as np
import torch

from ..utils.random import next_generator


def _fans(shape):
    shape = tuple(shape)
    if len(shape) < 1:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    rf = int(np.prod(shape[:-2]))
    return shape[-2] * rf, shape[-1] * rf


class Initializer:
    def __call__(self, shape, dtype=torch.float32):
        raise NotImplementedError

    def get_config(self):
        return {}

    @classmethod
    def class_name(cls):
        return cls.__name__


class Zeros(Initializer):
    def __call__(self, shape, dtype=torch.float32):
        return torch.zeros(shape, dtype=dtype)


class Ones(Initializer):
    def __call__(self, shape, dtype=torch.float32):
        return torch.ones(shape, dtype=dtype)


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.value = value

    def __call__(self, shape, dtype=torch.float32):
        return torch.full(shape, float(self.value), dtype=dtype)

    def get_config(self):
        return {"value": self.value}


class VarianceScaling(Initializer):
    def __init__(self, scale=1.0, mode="fan_in", distribution="truncated_normal", seed=None):
        self.scale, self.mode, self.distribution, self.seed = scale, mode, distribution, seed

    def __call__(self, shape, dtype=torch.float32):
        fan_in, fan_out = _fans(shape)
        n = {"fan_in": fan_in, "fan_out": fan_out, "fan_avg": (fan_in + fan_out) / 2.0}[self.mode]
        scale = self.scale / max(1.0, n)
        g = next_generator()
        if self.seed is not None:
            g.manual_seed(int(self.seed))
        if self.distribution == "uniform":
            lim = math.sqrt(3.0 * scale)
            return (torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1).mul_(lim).to(dtype)
        if self.distribution in ("truncated_normal", "normal"):
            std = math.sqrt(scale)
            if self.distribution == "truncated_normal":
                std = std / 0.87962566103423978
                t = torch.empty(shape, dtype=torch.float64)
                torch.nn.init.trunc_normal_(t, 0.0, 1.0, -2.0, 2.0, generator=g)
                return (t * std).to(dtype)
            return (torch.randn(shape, generator=g, dtype=torch.float64) * std).to(dtype)
        raise ValueError(self.distribution)

    def get_config(self):
        return {"scale": self.scale, "mode": self.mode, "distribution": self.distribution, "seed": self.seed}


class GlorotUniform(VarianceScaling):
    def __init__(self, seed=None):
        super().__init__(1.0, "fan_avg", "uniform", seed)

    def get_config(self):
        return {"seed": self.seed}


class GlorotNormal(VarianceScaling):
    def __init__(self, seed=None):
        super().__init__(1.0, "fan_avg", "truncated_normal", seed)

    def get_config(self):
        return {"seed": self.seed}


class HeNormal(VarianceScaling):
    def __init__(self, seed=None):
        super().__init__(2.0, "fan_in", "truncated_normal", seed)

    def get_config(self):
        return {"seed": self.seed}


class HeUniform(VarianceScaling):
    def __init__(self, seed=None):
        super().__init__(2.0, "fan_in", "uniform", seed)

    def get_config(self):
        return {"seed": self.seed}


class RandomNormal(Initializer):
    def __init__(self, mean=0.0, stddev=0.05, seed=None):
        self.mean, self.stddev, self.seed = mean, stddev, seed

    def __call__(self, shape, dtype=torch.float32):
        g = next_generator()
        return (torch.randn(shape, generator=g, dtype=torch.float64) * self.stddev + self.mean).to(dtype)

    def get_config(self):
        return {"mean": self.mean, "stddev": self.stddev, "seed": self.seed}


class RandomUniform(Initializer):
    def __init__(self, minval=-0.05, maxval=0.05, seed=None):
        self.minval, self.maxval, self.seed = minval, maxval, seed

    def __call__(self, shape, dtype=torch.float32):
        g = next_generator()
        u = torch.rand(shape, generator=g, dtype=torch.float64)
        return (u * (self.maxval - self.minval) + self.minval).to(dtype)

    def get_config(self):
        return {"minval": self.minval, "maxval": self.maxval, "seed": self.seed}


_ALIASES = {
    "zeros": Zeros, "ones": Ones, "constant": Constant,
    "glorot_uniform": GlorotUniform, "glorot_normal": GlorotNormal,
    "he_normal": HeNormal, "he_uniform": HeUniform,
    "random_normal": RandomNormal, "random_uniform": RandomUniform,
    "variance_scaling": VarianceScaling,
}
_CLASSES = {c.__name__: c for c in _ALIASES.values()}


def get(identifier):
    if isinstance(identifier, Initializer):
        return identifier
    if isinstance(identifier, str):
        if identifier in _ALIASES:
            return _ALIASES[identifier]()
        if identifier in _CLASSES:
            return _CLASSES[identifier]()
    if isinstance(identifier, dict):
        return _CLASSES[identifier["class_name"]](**identifier.get("config", {}))
    raise ValueError(f"unknown initializer {identifier!r}")


def serialize(init: Initializer) -> dict:
    return {"class_name": init.class_name(), "config": init.get_config()}


zeros = Zeros
ones = Ones
glorot_uniform = GlorotUniform
he_normal = HeNormal
