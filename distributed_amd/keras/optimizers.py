"""Keras optimizers (tf.keras 2.0 optimizer_v2 update rules) over flat fp32 buffers.

``SGD(learning_rate=0.001)`` is the reference optimizer (reference README.md:72, 302).
Master weights are always fp32 (an lr=1e-3 update is below bf16 resolution for most
weights).  ``apply_flat`` is the generic-engine update; the
fused ConvNet engine applies the same SGD/momentum rule inside its HIP kernels.
"""
from __future__ import annotations

import math

import torch


class Optimizer:
    def __init__(self, learning_rate=0.001, name="Optimizer", **kw):
        if "lr" in kw:  # Keras alias
            learning_rate = kw.pop("lr")
        self._lr = float(learning_rate)
        self.name = name
        self._iterations = 0
        self._iter_source = None  # callable returning device-side iteration count
        self.slots = {}  # name -> flat fp32 tensor

    @property
    def learning_rate(self) -> float:
        return self._lr

    @learning_rate.setter
    def learning_rate(self, v):
        self._lr = float(v)

    lr = learning_rate

    @property
    def iterations(self) -> int:
        if self._iter_source is not None:
            return int(self._iter_source())
        return self._iterations

    @iterations.setter
    def iterations(self, v):
        self._iterations = int(v)

    def slot_names(self):
        return []

    def ensure_slots(self, n: int, device):
        for s in self.slot_names():
            if s not in self.slots or self.slots[s].numel() != n or self.slots[s].device != device:
                self.slots[s] = torch.zeros(n, dtype=torch.float32, device=device)

    def apply_flat(self, p: torch.Tensor, g: torch.Tensor) -> None:
        raise NotImplementedError

    def get_config(self):
        return {"name": self.name, "learning_rate": self._lr}


class SGD(Optimizer):
    def __init__(self, learning_rate=0.01, momentum=0.0, nesterov=False, name="SGD", **kw):
        super().__init__(learning_rate, name, **kw)
        self.momentum = float(momentum)
        self.nesterov = bool(nesterov)

    def slot_names(self):
        return ["momentum"] if self.momentum else []

    @torch.no_grad()
    def apply_flat(self, p, g):
        if self.momentum == 0.0:
            p.add_(g, alpha=-self._lr)
        else:
            v = self.slots["momentum"]
            v.mul_(self.momentum).add_(g, alpha=-self._lr)
            if self.nesterov:
                p.add_(v, alpha=self.momentum).add_(g, alpha=-self._lr)
            else:
                p.add_(v)
        self._iterations += 1

    def get_config(self):
        c = super().get_config()
        c.update(decay=0.0, momentum=self.momentum, nesterov=self.nesterov)
        return c


class Adam(Optimizer):
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, amsgrad=False, name="Adam",
                 **kw):
        super().__init__(learning_rate, name, **kw)
        self.beta_1, self.beta_2, self.epsilon, self.amsgrad = beta_1, beta_2, epsilon, amsgrad

    def slot_names(self):
        return ["m", "v"] + (["vhat"] if self.amsgrad else [])

    @torch.no_grad()
    def apply_flat(self, p, g):
        t = self._iterations + 1
        m, v = self.slots["m"], self.slots["v"]
        m.mul_(self.beta_1).add_(g, alpha=1 - self.beta_1)
        v.mul_(self.beta_2).addcmul_(g, g, value=1 - self.beta_2)
        lr_t = self._lr * math.sqrt(1 - self.beta_2 ** t) / (1 - self.beta_1 ** t)
        if self.amsgrad:
            vh = self.slots["vhat"]
            torch.maximum(vh, v, out=vh)
            p.addcdiv_(m, vh.sqrt().add_(self.epsilon), value=-lr_t)
        else:
            p.addcdiv_(m, v.sqrt().add_(self.epsilon), value=-lr_t)
        self._iterations = t

    def get_config(self):
        c = super().get_config()
        c.update(decay=0.0, beta_1=self.beta_1, beta_2=self.beta_2, epsilon=self.epsilon, amsgrad=self.amsgrad)
        return c


class RMSprop(Optimizer):
    def __init__(self, learning_rate=0.001, rho=0.9, momentum=0.0, epsilon=1e-7, centered=False, name="RMSprop",
                 **kw):
        super().__init__(learning_rate, name, **kw)
        self.rho, self.momentum, self.epsilon, self.centered = rho, momentum, epsilon, centered

    def slot_names(self):
        return ["rms"] + (["momentum"] if self.momentum else []) + (["mg"] if self.centered else [])

    @torch.no_grad()
    def apply_flat(self, p, g):
        ms = self.slots["rms"]
        ms.mul_(self.rho).addcmul_(g, g, value=1 - self.rho)
        denom = ms
        if self.centered:
            mg = self.slots["mg"]
            mg.mul_(self.rho).add_(g, alpha=1 - self.rho)
            denom = ms - mg * mg
        upd = g / (denom.sqrt() + self.epsilon) * self._lr
        if self.momentum:
            mom = self.slots["momentum"]
            mom.mul_(self.momentum).add_(upd)
            p.sub_(mom)
        else:
            p.sub_(upd)
        self._iterations += 1

    def get_config(self):
        c = super().get_config()
        c.update(decay=0.0, rho=self.rho, momentum=self.momentum, epsilon=self.epsilon, centered=self.centered)
        return c


_ALIASES = {"sgd": SGD, "adam": Adam, "rmsprop": RMSprop}
_CLASSES = {c.__name__: c for c in _ALIASES.values()}


def get(identifier) -> Optimizer:
    if isinstance(identifier, Optimizer):
        return identifier
    if isinstance(identifier, str):
        return _ALIASES[identifier.lower()]()
    if isinstance(identifier, dict):
        cfg = dict(identifier.get("config", {}))
        cfg.pop("decay", None)
        return _CLASSES[identifier["class_name"]](**cfg)
    raise ValueError(f"unknown optimizer {identifier!r}")


def serialize(opt: Optimizer):
    return {"class_name": type(opt).__name__, "config": opt.get_config()}
