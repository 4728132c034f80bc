"""Keras losses.  ``per_sample`` gives the unreduced loss; ``__call__`` applies Keras'
default ``SUM_OVER_BATCH_SIZE`` reduction.  Under MultiWorkerMirroredStrategy the
engines divide the per-replica sum by the *global* batch, so the SUM all-reduce of
gradients yields the global mean."""
from __future__ import annotations

import torch
import torch.nn.functional as F

_EPS = 1e-7


class Reduction:
    AUTO = "auto"
    NONE = "none"
    SUM = "sum"
    SUM_OVER_BATCH_SIZE = "sum_over_batch_size"


class Loss:
    kind = "generic"

    def __init__(self, reduction=Reduction.AUTO, name=None):
        self.reduction = reduction
        self.name = name or type(self).__name__

    def per_sample(self, y_true, y_pred):
        raise NotImplementedError

    def __call__(self, y_true, y_pred, sample_weight=None):
        ls = self.per_sample(torch.as_tensor(y_true), y_pred)
        if sample_weight is not None:
            ls = ls * torch.as_tensor(sample_weight, dtype=ls.dtype, device=ls.device)
        if self.reduction == Reduction.NONE:
            return ls
        if self.reduction == Reduction.SUM:
            return ls.sum()
        return ls.sum() / max(1, ls.numel())

    def get_config(self):
        return {"reduction": self.reduction, "name": self.name}


def _probs_clip(p):
    p = p / p.sum(dim=-1, keepdim=True)
    return p.clamp(_EPS, 1 - _EPS)


class SparseCategoricalCrossentropy(Loss):
    kind = "sparse_categorical"

    def __init__(self, from_logits=False, reduction=Reduction.AUTO, name="sparse_categorical_crossentropy"):
        super().__init__(reduction, name)
        self.from_logits = from_logits

    def per_sample(self, y_true, y_pred):
        y = y_true.reshape(-1).to(y_pred.device).long()
        if self.from_logits:
            return F.cross_entropy(y_pred.float(), y, reduction="none")
        p = _probs_clip(y_pred.float())
        return -torch.log(p.gather(1, y[:, None])[:, 0])

    def get_config(self):
        c = super().get_config()
        c["from_logits"] = self.from_logits
        return c


class CategoricalCrossentropy(Loss):
    kind = "categorical"

    def __init__(self, from_logits=False, label_smoothing=0.0, reduction=Reduction.AUTO,
                 name="categorical_crossentropy"):
        super().__init__(reduction, name)
        self.from_logits, self.label_smoothing = from_logits, label_smoothing

    def per_sample(self, y_true, y_pred):
        y = y_true.to(y_pred.device).float()
        if self.label_smoothing:
            y = y * (1 - self.label_smoothing) + self.label_smoothing / y.shape[-1]
        logp = torch.log_softmax(y_pred.float(), -1) if self.from_logits else torch.log(_probs_clip(y_pred.float()))
        return -(y * logp).sum(-1)

    def get_config(self):
        c = super().get_config()
        c.update(from_logits=self.from_logits, label_smoothing=self.label_smoothing)
        return c


class BinaryCrossentropy(Loss):
    kind = "binary"

    def __init__(self, from_logits=False, reduction=Reduction.AUTO, name="binary_crossentropy"):
        super().__init__(reduction, name)
        self.from_logits = from_logits

    def per_sample(self, y_true, y_pred):
        y = y_true.to(y_pred.device).float().reshape(y_pred.shape)
        if self.from_logits:
            l = F.binary_cross_entropy_with_logits(y_pred.float(), y, reduction="none")
        else:
            p = y_pred.float().clamp(_EPS, 1 - _EPS)
            l = -(y * torch.log(p) + (1 - y) * torch.log(1 - p))
        return l.reshape(l.shape[0], -1).mean(-1)


class MeanSquaredError(Loss):
    def __init__(self, reduction=Reduction.AUTO, name="mean_squared_error"):
        super().__init__(reduction, name)

    def per_sample(self, y_true, y_pred):
        d = (y_pred.float() - y_true.to(y_pred.device).float().reshape(y_pred.shape)) ** 2
        return d.reshape(d.shape[0], -1).mean(-1)


class MeanAbsoluteError(Loss):
    def __init__(self, reduction=Reduction.AUTO, name="mean_absolute_error"):
        super().__init__(reduction, name)

    def per_sample(self, y_true, y_pred):
        d = (y_pred.float() - y_true.to(y_pred.device).float().reshape(y_pred.shape)).abs()
        return d.reshape(d.shape[0], -1).mean(-1)


_ALIASES = {
    "sparse_categorical_crossentropy": SparseCategoricalCrossentropy,
    "categorical_crossentropy": CategoricalCrossentropy,
    "binary_crossentropy": BinaryCrossentropy,
    "mse": MeanSquaredError, "mean_squared_error": MeanSquaredError,
    "mae": MeanAbsoluteError, "mean_absolute_error": MeanAbsoluteError,
}
_CLASSES = {c.__name__: c for c in _ALIASES.values()}


def get(identifier) -> Loss:
    if isinstance(identifier, Loss):
        return identifier
    if isinstance(identifier, str):
        return _ALIASES[identifier]()
    if isinstance(identifier, dict):
        return _CLASSES[identifier["class_name"]](**identifier.get("config", {}))
    raise ValueError(f"unknown loss {identifier!r}")


def serialize(loss: Loss):
    return {"class_name": type(loss).__name__, "config": loss.get_config()}
