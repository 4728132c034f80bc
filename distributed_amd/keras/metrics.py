"""Keras metrics.  ``'accuracy'`` resolves by loss kind like tf.keras 2.0
(sparse labels + logits -> sparse_categorical_accuracy; reference README.md:73)."""
from __future__ import annotations

import torch


class Metric:
    """Stateful mean metric: per-sample values accumulated as (total, count)."""

    name = "metric"

    def __init__(self, name=None):
        if name:
            self.name = name
        self.reset_states()

    def reset_states(self):
        self.total, self.count = 0.0, 0.0

    def per_sample(self, y_true, y_pred) -> torch.Tensor:
        raise NotImplementedError

    def update_state(self, y_true, y_pred):
        v = self.per_sample(torch.as_tensor(y_true), y_pred)
        self.total += float(v.sum())
        self.count += float(v.numel())

    def result(self):
        return self.total / self.count if self.count else 0.0


class SparseCategoricalAccuracy(Metric):
    name = "sparse_categorical_accuracy"

    def per_sample(self, y_true, y_pred):
        return (y_pred.argmax(-1) == y_true.reshape(-1).to(y_pred.device).long()).float()


class CategoricalAccuracy(Metric):
    name = "categorical_accuracy"

    def per_sample(self, y_true, y_pred):
        return (y_pred.argmax(-1) == y_true.to(y_pred.device).argmax(-1)).float()


class BinaryAccuracy(Metric):
    name = "binary_accuracy"

    def __init__(self, name=None, threshold=0.5):
        self.threshold = threshold
        super().__init__(name)

    def per_sample(self, y_true, y_pred):
        y = y_true.to(y_pred.device).float().reshape(y_pred.shape)
        return ((y_pred > self.threshold).float() == y).float().reshape(y.shape[0], -1).mean(-1)


class Mean(Metric):
    name = "mean"


def resolve(identifier, loss) -> Metric:
    """Resolve a metric identifier; 'accuracy'/'acc' depend on the loss (Keras rule)."""
    if isinstance(identifier, Metric):
        return identifier
    if identifier in ("accuracy", "acc"):
        kind = getattr(loss, "kind", "generic")
        m = {"sparse_categorical": SparseCategoricalAccuracy, "categorical": CategoricalAccuracy,
             "binary": BinaryAccuracy}.get(kind, SparseCategoricalAccuracy)()
        m.name = identifier
        return m
    table = {"sparse_categorical_accuracy": SparseCategoricalAccuracy,
             "categorical_accuracy": CategoricalAccuracy, "binary_accuracy": BinaryAccuracy}
    if identifier in table:
        return table[identifier]()
    raise ValueError(f"unknown metric {identifier!r}")
