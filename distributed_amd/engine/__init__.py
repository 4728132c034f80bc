"""Training engines behind ``Model.fit``.

* :class:`~.generic.GenericEngine` — any Keras model; per-layer ops, autograd backward,
  one flat gradient bucket (+ metric tail) all-reduced per step.
* :class:`~.fused_convnet.FusedConvNetEngine` — the reference CNN family on MI355X:
  3 fused HIP launches per step + RCCL all-reduce, captured into hipGraphs.
"""
from .base import Engine, select_engine  # noqa: F401
from .data import DataFeed  # noqa: F401
