"""Data-parallel runtime: cluster spec (TF_CONFIG), communicators, strategies."""
from . import cluster, communicator, runtime, strategy  # noqa: F401
from .strategy import MultiWorkerMirroredStrategy, get_strategy, ReduceOp  # noqa: F401
