"""Distribution strategies: ``MultiWorkerMirroredStrategy`` and the default strategy.

Reference behaviour:

* synchronous multi-worker data parallelism, one replica per worker, every worker runs
  the same program ("independent_worker" mode, reference README.md:395);
* variables created inside ``strategy.scope()`` are mirrored: initial values come from
  worker 0 (broadcast), and stay identical because every replica applies the same
  all-reduced (SUM of 1/global-batch scaled) gradient (README.md:403);
* loss and metrics are reduced globally, so every worker reports identical numbers
  (README.md:229-231);
* ``fit(batch_size=B)`` takes the *global* batch; each replica consumes
  ``B / num_replicas_in_sync`` rows per step (README.md:124-125, 413).

MI355X realisation: one process per GPU, RCCL all-reduce of one flat gradient buffer
(grads + metric tail) per step, issued on the step's HIP stream.
"""
from __future__ import annotations

import contextlib
import threading
from typing import Optional

import torch

from ..utils import logging as dlog
from . import cluster as _cluster
from . import runtime as _runtime


class ReduceOp:
    SUM = "sum"
    MEAN = "mean"
    MAX = "max"
    MIN = "min"


class CollectiveCommunication:
    """Kept for API parity (reference README.md:398); RCCL is the only GPU transport."""

    AUTO = "AUTO"
    RING = "RING"
    NCCL = "NCCL"


_tls = threading.local()


def _stack():
    if not hasattr(_tls, "stack"):
        _tls.stack = []
    return _tls.stack


class Strategy:
    """Base strategy.  ``extended`` mirrors tf.distribute's split, kept minimal."""

    mode = "independent_worker"

    def __init__(self):
        self._runtime: Optional[_runtime.Runtime] = None

    # --- runtime -------------------------------------------------------------
    @property
    def runtime(self) -> _runtime.Runtime:
        if self._runtime is None:
            self._runtime = _runtime.get()
        return self._runtime

    @property
    def num_replicas_in_sync(self) -> int:
        return self.runtime.world_size

    @property
    def device(self) -> torch.device:
        return self.runtime.device

    @property
    def communicator(self):
        return self.runtime.comm

    @property
    def rank(self) -> int:
        return self.runtime.rank

    @property
    def is_chief(self) -> bool:
        return self.runtime.rank == 0

    # --- scope ---------------------------------------------------------------
    @contextlib.contextmanager
    def scope(self):
        _stack().append(self)
        try:
            yield self
        finally:
            _stack().pop()

    # --- collectives on host values -------------------------------------------
    def reduce(self, op, value, axis=None):
        """Reduce a per-replica value across replicas (tf.distribute.Strategy.reduce).

        With ``axis`` the value is first reduced along that axis on each replica (SUM/MAX/MIN),
        and MEAN is the mean over every element along ``axis`` on every replica."""
        t = torch.as_tensor(value, dtype=torch.float64).clone()
        key = {ReduceOp.SUM: "sum", ReduceOp.MEAN: "mean"}.get(op, op)
        if key not in ("sum", "mean", "max", "min"):
            raise ValueError(f"unsupported reduce op {op!r}")
        count = 1.0
        if axis is not None:
            if key in ("sum", "mean"):
                count = float(t.shape[axis])
                t = t.sum(dim=axis)
            else:
                t = t.amax(dim=axis) if key == "max" else t.amin(dim=axis)
        n = self.num_replicas_in_sync
        if n > 1:  # world 1 has no process group: nothing to combine
            self.communicator.allreduce_(t, "sum" if key == "mean" else key)
        if key == "mean":
            t = t / (count * n)
        return t

    def broadcast_tensor_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        if self.num_replicas_in_sync > 1:
            self.communicator.broadcast_(t, root)
        return t

    def barrier(self):
        if self.num_replicas_in_sync > 1:
            self.communicator.barrier()


class DefaultStrategy(Strategy):
    """Single replica on this process's device (no scope needed)."""


class MultiWorkerMirroredStrategy(Strategy):
    """Synchronous multi-worker mirrored training over RCCL (gloo on CPU).

    ``communication`` is accepted for API parity with TF 2.0 and ignored: the
    transport is always RCCL on MI355X (ring/tree chosen by RCCL over xGMI).
    """

    def __init__(self, communication=CollectiveCommunication.AUTO, cluster_resolver=None):
        super().__init__()
        spec = cluster_resolver if isinstance(cluster_resolver, _cluster.ClusterSpec) else None
        self._runtime = _runtime.init(spec)
        self.communication = communication
        self.cluster_spec = self._runtime.spec
        dlog.info("Multi-worker MultiWorkerMirroredStrategy with %s", _runtime.describe())

    @property
    def cluster_resolver(self):
        return self.cluster_spec


_DEFAULT: Optional[DefaultStrategy] = None


def get_strategy() -> Strategy:
    st = _stack()
    if st:
        return st[-1]
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = DefaultStrategy()
    return _DEFAULT


def has_strategy() -> bool:
    return bool(_stack())


def _reset_default():
    global _DEFAULT
    _DEFAULT = None
