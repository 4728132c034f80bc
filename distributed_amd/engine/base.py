"""Engine interface and selection."""
from __future__ import annotations

from ..utils import env
from ..utils import logging as dlog


class ExchangeFault(RuntimeError):
    """A bounded in-kernel exchange wait expired mid-run on at least one rank (collective
    vote at the epoch's host sync, so EVERY rank raises it).  ``Model.fit`` answers with
    :meth:`~.fused_convnet.FusedConvNetEngine.rebuild_after_fault`: the epoch restarts from its start-of-epoch
    snapshot on the next transport, instead of the whole gang restarting."""



class Engine:
    """Executes training steps for one (model, strategy, batch) configuration."""

    name = "base"

    def __init__(self, model, strategy, per_replica_batch: int, global_batch: int):
        self.model, self.strategy = model, strategy
        self.per_replica, self.global_batch = per_replica_batch, global_batch
        self.world, self.rank = strategy.num_replicas_in_sync, strategy.rank
        self.device = strategy.device
        # every replica must draw the same epoch permutation (disjoint shards of one global
        # batch): the shuffle seed is rank 0's, broadcast once
        from ..utils import random as _r

        seed = _r._GLOBAL_SEED if _r._GLOBAL_SEED is not None else 0x5EED
        if self.world > 1:
            seed = strategy.communicator.broadcast_object(seed, 0)
        self.shuffle_seed = int(seed)

    def bind(self, x, y):  # -> DataFeed
        raise NotImplementedError

    def start_epoch(self, epoch: int, shuffle: bool):
        raise NotImplementedError

    def run(self, n_steps: int):
        raise NotImplementedError

    def prepare(self, n_steps: int):
        """Build whatever ``run(n_steps)`` will replay (HIP graphs) without executing a
        step, so a timed ``run`` measures replay only."""

    def metrics(self) -> dict:
        """Global epoch-so-far averages, e.g. {'loss':..., 'accuracy':...} (syncs)."""
        raise NotImplementedError

    def end_epoch(self) -> dict:
        return self.metrics()

    def finish(self):
        pass

    def lr_changed(self):
        pass

    def reload_optimizer_state(self):
        """Optimizer slots / iterations were replaced on the host (checkpoint restore)."""

    def sync(self):
        pass

    def completion_event(self):
        """An event that completes when the work enqueued so far has finished on the device
        (the watchdog beats on it), or None on the CPU: the host loop itself is the work."""
        if getattr(self.device, "type", "cpu") != "cuda":
            return None
        import torch

        ev = torch.cuda.Event()
        ev.record(self._work_stream())
        return ev

    def _work_stream(self):
        """The stream the engine's step work is enqueued on."""
        import torch

        return torch.cuda.current_stream(self.device)

    def phase_times(self, n_steps: int) -> dict:
        """Mean milliseconds per step of the step's phases (forward / backward / all-reduce /
        optimizer) over ``n_steps`` real training steps run eagerly with timing points between
        the phases.  Engines override; the base reports the whole step only."""
        import time

        self.sync()
        t0 = time.perf_counter()
        self.run(n_steps)
        self.sync()
        return {"step": (time.perf_counter() - t0) * 1e3 / max(n_steps, 1)}

    def _own_variables(self, variables):
        """Route host writes of these variables (set_weights, load_weights, layer-level
        assign) through before/after_external_write."""
        import weakref

        ref = weakref.ref(self)
        for v in variables:
            v._engine_ref = ref

    def before_external_write(self):
        """A model variable is about to be overwritten from the host."""
        self.sync()

    def after_external_write(self):
        """A model variable was overwritten from the host (refresh derived copies)."""


def select_engine(model, strategy, per_replica: int, global_batch: int) -> Engine:
    from .generic import GenericEngine

    if env.get_bool("DAMD_FUSED", True):
        from .fused_convnet import FusedConvNetEngine

        ok, why = FusedConvNetEngine.eligible(model, strategy)
        if ok:
            return FusedConvNetEngine(model, strategy, per_replica, global_batch)
        dlog.debug("fused ConvNet engine not used: %s", why)
    if env.get_bool("DAMD_NATIVE_GRAPH", True):
        from .native_graph import NativeGraphEngine

        ok, why = NativeGraphEngine.eligible(model, strategy)
        if ok:
            return NativeGraphEngine(model, strategy, per_replica, global_batch)
        dlog.debug("native graph engine not used: %s", why)
    else:
        why = "DAMD_NATIVE_GRAPH=0"
    if strategy.device.type == "cuda":
        # a GPU model outside the native engines' coverage trains through PyTorch eager ops
        # (vendor libraries): say so loudly, or refuse under DAMD_STRICT_NATIVE=1
        msg = f"model trains on the PyTorch eager fallback (GenericEngine), not the native HIP engines: {why}"
        if env.get_bool("DAMD_STRICT_NATIVE", False):
            raise RuntimeError(msg + " (DAMD_STRICT_NATIVE=1)")
        dlog.warning(msg)
    return GenericEngine(model, strategy, per_replica, global_batch)
