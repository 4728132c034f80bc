"""Race / divergence detection for synchronous data parallelism.

* :func:`param_fingerprint` — an order-sensitive fp64 fingerprint of every model variable
  (trainable + BN statistics), computed on the device.
* :func:`check_mirrored` — all-gathers the fingerprints and raises
  :class:`MirrorDivergenceError` if any replica differs: mirrored variables must stay
  bitwise identical on every worker (the reference's observable invariant: identical
  per-worker results, README.md:229-231).  Used by the ``MirrorCheck`` callback and by
  ``DAMD_CHECK_MIRRORS=N`` (check every N epochs inside ``fit``).
* :func:`debug_sync` — with ``DAMD_DEBUG_SYNC=1`` every engine chunk is followed by a
  device synchronize + error check, so an asynchronous kernel fault is reported at the
  chunk that caused it instead of at a later host read.
"""
from __future__ import annotations

from typing import List

import torch

from . import env
from . import logging as dlog


class MirrorDivergenceError(RuntimeError):
    pass


def param_fingerprint(model) -> List[float]:
    """[sum, sum|.|, sum(i*x) mod-weighted] in fp64 over all variables, in order."""
    s0 = s1 = s2 = 0.0
    acc = None
    for i, w in enumerate(model.weights):
        t = w.value.detach().reshape(-1).double()
        idx = torch.arange(t.numel(), device=t.device, dtype=torch.float64).remainder_(9973.0).add_(1.0 + i)
        v = torch.stack([t.sum(), t.abs().sum(), (t * idx).sum()])
        acc = v if acc is None else acc + v
    if acc is None:
        return [s0, s1, s2]
    return [float(x) for x in acc.cpu().tolist()]


def check_mirrored(model, strategy=None, tag: str = "") -> List[float]:
    st = strategy or model._strategy
    if getattr(model, "_engine", None) is not None:
        model._engine.sync()
    fp = param_fingerprint(model)
    if st.num_replicas_in_sync == 1:
        return fp
    allfp = st.communicator.allgather_object(fp)
    bad = [r for r, f in enumerate(allfp) if f != allfp[0]]
    if bad:
        raise MirrorDivergenceError(f"mirrored variables diverged{(' at ' + tag) if tag else ''}: replicas {bad} "
                                    f"differ from replica 0 ({allfp[0]} vs {[allfp[r] for r in bad]})")
    dlog.debug("mirror check ok%s: %s", f" ({tag})" if tag else "", fp)
    return fp


def mirror_check_every() -> int:
    return env.get_int("DAMD_CHECK_MIRRORS", 0)


def debug_sync(device) -> None:
    if device.type == "cuda" and env.get_bool("DAMD_DEBUG_SYNC", False):
        torch.cuda.synchronize(device)
