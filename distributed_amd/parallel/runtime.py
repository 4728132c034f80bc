"""Process-wide runtime: device selection, process group, communicator (one per process).

One process drives one GPU (``local_rank`` -> ``torch.cuda.set_device``), as in
SURVEY.md §3.1 "New".  The runtime is created lazily by the first strategy (or by
``fit`` on the default strategy) and torn down with :func:`shutdown`.
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass
from typing import Optional

import torch

from ..utils import env
from ..utils import logging as dlog
from . import cluster as _cluster
from .communicator import Communicator, LoopbackCommunicator, init_process_group, make_communicator


@dataclass
class Runtime:
    spec: _cluster.ClusterSpec
    device: torch.device
    comm: Communicator

    @property
    def world_size(self) -> int:
        return self.spec.num_workers

    @property
    def rank(self) -> int:
        return self.spec.task_id


_lock = threading.Lock()
_RT: Optional[Runtime] = None


def pick_device(local_rank: int) -> torch.device:
    want = env.get_str("DAMD_DEVICE", "auto")
    if want == "cpu" or (want == "auto" and not torch.cuda.is_available()):
        return torch.device("cpu")
    n = torch.cuda.device_count()
    if n == 0:
        raise RuntimeError("DAMD_DEVICE=cuda but no HIP device is visible")
    idx = local_rank % n
    torch.cuda.set_device(idx)
    return torch.device("cuda", idx)


def init(spec: Optional[_cluster.ClusterSpec] = None) -> Runtime:
    global _RT
    with _lock:
        if _RT is not None:
            return _RT
        spec = spec or _cluster.resolve()
        device = pick_device(spec.local_rank)
        world, rank = spec.num_workers, spec.task_id
        if world > 1:
            if spec.source == "torchrun":
                init_method = "env://"
            else:
                host, port = spec.workers[0].rsplit(":", 1)
                init_method = f"tcp://{host}:{port}"
            init_process_group(world, rank, init_method, env.get_float("DAMD_INIT_TIMEOUT_S", 600.0))
        comm = make_communicator(world, rank, device, env.get_str("DAMD_COMM", "auto"))
        _RT = Runtime(spec=spec, device=device, comm=comm)
        return _RT


def get() -> Runtime:
    return _RT if _RT is not None else init()


def current_or_none() -> Optional[Runtime]:
    return _RT


def shutdown() -> None:
    global _RT
    with _lock:
        if _RT is None:
            return
        try:
            _RT.comm.shutdown()
        finally:
            import torch.distributed as dist

            if dist.is_initialized():
                try:
                    dist.destroy_process_group()
                except Exception:  # pragma: no cover
                    pass
            _RT = None
            from . import strategy as _strategy

            _strategy._reset_default()  # the default strategy caches the runtime


def local_runtime_for_tests(device: str = "cpu") -> Runtime:
    """A world-1 runtime that never touches torch.distributed."""
    global _RT
    with _lock:
        _RT = Runtime(spec=_cluster.ClusterSpec(workers=["127.0.0.1:0"]), device=torch.device(device),
                      comm=LoopbackCommunicator())
        return _RT


def describe() -> str:
    rt = get()
    return (f"cluster_spec = {rt.spec.as_dict()}, task_type = '{rt.spec.task_type}', task_id = {rt.rank}, "
            f"num_workers = {rt.world_size}, local_devices = ('{rt.device}',), communication = {rt.comm.name.upper()}")


def fault_injection_step() -> Optional[int]:
    """``DAMD_FAIL_AT=rank:step[:attempt]`` -> the global step at which this rank raises.
    With ``attempt`` the failure fires only in that launcher attempt
    (``DAMD_RESTART_COUNT``), so a gang restart can then run to completion."""
    v = os.environ.get("DAMD_FAIL_AT")
    if not v:
        return None
    parts = v.split(":")
    r, s = int(parts[0]), int(parts[1])
    if len(parts) > 2 and int(os.environ.get("DAMD_RESTART_COUNT", "0")) != int(parts[2]):
        return None
    rt = get()
    return s if r == rt.rank else None
