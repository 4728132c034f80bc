"""Communicators: the collective layer under MultiWorkerMirroredStrategy.

Reference: TF CollectiveAllReduce over gRPC between CPU workers
(reference README.md:395 ``rpc_layer='grpc'``, :398 ``CollectiveCommunication.AUTO``,
:403-412 "Collective batch_all_reduce").  MI355X design:

* :class:`RcclCommunicator` — native RCCL communicator (``_C.RcclComm``) for device
  tensors, enqueued on the caller's HIP stream (capturable into hipGraphs); the
  unique id is exchanged once over the control-plane process group.
* :class:`TorchCommunicator` — ``torch.distributed`` (gloo on CPU; nccl=RCCL on GPU
  when ``DAMD_COMM=torch``).
* :class:`LoopbackCommunicator` — world size 1, every collective is a no-op.

All communicators expose the same in-place tensor API.
"""
from __future__ import annotations

import datetime
from typing import Any, List, Optional

import torch
import torch.distributed as dist

from ..utils import logging as dlog

_OPS = {"sum": 0, "max": 1, "min": 2, "avg": 3}
_DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3, torch.float64: 4, torch.int64: 5}


class Communicator:
    name = "base"
    world_size = 1
    rank = 0
    # control-plane collectives issued (barrier / object all-gather / object broadcast):
    # bench.py checks that none runs inside a timed window
    control_ops = 0

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        raise NotImplementedError

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        raise NotImplementedError

    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def barrier(self) -> None:
        raise NotImplementedError

    def allgather_object(self, obj: Any) -> List[Any]:
        raise NotImplementedError

    def broadcast_object(self, obj: Any, root: int = 0) -> Any:
        raise NotImplementedError

    def allreduce_async(self, t: torch.Tensor, op: str = "sum"):
        """Start an in-place all-reduce; returns a handle with ``wait()``."""
        self.allreduce_(t, op)
        return _Done()

    @property
    def native(self):
        """Native RCCL handle usable inside captured graphs (None if not RCCL)."""
        return None

    def shutdown(self) -> None:
        pass


class _Done:
    def wait(self):
        return True


class LoopbackCommunicator(Communicator):
    name = "loopback"

    def allreduce_(self, t, op="sum"):
        return t

    def broadcast_(self, t, root=0):
        return t

    def allgather(self, t):
        return t.unsqueeze(0).clone()

    def barrier(self):
        pass

    def allgather_object(self, obj):
        return [obj]

    def broadcast_object(self, obj, root=0):
        return obj


_TORCH_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


class TorchCommunicator(Communicator):
    """torch.distributed process group (gloo control plane; optional data-plane group)."""

    name = "torch"

    def __init__(self, world_size: int, rank: int, data_group=None, host_staging: bool = False):
        self.world_size, self.rank = world_size, rank
        self._data_group = data_group  # None -> default (gloo) group
        self.host_staging = host_staging

    def allreduce_(self, t, op="sum"):
        if self._staged(t):
            h = t.detach().cpu()
            self.allreduce_(h, op)
            t.copy_(h)
            return t
        if op == "avg":
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self._group_for(t))
            t.div_(self.world_size)
            return t
        dist.all_reduce(t, op=_TORCH_OPS[op], group=self._group_for(t))
        return t

    def allreduce_async(self, t, op="sum"):
        if self._staged(t) or op == "avg" or t.is_cuda:
            return super().allreduce_async(t, op)
        return dist.all_reduce(t, op=_TORCH_OPS[op], group=self._group_for(t), async_op=True)

    def broadcast_(self, t, root=0):
        if self._staged(t):
            h = t.detach().cpu()
            dist.broadcast(h, src=root)
            t.copy_(h)
            return t
        dist.broadcast(t, src=root, group=self._group_for(t))
        return t

    def _staged(self, t):
        # DAMD_COMM=gloo on a GPU: device tensors go through host memory (test/debug mode,
        # e.g. several ranks sharing one GPU, which RCCL does not allow)
        return t.is_cuda and self._data_group is None and self.host_staging

    def allgather(self, t):
        out = [torch.empty_like(t) for _ in range(self.world_size)]
        dist.all_gather(out, t.contiguous(), group=self._group_for(t))
        return torch.stack(out)

    def barrier(self):
        self.control_ops += 1
        dist.barrier()

    def allgather_object(self, obj):
        self.control_ops += 1
        out = [None] * self.world_size
        dist.all_gather_object(out, obj)
        return out

    def broadcast_object(self, obj, root=0):
        self.control_ops += 1
        box = [obj]
        dist.broadcast_object_list(box, src=root)
        return box[0]

    def _group_for(self, t):
        if t.is_cuda and self._data_group is not None:
            return self._data_group
        if t.is_cuda:
            raise RuntimeError("device tensor on a gloo-only communicator; use RcclCommunicator")
        return None

    def shutdown(self):
        pass


class RcclCommunicator(TorchCommunicator):
    """Native RCCL data plane + gloo control plane."""

    name = "rccl"

    def __init__(self, world_size: int, rank: int, device: int):
        super().__init__(world_size, rank)
        from ..native import require_C

        C = require_C()
        uid = C.rccl_unique_id() if rank == 0 else None
        uid = self.broadcast_object(uid, root=0) if world_size > 1 else uid
        self.uid = uid  # every rank holds rank 0's ncclUniqueId from here on
        self._comm = C.RcclComm(world_size, rank, uid, device)
        self.device = device
        dlog.debug("RCCL communicator up: rank %d/%d on hip device %d (RCCL %s)", rank, world_size, device,
                   C.rccl_version())

    @property
    def native(self):
        return self._comm

    def _stream(self):
        return torch.cuda.current_stream().cuda_stream

    def allreduce_(self, t, op="sum"):
        if not t.is_cuda:
            return super().allreduce_(t, op)
        if not t.is_contiguous():
            raise ValueError("allreduce_ needs a contiguous tensor")
        self._comm.allreduce(t.data_ptr(), t.data_ptr(), t.numel(), _DTYPES[t.dtype], _OPS[op], self._stream())
        return t

    def broadcast_(self, t, root=0):
        if not t.is_cuda:
            return super().broadcast_(t, root)
        self._comm.broadcast(t.data_ptr(), t.numel(), _DTYPES[t.dtype], root, self._stream())
        return t

    def allgather(self, t):
        if not t.is_cuda:
            return super().allgather(t)
        t = t.contiguous()
        out = torch.empty((self.world_size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self._comm.allgather(t.data_ptr(), out.data_ptr(), t.numel(), _DTYPES[t.dtype], self._stream())
        return out

    def shutdown(self):
        self._comm = None


def make_peer_allreduce(comm: Communicator, device: int, capacity: int, blocks: int = 64,
                        timeout_s: float = 120.0, selftest: bool = True):
    """Native xGMI two-shot all-reduce (csrc/runtime/peer_comm.h) for ``capacity`` fp32
    values per call, or None.  Every step is agreed by all ranks over the control plane
    (IPC export, mapping, and a device self-test against a closed-form result), so either
    every rank gets a working instance or every rank falls back to RCCL."""
    W, r = comm.world_size, comm.rank
    if W < 2:
        return None
    # IPC handles only map on the node that minted them: a multi-host cluster (TF_CONFIG
    # workers on several machines) must not even try -- it uses RCCL
    nodes = comm.allgather_object(node_id())
    if len(set(nodes)) != 1:
        dlog.info("peer all-reduce: ranks span %d hosts; gradient all-reduce via RCCL", len(set(nodes)))
        return None
    from ..native import require_C

    C = require_C()
    pa, h = None, None
    try:
        pa = C.PeerAllreduce(W, r, device, int(capacity), int(blocks), float(timeout_s))
        h = pa.handles()
    except Exception as e:  # pragma: no cover - exercised on hardware only
        dlog.warning("peer all-reduce unavailable on rank %d: %s", r, e)
    hs = comm.allgather_object(h)
    if any(x is None for x in hs):
        return None
    ok = True
    try:
        pa.open(list(hs))
    except Exception as e:  # pragma: no cover
        dlog.warning("peer all-reduce: mapping peer buffers failed on rank %d: %s", r, e)
        ok = False
    if not all(comm.allgather_object(ok)):
        return None
    if selftest:
        try:
            ok = _peer_selftest(pa, device, int(capacity), W, r)
        except Exception as e:  # pragma: no cover - every rank must reach the vote below
            dlog.warning("peer all-reduce self-test raised on rank %d: %s", r, e)
            ok = False
        if not all(comm.allgather_object(ok)):
            dlog.warning("peer all-reduce self-test failed; using RCCL")
            return None
    pa.set_timeout(float(timeout_s))
    return pa


def node_id() -> str:
    """Identity of this machine: hostname + kernel boot id (containers on one host that
    share a hostname but not a kernel still differ)."""
    import socket

    boot = ""
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        pass
    return f"{socket.gethostname()}/{boot}"


def _peer_selftest(pa, device: int, n: int, W: int, r: int) -> bool:
    """Three back-to-back all-reduces of rank-dependent data (exercises the per-block
    epochs) with a short wait deadline; exact comparison with the closed form."""
    dev = torch.device("cuda", device)
    pa.set_timeout(10.0)
    base = (torch.arange(n, device=dev, dtype=torch.float32) % 251) - 125.0
    s = torch.cuda.current_stream(dev)
    ok = True
    for it in range(3):
        x = base * float(r + 1 + it)
        pa.allreduce(x.data_ptr(), n, s.cuda_stream)
        torch.cuda.synchronize(dev)
        want = base * float(W * (W + 1) // 2 + W * it)
        ok = ok and bool(torch.equal(x, want))
    st = pa.status()
    pa.clear_status()
    torch.cuda.synchronize(dev)
    return ok and st == 0


def init_process_group(world_size: int, rank: int, init_method: str, timeout_s: float = 600.0) -> None:
    if dist.is_initialized():
        return
    dist.init_process_group(
        backend="gloo",
        init_method=init_method,
        world_size=world_size,
        rank=rank,
        timeout=datetime.timedelta(seconds=timeout_s),
    )


def make_communicator(world_size: int, rank: int, device: torch.device, kind: Optional[str] = None) -> Communicator:
    if world_size == 1 and kind in (None, "auto", "loopback"):
        if device.type == "cuda" and kind not in ("loopback",):
            # a size-1 RCCL comm keeps the world=1 run on exactly the same code path
            # (BASELINE.json:8 "single-replica MirroredStrategy path") without a PG.
            try:
                from ..native import require_C

                C = require_C()
                c = RcclCommunicator.__new__(RcclCommunicator)
                TorchCommunicator.__init__(c, 1, 0)
                c._comm = C.RcclComm(1, 0, C.rccl_unique_id(), device.index or 0)
                c.device = device.index or 0
                return c
            except Exception as e:  # pragma: no cover
                dlog.warning("size-1 RCCL communicator unavailable (%s); using loopback", e)
        return LoopbackCommunicator()
    if device.type == "cuda":
        if kind == "gloo":
            return TorchCommunicator(world_size, rank, host_staging=True)
        if kind == "torch":
            grp = dist.new_group(backend="nccl")
            return TorchCommunicator(world_size, rank, data_group=grp)
        return RcclCommunicator(world_size, rank, device.index or 0)
    return TorchCommunicator(world_size, rank)
