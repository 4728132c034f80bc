"""Start-up self-test of the fused MNIST step's gradient exchange, with in-process fallback.

Why: the default multi-GPU exchange of the fused engine runs INSIDE the step kernels
(sharded xGMI exchange, csrc/kernels/convnet_step2.hip) or as the standalone two-shot peer
kernel (csrc/kernels/peer_allreduce.hip).  A wrong reduction there would be invisible at
run time: every rank receives the same (wrong) reduced gradient, so the replicas stay
bitwise mirrored and MirrorCheck cannot see it.  The reference's contract is a synchronous
all-reduce with identical results on every worker (README.md:403-412, 229-231).

So before step 1, each candidate transport runs ``STEPS`` real training steps (SGD with
momentum, both step parities, an epoch flush) on synthetic rows through a scratch trainer,
and the SAME steps run through a second scratch trainer whose gradients are reduced on the
host: all-gathered over the gloo control plane and summed in rank order -- the order the
device transports sum in (fp32 addition in rank order; int64 fixed-point conv sums exactly;
with the bf16 exchange, every partial and the reduced unit rounded to bf16 as the kernel
does).  The two must agree BITWISE (parameters, velocities, epoch metric sums), on every
rank (gloo vote).  A transport that fails -- or whose bounded in-kernel waits expire -- is
dropped before it carries a single real step, and the next one is tried:
sharded -> xgmi -> rccl (RCCL, the library ring, is the last resort and is not re-verified
here: it is not ours).

``DAMD_XCHG_SELFTEST_INJECT=<kind>[:rank]`` (tests only) corrupts one parameter of that
transport's result on that rank (default rank 1), to exercise the fallback.
"""
from __future__ import annotations

import os
import struct
from typing import Optional, Tuple

import numpy as np
import torch

from ..utils import logging as dlog

NPARAM, NGRAD, NCONV, FEAT, HID = 347146, 347152, 320, 5408, 64
OFF_W1, OFF_B1 = NCONV, NCONV + FEAT * HID
C_LR, C_MOM, C_NEST, C_NS, C_ROW0, C_GB, C_WRAP = 0, 1, 2, 3, 4, 5, 13
C_AL, C_AC, C_AN = 10, 11, 12
STEPS = 3
TIMEOUT_S = 10.0


def _f2i(f: float) -> int:
    return struct.unpack("<i", struct.pack("<f", float(f)))[0]


class _Scratch:
    """One scratch trainer + buffers (what FusedConvNetEngine allocates), starting at P0."""

    def __init__(self, C, dev, B, GB, rank, P0, X, Y, ppb, PP, wrap=0):
        f32 = dict(dtype=torch.float32, device=dev)
        BP = (B + 63) // 64 * 64
        self.P = P0.clone()
        self.G = torch.zeros(NGRAD, **f32)
        self.V = torch.zeros(NGRAD, **f32)
        self.ctrl = torch.zeros(32, dtype=torch.int32, device=dev)
        self.w1alt = torch.zeros(FEAT * HID, **f32)
        self.v1alt = torch.zeros(FEAT * HID, **f32)
        self.w1bf = self.P[OFF_W1:OFF_B1].to(torch.bfloat16)
        self.pooled = torch.zeros(FEAT, BP, dtype=torch.bfloat16, device=dev)
        self.code = torch.zeros(B, FEAT, dtype=torch.uint8, device=dev)
        self.hacc = torch.zeros(C.convnet_hacc_elems(B), dtype=torch.int64, device=dev)
        self.hconv = torch.zeros(2 * NCONV, dtype=torch.int64, device=dev)
        self.calt = torch.zeros(2 * NCONV, **f32)
        self.hred = torch.zeros(2 * NCONV, dtype=torch.int64, device=dev)
        c = torch.zeros(32, dtype=torch.int32)
        c[C_LR], c[C_MOM], c[C_NEST] = _f2i(0.1), _f2i(0.9), 0
        c[C_NS], c[C_ROW0], c[C_GB], c[C_WRAP] = X.shape[0], rank * B, GB, int(wrap)
        self.ctrl.copy_(c.to(dev))
        bufs = dict(params=self.P.data_ptr(), grads=self.G.data_ptr(), velocity=self.V.data_ptr(),
                    ctrl=self.ctrl.data_ptr(), pooled=self.pooled.data_ptr(), code=self.code.data_ptr(),
                    w1alt=self.w1alt.data_ptr(), v1alt=self.v1alt.data_ptr(), w1bf=self.w1bf.data_ptr(),
                    hacc=self.hacc.data_ptr(), hconv=self.hconv.data_ptr(), calt=self.calt.data_ptr(),
                    eager_w1=0, ppb=ppb)
        torch.cuda.synchronize(dev)
        self.t = C.ConvNetTrainer(dev.index or 0, bufs, B, PP, 1)
        self.t.set_data(X.data_ptr(), Y.data_ptr(), 1)

    def result(self):
        c = self.ctrl.cpu()
        return (self.P[:NPARAM].cpu(), self.V[:NPARAM].cpu(), c[C_AL:C_AN + 1].clone())


def _rank_order_sum(comm, t: torch.Tensor, bf16_range: Optional[Tuple[int, int]] = None) -> torch.Tensor:
    """All-gather ``t`` over the control plane and sum in rank order (fp32 adds, or exact
    int64).  ``bf16_range``: that slice is exchanged as bf16 (each partial rounded, the sum
    rounded again), as the sharded exchange with DAMD_GRAD_DTYPE=bf16 does."""
    h = t.detach().cpu()
    parts = comm.allgather(h)  # [W, ...] over gloo (CPU tensors)
    if bf16_range is not None:
        lo, hi = bf16_range
        parts = parts.clone()
        parts[:, lo:hi] = parts[:, lo:hi].to(torch.bfloat16).float()
    acc = parts[0].clone()
    for r in range(1, parts.shape[0]):
        acc += parts[r]
    if bf16_range is not None:
        lo, hi = bf16_range
        acc[lo:hi] = acc[lo:hi].to(torch.bfloat16).float()
    return acc.to(t.device)


def _host_reference(C, comm, dev, B, GB, rank, P0, X, Y, ppb, PP, gbf16):
    s = _Scratch(C, dev, B, GB, rank, P0, X, Y, ppb, PP)
    for _ in range(STEPS):
        s.t.step(1)
        if not s.t.sync(60.0):
            raise RuntimeError("self-test reference step did not complete")
        s.G.copy_(_rank_order_sum(comm, s.G, (OFF_W1, OFF_B1) if gbf16 else None))
        s.hconv.copy_(_rank_order_sum(comm, s.hconv))
        torch.cuda.synchronize(dev)
    s.t.flush()
    s.t.sync(60.0)
    torch.cuda.synchronize(dev)
    return s.result()


def _setup(kind, C, comm, peer, native, dev, B, GB, rank, P0, X, Y, ppb, PP, gbf16, cu_split, wrap=0):
    """A scratch trainer wired to transport ``kind``.  Local only: the caller votes on
    the outcome BEFORE any collective that assumes every rank got this far."""
    s = _Scratch(C, dev, B, GB, rank, P0, X, Y, ppb, PP, wrap)
    if cu_split is not None:
        s.t.restrict_cus(*cu_split)
    if kind == "xgmi-sharded":
        s.t.set_sharded(peer, s.hred.data_ptr(), int(gbf16))
        s.t.set_exchange_timeout(TIMEOUT_S)
    elif kind == "xgmi-peer":
        peer.set_timeout(TIMEOUT_S)
        s.t.set_peer(peer, fold=True)
    elif kind == "rccl":
        if native is None:
            raise ValueError("rccl: no native RCCL communicator")
        s.t.set_comm(native)
    else:
        raise ValueError(kind)
    return s


def _voted_setup(kind, comm, *args):
    """(scratch, why) on every rank; scratch None on EVERY rank if any rank's set-up failed
    (restrict_cus / set_sharded / set_peer raising on one rank must not leave that rank
    in a different collective than the others)."""
    s, why = None, ""
    try:
        s = _setup(*args)
    except Exception as e:  # every rank must reach the vote below
        why = f"set-up raised {e!r}"
    votes = comm.allgather_object(why)
    bad = [(r, w) for r, w in enumerate(votes) if w]
    if bad:
        return None, "; ".join(f"rank {r}: {w}" for r, w in bad)
    if kind == "xgmi-sharded":
        comm.barrier()  # every rank's flags are cleared before any rank's first step
    return s, ""


def _run_under_test(s, peer):
    s.t.step(STEPS)
    done = s.t.sync(4 * TIMEOUT_S + 30.0)
    s.t.flush()
    done = s.t.sync(4 * TIMEOUT_S + 30.0) and done
    torch.cuda.synchronize()
    st = peer.status() if peer is not None else 0
    return s.result(), bool(done), int(st)


def _inject_target(kind: str, rank: int) -> bool:
    spec = os.environ.get("DAMD_XCHG_SELFTEST_INJECT", "")
    if not spec:
        return False
    k, _, r = spec.partition(":")
    return k == kind and rank == (int(r) if r else 1)


def verify(kind: str, C, comm, peer, dev, B: int, ppb: int, PP: int, P0: torch.Tensor, gbf16: bool = False,
           cu_split: Optional[Tuple[int, int]] = None) -> bool:
    """Self-test transport ``kind`` ('xgmi-sharded' | 'xgmi-peer') on every rank; True iff it
    matched the rank-order host reduction bitwise on EVERY rank (collective: every rank
    must call it with the same kind)."""
    W, rank = comm.world_size, comm.rank
    GB = B * W
    rng = np.random.default_rng(12345)  # the same synthetic rows on every rank
    n = GB * (STEPS + 1)
    X = torch.from_numpy(rng.integers(0, 256, size=(n, 784), dtype=np.uint8)).to(dev)
    Y = torch.from_numpy(rng.integers(0, 10, size=n).astype(np.int32)).to(dev)
    ok, why, got = True, "", None
    s, why = _voted_setup(kind, comm, kind, C, comm, peer, None, dev, B, GB, rank, P0, X, Y, ppb, PP, gbf16, cu_split)
    if s is None:  # identical on every rank: skip the run AND the host reference
        dlog.warning("gradient exchange %s: self-test set-up failed (%s)", kind, why)
        return False
    try:
        got, done, st = _run_under_test(s, peer)
        if _inject_target(kind, rank):
            got[0][0] = torch.nextafter(got[0][0], torch.tensor(float("inf")))
        if not done or st != 0:
            ok, why = False, f"exchange waits expired (status {st:#x})" if st else "step did not complete"
    except Exception as e:  # every rank must reach the vote below
        ok, why, got = False, f"raised {e!r}", None
    del s
    try:
        ref = _host_reference(C, comm, dev, B, GB, rank, P0, X, Y, ppb, PP, gbf16 and kind == "xgmi-sharded")
    except Exception as e:
        ok, why, ref = False, f"host reference raised {e!r}", None
    if ok:
        names = ("parameters", "velocities", "epoch metric sums")
        for nm, a, b in zip(names, got, ref):
            if not torch.equal(a, b):
                d = (a.double() - b.double()).abs()
                ok, why = False, f"{nm} differ from the host rank-order reduction (max |diff| {d.max().item():.3g}, " \
                                 f"{int((d > 0).sum())} values)"
                break
    votes = comm.allgather_object((ok, why))
    if peer is not None:
        peer.clear_status()
        torch.cuda.synchronize(dev)
    all_ok = all(v[0] for v in votes)
    if not all_ok:
        bad = [(r, v[1]) for r, v in enumerate(votes) if not v[0]]
        dlog.warning("gradient exchange %s failed its start-up self-test on rank(s) %s", kind,
                     "; ".join(f"{r}: {w}" for r, w in bad))
    else:
        dlog.info("gradient exchange %s: start-up self-test passed (%d steps bitwise equal to the host "
                  "rank-order reduction on %d ranks)", kind, STEPS, W)
    return all_ok


def time_transport(kind: str, C, comm, peer, native, dev, B: int, ppb: int, PP: int, P0: torch.Tensor,
                   gbf16: bool = False, cu_split: Optional[Tuple[int, int]] = None,
                   steps: int = 20) -> Optional[float]:
    """Seconds per step of transport ``kind`` ('xgmi-sharded' | 'xgmi-peer' | 'rccl'), max over
    ranks, or None on EVERY rank if it could not be timed (collective).

    Measured the way bench.py times its headline window: ``steps`` training steps + the
    flush of the last deferred update captured as ONE graph (capture_final), one untimed
    replay, then a barrier, one timed replay and a device synchronize.  Scratch buffers on
    synthetic rows, so the model's own state is untouched; the kernels are the ones a real
    step runs (reference README.md:398, ``CollectiveCommunication.AUTO``: the runtime, not
    the user, picks the collective implementation)."""
    import time

    W, rank = comm.world_size, comm.rank
    GB = B * W
    wrap = 4
    rng = np.random.default_rng(777)
    X = torch.from_numpy(rng.integers(0, 256, size=(GB * wrap, 784), dtype=np.uint8)).to(dev)
    Y = torch.from_numpy(rng.integers(0, 10, size=GB * wrap).astype(np.int32)).to(dev)
    s, why = _voted_setup(kind, comm, kind, C, comm, peer, native, dev, B, GB, rank, P0, X, Y, ppb, PP, gbf16,
                          cu_split, wrap)
    if s is None:
        dlog.warning("gradient exchange %s: not timed (%s)", kind, why)
        return None
    dt, ok = 0.0, True
    try:
        s.t.capture_final(int(steps))
        s.t.run_final(int(steps))  # untimed: first replay
        ok = bool(s.t.sync(4 * TIMEOUT_S + 30.0))
    except Exception as e:  # every rank must reach the collectives below
        dlog.warning("gradient exchange %s: timing run raised %r", kind, e)
        ok = False
    comm.barrier()
    if ok:
        t0 = time.perf_counter()
        s.t.run_final(int(steps))
        ok = bool(s.t.sync(4 * TIMEOUT_S + 30.0))
        dt = time.perf_counter() - t0
    st = peer.status() if (peer is not None and kind != "rccl") else 0
    votes = comm.allgather_object((ok and st == 0, dt))
    if peer is not None:
        peer.clear_status()
    torch.cuda.synchronize(dev)
    del s
    if not all(v[0] for v in votes):
        dlog.warning("gradient exchange %s: timing run failed on some rank", kind)
        return None
    return max(v[1] for v in votes) / steps
