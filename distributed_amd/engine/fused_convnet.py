"""Fused MI355X engine for the reference CNN family (reference README.md:58-73).

Pattern: ``Conv2D(32, 3, relu, input (28,28,1)) -> MaxPooling2D(2) -> Flatten ->
Dense(64, relu) -> Dense(10)`` + ``SparseCategoricalCrossentropy(from_logits=True)`` +
``SGD`` (any lr / momentum / nesterov) + accuracy metric.

Execution (csrc/kernels/convnet_step2.hip, csrc/runtime/step_executor.cpp): a step is
two HIP launches (fwd, bwd) plus, at world > 1, the per-step SUM all-reduce of the flat
gradient buffer (347,146 grads + [loss, correct, count] tail); the SGD update is applied
eagerly by bwd (world 1) or deferred into the next step's fwd; k steps are captured into
one hipGraph and replayed.  Model
variables are views of the fp32 master buffer, so ``get_weights``/checkpoints see the
trained values after ``finish()`` (which applies the last pending update).
"""
from __future__ import annotations

import struct

import numpy as np
import torch

from ..utils import env
from ..utils import logging as dlog
from .base import Engine, ExchangeFault  # noqa: F401  (ExchangeFault: re-exported)
from .data import DataFeed


class ExchangeSelfTestError(RuntimeError):
    """A pinned device gradient exchange (DAMD_ALLREDUCE=xgmi | sharded) failed its start-up
    self-test (engine/xchg_selftest.py).  Raised on EVERY rank (the outcome is a collective
    vote), so a caller may catch it and go on with another transport consistently."""

NPARAM = 347146
NGRAD = 347152
HID, NCLS, FEAT, NCONV = 64, 10, 5408, 320
# ctrl word indices (csrc/include/damd_common.h struct Ctrl)
(C_LR, C_MOM, C_NEST, C_NS, C_ROW0, C_GB, C_CUR, C_IT, C_CA, C_CB, C_AL, C_AC, C_AN, C_WRAP, C_CUR2, C_CUR3, C_WPAR,
 C_FLUSHT, C_PEND, C_PAR2, C_BAD, C_XCNT, C_XCNT2, C_TICKET, C_PEND2, C_XGEN) = range(26)
SHAPES = [(3, 3, 1, 32), (32,), (5408, 64), (64,), (64, 10), (10,)]


def _xchg_fault_at(rank: int, world: int):
    spec = env.get_str("DAMD_XCHG_FAULT_AT", "")
    if not spec or world < 2:
        return None
    r, _, st = spec.partition(":")
    return int(st) if int(r) == rank else None


def _f2i(f: float) -> int:
    return struct.unpack("<i", struct.pack("<f", float(f)))[0]


def _i2f(i: int) -> float:
    return struct.unpack("<f", struct.pack("<i", int(i)))[0]


class FusedConvNetEngine(Engine):
    name = "fused_convnet"

    @staticmethod
    def eligible(model, strategy):
        from ..keras import layers as L
        from ..keras import losses, optimizers

        if strategy.device.type != "cuda":
            return False, "not on a GPU"
        ls = [l for l in getattr(model, "layers", []) if not isinstance(l, L.InputLayer)]
        if len(ls) != 5:
            return False, "layer count"
        c, p, f, d1, d2 = ls
        if not (isinstance(c, L.Conv2D) and c.filters == 32 and c.kernel_size == (3, 3) and c.strides == (1, 1)
                and c.padding == "valid" and c.dilation_rate == (1, 1) and c.use_bias
                and c.activation.__name__ == "relu" and tuple(c.input_shape or ())[1:] == (28, 28, 1)):
            return False, "conv layer"
        if not (isinstance(p, L.MaxPooling2D) and p.pool_size == (2, 2) and p.strides == (2, 2)
                and p.padding == "valid"):
            return False, "pool layer"
        if not isinstance(f, L.Flatten):
            return False, "flatten"
        if not (isinstance(d1, L.Dense) and d1.units == 64 and d1.use_bias and d1.activation.__name__ == "relu"):
            return False, "dense"
        if not (isinstance(d2, L.Dense) and d2.units == 10 and d2.use_bias and d2.activation.__name__ == "linear"):
            return False, "dense_1"
        if not (isinstance(model.loss, losses.SparseCategoricalCrossentropy) and model.loss.from_logits):
            return False, "loss"
        if type(model.optimizer) is not optimizers.SGD:
            return False, "optimizer"
        if len(model.trainable_weights) != len(SHAPES):
            return False, "frozen layer weights"
        for m in model.compiled_metrics:
            if m.name not in ("accuracy", "acc", "sparse_categorical_accuracy"):
                return False, f"metric {m.name}"
        return True, ""

    def __init__(self, model, strategy, per_replica_batch, global_batch, exclude=()):
        super().__init__(model, strategy, per_replica_batch, global_batch)
        from ..native import require_C

        C = require_C()
        dev = self.device
        B = per_replica_batch
        # pooled positions per slice: 3 (57 slices, F3 on 57 CUs) measured 29.2 vs 30.0 us
        # per step for 4 (43 slices); 2 and 1 lose to the larger F1 grid
        self.PP = env.get_int("DAMD_PP", 3)
        if not 1 <= self.PP <= 4:
            raise ValueError("DAMD_PP must be in [1, 4]")
        # the backward kernel's own slicing (one block per slice): finer slices spread its
        # post-head work (dW1 / dP MFMAs, pool / ReLU backward, conv gradient) over more CUs.
        # rocprofv3 bwd duration, B=64: 13.32 us (1 position, 169 blocks), 12.53 us (2, 85),
        # 13.16 us (3, 57): more blocks also mean more same-address conv-gradient atomics
        # and redundant heads, so 2 is the default
        self.PPB = env.get_int("DAMD_PP_BWD", 2)
        if not 1 <= self.PPB <= 4:
            raise ValueError("DAMD_PP_BWD must be in [1, 4]")
        NS = C.convnet_num_slices(self.PP)
        f32 = dict(dtype=torch.float32, device=dev)
        BP = (B + 63) // 64 * 64  # padded batch pitch of the feature-major buffers
        self.P = torch.zeros(NGRAD, **f32)
        self.G = torch.zeros(C.convnet_grad_count(self.PP), **f32)  # grads + metric tail
        self.V = torch.zeros(NGRAD, **f32)
        self.ctrl = torch.zeros(32, dtype=torch.int32, device=dev)
        self.w1alt = torch.zeros(FEAT * HID, **f32)   # W1 double buffer (by step parity)
        self.v1alt = torch.zeros(FEAT * HID, **f32)
        self.w1bf = torch.zeros(FEAT * HID, dtype=torch.bfloat16, device=dev)
        self.pooled = torch.zeros(FEAT, BP, dtype=torch.bfloat16, device=dev)
        self.code = torch.zeros(B, FEAT, dtype=torch.uint8, device=dev)
        self.hacc = torch.zeros(C.convnet_hacc_elems(B), dtype=torch.int64, device=dev)  # by step parity
        self.hconv = torch.zeros(2 * NCONV, dtype=torch.int64, device=dev)
        self.calt = torch.zeros(2 * NCONV, **f32)  # alternate conv parameters + velocity
        # next-batch prefetch (B <= 64): bwd copies the next step's rows here for the next fwd,
        # tagged with the ctrl block's data generation + cursor (DAMD_XPREFETCH=0: off)
        self.xnext = self.xtag = self.xcur = self.ycur = None
        if B <= 64 and env.get_bool("DAMD_XPREFETCH", True):
            self.xnext = torch.zeros(B * 784, **f32)  # (u8 rows use the first quarter)
            self.xtag = torch.zeros(1, dtype=torch.int64, device=dev)
            # this step's rows / labels as the fwd read them, for the bwd (no cursor needed)
            self.xcur = torch.zeros(B * 784, **f32)
            self.ycur = torch.zeros(B, dtype=torch.int32, device=dev)
        # model variables -> views of the fp32 master buffer (Keras weight order)
        self.vars = model.trainable_weights
        off = 0
        for v, shp in zip(self.vars, SHAPES):
            if tuple(v.shape) != shp:
                raise RuntimeError(f"unexpected variable shape {v.shape} for {v.name}")
            n = int(np.prod(shp))
            v._rebind(self.P[off:off + n].view(shp))
            off += n
        self._own_variables(self.vars)
        opt = model.optimizer
        if opt.momentum and "momentum" in opt.slots and opt.slots["momentum"].numel() == NPARAM:
            self.V[:NPARAM].copy_(opt.slots["momentum"].to(dev))
        if self.world > 1:
            strategy.communicator.broadcast_(self.P, 0)  # mirrored variables start equal
        c = self.ctrl.cpu()
        c[C_IT] = int(opt.iterations)
        self.ctrl.copy_(c.to(dev))
        self._write_hparams()
        torch.cuda.synchronize(dev)
        bufs = dict(params=self.P.data_ptr(), grads=self.G.data_ptr(), velocity=self.V.data_ptr(),
                    ctrl=self.ctrl.data_ptr(),
                    pooled=self.pooled.data_ptr(), code=self.code.data_ptr(), w1alt=self.w1alt.data_ptr(),
                    v1alt=self.v1alt.data_ptr(), w1bf=self.w1bf.data_ptr(),
                    hacc=self.hacc.data_ptr(), hconv=self.hconv.data_ptr(), calt=self.calt.data_ptr(),
                    ppb=self.PPB)
        if self.xnext is not None:
            bufs.update(xnext=self.xnext.data_ptr(), xtag=self.xtag.data_ptr(), xcur=self.xcur.data_ptr(),
                        ycur=self.ycur.data_ptr())
        # world 1 (no gradient all-reduce): bwd applies the W1 update itself as soon as it
        # has the slice's gradient, and fwd reads only the bf16 copy (DAMD_EAGER_W1=0: the
        # deferred update in fwd, as with an all-reduce between the launches)
        force_ar = env.get_bool("DAMD_FORCE_ALLREDUCE", False)
        # (B <= 64: the single-chunk backward; the multi-chunk one has no registers to spare
        # for the slice's masters)
        self.eager_w1 = self.world == 1 and not force_ar and B <= 64 and env.get_bool("DAMD_EAGER_W1", True)
        bufs["eager_w1"] = int(self.eager_w1)
        self.stamps = None
        if env.get_bool("DAMD_STAMPS", False):  # diagnostics: per-phase s_memrealtime stamps
            self.stamps = torch.zeros(3, 256, 16, dtype=torch.int64, device=dev)
            bufs["stamps"] = self.stamps.data_ptr()
        self.trainer = C.ConvNetTrainer(dev.index or 0, bufs, B, self.PP, 1)
        self._refresh_w1bf()
        # DAMD_FORCE_ALLREDUCE=1 keeps the (size-1) RCCL all-reduce inside the captured step
        # at world 1: the multi-GPU graph path exercised on a single GPU
        force = env.get_bool("DAMD_FORCE_ALLREDUCE", False)
        native = strategy.communicator.native if (self.world > 1 or force) else None
        if "rccl" in (exclude or ()):
            native = None  # RCCL faulted mid-run on this gang: host all-reduce from here on
        # per-step gradient exchange at world > 1 (DAMD_ALLREDUCE):
        #   auto / sharded -- inside the two step kernels (convnet.h XArgs): each rank owns a
        #       quarter-slice unit of dW1 per 1/world of the units, bwd pushes partials to the
        #       owners over xGMI, owners reduce in rank order and push the reduced units back;
        #       the small gradients + metrics travel as one message per rank.  No extra launch.
        #   xgmi -- the standalone two-shot peer all-reduce kernel after bwd (folded staging)
        #   rccl -- RCCL inside the captured step; off -- no device transport (RCCL if the
        #       communicator has one, else the host-staged gloo all-reduce between steps)
        # Both peer modes need every rank to map every peer (one node); else RCCL.
        self.peer = None
        self.sharded = False
        # transports never to use again on this engine: the ones a mid-run exchange fault
        # was detected on (rebuild_after_fault)
        self.exclude = set(exclude or ())
        self.transport_us: dict = {}  # measured us / step per candidate exchange (auto mode)
        # start-up self-test outcome of the device exchange (None: no device exchange was
        # self-tested -- world 1, RCCL or the host all-reduce) and the transports that failed it
        self.exchange_verified = None
        self.exchange_fallback_from: list = []
        self.hred = torch.zeros(2 * NCONV, dtype=torch.int64, device=dev)  # sharded: conv sums for flush
        mode = env.get_str("DAMD_ALLREDUCE", "auto").lower()
        self._mode = mode
        if mode not in ("auto", "sharded", "xgmi", "rccl", "off"):
            raise ValueError("DAMD_ALLREDUCE must be auto, sharded, xgmi, rccl or off")
        # DAMD_GRAD_DTYPE=bf16: the exchanged dW1 travels as bf16 (fp32 accumulation by the
        # owner, fp32 master update); default fp32 (reference parity)
        self.grad_dtype = env.get_str("DAMD_GRAD_DTYPE", "fp32").lower()
        if self.grad_dtype not in ("fp32", "bf16"):
            raise ValueError("DAMD_GRAD_DTYPE must be fp32 or bf16")
        if self.world > 1 and mode not in ("rccl", "off") and not {"xgmi-sharded", "xgmi-peer"} <= self.exclude:
            from ..parallel.communicator import make_peer_allreduce

            # in-kernel wait deadline: the collective watchdog's (its default included), so a
            # missing peer is reported by the kernel's status word no later than the watchdog
            from ..utils.watchdog import deadline_for

            wd = deadline_for(self.world)
            want_sharded = mode in ("auto", "sharded") and self.world <= 8
            if want_sharded:
                NU = 4 * C.convnet_num_slices(self.PPB)
                cap = max(self.world * NU * 2048, 347648 + 2 * 8 * 1408 + 16384 + FEAT * HID // 2)
            else:
                cap = C.PeerAllreduce.message_words(C.convnet_grad_count(self.PP), 2 * NCONV)
            self.peer = make_peer_allreduce(strategy.communicator, dev.index or 0, cap,
                                            blocks=env.get_int("DAMD_PEER_BLOCKS", 64),
                                            timeout_s=wd if wd > 0 else 60.0)
            if self.peer is None and mode in ("xgmi", "sharded"):
                raise RuntimeError(f"DAMD_ALLREDUCE={mode} but the xGMI peer mapping is unavailable")
            if self.peer is not None:
                # ranks sharing one device (the 1-GPU rehearsal of a multi-GPU run): each
                # rank's step stream gets its own CUs -- the in-kernel waits of one rank must
                # not hold the CUs another rank needs to publish what they wait for
                # (two ranks need no split: one rank's waiting forward leaves the other's
                # 57-169-block backward enough CUs to finish -- measured 44.7 us/step shared
                # vs 78 us with halved CUs; from three ranks on, the waiting forwards of two
                # ranks can hold every CU)
                ndev = max(1, torch.cuda.device_count())
                share = [q for q in range(self.world) if q % ndev == (dev.index or 0)]
                cu_split = ((share.index(self.rank), len(share))
                            if len(share) > 2 and env.get_bool("DAMD_SHARED_CU_SPLIT", True) else None)
                # start-up self-test of each candidate transport against the host rank-order
                # reduction, bitwise, on every rank (engine/xchg_selftest.py); then, with the
                # transport not pinned, every candidate that passed (and RCCL) is TIMED the way
                # bench.py times its window, and the fastest carries the run (reference
                # README.md:398, communication = AUTO).  Without tuning: the first that passes,
                # sharded -> xgmi -> RCCL.
                cands = [k for k in ((["xgmi-sharded"] if want_sharded else [])
                                     + ([] if mode == "sharded" else ["xgmi-peer"])) if k not in self.exclude]
                tune = (mode == "auto" and env.get_bool("DAMD_XCHG_TUNE", True))
                from . import xchg_selftest

                passed = []
                selftested = env.get_bool("DAMD_XCHG_SELFTEST", True)
                if selftested:
                    for kind in cands:
                        if xchg_selftest.verify(kind, C, strategy.communicator, self.peer, dev, B, self.PPB, self.PP,
                                                self.P, gbf16=self.grad_dtype == "bf16" and kind == "xgmi-sharded",
                                                cu_split=cu_split):
                            passed.append(kind)
                            if not tune:
                                break
                        else:
                            self.exchange_fallback_from.append(kind)
                else:
                    passed = list(cands) if tune else cands[:1]
                chosen = passed[0] if passed else None
                timed = passed + (["rccl"] if (native is not None and "rccl" not in self.exclude) else [])
                if tune and len(timed) > 1:
                    for kind in timed:
                        t = xchg_selftest.time_transport(kind, C, strategy.communicator, self.peer, native, dev, B,
                                                         self.PPB, self.PP, self.P,
                                                         gbf16=self.grad_dtype == "bf16" and kind == "xgmi-sharded",
                                                         cu_split=cu_split)
                        if t is not None:
                            self.transport_us[kind] = round(t * 1e6, 2)
                    if self.transport_us:
                        chosen = min(self.transport_us, key=self.transport_us.get)
                # in-kernel wait deadline of the run (DAMD_XCHG_TIMEOUT_S: shorter, for tests)
                self.peer.set_timeout(env.get_float("DAMD_XCHG_TIMEOUT_S", wd if wd > 0 else 60.0))
                if selftested and chosen is not None and chosen != "rccl":
                    self.exchange_verified = True
                if chosen == "rccl":
                    self.peer = None  # RCCL measured fastest: set_comm below
                elif chosen is None:
                    if mode in ("xgmi", "sharded"):
                        raise ExchangeSelfTestError(f"DAMD_ALLREDUCE={mode}: the exchange failed its start-up self-test")
                    dlog.warning("fused ConvNet engine: no xGMI exchange passed its self-test; using %s",
                                 "RCCL" if native is not None else "the host (gloo) all-reduce")
                    self.peer = None
                elif chosen == "xgmi-sharded":
                    self.trainer.set_sharded(self.peer, self.hred.data_ptr(), int(self.grad_dtype == "bf16"))
                    self.sharded = True
                    if cu_split is not None:
                        self.trainer.restrict_cus(*cu_split)
                    # every rank's flags are zero before any rank's first step writes into them
                    strategy.communicator.barrier()
        if self.grad_dtype == "bf16" and not self.sharded:
            if self.world > 1:
                dlog.warning("DAMD_GRAD_DTYPE=bf16 applies to the sharded exchange only; exchanging fp32")
            self.grad_dtype = "fp32"
        # host-collective mode (DAMD_COMM=gloo, e.g. several ranks on one GPU): one step at a
        # time, the gradient/metric buffer all-reduced through the host between steps
        self.host_collective = self.world > 1 and native is None and self.peer is None
        self.allreduce_kind = ("none" if self.world == 1 and not force else
                               "xgmi-sharded" if self.sharded else
                               "xgmi-peer" if self.peer is not None else
                               "rccl" if native is not None else "host-gloo")
        if self.peer is not None and not self.sharded:
            # folded (default): bwd writes its gradient straight into the peer kernel's `in`
            # staging and fwd / flush read the reduced gradient from its `out`, so the peer
            # kernel only exchanges (no copy-in / copy-out passes over the 1.39 MB message)
            self.trainer.set_peer(self.peer, fold=env.get_bool("DAMD_PEER_FOLD", True))
        elif self.peer is None and native is not None:
            self.trainer.set_comm(native)
        if self.world > 1:
            dlog.info("fused ConvNet engine: gradient exchange via %s",
                      {"xgmi-sharded": "the step kernels (sharded xGMI exchange)",
                       "xgmi-peer": "xGMI peer-to-peer all-reduce kernel", "rccl": "RCCL",
                       "host-gloo": "host (gloo)"}[self.allreduce_kind])
            if self.transport_us:
                dlog.info("gradient exchange: %s (%s)", self.allreduce_kind,
                          ", ".join(f"{k} {v:.1f} us" for k, v in self.transport_us.items()))
        self.use_graph = env.get_bool("DAMD_GRAPH", True) and not self.host_collective
        self.graph_steps = max(1, env.get_int("DAMD_GRAPH_STEPS", 20))
        self.watchdog_s = env.get_float("DAMD_WATCHDOG_S", 0.0)
        opt._iter_source = self._iterations
        self.feed = None
        self._pending = False
        self.steps_done = 0
        self._fault_done = bool(exclude)  # the fault injection fires once per gang
        dlog.debug("fused ConvNet engine: B=%d, slices=%d, graph=%s", B, NS, self.use_graph)

    # --- host <-> ctrl ---------------------------------------------------------------
    def _ctrl_host(self, soft=False):
        self.trainer.sync(self.watchdog_s) or self._watchdog_fired()
        self._check_peer(soft)
        return self.ctrl.cpu().tolist()

    def _check_peer(self, soft=False):
        if self.peer is not None and self.peer.status():
            if soft:
                # mid-epoch read with fault recovery on: the epoch-end vote decides (every
                # rank together) -- raising here on one rank would strand the others
                if not getattr(self, "_fault_logged", False):
                    dlog.warning("gradient exchange %s: a bounded wait expired on rank %d; the epoch will be "
                                 "re-run on another transport", self.allreduce_kind, self.rank)
                    self._fault_logged = True
                return
            raise RuntimeError("xGMI peer all-reduce: a wait for a peer timed out (peer missing or wedged)")

    def _ctrl_write(self, updates: dict):
        self.trainer.sync(self.watchdog_s) or self._watchdog_fired()
        self._check_peer()
        c = self.ctrl.cpu()
        for k, v in updates.items():
            c[k] = v
        # any host write may move the cursor or follow new epoch rows: a batch the last bwd
        # prefetched must not match its tag any more
        c[C_XGEN] = (int(c[C_XGEN]) + 1) & 0x7fffffff
        self.ctrl.copy_(c.to(self.device))
        torch.cuda.synchronize(self.device)

    def _write_hparams(self):
        opt = self.model.optimizer
        c = self.ctrl.cpu()
        c[C_LR] = _f2i(opt.learning_rate)
        c[C_MOM] = _f2i(opt.momentum)
        c[C_NEST] = int(opt.nesterov)
        c[C_ROW0] = self.rank * self.per_replica
        c[C_GB] = self.global_batch
        self.ctrl.copy_(c.to(self.device))

    def _watchdog_fired(self):
        what = ("xGMI peer all-reduce wedged" if self.peer is not None else "RCCL communicator aborted")
        raise RuntimeError(f"collective watchdog: step did not complete within {self.watchdog_s}s; {what}")

    def _iterations(self):
        return self._ctrl_host()[C_IT]

    def reload_optimizer_state(self):
        self._flush()
        self.trainer.sync(0.0)
        opt = self.model.optimizer
        if opt.momentum and "momentum" in opt.slots and opt.slots["momentum"].numel() == NPARAM:
            self.V[:NPARAM].copy_(opt.slots["momentum"].to(self.device))
        opt._iter_source = None
        it = int(opt.iterations)
        opt._iter_source = self._iterations
        self._ctrl_write({C_IT: it})

    def lr_changed(self):
        self._flush()
        c = {C_LR: _f2i(self.model.optimizer.learning_rate)}
        self._ctrl_write(c)

    # --- data / epochs ---------------------------------------------------------------
    def bind(self, x, y):
        x = np.asarray(x)
        if tuple(x.shape[1:]) not in ((28, 28, 1), (28, 28), (784,)):
            raise ValueError(f"fused ConvNet engine expects 28x28x1 inputs, got {x.shape[1:]}")
        key = (id(x), id(y), len(x))
        if self.feed is None or getattr(self, "_feed_key", None) != key:
            self.trainer.sync(0.0)
            self.feed = DataFeed(x, y, self.device, flatten=True, allow_u8=env.get_bool("DAMD_X_U8", True))
            if self.feed.n * 784 * (1 if self.feed.x_u8 else 4) >= 2 ** 31:
                # the step kernels address the (epoch-permuted) dataset with 32-bit offsets
                raise ValueError(f"fused ConvNet engine: {self.feed.n} rows exceed the 2 GiB dataset limit")
            self._feed_key = key
            torch.cuda.synchronize(self.device)
            self.x_ep = torch.empty_like(self.feed.x)
            self.y_ep = torch.empty_like(self.feed.y)
            torch.cuda.synchronize(self.device)
            self.trainer.set_data(self.x_ep.data_ptr(), self.y_ep.data_ptr(), int(self.feed.x_u8))
            self._ctrl_write({C_NS: self.feed.n})
        return self.feed

    def start_epoch(self, epoch, shuffle, wrap_steps: int = 0):
        """``wrap_steps > 0`` makes the device cursor wrap (benchmark runs longer than an
        epoch without host round trips); fit() manages epochs on the host (wrap 0)."""
        self._flush()
        self.trainer.sync(0.0)
        self.feed.set_epoch(epoch, shuffle, self.shuffle_seed)
        # materialise the epoch order once (one gather per epoch instead of an index
        # indirection on every step's critical path)
        perm = self.feed.perm.long()
        torch.index_select(self.feed.x, 0, perm, out=self.x_ep)
        torch.index_select(self.feed.y, 0, perm, out=self.y_ep)
        opt = self.model.optimizer
        self._ctrl_write({C_CUR: 0, C_AL: 0, C_AC: 0, C_AN: 0, C_WRAP: int(wrap_steps),
                          C_LR: _f2i(opt.learning_rate), C_MOM: _f2i(opt.momentum), C_NEST: int(opt.nesterov)})

    def run(self, n_steps):
        fa = _xchg_fault_at(self.rank, self.world)
        if fa is not None and self.steps_done <= fa < self.steps_done + n_steps and not self._fault_done:
            # tests only (DAMD_XCHG_FAULT_AT=rank:step): this rank stalls before launching
            # global step `step`, so the other ranks' bounded exchange waits expire
            import time

            self._fault_done = True
            k = fa - self.steps_done
            if k:
                self.run(k)
            self.trainer.sync(0.0)
            time.sleep(env.get_float("DAMD_XCHG_FAULT_DELAY_S", 3.0))
            self.run(n_steps - k)
            return
        if self.host_collective:
            for _ in range(n_steps):
                self.trainer.step(1)
                self.trainer.sync(0.0)
                self.strategy.communicator.allreduce_(self.G, "sum")
                self.strategy.communicator.allreduce_(self.hconv, "sum")  # exact int64 sum
                torch.cuda.synchronize(self.device)
            self._pending = True
            self.steps_done += n_steps
            return
        if self.use_graph and n_steps >= self.graph_steps:
            self.trainer.capture(self.graph_steps)
        if self.use_graph:
            self.trainer.run(n_steps)
        else:
            self.trainer.step(n_steps)
        self._pending = True
        self.steps_done += n_steps

    def phase_times(self, n_steps: int) -> dict:
        """forward (incl. the fused SGD update of the previous step's gradient), backward and
        gradient all-reduce, from HIP events between the launches of eager 2-launch steps."""
        if self.host_collective:
            return super().phase_times(n_steps)
        self.sync()
        rows = self.trainer.phase_times(int(n_steps))
        self._pending = True
        self.steps_done += n_steps
        n = max(len(rows), 1)
        fwd = sum(r[0] for r in rows) / n
        bwd = sum(r[1] for r in rows) / n
        ar = sum(r[2] for r in rows) / n
        return {"forward": fwd, "backward": bwd, "allreduce": ar, "optimizer": 0.0,
                "step": fwd + bwd + ar,
                "note": ("W1 SGD update in the backward kernel, conv / b1 / W2 / b2 updates in the forward kernel"
                         if self.eager_w1 else "SGD update fused into the forward kernel"),
                "allreduce_kind": self.allreduce_kind}

    def prepare(self, n_steps):
        if self.use_graph and not self.host_collective and n_steps >= self.graph_steps:
            self.trainer.capture(self.graph_steps)

    def prepare_final(self, n_steps) -> bool:
        """Capture ``n_steps`` steps followed by the flush of the last deferred update as ONE
        graph, for a timed run that must end with every update applied (bench.py): one
        replay instead of n / graph_steps replays plus an eager flush launch."""
        if self.host_collective or not self.use_graph or n_steps <= 0:
            return False
        try:
            self.trainer.capture_final(int(n_steps))
            # one replay with every node disabled: the graph's first-launch cost (~9 us
            # measured, scripts/probe_cold_graph.py) is paid here, outside the timed window.
            # A graph whose nodes cannot be toggled is only not pre-warmed.
            if env.get_bool("DAMD_WARM_FINAL", True):
                self.trainer.warm_final(int(n_steps))
        except RuntimeError as e:
            dlog.warning("final-graph capture unavailable (%s): timed run replays step graphs + flush", e)
            return False
        return True

    def run_and_flush(self, n_steps):
        """``n_steps`` steps, then the pending update applied (run + _flush), through the
        prepare_final graph when one was captured for this count."""
        if (n_steps > 0 and not self.host_collective and self.use_graph
                and self.trainer.run_final(int(n_steps))):
            self._pending = False
            self.steps_done += n_steps
            return
        self.run(n_steps)
        self._flush()

    def _flush(self):
        if self._pending:
            self.trainer.flush()
            self._pending = False

    def metrics(self):
        soft = self.recovers_faults
        c = self._ctrl_host(soft)
        # the last step's reduced metric tail (in the peer `out` staging when folded)
        tail = list(self.trainer.metric_tail()) if self._pending else [0.0, 0.0, 0.0]
        # metric_tail's gather waits (bounded) for every rank's last message: a wait that
        # expired there leaves a stale tail -- never report it
        self._check_peer(soft)
        loss = _i2f(c[C_AL]) + tail[0]
        corr = _i2f(c[C_AC]) + tail[1]
        cnt = _i2f(c[C_AN]) + tail[2]
        d = max(cnt, 1.0)
        # a non-finite / out-of-range value met a fixed-point sum (ctrl.bad): NaN, like the
        # fp32 engines would show it (TerminateOnNaN must fire)
        out = {"loss": float("nan") if c[C_BAD] else loss / d, "_count": cnt}
        for m in self.model.compiled_metrics:
            out[m.name] = corr / d
        return out

    def end_epoch(self):
        self._flush()
        if self.recovers_faults:
            self._vote_exchange_health()
        return self.metrics()

    # --- mid-run exchange faults -------------------------------------------------------
    @property
    def recovers_faults(self) -> bool:
        """A device exchange whose waits are bounded (sharded / peer): a wait that expires is
        recovered from at the epoch's end (DAMD_XCHG_RECOVER=0: raise, gang restart)."""
        return (self.world > 1 and self.peer is not None and self._mode == "auto"
                and env.get_bool("DAMD_XCHG_RECOVER", True))

    def recovery_snapshot(self):
        """Host copy of the state an epoch restarts from after an exchange fault (parameters,
        momentum, iteration count), taken at the epoch's start; None without a device
        exchange to recover."""
        if not self.recovers_faults:
            return None
        self._flush()
        self.trainer.sync(self.watchdog_s) or self._watchdog_fired()
        return {"P": self.P[:NPARAM].cpu().clone(), "V": self.V[:NPARAM].cpu().clone(),
                "it": int(self.ctrl.cpu()[C_IT]), "kind": self.allreduce_kind}

    def _vote_exchange_health(self):
        done = bool(self.trainer.sync(self.watchdog_s if self.watchdog_s > 0 else 120.0))
        st = int(self.peer.status()) if self.peer is not None else 0
        votes = self.strategy.communicator.allgather_object((done, st))
        bad = [r for r, (d, q) in enumerate(votes) if not d or q]
        if bad:
            raise ExchangeFault(f"gradient exchange {self.allreduce_kind}: bounded waits expired on rank(s) {bad}")

    def rebuild_after_fault(self, snap):
        """A fresh engine on the next transport (the faulted one excluded), whose state is
        ``snap`` (recovery_snapshot of the epoch's start).  Collective: every rank calls it
        after the same ExchangeFault."""
        failed = snap["kind"]
        self.trainer.sync(5.0)
        if self.peer is not None:
            self.peer.clear_status()
        torch.cuda.synchronize(self.device)
        self.P[:NPARAM].copy_(snap["P"].to(self.device))  # the model's variables are views of P
        opt = self.model.optimizer
        opt._iter_source = None
        opt.iterations = snap["it"]
        if opt.momentum:
            opt.ensure_slots(NPARAM, self.device)
            opt.slots["momentum"].copy_(snap["V"].to(self.device))
        torch.cuda.synchronize(self.device)
        self.peer = None  # this engine is done: no host read may see its status again
        dlog.warning("gradient exchange %s faulted mid-run: re-running the epoch from its start on the next "
                     "transport", failed)
        new = FusedConvNetEngine(self.model, self.strategy, self.per_replica, self.global_batch,
                                 exclude=self.exclude | {failed})
        new.exchange_fallback_from = list(self.exchange_fallback_from) + [f"{failed} (mid-run)"]
        return new

    def finish(self):
        self._flush()
        self.trainer.sync(self.watchdog_s) or self._watchdog_fired()
        self._check_peer()  # never hand out weights built from a timed-out (partial) reduction
        opt = self.model.optimizer
        if opt.momentum:
            opt.ensure_slots(NPARAM, self.device)
            opt.slots["momentum"].copy_(self.V[:NPARAM])
        torch.cuda.synchronize(self.device)

    def _refresh_w1bf(self):
        """bf16 copy of W1 from the fp32 master (the eager step's fwd reads only the copy)."""
        torch.cuda.synchronize(self.device)
        self.w1bf.copy_(self.P[NCONV:NCONV + FEAT * HID])
        torch.cuda.synchronize(self.device)

    def after_external_write(self):
        self._refresh_w1bf()
        self._ctrl_write({C_BAD: 0})  # new weights: a past overflow no longer applies

    def _work_stream(self):
        # the step kernels run on the trainer's own HIP stream
        if getattr(self, "_ext_stream", None) is None:
            self._ext_stream = torch.cuda.ExternalStream(self.trainer.stream, device=self.device)
        return self._ext_stream

    def sync(self):
        # host readers (get_weights, checkpoints, callbacks) see the trained values: the
        # deferred update of the last step is applied first
        self._flush()
        self.trainer.sync(self.watchdog_s) or self._watchdog_fired()
        self._check_peer()  # never hand out weights built from a timed-out (partial) reduction
