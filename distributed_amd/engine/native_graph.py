"""Native graph engine: any supported Keras model lowered to a static plan of HIP kernel
launches (no autograd, no per-op Python on the hot path), captured as a HIP graph.

This is the generic-model counterpart of the fused MNIST trainer (fused_convnet.py),
used for ResNet-style networks (BASELINE.json config 4) and any
other model built from the supported layers.  What happens per step (one rank):

    gather_batch (device cursor, uint8/fp32 -> bf16 NHWC, channel padding)
    forward:  implicit-GEMM MFMA convs / dense (csrc/kernels/gemm.hip) with bias / ReLU /
              BatchNorm-statistics epilogues, fused BN(+residual)(+ReLU) apply, pooling
    loss:     softmax cross-entropy + accuracy -> dlogits and the metric tail of G
    backward: reverse plan: BN backward (3 passes), pooling backward, dgrad GEMMs
              (residual fan-in accumulated in the GEMM epilogue), wgrad GEMMs accumulated
              with fp32 atomics straight into the flat gradient buffer G (split-K)
    all-reduce G (RCCL, in the graph) -> flat SGD (+momentum) that also refreshes the
              bf16 weight shadow and advances the device cursor / epoch accumulators.

Memory is planned once at bind time (bf16 activations + gradients for every tensor —
small next to 288 GB of HBM), so the captured graph replays with no allocation.

Fusion rules (decided on the layer graph, not traced):
  Conv2D(no bias, linear) -> BatchNormalization : batch statistics from the conv epilogue
  BatchNormalization -> ReLU                    : ReLU in the BN apply
  BatchNormalization -> Add(other) [-> ReLU]    : residual add (+ the other branch's own
                                                  BN when it is BN-terminated) in one pass
"""
from __future__ import annotations

import gc
import math
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops import hip as H
from ..utils import env
from ..utils import logging as dlog
from .base import Engine
from .data import DataFeed

C_LR, C_MOM, C_NEST, C_NS, C_ROW0, C_GB, C_CUR, C_IT = 0, 1, 2, 3, 4, 5, 6, 7
C_AL, C_AC, C_AN, C_WRAP = 10, 11, 12, 13


def _f2i(f):
    return struct.unpack("<i", struct.pack("<f", float(f)))[0]


def _i2f(i):
    return struct.unpack("<f", struct.pack("<i", int(i)))[0]


def _pad8(c):
    return -(-c // 8) * 8


@dataclass
class T:
    """A planned tensor (per-replica batch)."""

    shape: tuple
    dtype: torch.dtype = torch.bfloat16
    buf: Optional[torch.Tensor] = None
    grad: Optional[torch.Tensor] = None
    needs_grad: bool = True
    alias_of: Optional["T"] = None
    consumers: List["Node"] = field(default_factory=list)
    written: bool = False  # backward bookkeeping

    def root(self):
        t = self
        while t.alias_of is not None:
            t = t.alias_of
        return t


@dataclass
class Node:
    kind: str
    layer: object
    inputs: List[T]
    out: T
    attrs: Dict = field(default_factory=dict)


def _layer_graph(model):
    """[(layer, [input keys], output key)], input key, output key."""
    from ..keras import layers as L

    if hasattr(model, "_layers") and not getattr(model, "_nodes", None):
        ls = [l for l in model._layers if not isinstance(l, L.InputLayer)]
        seq = []
        for i, l in enumerate(ls):
            seq.append((l, [i], i + 1))
        return seq, 0, len(ls), tuple(model.input_shape[1:])
    keys = {id(model._inputs[0]): 0}
    seq = []
    for t in model._nodes:
        keys[id(t)] = len(keys)
        seq.append((t.layer, [keys[id(i)] for i in t.inputs], keys[id(t)]))
    return seq, 0, keys[id(model._outputs[0])], tuple(model._inputs[0].shape[1:])


def _act_name(layer) -> str:
    act = getattr(layer, "activation", None)
    return getattr(act, "__name__", "linear") if act is not None else "linear"


def _param_weights(model):
    """Every layer weight the forward plan reads (kernels, biases, BN gamma / beta),
    trainable or frozen -- i.e. all weights except the BN moving statistics."""
    out = []
    for l in model.layers:
        stats = {id(getattr(l, "moving_mean", None)), id(getattr(l, "moving_variance", None))}
        out += [w for w in l.weights if id(w) not in stats]
    return out


def _opt_kernel_slots(opt):
    """(opt_step kind, slot names for S0..S2; '' = unused) of a Keras optimizer."""
    from ..keras import optimizers

    if isinstance(opt, optimizers.Adam):
        return 1, ["m", "v", "vhat" if opt.amsgrad else ""]
    if isinstance(opt, optimizers.RMSprop):
        return 2, ["rms", "momentum" if opt.momentum else "", "mg" if opt.centered else ""]
    return 0, ["momentum" if opt.momentum else "", "", ""]


class NativeGraphEngine(Engine):
    name = "native_graph"

    SUPPORTED = ("Conv2D", "BatchNormalization", "Activation", "ReLU", "Add", "MaxPooling2D",
                 "AveragePooling2D", "GlobalAveragePooling2D", "Flatten", "Dense", "Dropout")
    ACTIVATIONS = ("linear", "relu", "sigmoid", "tanh")
    _weights_static = False  # True for an inference plan: padded weight copies made once per call
    # DAMD_BN_FIN (default on): BatchNorm statistics through int64 fixed-point accumulators
    # (order-independent: bitwise the same sums whatever order the producer blocks arrive in) finalized
    # inside the consumer kernels (ops/hip.py BNFin): 40 fewer launches per ResNet-18 step.
    # Same-address fp64 atomics serialise at the memory side (~18 ns each: with one
    # accumulator bn_bwd_reduce took 8.6 -> 26 us, the step 3.02 ms), so the producers add
    # into DAMD_BN_REPS (8) replicas (block b -> replica b % 8) that the consumers sum in
    # order: 2.665 vs 2.712 ms/step with the partials + finalize launches (DAMD_BN_FIN=0).
    _bn_fin = True

    @staticmethod
    def eligible(model, strategy):
        from ..keras import losses, optimizers

        if strategy.device.type != "cuda":
            return False, "not on a GPU"
        if type(model.optimizer) not in (optimizers.SGD, optimizers.Adam, optimizers.RMSprop):
            return False, f"optimizer {type(model.optimizer).__name__}"
        if not (isinstance(model.loss, losses.SparseCategoricalCrossentropy) and model.loss.from_logits):
            return False, "loss"
        for m in model.compiled_metrics:
            if m.name not in ("accuracy", "acc", "sparse_categorical_accuracy"):
                return False, f"metric {m.name}"
        # the training plan keeps one flat buffer of trainable weights: a frozen kernel /
        # bias / gamma / beta (layer.trainable = False) trains on the generic path
        trainable = {id(w) for w in model.trainable_weights}
        if any(id(w) not in trainable for w in _param_weights(model)):
            return False, "frozen layer weights"
        return NativeGraphEngine.layers_eligible(model)

    @staticmethod
    def layers_eligible(model):
        """(ok, reason): every layer of ``model`` has a native forward + backward kernel
        and the model ends in a linear Dense (the logits)."""
        try:
            seq, _, out_key, in_shape = _layer_graph(model)
        except Exception as e:  # pragma: no cover
            return False, f"graph: {e}"
        if len(in_shape) != 3:
            return False, "input must be an image (H, W, C)"
        for l, ins, _ in seq:
            k = type(l).__name__
            if k not in NativeGraphEngine.SUPPORTED:
                return False, f"layer {k}"
            act = getattr(l, "activation", None)
            an = getattr(act, "__name__", "linear") if act is not None else "linear"
            if k in ("Conv2D", "Dense", "Activation") and an not in NativeGraphEngine.ACTIVATIONS:
                return False, f"activation {an}"
            if k == "ReLU" and (l.max_value is not None or l.negative_slope or l.threshold):
                return False, "ReLU options"
            if k == "Conv2D":
                if l.dilation_rate != (1, 1) or l.kernel_size[0] != l.kernel_size[1] or l.strides[0] != l.strides[1]:
                    return False, "conv geometry"
                if l.strides[0] not in (1, 2) or l.filters % 8:
                    return False, "conv stride/filters"
            if k == "MaxPooling2D" and l.pool_size[0] * l.pool_size[1] > 255:
                return False, "pool size"
            if k == "Dropout" and not 0.0 <= l.rate < 1.0:
                return False, "dropout rate"
            if k == "BatchNormalization" and l.axis not in (-1, 3):
                return False, "BN axis"
            if k == "Add" and len(ins) != 2:
                return False, "Add arity"
            if k == "Dense" and l is not seq[-1][0] and l.units % 8:
                return False, "hidden Dense units must be a multiple of 8"
        last = seq[-1][0]
        if type(last).__name__ != "Dense" or getattr(last.activation, "__name__", "") != "linear":
            return False, "the model must end in a linear Dense (logits)"
        return True, ""

    # ------------------------------------------------------------------------------------
    def __init__(self, model, strategy, per_replica_batch, global_batch):
        super().__init__(model, strategy, per_replica_batch, global_batch)
        from ..native import require_C

        self.C = require_C()
        dev = self.device
        self.B = B = per_replica_batch
        # flat fp32 master buffer P (Keras trainable-weight order), bf16 shadow, grads, momentum
        # every variable starts on an 8-element boundary: 16-byte aligned bf16 / 32-byte
        # aligned fp32 views for the kernels' vector accesses
        self.vars = model.trainable_weights
        self.sizes = [int(np.prod(v.shape)) for v in self.vars]
        offs, off = [], 0
        for sz in self.sizes:
            offs.append(off)
            off = _pad8(off + sz)
        self.nparam = n = off
        self.P = torch.zeros(n, dtype=torch.float32, device=dev)
        self.Pb = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        self.G = torch.zeros(n + 8, dtype=torch.float32, device=dev)  # + metric tail
        # optimizer slots (flat, same padded layout as P): SGD momentum; Adam m, v, vhat;
        # RMSprop rms, momentum, mean gradient -- S0..S2 of the opt_step kernel
        kind, names = _opt_kernel_slots(model.optimizer)
        self.opt_kind, self.slot_kernel_names = kind, names
        self.S = {nm: torch.zeros(n, dtype=torch.float32, device=dev) for nm in names if nm}
        self._slot_dummy = torch.zeros(8, dtype=torch.float32, device=dev)
        self.V = self.S.get("momentum", self._slot_dummy)
        self.views, self.bviews, self.gviews = {}, {}, {}
        self.offsets = offs
        for v, sz, off in zip(self.vars, self.sizes, offs):
            v._rebind(self.P[off:off + sz].view(v.shape))
            self.views[id(v)] = self.P[off:off + sz].view(v.shape)
            self.bviews[id(v)] = self.Pb[off:off + sz].view(v.shape)
            self.gviews[id(v)] = self.G[off:off + sz].view(v.shape)
        self._own_variables(self.vars)
        # non-trainable (BN moving statistics) live on the device as fp32
        for w in model.non_trainable_weights:
            if w.value.device != dev:
                w._rebind(torch.zeros(w.shape, dtype=torch.float32, device=dev))
        opt = model.optimizer
        self._load_momentum()
        if self.world > 1:
            comm = strategy.communicator
            comm.broadcast_(self.P, 0)
            for w in model.non_trainable_weights:
                comm.broadcast_(w.value, 0)
        H.cast_bf16(self.P, self.Pb)
        self.ctrl = torch.zeros(32, dtype=torch.int32, device=dev)
        c = self.ctrl.cpu()
        c[C_IT] = int(opt.iterations)
        self.ctrl.copy_(c.to(dev))
        self._write_hparams()
        force = env.get_bool("DAMD_FORCE_ALLREDUCE", False)  # exercise the RCCL path at world 1
        self.native_comm = strategy.communicator.native if (self.world > 1 or force) else None
        self.peer = None  # native xGMI peer all-reduce as the bucket transport (set below)
        # DAMD_GRAD_DTYPE=bf16: the RCCL buckets carry bf16 gradients (half the ring traffic;
        # the metric tail stays fp32, the master update fp32); default fp32 (reference parity)
        self.grad_bf16 = env.get_str("DAMD_GRAD_DTYPE", "fp32").lower() == "bf16"
        self.graph = None
        self._phase_events = None  # phase_times(): (name, event) marks of an eager step
        self.feed = None
        self._plan()
        self._plan_buckets(env.get_float("DAMD_BUCKET_MB", 8.0), env.get_float("DAMD_BUCKET_LAST_MB", 1.0))
        # bucket transport at world > 1 (DAMD_ALLREDUCE): RCCL (auto, when the RCCL
        # communicator exists), or the native xGMI peer all-reduce over IPC-mapped staging
        # (xgmi; auto without RCCL, e.g. ranks sharing one GPU in a rehearsal) -- both on the
        # side stream, overlapped with the rest of backward, inside the captured step
        mode = env.get_str("DAMD_ALLREDUCE", "auto").lower()
        if self.world > 1 and (mode == "xgmi" or (mode == "auto" and self.native_comm is None)):
            from ..parallel.communicator import make_peer_allreduce

            from ..utils.watchdog import deadline_for

            wd = deadline_for(self.world)  # in-kernel wait deadline = the watchdog's
            # one peer all-reduce (own IPC-mapped staging, own epochs) PER BUCKET, each on its
            # own side stream: the buckets' all-reduces then need no order among themselves, so
            # in the captured graph each depends on the backward kernels that wrote its bucket
            # only.  (One staging for all = a chain of all-reduce nodes, each with two parents
            # -- the previous all-reduce and the backward -- which the HIP graph executor ran in
            # line with the backward: profiles/r04_resnet18_dp, scripts/probe_graph_branches.py)
            self.peers = []
            for b in self._buckets:
                p = make_peer_allreduce(strategy.communicator, dev.index or 0, b["hi"] - b["lo"],
                                        blocks=env.get_int("DAMD_PEER_BLOCKS", 64), timeout_s=wd if wd > 0 else 60.0)
                if p is None:
                    self.peers = []
                    break
                self.peers.append(p)
            self.peer = self.peers[0] if self.peers else None
            if self.peer is None and mode == "xgmi":
                raise RuntimeError("DAMD_ALLREDUCE=xgmi but the xGMI peer mapping is unavailable")
        if self.peer is not None and self.grad_bf16:
            dlog.warning("DAMD_GRAD_DTYPE=bf16 applies to the RCCL buckets; the peer transport reduces fp32")
            self.grad_bf16 = False
        # RCCL buckets: one communicator PER BUCKET (a unique id each, exchanged over the gloo
        # control plane), each on its own stream.  Collectives on ONE communicator must run
        # in issue order, so a shared communicator forces the captured graph into a chain --
        # each all-reduce node waiting on the previous one AND on its backward -- which the
        # graph executor serialised with the backward (profiles/r05_graph_branches: no
        # overlap for the last buckets).  With a communicator per bucket every all-reduce
        # node depends only on the backward work that wrote its bucket.  DAMD_BUCKET_COMMS=0:
        # the single shared communicator and one comm stream (the round-5 chain).
        self.bucket_comms = []
        if (self.native_comm is not None and self.peer is None and len(self._buckets) > 1
                and env.get_bool("DAMD_BUCKET_COMMS", True)):
            comm = strategy.communicator
            uids = [self.C.rccl_unique_id() for _ in self._buckets] if self.rank == 0 else None
            if self.world > 1:
                uids = comm.broadcast_object(uids, 0)
            self.bucket_comms = [self.C.RcclComm(self.world, self.rank, u, dev.index or 0) for u in uids]
        self.host_collective = self.world > 1 and self.native_comm is None and self.peer is None
        self.allreduce_kind = ("none" if self.native_comm is None and self.peer is None else
                               "xgmi-peer-bucketed" if self.peer is not None else
                               "rccl-bucketed-bf16" if self.grad_bf16 else "rccl-bucketed")
        if self.host_collective:
            self.allreduce_kind = "host-gloo"
        self.use_graph = env.get_bool("DAMD_GRAPH", True) and not self.host_collective
        self.g16 = (torch.zeros(self.nparam, dtype=torch.bfloat16, device=dev)
                    if self.grad_bf16 and self.native_comm is not None else None)
        # created up front: no stream creation while a graph is being captured.  One stream
        # per bucket (peer staging or RCCL communicator per bucket); a single comm stream
        # when all buckets share one RCCL communicator (its collectives stay in order)
        per_bucket = self.peer is not None or bool(self.bucket_comms)
        self._comm_stream = (torch.cuda.Stream(dev) if (self.native_comm is not None or self.peer is not None)
                             else None)
        self._comm_streams = [torch.cuda.Stream(dev) for _ in self._buckets] if per_bucket else []
        # the SGD / Adam / RMSprop update of a bucket's variables runs right behind the
        # bucket's all-reduce on its own stream (it overlaps the rest of backward, and only
        # the update of the LAST bucket trails the step; DAMD_BUCKET_OPT=0: one optimizer
        # launch after the join).  The bucket holding the metric tail also does the step's
        # bookkeeping (metric fold, cursor, iterations).
        # (world 1, no all-reduce: off by default -- the 4096-block update launches on side
        # streams took CUs from the backward kernels, measured +170 us per ResNet-18 step;
        # the persistent direct convs need every CU)
        reduce = self.native_comm is not None or self.peer is not None
        self.bucket_opt = (env.get_bool("DAMD_BUCKET_OPT", reduce) and not self.host_collective
                           and len(self._buckets) > 1)
        if self.bucket_opt and not self._comm_streams:
            self._comm_streams = [torch.cuda.Stream(dev) for _ in self._buckets]
        # convolution weight gradients on a side stream (DAMD_WGRAD_STREAM): a conv's
        # weight gradient and its backprop-input read the same dy and are independent, so
        # the weight-gradient kernel (+ its split-K reduce) runs beside the backprop-input /
        # BatchNorm-backward chain of the main stream (own workspace); joined before the
        # optimizer, and every bucket all-reduce waits for it
        self._wgrad_stream = torch.cuda.Stream(dev) if env.get_bool("DAMD_WGRAD_STREAM", False) else None
        self.gemm_ws_w = torch.zeros_like(self.gemm_ws) if self._wgrad_stream is not None else None
        self._wgrad_side_minc = env.get_int("DAMD_WGRAD_STREAM_MINC", 0)  # convs with fewer outputs stay inline
        for k, b in enumerate(self._buckets):
            b["k"] = k
        opt._iter_source = self._iterations
        torch.cuda.synchronize(dev)
        dlog.info("native graph engine: %d nodes, %d params, %.1f MB planned activations", len(self.nodes), n,
                  self.act_bytes / 2**20)

    # --- planning --------------------------------------------------------------------------
    def _plan(self):
        self._build()
        self._allocate()

    @classmethod
    def plan_only(cls, model, batch: int):
        """The fused plan of ``model`` at per-replica batch ``batch`` without touching a
        device (planner inspection / CPU tests)."""
        self = cls.__new__(cls)
        self.model, self.B = model, batch
        self._build()
        return self

    def describe_plan(self) -> dict:
        live = [nd for nd in self.nodes if not nd.attrs.get("dead")]
        return {
            "nodes": len(self.nodes),
            "kernels_fwd": len(live),
            "conv_bn_stats": sum(1 for nd in self.nodes if nd.attrs.get("stats")),
            "bn_relu": sum(1 for nd in self.nodes if nd.kind == "BatchNormalization" and nd.attrs.get("relu")),
            "add_fused_raw": sum(1 for nd in self.nodes if nd.attrs.get("fused") and nd.attrs["fused"][1][0] == "raw"),
            "add_fused_bn": sum(1 for nd in self.nodes if nd.attrs.get("fused") and nd.attrs["fused"][1][0] == "bn"),
            "add_relu": sum(1 for nd in self.nodes if nd.kind == "Add" and nd.attrs.get("relu")),
            "dead": sum(1 for nd in self.nodes if nd.attrs.get("dead")),
        }

    def _build(self):
        model, B = self.model, self.B
        seq, in_key, out_key, in_shape = _layer_graph(model)
        tensors: Dict[int, T] = {}
        h, w, c = in_shape
        self.in_shape = (h, w, c)
        self.cin_pad = _pad8(c)
        x0 = T((B, h, w, self.cin_pad), needs_grad=False)
        tensors[in_key] = x0
        self.x0 = x0
        nodes = []
        for layer, ins, ok in seq:
            kind = type(layer).__name__
            xs = [tensors[i] for i in ins]
            shp = self._out_shape(kind, layer, xs)
            out = T(shp)
            nd = Node(kind, layer, xs, out)
            for x in xs:
                x.consumers.append(nd)
            tensors[ok] = out
            nodes.append(nd)
        self.logits_t = tensors[out_key]
        self.nodes = nodes
        # packed-tap stem: a <= 4-channel input read only by stride-2 convs of <= 8 columns
        # is stored with 4 channels and those convs run K = KH x 32 (ops/hip.py stem4_ok)
        if c <= 4 and x0.consumers and env.get_bool("DAMD_STEM4", True) and all(
                nd.kind == "Conv2D" and H.stem4_ok((B, h, w, 4), (nd.layer.kernel.shape[0], nd.layer.kernel.shape[1],
                                                                  4, nd.layer.kernel.shape[3]),
                                                    nd.layer.strides, nd.layer.padding)
                for nd in x0.consumers):
            self.cin_pad = 4
            x0.shape = (B, h, w, 4)
        self._fuse()

    def _out_shape(self, kind, l, xs):
        x = xs[0].shape
        B = self.B
        if kind == "Conv2D":
            ho, _ = H.conv_out(x[1], l.kernel_size[0], l.strides[0], l.padding)
            wo, _ = H.conv_out(x[2], l.kernel_size[1], l.strides[1], l.padding)
            return (B, ho, wo, l.filters)
        if kind in ("MaxPooling2D", "AveragePooling2D"):
            g = H.pool_geo(x, l.pool_size, l.strides, l.padding)
            return (B, g[10], g[11], x[3])
        if kind == "GlobalAveragePooling2D":
            return (B, x[3])
        if kind == "Flatten":
            return (B, int(np.prod(x[1:])))
        if kind == "Dense":
            return (B, l.units)
        return x

    def _fuse(self):
        def relu_node(nd):
            if nd.kind == "ReLU":
                return True
            return nd.kind == "Activation" and getattr(nd.layer.activation, "__name__", "") == "relu"

        for i, nd in enumerate(self.nodes):
            nd.attrs.setdefault("dead", False)
            if nd.kind == "Activation" and _act_name(nd.layer) == "linear":
                nd.attrs["dead"] = True  # linear activation: identity
                self._alias(nd.out, nd.inputs[0])
            if nd.kind == "Dropout":
                if nd.layer.rate == 0.0:
                    nd.attrs["dead"] = True
                    self._alias(nd.out, nd.inputs[0])
                # per-layer, per-replica mask stream (TF draws independent masks per replica)
                s0 = nd.layer.seed if getattr(nd.layer, "seed", None) is not None else 0x5EED
                nd.attrs["seed"] = (int(s0) * 0x9E3779B1 + (i + 1) * 0x85EBCA77
                                    + getattr(self, "rank", 0) * 0xC2B2AE3D) & 0xFFFFFFFF
            if nd.kind == "Flatten":
                nd.attrs["dead"] = True  # NHWC flatten is a view
                self._alias(nd.out, nd.inputs[0])
        for nd in self.nodes:
            if nd.kind != "BatchNormalization":
                continue
            x = nd.inputs[0]
            prod = self._producer(x)
            if (prod is not None and prod.kind == "Conv2D" and not prod.layer.use_bias
                    and getattr(prod.layer.activation, "__name__", "linear") == "linear" and len(x.consumers) == 1):
                prod.attrs["stats"] = True
                nd.attrs["stats_from_conv"] = True
        for nd in self.nodes:
            if nd.kind != "BatchNormalization" or nd.attrs.get("stats_only"):
                continue
            y = nd.out
            if len(y.consumers) == 1 and y.consumers[0].kind == "Add":
                # BN -> Add(other) [-> ReLU]: one pass at the Add's position (after both branches)
                add = y.consumers[0]
                other = add.inputs[1] if add.inputs[0] is y else add.inputs[0]
                op = self._producer(other)
                nd.attrs["stats_only"] = True
                if (op is not None and op.kind == "BatchNormalization" and len(other.consumers) == 1
                        and not op.attrs.get("stats_only")):
                    op.attrs["stats_only"] = True
                    add.attrs["fused"] = (nd, ("bn", op))
                else:
                    add.attrs["fused"] = (nd, ("raw", other))
                out = add.out
                if len(out.consumers) == 1 and relu_node(out.consumers[0]):
                    r = out.consumers[0]
                    add.attrs["relu"] = True
                    r.attrs["dead"] = True
                    self._alias(r.out, out)
                continue
            if len(y.consumers) == 1 and relu_node(y.consumers[0]):
                r = y.consumers[0]
                nd.attrs["relu"] = True
                r.attrs["dead"] = True
                self._alias(r.out, y)
                # BN -> ReLU -> MaxPool (the ResNet stem): the pool normalises on the fly and
                # the BN+ReLU output is never stored (layer_ops.hip stem fusion)
                outs = r.out.consumers
                if (len(outs) == 1 and outs[0].kind == "MaxPooling2D"
                        and env.get_bool("DAMD_STEM_FUSE", True)):
                    nd.attrs["pool"] = outs[0]
                    outs[0].attrs["bn"] = nd

    def _producer(self, t):
        for nd in self.nodes:
            if nd.out is t:
                return nd
        return None

    @staticmethod
    def _alias(t, target):
        t.alias_of = target

    def _allocate(self):
        dev = self.device
        nbytes = 0

        def alloc(t: T, dtype=torch.bfloat16):
            nonlocal nbytes
            if t.alias_of is not None:
                return
            t.buf = torch.zeros(t.shape, dtype=dtype, device=dev)
            t.dtype = dtype
            nbytes += t.buf.numel() * t.buf.element_size()
            if t.needs_grad:
                t.grad = torch.zeros(t.shape, dtype=torch.bfloat16, device=dev)
                nbytes += t.grad.numel() * 2

        alloc(self.x0)
        self.labels = torch.zeros(self.B, dtype=torch.int32, device=dev)
        last = self.nodes[-1]
        for nd in self.nodes:
            if nd is last or nd.attrs.get("pool") is not None:  # stem-fused BN: no output tensor
                continue
            alloc(nd.out)
        # logits: fp32, row pitch padded to 8
        K = last.layer.units
        self.K, self.Kp = K, _pad8(K)
        self.logits = torch.zeros(self.B, self.Kp, dtype=torch.float32, device=dev)
        self.dlogits = torch.zeros(self.B, self.Kp, dtype=torch.bfloat16, device=dev)
        self.xent_rows = H.xent_rows(self.B, dev)  # fixed-order loss / metric sums
        last.attrs["logits"] = True
        # per-node scratch
        self.st_ident = torch.cat([torch.zeros(1, 1), torch.ones(1, 1), torch.ones(1, 1), torch.zeros(1, 1)])
        self._ident_cache = {}
        maxM_C = 0
        ws = 0  # fp32 split-K slabs, shared by every split GEMM (they run in order on one stream)
        for nd in self.nodes:
            if nd.attrs.get("dead"):
                continue
            k = nd.kind
            if k == "Conv2D":
                l = nd.layer
                cin = nd.inputs[0].root().shape[3]
                kh, kw, cin0, cout = l.kernel.shape
                ws = max(ws, H.conv_wgrad_workspace_elems(nd.inputs[0].root().shape, (kh, kw, cin, cout), l.strides,
                                                          l.padding))
                nd.attrs["cin_pad"] = cin
                if cin == 4 and H.stem4_ok(nd.inputs[0].root().shape, (kh, kw, 4, cout), l.strides, l.padding):
                    wsh = H.stem4_weight_shape((kh, kw, 4, cout))
                    nd.attrs["stem4"] = True
                    nd.attrs["w_pad"] = torch.zeros(wsh, dtype=torch.bfloat16, device=dev)
                    nd.attrs["dw_pad"] = torch.zeros(wsh, dtype=torch.float32, device=dev)
                elif cin != cin0:
                    nd.attrs["w_pad"] = torch.zeros(kh, kw, cin, cout, dtype=torch.bfloat16, device=dev)
                    nd.attrs["dw_pad"] = torch.zeros(kh, kw, cin, cout, dtype=torch.float32, device=dev)
                xshape, wshape = nd.inputs[0].root().shape, (kh, kw, cin, cout)
                fplan = H.conv_fwd_plan(xshape, wshape, l.strides, l.padding)
                ws = max(ws, fplan["ws"], H.conv_dgrad_plan(xshape, wshape, l.strides, l.padding)["ws"])
                if nd.attrs.get("stats"):
                    nd.attrs["stats_buf"] = torch.zeros(fplan["stats_T"], 2, cout, device=dev)
                if l.use_bias:  # bias gradient = column sums of dy, fixed order
                    ws = max(ws, H.colsum_workspace_elems(int(np.prod(nd.out.shape[:-1])), cout))
                if _act_name(l) != "linear":
                    nd.attrs["dz"] = torch.zeros(nd.out.shape, dtype=torch.bfloat16, device=dev)
            elif k == "BatchNormalization":
                C = nd.out.shape[-1]
                M = int(np.prod(nd.out.shape[:-1]))
                nd.attrs["st"] = torch.zeros(4, C, device=dev)
                T_ = self.C.bn_bwd_blocks(M, C)
                nd.attrs["T"] = T_
                nd.attrs["part"] = torch.zeros(max(T_, 1), 2, C, device=dev)
                nd.attrs["co"] = torch.zeros(3, C, device=dev)
                maxM_C = max(maxM_C, M * C)
            elif k == "MaxPooling2D":
                nd.attrs["arg"] = torch.zeros(nd.out.shape, dtype=torch.uint8, device=dev)
            elif k == "Dense":
                l = nd.layer
                kin, units = l.kernel.shape
                ws = max(ws, H.wgrad_workspace_elems(kin, _pad8(units), self.B),
                         H.dense_workspace_elems(self.B, _pad8(units), kin),
                         H.colsum_workspace_elems(self.B, units))
                if nd.attrs.get("logits") and units % 8:
                    up = _pad8(units)
                    nd.attrs["w_pad"] = torch.zeros(kin, up, dtype=torch.bfloat16, device=dev)
                    nd.attrs["dw_pad"] = torch.zeros(kin, up, dtype=torch.float32, device=dev)
                    if l.use_bias:
                        nd.attrs["b_pad"] = torch.zeros(up, dtype=torch.float32, device=dev)
                if _act_name(l) != "linear":
                    nd.attrs["dz"] = torch.zeros(nd.out.shape, dtype=torch.bfloat16, device=dev)
        self._plan_bn_fin()
        self._plan_bn_dgrad_fusion()
        self._plan_bn_conv_fold()
        # one scratch bf16 buffer for "second writer" gradient accumulation
        big = max([int(np.prod(t.shape)) for t in self._all_tensors()] + [1])
        self.scratch = torch.zeros(big, dtype=torch.bfloat16, device=dev)
        self.scratch2 = torch.zeros(big, dtype=torch.bfloat16, device=dev)
        nbytes += big * 4
        self.gemm_ws = torch.zeros(max(ws, 4), dtype=torch.float32, device=dev)
        nbytes += self.gemm_ws.numel() * 4
        self.act_bytes = nbytes

    def _plan_bn_fin(self):
        """Fixed-point statistics accumulators of every BatchNorm ([2][C] forward sums, [2][C]
        backward sums) in one buffer, cleared by the step's gather_batch launch; the conv
        producing a BN input accumulates into it from its epilogue."""
        bns = [nd for nd in self.nodes if nd.kind == "BatchNormalization" and not nd.attrs.get("dead")]
        use = (self._bn_fin and env.get_bool("DAMD_BN_FIN", True)
               and all(nd.out.shape[-1] <= H.FIN_MAX_C for nd in bns))
        self.bn_acc = None
        if not use or not bns:
            return
        R = max(1, env.get_int("DAMD_BN_REPS", 8))
        # int64 fixed point (ops/hip.py bn_acc_encode): forward [R][2C] one word per value,
        # backward [R][4C] two words per value, each followed by its sticky flag plane
        # (damd_common.h bnacc_flag)
        tot = sum(6 * (R + 1) * nd.out.shape[-1] for nd in bns)
        self.bn_acc = torch.zeros(tot, dtype=torch.int64, device=self.device)
        o = 0
        for nd in bns:
            C = nd.out.shape[-1]
            nf, nb = 2 * C * (R + 1), 4 * C * (R + 1)
            nd.attrs["acc_f"] = self.bn_acc[o:o + nf].view(R + 1, 2 * C)
            nd.attrs["acc_b"] = self.bn_acc[o + nf:o + nf + nb].view(R + 1, 4 * C)
            o += nf + nb
            if nd.attrs.get("stats_from_conv"):
                self._producer(nd.inputs[0]).attrs["stats_buf"] = nd.attrs["acc_f"]
            l = nd.layer
            M = int(np.prod(nd.inputs[0].shape[:-1]))
            nd.attrs["fin"] = H.BNFin(nd.attrs["acc_f"], self._view_or_none(l.gamma), self._view_or_none(l.beta),
                                      nd.attrs["st"], l.moving_mean.value, l.moving_variance.value, M, l.epsilon,
                                      l.momentum)

    def _plan_bn_dgrad_fusion(self):
        """BN -> ReLU -> Conv2D with the conv as the ReLU output's only consumer (the first
        conv of every ResNet basic block's second half): the conv's backprop-input, when the
        direct 3x3 kernel runs it, also writes the BN-backward partials in its epilogue
        (E_BNRED), so that BN's backward skips its reduce pass (one read of dy and x less)."""
        if not env.get_bool("DAMD_BN_DGRAD_FUSE", True) or not env.get_bool("DAMD_BN_MASK_FROM_X", True):
            return
        for bn in self.nodes:
            a = bn.attrs
            if (bn.kind != "BatchNormalization" or a.get("dead") or not a.get("relu") or a.get("stats_only")
                    or a.get("pool") is not None):
                continue
            outs = bn.out.consumers
            if len(outs) != 1 or not outs[0].attrs.get("dead") or len(outs[0].out.consumers) != 1:
                continue
            conv = outs[0].out.consumers[0]
            if conv.kind != "Conv2D" or conv.attrs.get("dead") or "w_pad" in conv.attrs:
                continue
            l = conv.layer
            plan = H.conv_dgrad_plan(bn.out.shape, tuple(l.kernel.shape), l.strides, l.padding)
            if plan["amode"] != H.A_DGRAD3:
                continue
            # with the in-consumer finalize the epilogue adds into the fixed-point accumulator
            a["dgrad_part"] = (a["acc_b"] if a.get("fin") is not None else
                               torch.zeros(plan["stats_T"], 2, bn.out.shape[-1], device=self.device))
            conv.attrs["bnred"] = bn

    def _plan_bn_conv_fold(self):
        """BN -> ReLU -> Conv2D with the conv as the ReLU output's only consumer and a direct
        3x3 forward plan (the second conv of every ResNet basic block on layers 1-3): the conv
        reads the BN INPUT, finalizes the statistics and applies BN + ReLU to its staged halo
        in LDS, and stores y for the weight gradient -- the bn_apply launch (a read of x and a
        write of y) disappears.  Needs the in-consumer finalize (bn_acc).  DAMD_BN_CONV_FOLD=0
        keeps the apply launch."""
        if self.bn_acc is None or not env.get_bool("DAMD_BN_CONV_FOLD", True):
            return
        for bn in self.nodes:
            a = bn.attrs
            if (bn.kind != "BatchNormalization" or a.get("dead") or not a.get("relu") or a.get("stats_only")
                    or a.get("pool") is not None or a.get("fin") is None or not a.get("stats_from_conv")):
                continue
            outs = bn.out.consumers
            if len(outs) != 1 or not outs[0].attrs.get("dead") or len(outs[0].out.consumers) != 1:
                continue
            conv = outs[0].out.consumers[0]
            if (conv.kind != "Conv2D" or conv.attrs.get("dead") or "w_pad" in conv.attrs or conv.attrs.get("stem4")
                    or conv.inputs[0].root() is not bn.out.root()):
                continue
            l = conv.layer
            plan = H.conv_fwd_plan(tuple(bn.out.shape), tuple(l.kernel.shape), l.strides, l.padding)
            if plan["amode"] != H.A_CONV3 or plan["splits"] != 1:
                continue
            a["conv_fold"] = conv
            conv.attrs["bnin"] = bn

    def _view_or_none(self, var):
        return self.views[id(var)] if var is not None else None

    # --- gradient buckets (all-reduce overlapped with the rest of backward) ------------------
    def _plan_buckets(self, bucket_mb: float, last_mb: float = 1.0):
        """Contiguous ranges of G, filled from the END of the Keras weight order (backward
        produces the last layers' gradients first); the metric tail rides in the first
        bucket.  A bucket is all-reduced on a side stream as soon as the backward ops that
        write its variables have been enqueued.  The bucket of the FIRST
        layers (written last, its all-reduce trails the whole backward) is cut at
        ``last_mb``, so the exposed tail of the step is one small all-reduce."""
        writers = {}
        for nd in self.nodes:
            if nd.attrs.get("dead"):
                continue
            l = nd.layer
            if nd.kind in ("Conv2D", "Dense"):
                vs = [l.kernel] + ([l.bias] if l.use_bias else [])
                writers[id(nd)] = vs
            elif nd.kind == "BatchNormalization" and not nd.attrs.get("stats_only"):
                writers[id(nd)] = [w for w in (l.gamma, l.beta) if w is not None]
            elif nd.kind == "Add" and nd.attrs.get("fused"):
                main, (mode, other) = nd.attrs["fused"]
                vs = [w for w in (main.layer.gamma, main.layer.beta) if w is not None]
                if mode == "bn":
                    vs += [w for w in (other.layer.gamma, other.layer.beta) if w is not None]
                writers[id(nd)] = vs
        self._writes = {k: [id(v) for v in vs] for k, vs in writers.items()}
        limit = max(1, int(bucket_mb * 2**20 / 4))
        first = []  # the first layers' variables, up to last_mb (reduced last)
        n_first, lim_first = 0, max(1, int(min(last_mb, bucket_mb) * 2**20 / 4))
        for i in range(len(self.vars)):
            if first and n_first + self.sizes[i] > lim_first:
                break
            first.append(i)
            n_first += self.sizes[i]
        order = list(range(len(first), len(self.vars)))[::-1]
        buckets, cur, cur_n = [], [], 0
        for i in order:
            cur.append(i)
            cur_n += self.sizes[i]
            if cur_n >= limit:
                buckets.append(cur)
                cur, cur_n = [], 0
        if cur:
            buckets.append(cur)
        if first:
            buckets.append(first)
        self._buckets = []
        for bi, idxs in enumerate(buckets):
            lo = min(self.offsets[i] for i in idxs)
            hi = max(self.offsets[i] + self.sizes[i] for i in idxs)
            hi = _pad8(hi)
            if bi == 0:
                hi = self.G.numel()  # + metric tail
            self._buckets.append({"lo": lo, "hi": hi, "vars": {id(self.vars[i]) for i in idxs}})
        # buckets must tile G exactly
        spans = sorted((b["lo"], b["hi"]) for b in self._buckets)
        assert spans[0][0] == 0 and all(a[1] == b[0] for a, b in zip(spans, spans[1:])), spans

    def _bucket_begin(self):
        for b in self._buckets:
            b["left"] = set(b["vars"])
            b["sent"] = False

    def _reduce_bucket(self, b, st: int):
        """SUM all-reduce of G[lo:hi] on stream ``st`` by the configured transport."""
        lo, hi = b["lo"], b["hi"]
        gp = self.G.data_ptr()
        comm = self.bucket_comms[b["k"]] if self.bucket_comms else self.native_comm
        if self.peer is not None:
            self.peers[b["k"]].allreduce(gp + 4 * lo, hi - lo, st)
        elif self.g16 is not None:
            n = min(hi, self.nparam) - lo  # the parameter part travels as bf16 ...
            g16 = self.g16.data_ptr() + 2 * lo
            self.C.cast_f32_bf16(gp + 4 * lo, g16, n, st)
            comm.allreduce(g16, g16, n, 1, 0, st)
            self.C.cast_bf16_f32(g16, gp + 4 * lo, n, st)
            if hi > self.nparam:  # ... the metric tail (counts, sums) as fp32
                comm.allreduce(gp + 4 * self.nparam, gp + 4 * self.nparam, hi - self.nparam, 0, 0, st)
        else:
            comm.allreduce(gp + 4 * lo, gp + 4 * lo, hi - lo, 0, 0, st)

    def _bucket_stream(self, b):
        return self._comm_streams[b["k"]] if self._comm_streams else self._comm_stream

    def _bucket_progress(self, nd, final=False):
        reduce = self.native_comm is not None or self.peer is not None
        if not reduce and not self.bucket_opt:
            return
        done = set(self._writes.get(id(nd), ())) if nd is not None else set()
        main = torch.cuda.current_stream(self.device)
        for b in self._buckets:
            if b["sent"]:
                continue
            b["left"] -= done
            if b["left"] and not final:
                continue
            cs = self._bucket_stream(b)
            cs.wait_stream(main)
            if self._wgrad_stream is not None:
                cs.wait_stream(self._wgrad_stream)
            if reduce:
                self._reduce_bucket(b, cs.cuda_stream)
            if self.bucket_opt:
                with torch.cuda.stream(cs):
                    self._optimizer_step(b)
            b["sent"] = True
        if final:
            for cs in (self._comm_streams or [self._comm_stream]):
                main.wait_stream(cs)

    def graph_nodes(self):
        """Structure of one captured step (tests): [(node type, kernel name, [dependency
        indices])] of a fresh capture whose hipGraph is kept (C.graph_nodes)."""
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph(keep_graph=True)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        gc.collect()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                self._step_body()
        torch.cuda.synchronize(self.device)
        nodes = self.C.graph_nodes(g.raw_cuda_graph())
        del g
        return nodes

    def _all_tensors(self):
        out = [self.x0]
        for nd in self.nodes:
            out.append(nd.out)
        return out

    def _ident(self, C):
        t = self._ident_cache.get(C)
        if t is None:
            t = self.st_ident.expand(4, C).contiguous().to(self.device)
            self._ident_cache[C] = t
        return t

    # --- gradient write protocol ----------------------------------------------------------
    def _grad_target(self, t: T):
        """(buffer to write, finish fn) for a producer of t's gradient."""
        r = t.root()
        if not r.needs_grad:
            return None, None
        if not r.written:
            r.written = True
            return r.grad, None
        tmp = self.scratch[: r.grad.numel()].view(r.grad.shape)

        def finish():
            H.add_bf16(r.grad, tmp, r.grad)

        return tmp, finish

    # --- hyper-parameters / ctrl -------------------------------------------------------------
    def _write_hparams(self):
        opt = self.model.optimizer
        c = self.ctrl.cpu()
        c[C_LR] = _f2i(opt.learning_rate)
        c[C_MOM] = _f2i(getattr(opt, "momentum", 0.0))
        c[C_NEST] = int(getattr(opt, "nesterov", False))
        c[C_ROW0] = self.rank * self.per_replica
        c[C_GB] = self.global_batch
        self.ctrl.copy_(c.to(self.device))

    def _ctrl_write(self, updates):
        torch.cuda.synchronize(self.device)
        c = self.ctrl.cpu()
        for k, v in updates.items():
            c[k] = v
        self.ctrl.copy_(c.to(self.device))
        torch.cuda.synchronize(self.device)

    def _iterations(self):
        torch.cuda.synchronize(self.device)
        return int(self.ctrl[C_IT].item())

    def lr_changed(self):
        self._ctrl_write({C_LR: _f2i(self.model.optimizer.learning_rate)})

    def _load_momentum(self):
        # optimizer slots are dense over the unpadded weights (Keras order)
        opt = self.model.optimizer
        tot = int(sum(self.sizes))
        for nm, buf in self.S.items():
            if nm in opt.slots and opt.slots[nm].numel() == tot:
                src = opt.slots[nm].to(self.device)
                o = 0
                for sz, off in zip(self.sizes, self.offsets):
                    buf[off:off + sz].copy_(src[o:o + sz])
                    o += sz

    def reload_optimizer_state(self):
        opt = self.model.optimizer
        torch.cuda.synchronize(self.device)
        self._load_momentum()
        opt._iter_source = None
        it = int(opt.iterations)
        opt._iter_source = self._iterations
        H.cast_bf16(self.P, self.Pb)
        self._ctrl_write({C_IT: it})

    # --- data -------------------------------------------------------------------------------
    def bind(self, x, y):
        x = np.asarray(x)
        h, w, c = self.in_shape
        if tuple(x.shape[1:]) not in ((h, w, c),) and not (c == 1 and tuple(x.shape[1:]) == (h, w)):
            raise ValueError(f"native graph engine expects inputs of shape {(h, w, c)}, got {x.shape[1:]}")
        key = (id(x), id(y), len(x))
        if self.feed is None or getattr(self, "_feed_key", None) != key:
            torch.cuda.synchronize(self.device)
            self.feed = DataFeed(x, y, self.device, flatten=True, allow_u8=env.get_bool("DAMD_X_U8", True))
            self._feed_key = key
            self.x_ep = torch.empty_like(self.feed.x)
            self.y_ep = torch.empty_like(self.feed.y)
            self.graph = None  # data pointers changed
            self._ctrl_write({C_NS: self.feed.n})
        return self.feed

    def start_epoch(self, epoch, shuffle, wrap_steps: int = 0):
        torch.cuda.synchronize(self.device)
        self.feed.set_epoch(epoch, shuffle, self.shuffle_seed)
        perm = self.feed.perm.long()
        torch.index_select(self.feed.x, 0, perm, out=self.x_ep)
        torch.index_select(self.feed.y, 0, perm, out=self.y_ep)
        opt = self.model.optimizer
        self._ctrl_write({C_CUR: 0, C_AL: 0, C_AC: 0, C_AN: 0, C_WRAP: int(wrap_steps),
                          C_LR: _f2i(opt.learning_rate), C_MOM: _f2i(getattr(opt, "momentum", 0.0)),
                          C_NEST: int(getattr(opt, "nesterov", False))})

    # --- the step ----------------------------------------------------------------------------
    def _mark(self, name):
        ev = self._phase_events
        if ev is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ev.append((name, e))

    def _step_body(self):
        C, B = self.C, self.B
        s = H.stream_handle()
        self._mark("start")
        h, w, c = self.in_shape
        # the step's first launch also clears the gradient buffer (and the BN statistics
        # accumulators): no memset launch in the step
        acc = self.bn_acc
        live = [nd for nd in self.nodes if not nd.attrs.get("dead")]
        # the first padded conv's bf16 weight copy (the packed-tap stem) is refreshed inside
        # the gather launch (no pad_cast launch of its own): nothing writes the masters
        # between this launch and that conv
        self._pad_folded = next((nd for nd in live if nd.kind == "Conv2D" and self._pad_job(nd) is not None), None)
        job = self._pad_job(self._pad_folded) if self._pad_folded is not None else None
        C.gather_batch(self.x_ep.data_ptr(), int(self.feed.x_u8), 255.0, self.y_ep.data_ptr(), self.ctrl.data_ptr(),
                       B, h * w, c, self.cin_pad, self.x0.buf.data_ptr(), self.labels.data_ptr(), s,
                       zero=self.G.data_ptr(), zero_bytes=self.G.numel() * 4,
                       zero2=acc.data_ptr() if acc is not None else 0, zero2_bytes=acc.numel() * 8 if acc is not None else 0,
                       pc_src=job[0].data_ptr() if job else 0, pc_dst=job[1].data_ptr() if job else 0,
                       pc_dims=list(job[2:]) if job else [])
        for nd in live:
            getattr(self, "_fwd_" + nd.kind)(nd)
        last = self.nodes[-1]
        # the logits layer's bias gradient comes out of the loss launch (no colsum launch;
        # DAMD_XENT_BIAS=0: the colsum launch, the same bits)
        fold = (last.kind == "Dense" and last.layer.use_bias and "dz" not in last.attrs
                and H.softmax_bias_fold_ok(self.B, self.K) and env.get_bool("DAMD_XENT_BIAS", True))
        last.attrs["bias_folded"] = fold
        H.softmax_xent(self.logits, self.labels, self.K, 1.0 / self.global_batch, self.dlogits, self.G[self.nparam:],
                       ctrl=self.ctrl, rows=self.xent_rows, bias_grad=self.gviews[id(last.layer.bias)] if fold else None)
        self._mark("forward")
        for t in self._all_tensors():
            t.root().written = False
        self._bucket_begin()
        for nd in reversed(live):
            getattr(self, "_bwd_" + nd.kind)(nd)
            self._bucket_progress(nd)
        if self._wgrad_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._wgrad_stream)
        self._mark("backward")
        self._bucket_progress(None, final=True)
        self._mark("allreduce")  # the part of the all-reduce not hidden behind backward
        if not self.host_collective and not self.bucket_opt:
            self._optimizer_step()
        self._mark("optimizer")

    def _optimizer_step(self, b=None):
        """The optimizer update of every parameter (b None), or of bucket b's range only --
        the bucket whose range holds the metric tail also does the step's bookkeeping."""
        opt = self.model.optimizer
        ptr = [self.S[nm].data_ptr() if nm else self._slot_dummy.data_ptr() for nm in self.slot_kernel_names]
        if self.opt_kind == 1:
            args = (float(opt.beta_1), float(opt.beta_2), float(opt.epsilon), 0.0, 0.0, int(opt.amsgrad))
        elif self.opt_kind == 2:
            args = (0.0, 0.0, float(opt.epsilon), float(opt.rho), float(opt.momentum), int(opt.centered))
        else:
            args = (0.0, 0.0, 0.0, 0.0, float(opt.momentum), int(opt.nesterov))
        lo, hi, book = 0, self.nparam, 1
        if b is not None:
            lo, hi = b["lo"], min(b["hi"], self.nparam)
            book = int(b["hi"] > self.nparam)
        # (a slot pointer of an unused slot is the dummy: offset, never dereferenced)
        o4 = 4 * lo
        self.C.opt_step(self.P.data_ptr() + o4, self.G.data_ptr() + o4, ptr[0] + o4, ptr[1] + o4, ptr[2] + o4,
                        self.Pb.data_ptr() + 2 * lo, max(hi - lo, 0), self.ctrl.data_ptr(),
                        self.G[self.nparam:].data_ptr(), self.opt_kind, *args, H.stream_handle(), book=book)

    # forward ops
    def _w(self, nd, var):
        return self.bviews[id(var)]

    def _fwd_Conv2D(self, nd):
        l = nd.layer
        x = nd.inputs[0].root().buf
        wb = self._w(nd, l.kernel)
        bias = self.views[id(l.bias)] if l.use_bias else None
        relu = getattr(l.activation, "__name__", "linear") == "relu"
        if not self._weights_static and nd is not getattr(self, "_pad_folded", None):
            self._pad_weights(nd)
        if nd.attrs.get("stem4"):
            kh = l.kernel.shape[0]
            wp = nd.attrs["w_pad"]
            H.conv_fwd_stem4(x, wp, nd.out.root().buf, kh, l.strides, l.padding, bias=bias, relu=relu,
                             stats=nd.attrs.get("stats_buf"), workspace=self.gemm_ws)
        else:
            if "w_pad" in nd.attrs:
                wb = nd.attrs["w_pad"]
            bn = nd.attrs.get("bnin")
            if bn is not None:  # BN -> ReLU of the input applied on load (_plan_bn_conv_fold)
                H.conv_fwd(bn.inputs[0].root().buf, wb, nd.out.root().buf, l.strides, l.padding, bias=bias,
                           relu=relu, stats=nd.attrs.get("stats_buf"), workspace=self.gemm_ws,
                           bnin=(bn.attrs["fin"], x))
            else:
                H.conv_fwd(x, wb, nd.out.root().buf, l.strides, l.padding, bias=bias, relu=relu,
                           stats=nd.attrs.get("stats_buf"), workspace=self.gemm_ws)
        self._act_epilogue(nd)

    def _pad_job(self, nd):
        """(fp32 master view, padded bf16 copy, R, C1, C2, C1p, C2p) of a padded conv's
        pad_cast, or None."""
        if nd.kind != "Conv2D" or "w_pad" not in nd.attrs:
            return None
        kh, kw, cin, cout = nd.layer.kernel.shape
        src, dst = self.views[id(nd.layer.kernel)], nd.attrs["w_pad"]
        if nd.attrs.get("stem4"):
            # [KH][KW][cin][cout] -> [KH][8][4][cout]: the (cin, cout) rows padded at their tail
            return (src, dst, kh, kw, cin * cout, 8, 4 * cout)
        return (src, dst, kh * kw, cin, cout, nd.attrs["cin_pad"], cout)

    def _pad_weights(self, nd):
        """Refresh a layer's padded bf16 weight copy from the fp32 masters (every training
        step; once per call for an inference plan, whose weights do not move)."""
        l = nd.layer
        if "w_pad" not in nd.attrs:
            return
        if nd.kind == "Conv2D":
            src, dst, *dims = self._pad_job(nd)
            H.pad_cast(src, *dims, dst)
        elif nd.kind == "Dense":
            kin, units = l.kernel.shape
            H.pad_cast(self.views[id(l.kernel)], 1, kin, units, kin, nd.attrs["w_pad"].shape[1], nd.attrs["w_pad"])
            if l.use_bias:
                nd.attrs["b_pad"][:units].copy_(self.views[id(l.bias)])

    def _act_epilogue(self, nd):
        """sigmoid / tanh of a Conv2D / Dense: in place over the GEMM's bf16 output (ReLU
        rides in the GEMM epilogue itself)."""
        an = _act_name(nd.layer)
        if an in ("sigmoid", "tanh"):
            y = nd.out.root().buf
            H.act_fwd(y, y, an)

    def _fwd_BatchNormalization(self, nd):
        l = nd.layer
        x = nd.inputs[0].root()
        C = x.shape[-1]
        M = int(np.prod(x.shape[:-1]))
        st = nd.attrs["st"]
        gamma = self.views[id(l.gamma)] if l.gamma is not None else None
        beta = self.views[id(l.beta)] if l.beta is not None else None
        fin = nd.attrs.get("fin")
        if fin is not None:
            if not nd.attrs.get("stats_from_conv"):  # sum / sum of squares of x into acc_f
                self.C.bn_bwd_reduce_acc(x.buf.data_ptr(), 0, 0, x.buf.data_ptr(), self._ident(C).data_ptr(), 0,
                                         nd.attrs["acc_f"].data_ptr(), nd.attrs["T"], M, C, H.stream_handle(),
                                         H.acc_reps(nd.attrs["acc_f"]))
            if nd.attrs.get("stats_only") or nd.attrs.get("pool") is not None or nd.attrs.get("conv_fold"):
                return  # finalized and applied by the fused Add / MaxPool / direct conv that consumes it
            H.bn_apply_fin(x.buf, nd.out.root().buf, fin, relu=nd.attrs.get("relu", False))
            return
        if nd.attrs.get("stats_from_conv"):
            part = self._producer(x).attrs["stats_buf"]
            Tn = part.shape[0]
        else:
            part, Tn = nd.attrs["part"], nd.attrs["T"]
            ident = self._ident(C)
            self.C.bn_bwd_reduce(x.buf.data_ptr(), 0, 0, x.buf.data_ptr(), ident.data_ptr(), 0, part.data_ptr(), Tn,
                                 M, C, H.stream_handle())
        H.bn_finalize(part, Tn, C, M, gamma, beta, l.epsilon, l.momentum, l.moving_mean.value,
                      l.moving_variance.value, st)
        if nd.attrs.get("stats_only") or nd.attrs.get("pool") is not None:
            return  # applied by the fused Add / MaxPool that consumes it
        H.bn_apply(x.buf, st, nd.out.root().buf, relu=nd.attrs.get("relu", False))

    def _fwd_Activation(self, nd):
        C = nd.out.shape[-1]
        x = nd.inputs[0].root()
        an = _act_name(nd.layer) if nd.kind == "Activation" else "relu"
        if an == "relu" and C % 8 == 0:
            H.bn_apply(x.buf, self._ident(C), nd.out.root().buf, relu=True)
        else:
            H.act_fwd(x.buf, nd.out.root().buf, an)

    def _fwd_Dropout(self, nd):
        H.dropout(nd.inputs[0].root().buf, nd.out.root().buf, self.ctrl, nd.attrs["seed"], nd.layer.rate)

    def _fwd_AveragePooling2D(self, nd):
        l = nd.layer
        H.avgpool_fwd(nd.inputs[0].root().buf, nd.out.root().buf, l.pool_size, l.strides, l.padding)

    _fwd_ReLU = _fwd_Activation

    def _fwd_Add(self, nd):
        fused = nd.attrs.get("fused")
        if fused is None:
            a, b = nd.inputs[0].root().buf, nd.inputs[1].root().buf
            H.add_bf16(a, b, nd.out.root().buf)
            return
        main, (mode, other) = fused
        x = main.inputs[0].root()
        if mode == "raw":
            r, st2 = other.root().buf, None
        else:
            r, st2 = other.inputs[0].root().buf, other.attrs["st"]
        if main.attrs.get("fin") is not None:
            H.bn_apply_fin(x.buf, nd.out.root().buf, main.attrs["fin"], relu=nd.attrs.get("relu", False), r=r,
                           fin2=other.attrs["fin"] if mode == "bn" else None)
            return
        H.bn_apply(x.buf, main.attrs["st"], nd.out.root().buf, relu=nd.attrs.get("relu", False), r=r, st2=st2)

    def _fwd_MaxPooling2D(self, nd):
        l = nd.layer
        bn = nd.attrs.get("bn")
        if bn is not None and bn.attrs.get("fin") is not None:
            H.bn_relu_maxpool_fwd_fin(bn.inputs[0].root().buf, nd.out.root().buf, nd.attrs["arg"], l.pool_size,
                                      l.strides, l.padding, bn.attrs["fin"])
            return
        if bn is not None:  # stem fusion: pool(relu(BN(x))) straight from the conv output
            H.bn_relu_maxpool_fwd(bn.inputs[0].root().buf, bn.attrs["st"], nd.out.root().buf, nd.attrs["arg"],
                                  l.pool_size, l.strides, l.padding)
            return
        H.maxpool_fwd(nd.inputs[0].root().buf, nd.out.root().buf, nd.attrs["arg"], l.pool_size, l.strides, l.padding)

    def _fwd_GlobalAveragePooling2D(self, nd):
        H.gap_fwd(nd.inputs[0].root().buf, nd.out.root().buf)

    def _fwd_Dense(self, nd):
        l = nd.layer
        x = nd.inputs[0].root().buf
        x2 = x.view(x.shape[0], -1)
        wb = self._w(nd, l.kernel)
        bias = self.views[id(l.bias)] if l.use_bias else None
        if not self._weights_static:
            self._pad_weights(nd)
        if "w_pad" in nd.attrs:
            wb = nd.attrs["w_pad"]
            if bias is not None:
                bias = nd.attrs["b_pad"]
        relu = getattr(l.activation, "__name__", "linear") == "relu"
        out = self.logits if nd.attrs.get("logits") else nd.out.root().buf
        H.dense_fwd(x2, wb, out, bias=bias, relu=relu, workspace=self.gemm_ws)
        if not nd.attrs.get("logits"):
            self._act_epilogue(nd)

    # backward ops
    def _dy(self, nd):
        if nd.attrs.get("logits"):
            return self.dlogits
        return nd.out.root().grad

    def _bwd_Conv2D(self, nd):
        l = nd.layer
        xt = nd.inputs[0].root()
        y = nd.out.root()
        dy = y.grad
        if "dz" in nd.attrs:
            self._act_bwd(nd, dy, y.buf, nd.attrs["dz"])
            dy = nd.attrs["dz"]
        side = self._wgrad_stream
        if side is not None and l.kernel.shape[-1] >= self._wgrad_side_minc:
            side.wait_stream(torch.cuda.current_stream(self.device))  # dy and x are final
            with torch.cuda.stream(side):
                self._conv_wgrad(nd, xt, dy, self.gemm_ws_w)
        else:
            self._conv_wgrad(nd, xt, dy, self.gemm_ws)
        if xt.needs_grad:
            wb = nd.attrs.get("w_pad", self._w(nd, l.kernel))
            acc = xt.written
            xt.written = True
            bn = nd.attrs.get("bnred")
            if bn is not None:
                # first (only) writer of the BN -> ReLU output gradient: the BN-backward
                # partials come out of this launch's epilogue
                bn.attrs["dgrad_fused"] = not acc and H.conv_dgrad(
                    dy, wb, xt.grad, l.strides, l.padding, accumulate=acc, workspace=self.gemm_ws,
                    bnred=(bn.inputs[0].root().buf, bn.attrs["st"], bn.attrs["dgrad_part"]))
                if acc:
                    H.conv_dgrad(dy, wb, xt.grad, l.strides, l.padding, accumulate=acc, workspace=self.gemm_ws)
            else:
                H.conv_dgrad(dy, wb, xt.grad, l.strides, l.padding, accumulate=acc, workspace=self.gemm_ws)

    def _conv_wgrad(self, nd, xt, dy, ws):
        """Bias and weight gradient of conv node nd (current stream, workspace ws)."""
        l = nd.layer
        if l.use_bias:
            H.colsum(dy, self.gviews[id(l.bias)], workspace=ws)
        if nd.attrs.get("stem4"):
            kh, kw, cin, cout = l.kernel.shape
            dwp = nd.attrs["dw_pad"]
            # split-K: the reduce adds straight into the gradient view (0 + sum, as
            # unpad_add(reduce) did: the same bits); one split: the atomic GEMM into dw_pad
            if not H.conv_wgrad_stem4(xt.buf, dy, dwp, kh, l.strides, l.padding, workspace=ws, accumulate=False,
                                      dw=self.gviews[id(l.kernel)]):
                H.unpad_add(dwp, kh, kw, cin * cout, 8, 4 * cout, self.gviews[id(l.kernel)])
        elif "dw_pad" in nd.attrs:
            dwp = nd.attrs["dw_pad"]
            H.conv_wgrad(xt.buf, dy, dwp, l.strides, l.padding, workspace=ws, accumulate=False)
            kh, kw, cin, cout = l.kernel.shape
            H.unpad_add(dwp, kh * kw, cin, cout, nd.attrs["cin_pad"], cout, self.gviews[id(l.kernel)])
        else:
            H.conv_wgrad(xt.buf, dy, self.gviews[id(l.kernel)], l.strides, l.padding, workspace=ws)

    def _bn_backward(self, bn, dy, ymask, relu, dz_out=None, mask_from_x=False):
        """BatchNorm backward of node ``bn`` for upstream gradient dy (masked by
        [ymask > 0] when relu); dgamma/dbeta into the gradient sinks, dx into the input's
        gradient; optionally also writes the masked dy to dz_out.  ``mask_from_x``: the
        output is bn_apply(x, relu) with no residual, so the kernels recompute the ReLU
        mask from x (already read) instead of reading the stored output."""
        l = bn.layer
        C_ = self.C
        s = H.stream_handle()
        x = bn.inputs[0].root()
        C = x.shape[-1]
        M = int(np.prod(x.shape[:-1]))
        st, part, co, Tn = bn.attrs["st"], bn.attrs["part"], bn.attrs["co"], bn.attrs["T"]
        ym = ymask.data_ptr() if relu else 0
        mode = (2 if mask_from_x else 1) if relu else 0
        dx, fin = self._grad_target(x)
        fused = bn.attrs.get("dgrad_fused") and mode == 2 and dz_out is None
        if bn.attrs.get("fin") is not None and dx is not None:
            H.bn_bwd_fin(dy, ymask if relu else None, mode, x.buf, st, bn.attrs["acc_b"], co, dx,
                         dgamma=self.gviews[id(l.gamma)] if l.gamma is not None else None,
                         dbeta=self.gviews[id(l.beta)] if l.beta is not None else None,
                         dz_out=dz_out if relu else None, reduce=not fused)
            if fin:
                fin()
            return
        if fused:
            part = bn.attrs["dgrad_part"]  # written by the consuming conv's backprop-input epilogue
            Tn = part.shape[0]
        else:
            C_.bn_bwd_reduce(dy.data_ptr(), ym, mode, x.buf.data_ptr(), st.data_ptr(),
                             dz_out.data_ptr() if (dz_out is not None and relu) else 0, part.data_ptr(), Tn, M, C, s)
        C_.bn_bwd_finalize(part.data_ptr(), Tn, C, float(M), st.data_ptr(), 0,
                           self.gviews[id(l.gamma)].data_ptr() if l.gamma is not None else 0,
                           self.gviews[id(l.beta)].data_ptr() if l.beta is not None else 0, co.data_ptr(), s)
        if dx is not None:
            C_.bn_bwd_apply(dy.data_ptr(), ym, mode, x.buf.data_ptr(), st.data_ptr(), co.data_ptr(),
                            dx.data_ptr(), M, C, s)
            if fin:
                fin()

    def _bwd_BatchNormalization(self, nd):
        if nd.attrs.get("stats_only") or nd.attrs.get("pool") is not None:
            return  # handled by the fused Add / MaxPool
        y = nd.out.root()
        self._bn_backward(nd, y.grad, y.buf, bool(nd.attrs.get("relu")),
                          mask_from_x=env.get_bool("DAMD_BN_MASK_FROM_X", True))

    def _act_bwd(self, nd, dy, y, dx):
        an = _act_name(nd.layer) if nd.kind != "ReLU" else "relu"
        if an == "relu" and dy.numel() % 8 == 0:
            H.relu_bwd(dy, y, dx)
        else:
            H.act_bwd(dy, y, dx, an)

    def _bwd_Activation(self, nd):
        x = nd.inputs[0].root()
        y = nd.out.root()
        dx, fin = self._grad_target(x)
        if dx is not None:
            self._act_bwd(nd, y.grad, y.buf, dx)
            if fin:
                fin()

    def _bwd_Dropout(self, nd):
        x = nd.inputs[0].root()
        dx, fin = self._grad_target(x)
        if dx is not None:
            # the same counter-hash mask and scale as the forward (same seed, same step t)
            H.dropout(nd.out.root().grad, dx, self.ctrl, nd.attrs["seed"], nd.layer.rate)
            if fin:
                fin()

    def _bwd_AveragePooling2D(self, nd):
        l = nd.layer
        x = nd.inputs[0].root()
        dx, fin = self._grad_target(x)
        if dx is not None:
            H.avgpool_bwd(nd.out.root().grad, dx, l.pool_size, l.strides, l.padding)
            if fin:
                fin()

    _bwd_ReLU = _bwd_Activation

    def _bwd_Add(self, nd):
        out = nd.out.root()
        fused = nd.attrs.get("fused")
        if fused is None:
            for x in nd.inputs:
                dx, fin = self._grad_target(x)
                if dx is not None:
                    dx.copy_(out.grad)
                    if fin:
                        fin()
            return
        main, (mode, other) = fused
        relu = bool(nd.attrs.get("relu"))
        dy = out.grad
        M = int(np.prod(out.shape[:-1]))
        C = out.shape[-1]
        if mode == "raw":
            # the residual input's gradient is the (masked) dy itself
            dz, fin = self._grad_target(other)
            if relu:
                self._bn_backward(main, dy, out.buf, True, dz_out=dz)
            else:
                if dz is not None:
                    dz.copy_(dy)
                self._bn_backward(main, dy, out.buf, False)
            if fin:
                fin()
        else:
            # both BN backwards mask dy by [out > 0] themselves (no separate ReLU-backward pass)
            if not self._bn_backward_dual(main, other, dy, out.buf, relu):
                self._bn_backward(main, dy, out.buf, relu)
                self._bn_backward(other, dy, out.buf, relu)

    def _bn_backward_dual(self, b1, b2, dy, ymask, relu):
        """Both BatchNorms of relu(BN(x) + BN(xd)) in one reduce and one apply launch
        (H.bn_bwd_fin_dual) when both finalize in their consumers and own their inputs'
        gradients (DAMD_BN_DUAL=0: four launches)."""
        if not env.get_bool("DAMD_BN_DUAL", True):
            return False
        xs = [b.inputs[0].root() for b in (b1, b2)]
        if (any(b.attrs.get("fin") is None or b.attrs.get("dgrad_fused") for b in (b1, b2))
                or xs[0] is xs[1] or any(x.written or not x.needs_grad for x in xs)
                or xs[0].shape != xs[1].shape or xs[0].shape[-1] % 8 or 256 % (xs[0].shape[-1] // 8)):
            return False
        args = []
        for b, x in zip((b1, b2), xs):
            dx, fin = self._grad_target(x)
            assert fin is None  # first writer (checked above)
            l = b.layer
            args.append({"x": x.buf, "st": b.attrs["st"], "acc": b.attrs["acc_b"], "co": b.attrs["co"], "dx": dx,
                         "dgamma": self.gviews[id(l.gamma)] if l.gamma is not None else None,
                         "dbeta": self.gviews[id(l.beta)] if l.beta is not None else None})
        H.bn_bwd_fin_dual(dy, ymask if relu else None, 1 if relu else 0, args)
        return True

    def _bwd_MaxPooling2D(self, nd):
        l = nd.layer
        bn = nd.attrs.get("bn")
        if bn is not None:  # the whole BN(+ReLU) backward of the fused stem
            x = bn.inputs[0].root()
            bl = bn.layer
            dx, fin = self._grad_target(x)
            if bn.attrs.get("fin") is not None and dx is not None:
                H.pool_bn_bwd_fin(nd.out.root().grad, nd.attrs["arg"], x.buf, bn.attrs["st"], bn.attrs["acc_b"],
                                  bn.attrs["co"], dx, l.pool_size, l.strides, l.padding,
                                  dgamma=self.gviews[id(bl.gamma)] if bl.gamma is not None else None,
                                  dbeta=self.gviews[id(bl.beta)] if bl.beta is not None else None)
                if fin:
                    fin()
                return
            H.pool_bn_bwd(nd.out.root().grad, nd.attrs["arg"], x.buf, bn.attrs["st"], bn.attrs["part"],
                          bn.attrs["co"], dx, l.pool_size, l.strides, l.padding,
                          dgamma=self.gviews[id(bl.gamma)] if bl.gamma is not None else None,
                          dbeta=self.gviews[id(bl.beta)] if bl.beta is not None else None)
            if fin:
                fin()
            return
        x = nd.inputs[0].root()
        dx, fin = self._grad_target(x)
        if dx is not None:
            H.maxpool_bwd(nd.out.root().grad, nd.attrs["arg"], dx, l.pool_size, l.strides, l.padding)
            if fin:
                fin()

    def _bwd_GlobalAveragePooling2D(self, nd):
        x = nd.inputs[0].root()
        dx, fin = self._grad_target(x)
        if dx is not None:
            H.gap_bwd(nd.out.root().grad, dx)
            if fin:
                fin()

    def _bwd_Dense(self, nd):
        l = nd.layer
        xt = nd.inputs[0].root()
        x2 = xt.buf.view(xt.buf.shape[0], -1)
        dy = self._dy(nd)
        if "dz" in nd.attrs:
            y = nd.out.root()
            self._act_bwd(nd, dy, y.buf, nd.attrs["dz"])
            dy = nd.attrs["dz"]
        units = l.units
        if l.use_bias and not nd.attrs.get("bias_folded"):
            H.colsum(dy, self.gviews[id(l.bias)], workspace=self.gemm_ws, M=dy.shape[0], N=units, ld=dy.shape[1])
        if "dw_pad" in nd.attrs:
            dwp = nd.attrs["dw_pad"]
            H.dense_wgrad(x2, dy, dwp, workspace=self.gemm_ws, accumulate=False)
            kin = l.kernel.shape[0]
            H.unpad_add(dwp, 1, kin, units, kin, dwp.shape[1], self.gviews[id(l.kernel)])
        else:
            H.dense_wgrad(x2, dy, self.gviews[id(l.kernel)], workspace=self.gemm_ws)
        if xt.needs_grad:
            wb = nd.attrs.get("w_pad", self._w(nd, l.kernel))
            acc = xt.written
            xt.written = True
            H.dense_dgrad(dy, wb, xt.grad.view(xt.grad.shape[0], -1), accumulate=acc, workspace=self.gemm_ws)

    # --- driver ---------------------------------------------------------------------------------
    def run(self, n_steps):
        if self.host_collective:
            for _ in range(n_steps):
                self._step_body()
                torch.cuda.synchronize(self.device)
                self.strategy.communicator.allreduce_(self.G, "sum")
                self._optimizer_step()
            return
        if not self.use_graph:
            for _ in range(n_steps):
                self._step_body()
            return
        done = 0
        if self.graph is None:
            # eager first step (also validates the plan), then capture
            self._step_body()
            done = 1
            if n_steps > 1:
                self._capture_safe()
                # capture does not execute; replay below
        for _ in range(n_steps - done):
            if self.graph is None:
                self._capture_safe()
            self.graph.replay()

    def phase_times(self, n_steps: int) -> dict:
        """Per-phase device time of eager steps: forward (incl. loss), backward, the exposed
        all-reduce (what is left after the buckets overlapped backward), optimizer."""
        if self.host_collective:
            return super().phase_times(n_steps)
        self.sync()
        acc = {}
        for _ in range(n_steps):
            self._phase_events = []
            self._step_body()
            evs, self._phase_events = self._phase_events, None
            torch.cuda.synchronize(self.device)
            for (_, a), (name, b) in zip(evs, evs[1:]):
                acc[name] = acc.get(name, 0.0) + a.elapsed_time(b)
        out = {k: v / max(n_steps, 1) for k, v in acc.items()}
        out["step"] = sum(out.values())
        out["allreduce_kind"] = self.allreduce_kind
        return out

    def prepare(self, n_steps):
        if self.use_graph and not self.host_collective and self.graph is None and n_steps > 0:
            self._capture_safe()

    def _capture_safe(self):
        # capturing would run allocator/stream ops; make sure no work is pending
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        # no garbage collection inside the capture: a finalizer that synchronises or frees
        # device resources (an old engine's communicator, graph, events) is illegal while a
        # stream captures and aborts the process (seen on the GPU tier)
        gc.collect()
        was = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    self._step_body()
        finally:
            if was:
                gc.enable()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self.graph = g

    def _check_peer(self):
        if self.peer is not None and any(p.status() for p in self.peers):
            raise RuntimeError("xGMI peer all-reduce: a wait for a peer timed out (peer missing or wedged)")

    def metrics(self):
        torch.cuda.synchronize(self.device)
        self._check_peer()
        c = self.ctrl.cpu().tolist()
        loss, corr, cnt = _i2f(c[C_AL]), _i2f(c[C_AC]), _i2f(c[C_AN])
        d = max(cnt, 1.0)
        out = {"loss": loss / d, "_count": cnt}
        for m in self.model.compiled_metrics:
            out[m.name] = corr / d
        return out

    def end_epoch(self):
        return self.metrics()

    def finish(self):
        torch.cuda.synchronize(self.device)
        opt = self.model.optimizer
        if self.S:
            tot = int(sum(self.sizes))
            opt.ensure_slots(tot, self.device)
            for nm, buf in self.S.items():
                o = 0
                for sz, off in zip(self.sizes, self.offsets):
                    opt.slots[nm][o:o + sz].copy_(buf[off:off + sz])
                    o += sz

    def sync(self):
        torch.cuda.synchronize(self.device)
        self._check_peer()  # never hand out weights built from a timed-out (partial) reduction

    def after_external_write(self):
        # the forward/backward GEMMs read the bf16 shadow Pb: re-derive it from the
        # overwritten fp32 masters before the next step
        H.cast_bf16(self.P, self.Pb)
        torch.cuda.synchronize(self.device)
