"""Native inference: ``predict`` / ``evaluate`` through the native forward plan.

The reference scores its trained model on a held-out split (README.md:286-290, 369-373:
``model.evaluate`` / ``predict`` after ``fit``; ``fit(validation_split=...)`` evaluates
every epoch).  Here that runs on the same lowered plan as training
(:class:`~distributed_amd.engine.native_graph.NativeGraphEngine`), forward only:

* the inputs of the whole call are uploaded once (uint8 or fp32 rows; 288 GB of HBM holds
  any evaluation split whole) and ``gather_batch`` cuts batch ``cursor`` on the device;
* BatchNorm runs with the MOVING statistics: ``bn_infer_st`` turns them into the same
  (mean, invstd, scale, shift) rows the training plan derives from batch statistics, so
  the fused BN / residual / stem-pool kernels are reused unchanged; Dropout is identity;
* one step = gather -> forward -> (``logits_store`` | ``softmax_xent``) -> ``step_fold``
  (cursor + metric accumulators in the device ``Ctrl`` block), captured once as a HIP
  graph and replayed ceil(n / batch) times: no host synchronisation per batch, one at
  the end of the call.

Plans are cached per (model, batch size); weights are re-read at the start of every call
(fp32 copy into the plan's flat buffer, one bf16 cast, the padded copies, the BN rows).
"""
from __future__ import annotations

import gc
from typing import Dict, Tuple

import numpy as np
import torch

from ..ops import hip as H
from ..utils import logging as dlog
from .native_graph import (C_AL, C_AC, C_AN, C_CUR, C_GB, C_NS, C_ROW0, C_WRAP, NativeGraphEngine, _i2f, _pad8,
                           _param_weights)


class NativeInference(NativeGraphEngine):
    name = "native_infer"
    _weights_static = True
    _bn_fin = False  # BN runs from the moving statistics (bn_infer_st)

    @staticmethod
    def eligible(model, device, evaluate: bool = False) -> Tuple[bool, str]:
        from ..keras import losses

        if torch.device(device).type != "cuda":
            return False, "not on a GPU"
        if evaluate:
            if not (isinstance(model.loss, losses.SparseCategoricalCrossentropy) and model.loss.from_logits):
                return False, "loss"
            for m in model.compiled_metrics:
                if m.name not in ("accuracy", "acc", "sparse_categorical_accuracy"):
                    return False, f"metric {m.name}"
        return NativeGraphEngine.layers_eligible(model)

    def __init__(self, model, batch: int, device):
        # no Engine.__init__: an inference plan owns no strategy, gradients or optimizer
        from ..native import require_C

        self.model, self.B, self.device = model, int(batch), torch.device(device)
        self.C = require_C()
        self.rank = 0
        self._build()
        for nd in self.nodes:
            if nd.kind == "Dropout" and not nd.attrs.get("dead"):
                nd.attrs["dead"] = True  # identity at inference
                self._alias(nd.out, nd.inputs[0])
            nd.attrs.pop("stats", None)  # BN uses the moving statistics: no batch statistics
            nd.attrs.pop("stats_from_conv", None)
        for t in self._all_tensors():
            t.needs_grad = False
        self._allocate()
        dev = self.device
        # every weight the forward reads, frozen layers included (not only trainable_weights)
        self.vars = _param_weights(model)
        self.sizes = [int(np.prod(v.shape)) for v in self.vars]
        offs, off = [], 0
        for sz in self.sizes:
            offs.append(off)
            off = _pad8(off + sz)
        self.nparam = off
        self.offsets = offs
        self.P = torch.zeros(off, dtype=torch.float32, device=dev)
        self.Pb = torch.zeros(off, dtype=torch.bfloat16, device=dev)
        self.views, self.bviews = {}, {}
        for v, sz, o in zip(self.vars, self.sizes, offs):
            self.views[id(v)] = self.P[o:o + sz].view(v.shape)
            self.bviews[id(v)] = self.Pb[o:o + sz].view(v.shape)
        self.tail = torch.zeros(8, dtype=torch.float32, device=dev)
        self.ctrl = torch.zeros(32, dtype=torch.int32, device=dev)
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        self._bufs: Dict[str, torch.Tensor] = {}
        self._bn = [nd for nd in self.nodes if nd.kind == "BatchNormalization" and not nd.attrs.get("dead")]
        self._stream = torch.cuda.Stream(dev)

    # --- weights --------------------------------------------------------------------------
    def _refresh_weights(self):
        for v in self.vars:
            self.views[id(v)].copy_(v.value.detach().reshape(v.shape))
        H.cast_bf16(self.P, self.Pb)
        for nd in self.nodes:
            if not nd.attrs.get("dead"):
                self._pad_weights(nd)
        keep = []  # moving statistics moved to the device for this call: alive until the sync
        for nd in self._bn:
            l = nd.layer
            C = nd.out.shape[-1]
            mean, var = (w.value.detach().to(self.device, torch.float32).contiguous()
                         for w in (l.moving_mean, l.moving_variance))
            keep += [mean, var]
            g = self.views[id(l.gamma)] if l.gamma is not None else None
            b = self.views[id(l.beta)] if l.beta is not None else None
            self.C.bn_infer_st(mean.data_ptr(), var.data_ptr(), g.data_ptr() if g is not None else 0,
                               b.data_ptr() if b is not None else 0, float(l.epsilon), C, nd.attrs["st"].data_ptr(),
                               H.stream_handle())
        torch.cuda.current_stream(self.device).synchronize()

    # --- the step ---------------------------------------------------------------------------
    def _fwd_BatchNormalization(self, nd):
        if nd.attrs.get("stats_only") or nd.attrs.get("pool") is not None:
            return  # applied by the fused Add / MaxPool that consumes it
        H.bn_apply(nd.inputs[0].root().buf, nd.attrs["st"], nd.out.root().buf, relu=nd.attrs.get("relu", False))

    def _infer_step(self, mode: str):
        C, B = self.C, self.B
        s = H.stream_handle()
        h, w, c = self.in_shape
        x, y = self._bufs["x"], self._bufs["y"]
        # uint8 inputs are fed as their raw values (Keras casts them), scale 1
        C.gather_batch(x.data_ptr(), int(x.dtype == torch.uint8), 1.0, y.data_ptr(), self.ctrl.data_ptr(), B,
                       h * w, c, self.cin_pad, self.x0.buf.data_ptr(), self.labels.data_ptr(), s)
        for nd in self.nodes:
            if not nd.attrs.get("dead"):
                getattr(self, "_fwd_" + nd.kind)(nd)
        if mode == "predict":
            C.logits_store(self.logits.data_ptr(), self.Kp, self.K, B, self.ctrl.data_ptr(),
                           self._bufs["out"].data_ptr(), s)
            C.step_fold(self.ctrl.data_ptr(), 0, s)
        else:
            H.softmax_xent(self.logits, self.labels, self.K, 1.0 / B, self.dlogits, self.tail, ctrl=self.ctrl,
                           rows=self.xent_rows)
            C.step_fold(self.ctrl.data_ptr(), self.tail.data_ptr(), s)

    def _stage(self, x, y=None):
        """Upload the call's inputs into (grown-only) device buffers; (re)capture happens
        only when a buffer had to be reallocated."""
        n = len(x)
        h, w, c = self.in_shape
        x = np.asarray(x)
        u8 = x.dtype == np.uint8
        rows = x.reshape(n, h * w * c)
        if not u8:
            rows = rows.astype(np.float32, copy=False)
        dt = torch.uint8 if u8 else torch.float32
        realloc = False
        cap = self._bufs.get("x")
        if cap is None or cap.dtype != dt or cap.shape[0] < n:
            self._bufs["x"] = torch.empty((max(n, 1), h * w * c), dtype=dt, device=self.device)
            realloc = True
        self._bufs["x"][:n].copy_(torch.from_numpy(np.ascontiguousarray(rows)), non_blocking=False)
        yb = self._bufs.get("y")
        if yb is None or yb.shape[0] < n:
            self._bufs["y"] = torch.zeros(max(n, 1), dtype=torch.int32, device=self.device)
            realloc = True
        if y is not None:
            self._bufs["y"][:n].copy_(torch.from_numpy(np.asarray(y).astype(np.int32).reshape(n)))
        ob = self._bufs.get("out")
        if ob is None or ob.shape[0] < n:
            self._bufs["out"] = torch.zeros((max(n, 1), self.K), dtype=torch.float32, device=self.device)
            realloc = True
        if realloc:
            self._graphs.clear()
        return n

    def _ctrl_reset(self, n):
        c = torch.zeros(32, dtype=torch.int32)
        c[C_NS], c[C_GB], c[C_ROW0], c[C_CUR], c[C_WRAP] = n, self.B, 0, 0, 0
        self.ctrl.copy_(c.to(self.device))
        self.tail.zero_()

    def _run(self, mode: str, n: int):
        steps = -(-n // self.B)
        dev = self.device
        torch.cuda.synchronize(dev)
        with torch.cuda.stream(self._stream):
            self._refresh_weights()
            self._ctrl_reset(n)
            g = self._graphs.get(mode)
            if g is None:
                g = torch.cuda.CUDAGraph()
                gc.collect()
                was = gc.isenabled()
                gc.disable()
                try:
                    with torch.cuda.graph(g, stream=self._stream):
                        self._infer_step(mode)
                finally:
                    if was:
                        gc.enable()
                self._graphs[mode] = g
            for _ in range(steps):
                g.replay()
        torch.cuda.synchronize(dev)

    # --- public ----------------------------------------------------------------------------
    @torch.no_grad()
    def predict(self, x) -> np.ndarray:
        n = self._stage(x)
        if n == 0:
            return np.zeros((0, self.K), dtype=np.float32)
        self._run("predict", n)
        return self._bufs["out"][:n].cpu().numpy()

    @torch.no_grad()
    def evaluate_sums(self, x, y) -> Tuple[float, float, float]:
        """(sum of per-sample loss, number of samples, number correct) over (x, y)."""
        n = self._stage(x, y)
        if n == 0:
            return 0.0, 0.0, 0.0
        self._run("evaluate", n)
        c = self.ctrl.cpu().tolist()
        return _i2f(c[C_AL]), _i2f(c[C_AN]), _i2f(c[C_AC])


def plan_for(model, batch: int, device, evaluate: bool = False):
    """The cached inference plan of ``model`` at ``batch`` (None when ineligible)."""
    ok, why = NativeInference.eligible(model, device, evaluate)
    if not ok:
        dlog.warning("native inference unavailable (%s): %s runs on PyTorch ops", why,
                     "evaluate" if evaluate else "predict")
        return None
    cache = model.__dict__.setdefault("_infer_plans", {})
    key = (int(batch), str(device))
    p = cache.get(key)
    if p is None:
        p = NativeInference(model, batch, device)
        cache[key] = p
    return p
