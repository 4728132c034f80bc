"""Generic engine: any Keras model, per-layer ops, autograd backward, flat-bucket DP.

Per step (per replica): gather the local rows of the global batch from the
device-resident feed, forward, per-sample loss, ``sum / global_batch`` so that a SUM
all-reduce gives the global-mean gradient, write all gradients into ONE
flat fp32 buffer whose tail carries [loss_sum, count, metric sums...] (SURVEY.md D6:
one collective per step for grads + metrics), all-reduce it, apply the optimizer on the
flat master buffer, and accumulate the metric tail on device (no host sync per step).
"""
from __future__ import annotations

import numpy as np
import torch

from .base import Engine
from .data import DataFeed


class GenericEngine(Engine):
    name = "generic"

    def __init__(self, model, strategy, per_replica_batch, global_batch):
        super().__init__(model, strategy, per_replica_batch, global_batch)
        self.vars = model.trainable_weights
        self.sizes = [int(np.prod(v.shape)) for v in self.vars]
        self.n = int(sum(self.sizes))
        dev = self.device
        self.P = torch.zeros(self.n, dtype=torch.float32, device=dev)
        off = 0
        self.leaves = []
        for v, sz in zip(self.vars, self.sizes):
            view = self.P[off:off + sz].view(v.shape)
            with torch.no_grad():
                view.copy_(v.value.detach().to(dev, torch.float32))
            leaf = torch.empty(0, device=dev)
            leaf.data = view
            leaf.requires_grad_(True)
            v._t = leaf
            self.leaves.append(leaf)
            off += sz
        self.loss = model.loss
        self.metric_objs = model.compiled_metrics
        self.ntail = 2 + len(self.metric_objs)
        self.G = torch.zeros(self.n + self.ntail, dtype=torch.float32, device=dev)
        self.acc = torch.zeros(self.ntail, dtype=torch.float64, device=dev)
        model.optimizer.ensure_slots(self.n, dev)
        # mirrored variables: replicas start from worker 0's values
        if self.world > 1:
            comm = strategy.communicator
            comm.broadcast_(self.P, 0)
            for w in model.non_trainable_weights:
                comm.broadcast_(w.value.data if w.value.requires_grad else w.value, 0)
        self.feed = None
        self.step_in_epoch = 0
        self._plan_buckets()

    def _plan_buckets(self):
        """Gradient buckets (SURVEY.md §3.3 / N3'): contiguous ranges of G filled from the
        last layer backwards, the metric tail in the first one.  During backward each
        parameter's gradient is copied into G by a hook; when a bucket is complete its
        all-reduce starts asynchronously while autograd computes the earlier layers."""
        from ..utils import env

        self.bucketed = self.world > 1 and env.get_float("DAMD_BUCKET_MB", 8.0) > 0
        self.allreduce_kind = ("none" if self.world == 1 else
                               f"{self.strategy.communicator.name}{'-bucketed' if self.bucketed else ''}")
        limit = max(1, int(env.get_float("DAMD_BUCKET_MB", 8.0) * 2**20 / 4))
        offs, off = [], 0
        for sz in self.sizes:
            offs.append(off)
            off += sz
        self.offs = offs
        buckets, cur, n = [], [], 0
        for i in reversed(range(len(self.sizes))):
            cur.append(i)
            n += self.sizes[i]
            if n >= limit:
                buckets.append(cur)
                cur, n = [], 0
        if cur:
            buckets.append(cur)
        self.buckets = []
        for bi, idxs in enumerate(buckets):
            lo = min(offs[i] for i in idxs)
            hi = self.n + self.ntail if bi == 0 else max(offs[i] + self.sizes[i] for i in idxs)
            self.buckets.append((lo, hi, set(idxs)))
        self.bucket_of = {i: b for b, (_, _, idxs) in enumerate(self.buckets) for i in idxs}

    def bind(self, x, y):
        key = (id(x), id(y), len(x))
        if self.feed is None or getattr(self, "_feed_key", None) != key:
            self.feed = DataFeed(x, y, self.device)
            self._feed_key = key
        return self.feed

    def start_epoch(self, epoch, shuffle):
        self.feed.set_epoch(epoch, shuffle, self.shuffle_seed)
        self.step_in_epoch = 0
        self.acc.zero_()

    def _tick(self, name):
        ph = getattr(self, "_phases", None)
        if ph is None:
            return
        import time

        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t = time.perf_counter()
        ph[name] = ph.get(name, 0.0) + (t - self._t_last) * 1e3
        self._t_last = t

    def phase_times(self, n_steps: int) -> dict:
        """Host-timed phases (device synchronised at each point): forward + loss, backward
        (bucketed all-reduces already launched inside it), the wait for the all-reduce,
        optimizer."""
        import time

        self.sync()
        self._phases = {}
        try:
            for _ in range(n_steps):
                left = self.feed.n // max(self.global_batch, 1) - self.step_in_epoch
                if left <= 0:
                    self.start_epoch(0, False)
                self._t_last = time.perf_counter()
                self._one_step()
            out = {k: v / max(n_steps, 1) for k, v in self._phases.items()}
        finally:
            self._phases = None
        out["step"] = sum(out.values())
        out["allreduce_kind"] = self.allreduce_kind
        return out

    def _one_step(self):
        feed, model = self.feed, self.model
        s = self.step_in_epoch
        idx = feed.batch_indices(s, self.global_batch, self.rank * self.per_replica, self.per_replica)
        gstart = s * self.global_batch
        gcount = max(0, min(self.global_batch, feed.n - gstart))
        G = self.G
        G.zero_()
        works = None
        if idx.numel() > 0 and gcount > 0:
            xb, yb = feed.x[idx], feed.y[idx]
            out = model(xb, training=True)
            ls = self.loss.per_sample(yb, out)
            loss = ls.sum() * (1.0 / gcount)
            self._tick("forward")
            with torch.no_grad():
                G[self.n] = ls.detach().sum()
                G[self.n + 1] = float(idx.numel())
                for i, m in enumerate(self.metric_objs):
                    G[self.n + 2 + i] = m.per_sample(yb, out.detach()).sum()
            if self.bucketed:
                works = self._backward_bucketed(loss)
            else:
                grads = torch.autograd.grad(loss, self.leaves, allow_unused=True)
                for g, sz, off in zip(grads, self.sizes, self.offs):
                    if g is not None:
                        G[off:off + sz].copy_(g.reshape(-1))
        elif self.bucketed:
            # a replica with no rows (short last batch) still issues the same bucket
            # sequence as the others: one all-reduce per bucket, in bucket order
            comm = self.strategy.communicator
            works = [comm.allreduce_async(G[lo:hi], "sum") for (lo, hi, _) in self.buckets]
        self._tick("backward")
        if works is not None:
            for w in works:
                w.wait()
        elif self.world > 1:
            self.strategy.communicator.allreduce_(G, "sum")
        self._tick("allreduce")
        self.model.optimizer.apply_flat(self.P, G[: self.n])
        self.acc += G[self.n:].double()
        self.step_in_epoch += 1
        self._tick("optimizer")

    def _backward_bucketed(self, loss):
        comm, G = self.strategy.communicator, self.G
        left = [set(idxs) for (_, _, idxs) in self.buckets]
        works = [None] * len(self.buckets)

        def launch(b):
            lo, hi, _ = self.buckets[b]
            works[b] = comm.allreduce_async(G[lo:hi], "sum")

        nxt = [0]

        def launch_ready():
            # buckets start strictly in index order (a complete bucket waits for the
            # earlier ones), so every rank issues the identical collective sequence even
            # if autograd finishes parameters in a different order
            while nxt[0] < len(self.buckets) and not left[nxt[0]]:
                launch(nxt[0])
                nxt[0] += 1

        def make_hook(i):
            def hook(g):
                off, sz = self.offs[i], self.sizes[i]
                with torch.no_grad():
                    G[off:off + sz].copy_(g.reshape(-1))
                left[self.bucket_of[i]].discard(i)
                launch_ready()
                return g
            return hook

        handles = [leaf.register_hook(make_hook(i)) for i, leaf in enumerate(self.leaves)]
        try:
            torch.autograd.backward(loss, inputs=self.leaves)
        finally:
            for h in handles:
                h.remove()
        for b in range(nxt[0], len(self.buckets)):  # parameters that received no gradient
            launch(b)
        for leaf in self.leaves:
            leaf.grad = None
        return works

    def run(self, n_steps):
        for _ in range(n_steps):
            self._one_step()

    def metrics(self):
        a = self.acc.cpu().tolist()
        cnt = a[1] if a[1] else 1.0
        out = {"loss": a[0] / cnt}
        for i, m in enumerate(self.metric_objs):
            out[m.name] = a[2 + i] / cnt
        out["_count"] = a[1]
        return out

    def sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
