"""Keras callbacks: History, ProgbarLogger, ModelCheckpoint, BackupAndRestore,
LearningRateScheduler, TerminateOnNaN, EarlyStopping.

The reference configures no recovery ("ModelCheckpoint callback is not provided.
Workers will need to restart training if any fails.", README.md:400); here
ModelCheckpoint / BackupAndRestore give epoch-granular checkpoint + resume that the
launcher's gang restart relies on.  Only the chief writes
 unless a per-worker path pattern contains ``{rank}``.
"""
from __future__ import annotations

import json
import math
import os
import sys

from ..utils import logging as dlog
from .utils import Progbar


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_model(self, model):
        self.model = model

    def set_params(self, params):
        self.params = params

    def on_train_begin(self, logs=None): pass
    def on_train_end(self, logs=None): pass
    def on_epoch_begin(self, epoch, logs=None): pass
    def on_epoch_end(self, epoch, logs=None): pass
    def on_train_batch_begin(self, batch, logs=None): pass
    def on_train_batch_end(self, batch, logs=None): pass
    on_batch_begin = on_train_batch_begin
    on_batch_end = on_train_batch_end
    # whether this callback needs per-step host callbacks (forces small replay chunks)
    needs_batch_hooks = False


class CallbackList:
    def __init__(self, callbacks, model, params):
        self.callbacks = list(callbacks)
        for c in self.callbacks:
            c.set_model(model)
            c.set_params(params)

    @property
    def needs_batch_hooks(self):
        return any(c.needs_batch_hooks for c in self.callbacks)

    def __getattr__(self, name):
        if name.startswith("on_"):
            def f(*a, **kw):
                for c in self.callbacks:
                    getattr(c, name)(*a, **kw)
            return f
        raise AttributeError(name)


class History(Callback):
    """``fit`` return value: ``history`` dict; ``metrics`` alias for the R API
    (``result$metrics$accuracy``, reference README.md:220)."""

    def on_train_begin(self, logs=None):
        self.epoch = []
        self.history = {}

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)

    @property
    def metrics(self):
        return self.history


class ProgbarLogger(Callback):
    def __init__(self, count_mode="samples", stream=None):
        super().__init__()
        self.stream = stream or sys.stdout
        self.progbar = None

    def on_train_begin(self, logs=None):
        self.verbose = self.params.get("verbose", 1)
        self.epochs = self.params.get("epochs", 1)
        if self.verbose and self.params.get("samples") is not None:
            self.stream.write("Train on %d samples\n" % self.params["samples"])
            self.stream.flush()

    def on_epoch_begin(self, epoch, logs=None):
        if self.verbose:
            self.stream.write("Epoch %d/%d\n" % (epoch + 1, self.epochs))
            self.stream.flush()
        self.progbar = Progbar(self.params.get("samples"), verbose=self.verbose, stream=self.stream)
        self.seen = 0

    def on_train_batch_end(self, batch, logs=None):
        logs = logs or {}
        self.seen = logs.get("seen", self.seen)
        vals = [(k, logs[k]) for k in self.params.get("metrics", []) if k in logs]
        self.progbar.update(self.seen, vals)

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        vals = [(k, logs[k]) for k in self.params.get("metrics", []) if k in logs]
        self.progbar.update(logs.get("seen", self.seen), vals, finalize=True)


class TerminateOnNaN(Callback):
    def on_epoch_end(self, epoch, logs=None):
        l = (logs or {}).get("loss")
        if l is not None and (math.isnan(l) or math.isinf(l)):
            dlog.warning("Epoch %d: invalid loss, terminating training", epoch)
            self.model.stop_training = True


class EarlyStopping(Callback):
    def __init__(self, monitor="loss", min_delta=0.0, patience=0, mode="auto", restore_best_weights=False):
        super().__init__()
        self.monitor, self.min_delta, self.patience = monitor, abs(min_delta), patience
        self.mode = mode if mode != "auto" else ("max" if "acc" in monitor else "min")
        self.restore_best_weights = restore_best_weights

    def on_train_begin(self, logs=None):
        self.wait, self.best, self.best_weights, self.stopped_epoch = 0, None, None, 0

    def on_epoch_end(self, epoch, logs=None):
        cur = (logs or {}).get(self.monitor)
        if cur is None:
            return
        better = self.best is None or (cur < self.best - self.min_delta if self.mode == "min"
                                       else cur > self.best + self.min_delta)
        if better:
            self.best, self.wait = cur, 0
            if self.restore_best_weights:
                self.best_weights = self.model.get_weights()
        else:
            self.wait += 1
            if self.wait > self.patience:
                self.stopped_epoch = epoch
                self.model.stop_training = True
                if self.restore_best_weights and self.best_weights is not None:
                    self.model.set_weights(self.best_weights)


class LearningRateScheduler(Callback):
    def __init__(self, schedule, verbose=0):
        super().__init__()
        self.schedule, self.verbose = schedule, verbose

    def on_epoch_begin(self, epoch, logs=None):
        opt = self.model.optimizer
        try:
            lr = self.schedule(epoch, opt.learning_rate)
        except TypeError:
            lr = self.schedule(epoch)
        opt.learning_rate = float(lr)
        if self.verbose:
            dlog.info("Epoch %05d: LearningRateScheduler setting learning rate to %s.", epoch + 1, lr)


def _is_chief(model) -> bool:
    st = getattr(model, "_strategy", None)
    return st is None or st.is_chief


class ModelCheckpoint(Callback):
    """Save the model (Keras HDF5) at the end of every epoch (``save_freq='epoch'``)."""

    def __init__(self, filepath, monitor="val_loss", verbose=0, save_best_only=False, save_weights_only=False,
                 mode="auto", save_freq="epoch", all_workers=False):
        super().__init__()
        if save_freq != "epoch":
            raise ValueError("only save_freq='epoch' is supported")
        self.filepath, self.monitor, self.verbose = filepath, monitor, verbose
        self.save_best_only, self.save_weights_only = save_best_only, save_weights_only
        self.mode = mode if mode != "auto" else ("max" if "acc" in monitor else "min")
        self.all_workers = all_workers or "{rank}" in str(filepath)
        self.best = None

    def _path(self, epoch, logs):
        st = getattr(self.model, "_strategy", None)
        rank = st.rank if st is not None else 0
        return str(self.filepath).format(epoch=epoch + 1, rank=rank, **(logs or {}))

    def on_epoch_end(self, epoch, logs=None):
        if not (self.all_workers or _is_chief(self.model)):
            return
        if self.save_best_only:
            cur = (logs or {}).get(self.monitor)
            if cur is None:
                return
            if self.best is not None and not (cur < self.best if self.mode == "min" else cur > self.best):
                return
            self.best = cur
        path = self._path(epoch, logs)
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        if self.save_weights_only:
            self.model.save_weights(path)
        else:
            self.model.save(path)
        if self.verbose:
            dlog.info("Epoch %05d: saving model to %s", epoch + 1, path)


class BackupAndRestore(Callback):
    """Fault-tolerance callback: back up the full training state at each epoch end and
    restore it (weights, optimizer slots, iterations, next epoch) when training restarts
    after a failure — e.g. after the launcher's gang restart."""

    def __init__(self, backup_dir):
        super().__init__()
        self.backup_dir = backup_dir
        self._ckpt = os.path.join(backup_dir, "chief.h5")
        self._meta = os.path.join(backup_dir, "state.json")

    def on_train_begin(self, logs=None):
        if os.path.exists(self._meta) and os.path.exists(self._ckpt):
            with open(self._meta) as f:
                meta = json.load(f)
            from . import saving

            saving.load_weights_into(self.model, self._ckpt, with_optimizer=True)
            self.model._initial_epoch_override = int(meta["epoch"]) + 1
            dlog.info("BackupAndRestore: resumed from epoch %d (%s)", meta["epoch"] + 1, self._ckpt)

    def on_epoch_end(self, epoch, logs=None):
        if _is_chief(self.model):
            os.makedirs(self.backup_dir, exist_ok=True)
            tmp = self._ckpt + ".tmp"
            self.model.save(tmp)
            os.replace(tmp, self._ckpt)
            with open(self._meta + ".tmp", "w") as f:
                json.dump({"epoch": epoch, "logs": {k: float(v) for k, v in (logs or {}).items()}}, f)
            os.replace(self._meta + ".tmp", self._meta)
        st = getattr(self.model, "_strategy", None)
        if st is not None:
            st.barrier()

    def on_train_end(self, logs=None):
        if _is_chief(self.model) and not getattr(self.model, "_failed", False):
            for p in (self._ckpt, self._meta):
                if os.path.exists(p):
                    os.remove(p)


class MirrorCheck(Callback):
    """Assert after every ``every`` epochs that all replicas hold bitwise-identical
    variables (distributed_amd/utils/debug.py); raises MirrorDivergenceError otherwise."""

    def __init__(self, every: int = 1):
        super().__init__()
        self.every = max(1, int(every))
        self.fingerprints = []

    def on_epoch_end(self, epoch, logs=None):
        if (epoch + 1) % self.every == 0:
            from ..utils.debug import check_mirrored

            self.fingerprints.append(check_mirrored(self.model, tag=f"epoch {epoch + 1}"))


class JSONMetricsLogger(Callback):
    """One JSON line per epoch (SURVEY.md §5 observability): epoch, the global metrics,
    images/sec and ms/step from the host wall clock of the epoch.  Written by the chief
    only (metrics are already global) to ``path`` (appended) or stdout."""

    def __init__(self, path=None, all_workers=False):
        super().__init__()
        self.path, self.all_workers = path, all_workers
        self._t0 = None

    def on_epoch_begin(self, epoch, logs=None):
        import time

        if self.model is not None and getattr(self.model, "_engine", None) is not None:
            self.model._engine.sync()
        self._t0 = time.perf_counter()

    def on_epoch_end(self, epoch, logs=None):
        import sys
        import time

        if not (self.all_workers or _is_chief(self.model)):
            return
        if getattr(self.model, "_engine", None) is not None:
            self.model._engine.sync()
        dt = time.perf_counter() - (self._t0 or time.perf_counter())
        steps = int(self.params.get("steps") or 0)
        bs = int(self.params.get("batch_size") or 0)
        rec = {"epoch": epoch + 1, **{k: float(v) for k, v in (logs or {}).items() if k != "seen"},
               "seconds": dt, "ms_per_step": 1e3 * dt / steps if steps else None,
               "images_per_sec": steps * bs / dt if dt > 0 else None,
               "engine": getattr(getattr(self.model, "_engine", None), "name", None)}
        eng = getattr(self.model, "_engine", None)
        if getattr(eng, "world", 1) > 1:
            # which gradient exchange carried the epoch, and what each candidate measured
            rec["gradient_exchange"] = getattr(eng, "allreduce_kind", None)
            if getattr(eng, "transport_us", None):
                rec["exchange_us_per_step"] = dict(eng.transport_us)
        line = json.dumps(rec)
        if self.path:
            with open(self.path, "a") as f:
                f.write(line + "\n")
        else:
            sys.stdout.write(line + "\n")
            sys.stdout.flush()
