"""keras.utils: Progbar (TF 2.0 format, reference README.md:307-311, 413-415), to_categorical."""
from __future__ import annotations

import sys
import time

import numpy as np


def _fmt_eta(eta: float) -> str:
    eta = int(eta)
    if eta > 3600:
        return "%d:%02d:%02d" % (eta // 3600, (eta % 3600) // 60, eta % 60)
    if eta > 60:
        return "%d:%02d" % (eta // 60, eta % 60)
    return "%ds" % eta


class Progbar:
    """Keras Progbar.  ``update(current, values)``; unit = samples like TF 2.0's fit on
    numpy input ("Train on 60000 samples", "320/60000 [....] - ETA: 2:25 - loss: ...")."""

    def __init__(self, target, width=30, verbose=1, interval=0.05, stateful_metrics=None, unit_name="sample",
                 stream=None):
        self.target, self.width, self.verbose, self.interval = target, width, verbose, interval
        self.unit_name = unit_name
        self.stream = stream or sys.stdout
        self._dynamic = hasattr(self.stream, "isatty") and self.stream.isatty()
        self._start = time.time()
        self._last_update = 0.0
        self._total_width = 0
        self._seen = 0
        self.last_line = ""

    def _bar(self, current):
        if self.target is None:
            return "%7d/Unknown" % current
        nd = int(np.log10(self.target)) + 1
        s = ("%" + str(nd) + "d/%d [") % (current, self.target)
        prog = float(current) / self.target
        w = int(self.width * prog)
        if w > 0:
            s += "=" * (w - 1) + (">" if current < self.target else "=")
        s += "." * (self.width - w) + "]"
        return s

    def format_line(self, current, values, now=None):
        now = time.time() if now is None else now
        line = self._bar(current)
        elapsed = now - self._start
        per_unit = elapsed / current if current else 0.0
        if self.target is not None and current < self.target:
            line += " - ETA: %s" % _fmt_eta(per_unit * (self.target - current))
        else:
            line += " - %ds" % elapsed
            if per_unit >= 1:
                line += " %.0fs/%s" % (per_unit, self.unit_name)
            elif per_unit >= 1e-3:
                line += " %.0fms/%s" % (per_unit * 1e3, self.unit_name)
            else:
                line += " %.0fus/%s" % (per_unit * 1e6, self.unit_name)
        for k, v in values:
            line += " - %s: %.4f" % (k, v) if abs(v) > 1e-3 else " - %s: %.4e" % (k, v)
        return line

    def update(self, current, values=None, finalize=False):
        values = values or []
        self._seen = current
        if self.verbose != 1:
            if finalize and self.verbose == 2:
                self.stream.write(self.format_line(current, values) + "\n")
                self.stream.flush()
            return
        now = time.time()
        if not finalize and now - self._last_update < self.interval and (self.target is None or current < self.target):
            return
        line = self.format_line(current, values, now)
        self.last_line = line
        if self._dynamic:
            pad = max(0, self._total_width - len(line))
            self.stream.write("\r" + line + " " * pad)
            self._total_width = len(line)
            if finalize:
                self.stream.write("\n")
        elif finalize:
            self.stream.write(line + "\n")
        self.stream.flush()
        self._last_update = now

    def add(self, n, values=None):
        self.update(self._seen + n, values)


def to_categorical(y, num_classes=None, dtype="float32"):
    y = np.asarray(y, dtype="int64").reshape(-1)
    n = num_classes or int(y.max()) + 1
    out = np.zeros((y.shape[0], n), dtype=dtype)
    out[np.arange(y.shape[0]), y] = 1
    return out
