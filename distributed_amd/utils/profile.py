"""Step-time profiling (SURVEY.md §5 "Tracing / profiling").

``with distributed_amd.utils.profile.profile("out.json"):`` around ``model.fit`` records,
per engine chunk (a run of k training steps), device time from HIP events and host wall
time, and writes a JSON summary (steps, mean/min/max ms per step, images/sec).  Chunks
are also bracketed by roctx ranges (``torch.cuda.nvtx`` maps to roctx on ROCm), so a
``rocprofv3 --marker-trace`` run shows them on the timeline next to the kernels.

:func:`step_phases` breaks a training step into forward / backward / all-reduce /
optimizer time (HIP events between the phases of eager steps; the engines'
``phase_times``), which is how the all-reduce share of a multi-GPU step is reported
(``bench.py --phases``).
"""
from __future__ import annotations

import contextlib
import json
import time
from typing import List, Optional

import torch

_ACTIVE: Optional["Profiler"] = None


class Profiler:
    def __init__(self, path: Optional[str] = None):
        self.path = path
        self.chunks: List[dict] = []

    def begin(self, steps: int, batch: int, device):
        rec = {"steps": steps, "batch": batch, "t0": time.perf_counter()}
        if device.type == "cuda":
            rec["e0"] = torch.cuda.Event(enable_timing=True)
            rec["e1"] = torch.cuda.Event(enable_timing=True)
            rec["e0"].record()
            try:
                torch.cuda.nvtx.range_push(f"damd.steps[{steps}]")
                rec["nvtx"] = True
            except Exception:  # pragma: no cover
                pass
        return rec

    def end(self, rec):
        if "e1" in rec:
            rec["e1"].record()
            if rec.pop("nvtx", False):
                torch.cuda.nvtx.range_pop()
        rec["t1"] = time.perf_counter()
        self.chunks.append(rec)

    def summary(self) -> dict:
        per = []
        steps = imgs = 0
        wall = 0.0
        for r in self.chunks:
            if "e0" in r:
                r["e1"].synchronize()
                ms = r["e0"].elapsed_time(r["e1"])
            else:
                ms = (r["t1"] - r["t0"]) * 1e3
            per.append(ms / max(r["steps"], 1))
            steps += r["steps"]
            imgs += r["steps"] * r["batch"]
            wall += r["t1"] - r["t0"]
        out = {"chunks": len(self.chunks), "steps": steps}
        if per:
            dev_ms = sum(p * r["steps"] for p, r in zip(per, self.chunks))
            out.update(mean_ms_per_step=dev_ms / steps, min_ms_per_step=min(per), max_ms_per_step=max(per),
                       images_per_sec=imgs / (dev_ms / 1e3) if dev_ms else None, host_wall_s=wall)
        return out

    def write(self):
        if self.path:
            with open(self.path, "w") as f:
                json.dump(self.summary(), f, indent=1)


def active() -> Optional[Profiler]:
    return _ACTIVE


@contextlib.contextmanager
def profile(path: Optional[str] = None):
    global _ACTIVE
    prev, _ACTIVE = _ACTIVE, Profiler(path)
    try:
        yield _ACTIVE
    finally:
        p, _ACTIVE = _ACTIVE, prev
        p.write()


def step_phases(model, x, y, batch_size: int, steps: int = 20, path: Optional[str] = None) -> dict:
    """Mean ms per step of each phase over ``steps`` real training steps of ``model`` on
    (x, y) at global ``batch_size`` (the model trains: run it on a copy if that matters).
    Every replica must call it (the steps contain the gradient all-reduce)."""
    st = model._strategy
    per = batch_size // st.num_replicas_in_sync
    eng = model._get_engine(per, batch_size)
    eng.bind(x, y)
    eng.start_epoch(0, False)
    eng.run(1)  # warm (plans, graph capture of the timed engines is not used here)
    eng.sync()
    out = eng.phase_times(steps)
    out = {k: (round(v, 5) if isinstance(v, float) else v) for k, v in out.items()}
    out["engine"] = eng.name
    out["steps"] = steps
    if path:
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
    return out

