"""Cluster specification / rendezvous: ``TF_CONFIG`` and launcher environments.

Reference behaviour:

* ``TF_CONFIG = {"cluster": {"worker": ["host:port", ...]}, "task": {"type": "worker",
  "index": i}}`` — the same worker list on every host, only ``index`` differs
  (reference README.md:84-113 (R), 319-357 (Python)).
* R's ``jsonlite::toJSON(..., auto_unbox=TRUE)`` turns length-1 vectors into scalars,
  so a one-worker cluster serialises ``worker`` as a bare string, and the Spark path
  builds ``index = barrier$partition`` (README.md:180-183) — both forms are accepted.
* Index 0 is the chief ("main worker", README.md:83, 319).

When TF_CONFIG is absent, torchrun-style ``RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT``
(used by ``bench.py`` under ``torch.distributed.run``) or the framework launcher's
``DAMD_*`` variables are honoured; with none of them the job is single-worker.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import List, Mapping, Optional

SUPPORTED_TASK_TYPES = ("worker",)
UNSUPPORTED_TASK_TYPES = ("chief", "ps", "evaluator")


class ClusterConfigError(ValueError):
    pass


@dataclass
class ClusterSpec:
    workers: List[str] = field(default_factory=list)  # "host:port" per rank
    task_type: str = "worker"
    task_id: int = 0
    source: str = "default"  # tf_config | torchrun | launcher | default
    local_rank: int = 0

    @property
    def num_workers(self) -> int:
        return max(1, len(self.workers))

    @property
    def rank(self) -> int:
        return self.task_id

    @property
    def is_chief(self) -> bool:
        return self.task_id == 0

    @property
    def chief_address(self) -> Optional[str]:
        return self.workers[0] if self.workers else None

    def as_dict(self) -> dict:
        return {"worker": list(self.workers)}


def _split_hostport(a: str):
    if ":" not in a:
        raise ClusterConfigError(f"worker address {a!r} is not host:port")
    host, port = a.rsplit(":", 1)
    try:
        p = int(port)
    except ValueError as e:
        raise ClusterConfigError(f"bad port in worker address {a!r}") from e
    if not (0 < p < 65536):
        raise ClusterConfigError(f"port out of range in {a!r}")
    return host, p


def parse_tf_config(raw: str) -> ClusterSpec:
    """Parse a TF_CONFIG JSON string into a :class:`ClusterSpec`."""
    try:
        cfg = json.loads(raw)
    except json.JSONDecodeError as e:
        raise ClusterConfigError(f"TF_CONFIG is not valid JSON: {e}") from e
    if not isinstance(cfg, dict):
        raise ClusterConfigError("TF_CONFIG must be a JSON object")
    cluster = cfg.get("cluster", {}) or {}
    if not isinstance(cluster, dict):
        raise ClusterConfigError("TF_CONFIG.cluster must be an object")
    for jt in cluster:
        if jt not in SUPPORTED_TASK_TYPES:
            raise ClusterConfigError(
                f"cluster job {jt!r} is not supported (only synchronous 'worker' jobs, "
                "as in the reference; parameter servers / evaluators are out of scope)"
            )
    workers = cluster.get("worker", [])
    if isinstance(workers, str):  # jsonlite auto_unbox of a length-1 vector
        workers = [workers]
    if not isinstance(workers, list) or not all(isinstance(w, str) for w in workers):
        raise ClusterConfigError("TF_CONFIG.cluster.worker must be a list of 'host:port' strings")
    for w in workers:
        _split_hostport(w)
    task = cfg.get("task", {}) or {}
    ttype = task.get("type", "worker")
    if isinstance(ttype, list):
        ttype = ttype[0]
    if ttype in UNSUPPORTED_TASK_TYPES:
        raise ClusterConfigError(f"task type {ttype!r} is not supported (only 'worker')")
    if ttype not in SUPPORTED_TASK_TYPES:
        raise ClusterConfigError(f"unknown task type {ttype!r}")
    idx = task.get("index", 0)
    if isinstance(idx, list):  # auto_unbox=FALSE style [0]
        if len(idx) != 1:
            raise ClusterConfigError("task.index list must have exactly one element")
        idx = idx[0]
    try:
        idx = int(idx)
    except (TypeError, ValueError) as e:
        raise ClusterConfigError(f"task.index {idx!r} is not an integer") from e
    if workers and not (0 <= idx < len(workers)):
        raise ClusterConfigError(f"task.index {idx} out of range for {len(workers)} workers")
    if not workers:
        workers = []
    lr = int(os.environ.get("DAMD_LOCAL_RANK", os.environ.get("LOCAL_RANK", idx if _all_local(workers) else 0)))
    return ClusterSpec(workers=workers, task_type=ttype, task_id=idx, source="tf_config", local_rank=lr)


def _all_local(workers) -> bool:
    hosts = {w.rsplit(":", 1)[0] for w in workers}
    return hosts <= {"127.0.0.1", "localhost", "::1"} or len(hosts) == 1


def resolve(env: Optional[Mapping[str, str]] = None) -> ClusterSpec:
    """Cluster spec from the environment: TF_CONFIG > torchrun > single worker."""
    env = os.environ if env is None else env
    raw = env.get("TF_CONFIG")
    if raw:
        spec = parse_tf_config(raw)
        if spec.workers:
            return spec
    if "WORLD_SIZE" in env and "RANK" in env:
        world, rank = int(env["WORLD_SIZE"]), int(env["RANK"])
        addr = env.get("MASTER_ADDR", "127.0.0.1")
        port = int(env.get("MASTER_PORT", "29500"))
        workers = [f"{addr}:{port + i}" for i in range(world)]
        return ClusterSpec(workers=workers, task_id=rank, source="torchrun",
                           local_rank=int(env.get("LOCAL_RANK", rank)))
    return ClusterSpec(workers=["127.0.0.1:0"], task_id=0, source="default", local_rank=0)


def tf_config_json(workers: List[str], index: int) -> str:
    """Build the TF_CONFIG string (Python form of README.md:322-327)."""
    return json.dumps({"cluster": {"worker": list(workers)}, "task": {"type": "worker", "index": int(index)}})
