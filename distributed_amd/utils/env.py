"""Environment flags (SURVEY.md §5 config/flag system).

TF_CONFIG keeps the reference schema (reference README.md:84-113, 319-357); framework
knobs use the ``DAMD_`` prefix.  NCCL_* / RCCL_* pass through untouched to RCCL.
"""
from __future__ import annotations

import os


def get_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return default if v in (None, "") else int(v)


def get_float(name: str, default: float) -> float:
    v = os.environ.get(name)
    return default if v in (None, "") else float(v)


def get_bool(name: str, default: bool) -> bool:
    v = os.environ.get(name)
    if v in (None, ""):
        return default
    return v.strip().lower() not in ("0", "false", "no", "off")


def get_str(name: str, default: str) -> str:
    v = os.environ.get(name)
    return default if v in (None, "") else v


# Documented knobs (README "Configuration"):
#   DAMD_DEVICE            cpu | cuda          force the compute device
#   DAMD_FUSED             0/1                 allow the fused native ConvNet engine (default 1)
#   DAMD_BUCKET_MB         float               gradient all-reduce bucket size, native graph engine (8)
#   DAMD_FORCE_ALLREDUCE   0/1                 keep the RCCL all-reduce in the step at world 1 (testing)
#   DAMD_NATIVE_GRAPH      0/1                 allow the native graph engine (HIP plan + graph, default 1)
#   DAMD_GRAPH             0/1                 capture steps into hipGraphs (default 1)
#   DAMD_GRAPH_STEPS       int                 steps per captured graph (default 20)
#   DAMD_PP                1..4                pooled positions per fused slice (default 3)
#   DAMD_DEBUG_SYNC        0/1                 synchronize + error-check after every engine chunk
#   DAMD_COMM              rccl | torch | gloo | auto   data-plane communicator on GPU (default auto=rccl;
#                          gloo stages device tensors through host memory: test/debug only)
#   DAMD_ALLREDUCE         auto | xgmi | off    per-step gradient all-reduce of the fused trainer: native
#                          xGMI peer-to-peer two-shot kernel (IPC-mapped peers, self-tested at start; auto
#                          falls back if any rank cannot use it) or off = the communicator's own (RCCL)
#   DAMD_PEER_BLOCKS       int                 workgroups of the xGMI all-reduce kernel (64)
#   DAMD_WATCHDOG_S        float               collective watchdog deadline (0 = off)
#   DAMD_FAIL_AT           "rank:step[:attempt]"  fault injection (raise inside fit; only in that launcher attempt)
#   DAMD_CHECK_MIRRORS     int                 mirror-divergence check every N epochs (0=off)
#   DAMD_LOCAL_RANK        int                 local GPU index (set by the launcher)
