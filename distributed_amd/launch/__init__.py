"""Gang launcher for local ranks (one process per GPU).

Replaces two reference launch paths:

* manual multi-host launch — set ``TF_CONFIG`` on every host and run the same script
  (reference README.md:80-113, 316-358): :func:`launch_script` / ``python -m
  distributed_amd.launch --nproc N script.py`` builds the TF_CONFIG of every rank
  (``127.0.0.1:<port_base+i>``) and starts all ranks at once;
* sparklyr ``spark_apply(f, barrier = TRUE)`` (README.md:171-223): :func:`barrier_apply`
  gang-schedules N tasks, hands each ``barrier = {"address": [...], "partition": i}``,
  collects one result per partition in partition order, returns errors as strings
  (the ``tryCatch`` contract, README.md:176, 221), and on a task crash kills the gang
  and retries it all-or-nothing (Spark barrier-stage semantics).

Ranks get ``DAMD_LOCAL_RANK=i`` (GPU index) and ``DAMD_RESTART_COUNT`` (attempt number).
"""
from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import sys
import time
import traceback
from dataclasses import dataclass
from typing import Any, Callable, List, Optional, Sequence

from ..parallel.cluster import tf_config_json


def free_port_base(n: int, host: str = "127.0.0.1", start: int = 20000, end: int = 32000) -> int:
    """First base port such that [base, base+n) are all bindable right now.  The range sits
    below Linux's ephemeral ports (32768-60999), which outgoing connections of any process
    may take between this check and the rank's bind."""
    import random

    rng = random.Random(os.getpid() ^ int(time.time() * 1000))
    for _ in range(200):
        base = rng.randrange(start, end - n)
        socks = []
        try:
            for i in range(n):
                s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
                s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                s.bind((host, base + i))
                socks.append(s)
            return base
        except OSError:
            continue
        finally:
            for s in socks:
                s.close()
    raise RuntimeError("no free port range found")


def rank_env(rank: int, nproc: int, port_base: int, attempt: int = 0, host: str = "127.0.0.1") -> dict:
    workers = [f"{host}:{port_base + i}" for i in range(nproc)]
    return {
        "TF_CONFIG": tf_config_json(workers, rank),
        "DAMD_LOCAL_RANK": str(rank),
        "DAMD_RESTART_COUNT": str(attempt),
        "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
    }


@dataclass
class GangResult:
    returncodes: List[int]
    attempts: int

    @property
    def ok(self) -> bool:
        return all(rc == 0 for rc in self.returncodes)


def _kill_all(procs):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
    deadline = time.time() + 10
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()


def launch_script(argv: Sequence[str], nproc: int, port_base: Optional[int] = None, max_restarts: int = 0,
                  timeout: Optional[float] = None, env: Optional[dict] = None, python: str = sys.executable,
                  stdout=None, stderr=None, on_failure=None) -> GangResult:
    """Run ``python argv...`` as ``nproc`` ranks; gang-restart on any failure.
    ``on_failure(returncodes)`` is called for every failed attempt (after the gang is
    killed): a rank's own exit status is kept, the killed survivors read -15 / -9."""
    return launch_command([python] + list(argv), nproc, port_base=port_base, max_restarts=max_restarts,
                          timeout=timeout, env=env, stdout=stdout, stderr=stderr, on_failure=on_failure)


def launch_command(cmd: Sequence[str], nproc: int, port_base: Optional[int] = None, max_restarts: int = 0,
                   timeout: Optional[float] = None, env: Optional[dict] = None, stdout=None, stderr=None,
                   on_failure=None, rank_arg: bool = False) -> GangResult:
    """Gang-run any command (an ``Rscript`` runner for the R ``spark_apply``, a Python script,
    ...) as ``nproc`` ranks with the per-rank environment of :func:`rank_env`
    (``rank_arg=True`` also appends the rank to the command line).  All-or-nothing: the
    gang's exit statuses are polled; the first failure (or the ``timeout``) kills every
    survivor's process group and the whole gang restarts, up to ``max_restarts`` times
    (Spark barrier-stage semantics, reference README.md:171-223)."""
    attempt = 0
    while True:
        base = port_base if port_base is not None else free_port_base(nproc)
        procs = []
        for r in range(nproc):
            e = dict(os.environ)
            e.update(env or {})
            e.update(rank_env(r, nproc, base, attempt))
            argv = list(cmd) + ([str(r)] if rank_arg else [])
            procs.append(subprocess.Popen(argv, env=e, stdout=stdout, stderr=stderr, start_new_session=True))
        t0 = time.time()
        failed = False
        while True:
            rcs = [p.poll() for p in procs]
            if any(rc not in (None, 0) for rc in rcs):
                failed = True
                break
            if all(rc == 0 for rc in rcs):
                break
            if timeout is not None and time.time() - t0 > timeout:
                failed = True
                break
            time.sleep(0.05)
        if failed:
            _kill_all(procs)
        rcs = [p.returncode if p.returncode is not None else -9 for p in procs]
        if failed and on_failure is not None:
            on_failure(rcs)
        if not failed or attempt >= max_restarts:
            return GangResult(rcs, attempt + 1)
        attempt += 1
        sys.stderr.write(f"[distributed_amd.launch] gang failed (rcs={rcs}); restart {attempt}/{max_restarts}\n")


# --------------------------------------------------------------------------------------
# barrier_apply: Spark-barrier-style gang of python callables
# --------------------------------------------------------------------------------------
def _task_main(fn, df, barrier, conn, env):
    os.environ.update(env)
    try:
        res = ("ok", fn(df, barrier))
    except BaseException as e:  # tryCatch(..., error = function(e) e$message)
        res = ("error", f"{type(e).__name__}: {e}", traceback.format_exc())
    try:
        conn.send(res)
    except Exception as e:  # unpicklable result
        conn.send(("error", f"result not transferable: {e}", ""))
    conn.close()


def barrier_apply(fn: Callable[[Any, dict], Any], nproc: int, partitions: Optional[Sequence[Any]] = None,
                  port_base: Optional[int] = None, max_restarts: int = 0, timeout: Optional[float] = None,
                  on_error: str = "return", env: Optional[dict] = None) -> List[Any]:
    """Gang-run ``fn(partition_data, barrier)`` on ``nproc`` local processes.

    ``barrier = {"address": ["127.0.0.1:<p0>", ...], "partition": i}`` like sparklyr's
    barrier context.  Returns the per-partition results in partition order.  If ``fn``
    raises: ``on_error="return"`` puts the error message in that slot (tryCatch
    contract), ``"raise"`` raises, ``"restart"`` retries the whole gang.  A crashed or
    timed-out task always kills the gang and retries it (up to ``max_restarts``).
    """
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    parts = list(partitions) if partitions is not None else [None] * nproc
    if len(parts) != nproc:
        raise ValueError("len(partitions) must equal nproc")
    attempt = 0
    while True:
        base = port_base if port_base is not None else free_port_base(nproc)
        addrs = [f"127.0.0.1:{base + i}" for i in range(nproc)]
        procs, conns = [], []
        for i in range(nproc):
            parent, child = ctx.Pipe(duplex=False)
            e = dict(env or {})
            e.update({"DAMD_LOCAL_RANK": str(i), "DAMD_RESTART_COUNT": str(attempt)})
            p = ctx.Process(target=_task_main, args=(fn, parts[i], {"address": list(addrs), "partition": i}, child, e),
                            daemon=False)
            p.start()
            child.close()
            procs.append(p)
            conns.append(parent)
        results: List[Any] = [None] * nproc
        got = [False] * nproc
        t0 = time.time()
        crashed = False
        while not all(got):
            for i, (p, c) in enumerate(zip(procs, conns)):
                if got[i]:
                    continue
                if c.poll():
                    try:
                        results[i] = c.recv()
                    except EOFError:
                        crashed = True
                    got[i] = True
                elif not p.is_alive() and not c.poll():
                    crashed = True
                    got[i] = True
            if crashed or (timeout is not None and time.time() - t0 > timeout):
                crashed = True
                break
            time.sleep(0.02)
        for p in procs:
            if crashed and p.is_alive():
                p.terminate()
        for p in procs:
            p.join(10)
            if p.is_alive():
                p.kill()
                p.join()
        errs = [r for r in results if isinstance(r, tuple) and r and r[0] == "error"]
        retry = crashed or (errs and on_error == "restart")
        if retry and attempt < max_restarts:
            attempt += 1
            continue
        if crashed:
            raise RuntimeError(f"barrier stage failed after {attempt + 1} attempt(s): a task crashed or timed out")
        if errs and on_error == "raise":
            raise RuntimeError(errs[0][1] + "\n" + errs[0][2])
        return [r[1] for r in results]


# --------------------------------------------------------------------------------------
# sparklyr-shaped helpers (local, no JVM): sdf_len / spark_apply / collect
# --------------------------------------------------------------------------------------
class LocalDataFrame:
    """A partitioned local table standing in for a Spark DataFrame."""

    def __init__(self, partitions: List[List[dict]]):
        self.partitions = partitions

    def collect(self) -> List[dict]:
        return [row for p in self.partitions for row in p]

    def num_partitions(self) -> int:
        return len(self.partitions)


def sdf_len(length: int, repartition: Optional[int] = None) -> LocalDataFrame:
    """``sdf_len(sc, length, repartition)`` (README.md:174): rows id=1..length."""
    n = repartition or 1
    rows = [{"id": i + 1} for i in range(length)]
    parts = [rows[(length * k) // n:(length * (k + 1)) // n] for k in range(n)]
    return LocalDataFrame(parts)


def spark_apply(sdf: LocalDataFrame, f: Callable, barrier: bool = True, columns=None, max_restarts: int = 0,
                timeout: Optional[float] = None, env: Optional[dict] = None) -> LocalDataFrame:
    """``spark_apply(sdf, f, barrier = TRUE, columns = c(address = "character"))``.

    ``f(df, barrier)`` runs once per partition (all partitions gang-scheduled); its
    return value becomes the row(s) of the result, under ``columns`` names."""
    if not barrier:
        raise NotImplementedError("only barrier execution is supported (the reference's mode)")
    n = sdf.num_partitions()
    outs = barrier_apply(f, n, partitions=sdf.partitions, max_restarts=max_restarts, timeout=timeout, env=env)
    col = list(columns.keys())[0] if isinstance(columns, dict) else (columns[0] if columns else "result")
    parts = []
    for o in outs:
        vals = o if isinstance(o, list) else [o]
        parts.append([{col: v} for v in vals])
    return LocalDataFrame(parts)


def collect(sdf: LocalDataFrame) -> List[dict]:
    return sdf.collect()
