#!/usr/bin/env python
"""Headline benchmark: MNIST-CNN data-parallel training throughput on MI355X.

Metric / config from BASELINE.json: whole-node images/sec of the reference MNIST CNN
(Conv2D(32,3,relu) -> MaxPool -> Flatten -> Dense(64,relu) -> Dense(10), 347,146
params, SparseCategoricalCrossentropy(from_logits) + SGD(lr=1e-3), README.md:58-73)
at 64 images per GPU (weak scaling: global batch = 64 x N), bf16 MFMA compute with fp32
master weights, synthetic 28x28x1 data (60000 rows, no network), random-init weights.

Every timed step is a full training step: forward, loss, backward, RCCL all-reduce of
the gradient (N > 1) and the SGD update (the last deferred update is flushed inside the
timed region).  Run:  python bench.py --gpus N --steps K --warmup W
N > 1: either under ``python -m torch.distributed.run --nproc-per-node N ... bench.py``
(RANK / WORLD_SIZE / MASTER_* in the environment), or plainly -- then this process
spawns the N ranks itself (one child process per GPU, torchrun-style environment,
started before anything touches the GPU), prints rank 0's JSON line and exits non-zero
if any rank fails.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

BASELINE_IMG_S = 6198.0  # reference 4-worker MWMS steady-state global rate (5,872-6,524)
METRIC = "images/sec (whole node) MNIST CNN at 1/2/4/8 MI355X; DP scaling efficiency"


def spawn_ranks(n: int, argv) -> int:
    """Run ``bench.py argv`` as ``n`` local ranks (reference README.md:363-392: the same
    script on every worker); returns the gang's exit code.  Rank 0's stdout is relayed; its
    JSON result line only once the whole gang has exited cleanly.

    The default gradient exchange at N > 1 is the sharded xGMI exchange inside the step
    kernels, whose peer waits are bounded (a short in-kernel deadline here: a step takes
    microseconds).  If that gang fails and the user did not pin DAMD_ALLREDUCE, the bench is
    run once more with the exchange on RCCL, so a node whose peer mappings misbehave still
    yields a measurement (the JSON line's "allreduce" field names the transport used)."""
    rc, out = _spawn_once(n, argv, {})
    if rc != 0 and "DAMD_ALLREDUCE" not in os.environ:
        print(f"bench.py: the {n}-rank run failed (exit {rc}); retrying with DAMD_ALLREDUCE=rccl",
              file=sys.stderr, flush=True)
        # the JSON line of the retry names the failed first attempt ("fallback_from"), so a
        # regression of the default transport stays visible in the record
        rc, out = _spawn_once(n, argv, {"DAMD_ALLREDUCE": "rccl", "DAMD_RESTART_COUNT": "1",
                                        "DAMD_BENCH_FALLBACK_FROM": f"gang-exit-{rc}"})
    if rc == 0:
        for line in out:
            print(line, end="", flush=True)
    return rc


def _spawn_once(n: int, argv, extra_env):
    import signal
    import subprocess

    from distributed_amd.launch import free_port_base

    port = free_port_base(1)
    procs = []
    held = []
    for r in range(n):
        env = dict(os.environ)
        env.setdefault("DAMD_WATCHDOG_S", "60")  # in-kernel peer-wait deadline (and host sync deadline)
        env.update(extra_env)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                    "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")})
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      start_new_session=True, text=True))
    import threading

    def relay():  # rank 0's stdout, relayed on a thread: the main loop keeps polling every rank
        for line in procs[0].stdout:
            if line.startswith('{"metric"'):
                held.append(line)  # printed by the caller once every rank exited cleanly
            else:
                print(line, end="", flush=True)

    th = threading.Thread(target=relay, daemon=True)
    th.start()
    try:
        deadline = None
        while any(p.poll() is None for p in procs):
            if any(p.returncode not in (None, 0) for p in procs):
                # a rank failed: the others may be blocked in a collective with it -- give
                # them a moment to exit on their own, then kill the gang
                if deadline is None:
                    deadline = time.time() + 10
                if time.time() > deadline:
                    break
            time.sleep(0.1)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
                p.wait()
        th.join(timeout=5)
    rc = 0
    rcs = [p.returncode for p in procs]
    if any(rcs):
        print(f"bench.py: rank exit codes {rcs}", file=sys.stderr)
        rc = next(c for c in rcs if c) or 1
        rc = rc if rc > 0 else 1
    return rc, held


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--per-gpu-batch", type=int, default=64)
    ap.add_argument("--engine", choices=["auto", "fused", "native", "generic"], default="auto")
    ap.add_argument("--model", choices=["mnist", "resnet18"], default="mnist",
                    help="mnist = the headline config (BASELINE.json); resnet18 = BASELINE.json config 4")
    ap.add_argument("--samples", type=int, default=None, help="synthetic dataset rows")
    ap.add_argument("--graph-steps", type=int, default=None)
    ap.add_argument("--phases", type=int, default=0,
                    help="after the timed run, time N more eager steps phase by phase (forward / backward / "
                         "all-reduce / optimizer) and add them to the JSON line as phases_ms")
    args = ap.parse_args()

    probes = sorted(k for k in os.environ if k.startswith("DAMD_PROBE_"))
    if probes:
        # timing probes skip work inside the step (wrong numerics): a number measured with
        # one is not a training step, so it never reaches a benchmark line
        print(f"bench.py: refusing to run with timing-probe variables set ({', '.join(probes)})", file=sys.stderr)
        sys.exit(2)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and "TF_CONFIG" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))

    if args.engine in ("generic", "native"):
        os.environ["DAMD_FUSED"] = "0"
    if args.engine == "generic":
        os.environ["DAMD_NATIVE_GRAPH"] = "0"
    if args.graph_steps:
        os.environ["DAMD_GRAPH_STEPS"] = str(args.graph_steps)
    elif "DAMD_GRAPH_STEPS" not in os.environ and args.steps > 0:
        # replayed graph length: a common divisor of the warmup and timed step counts, so the
        # warmup already replays the very graph the timed loop replays (its first launch
        # pays one-time costs) -- e.g. 5 for --steps 20 --warmup 5
        g = math.gcd(args.steps, args.warmup)
        os.environ["DAMD_GRAPH_STEPS"] = str(g if g >= 5 else min(args.steps, 20))

    import numpy as np
    import torch

    import distributed_amd as tf
    from distributed_amd.parallel import runtime

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        if args.gpus > 1:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}; launch with torch.distributed.run",
                  file=sys.stderr)
            sys.exit(2)
    strategy = tf.distribute.experimental.MultiWorkerMirroredStrategy()
    rt = runtime.get()
    n = strategy.num_replicas_in_sync
    B = args.per_gpu_batch
    GB = B * n

    comm = strategy.communicator
    on_gpu = rt.device.type == "cuda"

    def barrier():
        if n > 1:
            comm.barrier()

    def device_sync():
        if on_gpu:
            torch.cuda.synchronize()

    if args.model == "mnist":
        (x, y), _ = tf.keras.datasets.mnist.load_data()
        x = x.reshape(len(x), 28, 28, 1) / 255.0
    else:
        rows = args.samples or max(4 * GB, 256)
        rng = np.random.default_rng(1234)
        x = (rng.integers(0, 256, size=(rows, 224, 224, 3), dtype=np.uint8) / np.float32(255.0)).astype(np.float32)
        y = rng.integers(0, 1000, size=rows).astype(np.int64)
    wrap = len(x) // GB

    def make_engine(transport=None):
        """A fresh model (random init, broadcast from rank 0) and its engine; ``transport``
        pins the fused engine's gradient exchange (DAMD_ALLREDUCE) for that engine only."""
        old = os.environ.get("DAMD_ALLREDUCE")
        if transport is not None:
            os.environ["DAMD_ALLREDUCE"] = transport
        try:
            with strategy.scope():
                if args.model == "mnist":
                    model = tf.models.mnist_cnn()
                    tf.models.compile_reference(model, 0.001)
                else:
                    model = tf.models.resnet18()
                    tf.models.compile_resnet(model, 0.1, 0.9)
            eng = model._get_engine(B, GB)
        finally:
            if transport is not None:
                if old is None:
                    os.environ.pop("DAMD_ALLREDUCE", None)
                else:
                    os.environ["DAMD_ALLREDUCE"] = old
        eng.bind(x, y)
        if eng.name in ("fused_convnet", "native_graph"):
            eng.start_epoch(0, True, wrap_steps=wrap)
        else:
            eng.start_epoch(0, True)
        return model, eng

    def run(eng, k):
        # generic engine has no device-side wrap: restart epochs on the host
        if eng.name not in ("fused_convnet", "native_graph"):
            while k > 0:
                left = wrap - eng.step_in_epoch
                if left <= 0:
                    eng.start_epoch(1, True)
                    left = wrap
                d = min(k, left)
                eng.run(d)
                k -= d
        else:
            eng.run(k)

    diag_extra = int(os.environ.get("DAMD_BENCH_EXTRA", "0")) > 0

    def ctl_ops():  # control-plane collectives (barrier / object all-gather) issued so far
        return int(getattr(comm, "control_ops", 0))

    def timed(eng, k, final):
        """(seconds for k full steps, barrier seconds, control collectives in the window).

        The window: a barrier + device synchronize BEFORE t0 (every rank starts together),
        the k steps (the last deferred SGD update included), then each rank's device
        synchronize ends ITS window (t1).  The barrier after t1 is outside the window (its
        cost is reported separately as ``barrier_us``): a host TCP round trip among N ranks
        is not training work.  Value = max over ranks of t1 - t0."""
        barrier()
        device_sync()
        c0 = ctl_ops()
        t0 = time.perf_counter()
        if final:
            eng.run_and_flush(k)  # K steps + the last deferred SGD update, one graph
        else:
            run(eng, k)
            if eng.name == "fused_convnet":
                eng._flush()  # the last deferred SGD update is part of the timed work
        if diag_extra:
            print(f"[bench] host launch call {(time.perf_counter() - t0) * 1e6:.1f} us", file=sys.stderr)
        if not on_gpu:
            eng.sync()
        # on the GPU the device-wide synchronize waits for every stream, the engines' own
        # (C++-created) step streams included: a second, engine-level host wait would only
        # add a round trip to the timed window
        device_sync()
        t1 = time.perf_counter()
        inwin = ctl_ops() - c0  # must stay 0: no host collective inside a timed window
        barrier()
        tb = time.perf_counter() - t1
        if n > 1:
            rows = comm.allgather_object((t1 - t0, tb, inwin))
            return max(r[0] for r in rows), max(r[1] for r in rows), sum(r[2] for r in rows)
        return t1 - t0, tb, inwin

    fail_at = runtime.fault_injection_step()  # DAMD_FAIL_AT=rank:step (launcher / gang tests)
    if fail_at is not None and fail_at <= args.warmup:
        raise RuntimeError(f"injected failure on rank {rt.rank} at step {fail_at} (DAMD_FAIL_AT)")

    # N > 1, fused engine, transport not pinned: the engine itself self-tests every candidate
    # gradient exchange and times each (sharded, peer, RCCL) with this bench's own window
    # protocol -- K steps + flush as one graph -- keeping the fastest
    # (engine/xchg_selftest.time_transport); fit() gets the same choice.  A candidate whose
    # self-test fails is skipped on every rank (collective vote).
    model, engine = make_engine()
    # build the replayed HIP graph(s) first: capture is setup, not part of a timed step
    engine.prepare(max(args.steps, args.warmup))
    # fused engine: the K timed steps and the final flush as one graph (setup, untimed)
    final = (engine.name == "fused_convnet" and 0 < args.steps <= 64
             and os.environ.get("DAMD_BENCH_FINAL_GRAPH", "1") != "0" and engine.prepare_final(args.steps))
    import gc

    # nothing left for the collector to finalize inside the window -- collected BEFORE the
    # warmup: a collection right before the window left the host's caches cold for the
    # graph launch (first window +2 us/step at K = 20 against the same window repeated)
    gc.collect()
    run(engine, args.warmup)
    engine.sync()
    dt, bar_s, ctl_in_window = timed(engine, args.steps, final)
    # diagnostics only (stderr, never the reported value): DAMD_BENCH_EXTRA=n repeats the
    # warmup + timed window n more times, to separate a first-window cost from the steady one
    for _ in range(int(os.environ.get("DAMD_BENCH_EXTRA", "0"))):
        if final:
            engine.prepare_final(args.steps)  # (the variant for the current step phase)
        run(engine, args.warmup)
        engine.sync()
        print(f"[bench] extra window: {timed(engine, args.steps, final)[0] * 1e3 / args.steps:.5f} ms/step",
              file=sys.stderr, flush=True)
    phases = engine.phase_times(args.phases) if args.phases > 0 else None
    m = engine.metrics()
    # MirrorCheck after the window: every rank holds bitwise the same parameters
    mirrored = None
    if n > 1 and hasattr(engine, "P"):
        import hashlib

        engine.sync()
        dig = hashlib.sha1(engine.P.detach().cpu().numpy().tobytes()).hexdigest()
        mirrored = len(set(comm.allgather_object(dig))) == 1
    ms = dt * 1e3 / args.steps
    value = GB * args.steps / dt
    if rt.rank == 0:
        resnet = args.model == "resnet18"
        out = {
            "metric": METRIC if not resnet else "images/sec (whole node) ResNet-18 synthetic 224x224x3",
            "value": round(value, 1),
            "unit": "images/sec",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if resnet else round(value / BASELINE_IMG_S, 2),
            # bf16 MFMA compute (fp32 master weights / accumulation) on the native engines;
            # the PyTorch generic engine computes in fp32
            "dtype": "bf16" if engine.name in ("fused_convnet", "native_graph") else "fp32",
            "data": (f"synthetic ({len(x)} rows 224x224x3 k/255, 1000 classes, random-init weights)" if resnet else
                     "synthetic (28x28x1 MNIST-shaped, 60000 rows, random-init weights)"),
            "config": {
                "model": ("ResNet-18 (11,689,512 params, BN, 1000 classes)" if resnet else
                          "MNIST CNN (Conv2D32-3x3-relu, MaxPool2, Dense64-relu, Dense10; 347,146 params)"),
                "global_batch": GB,
                "per_gpu_batch": B,
                "seq_len": None,
                "parallelism": f"dp{n}",
                "engine": engine.name,
                "optimizer": ("SGD(lr=0.1, momentum=0.9)" if resnet else "SGD(lr=1e-3)") + ", fp32 master weights",
            },
            "final_epoch_loss": round(m.get("loss", float("nan")), 4),
            # how the per-step gradient all-reduce ran, and how many ranks RCCL itself counts
            "allreduce": getattr(engine, "allreduce_kind", "none"),
            # dtype of the exchanged gradient (DAMD_GRAD_DTYPE; fp32 = reference parity)
            "grad_dtype": ("bf16" if (getattr(engine, "grad_dtype", "fp32") == "bf16"
                                      or getattr(engine, "grad_bf16", False)) and n > 1 else "fp32"),
            "rccl_ranks": _rccl_ranks(comm),
        }
        if n > 1:
            # the barrier AFTER the window (outside it) and the control-plane collectives
            # inside the window (0 by construction; tests/test_bench_cpu.py asserts it)
            out["barrier_us"] = round(bar_s * 1e6, 1)
            out["control_collectives_in_window"] = ctl_in_window
            ev = getattr(engine, "exchange_verified", None)
            # the device exchange passed its start-up self-test (bitwise vs the host rank-order
            # reduction) AND the replicas are bitwise mirrored after the window; None: the
            # transport (RCCL / host) is not self-tested
            out["exchange_verified"] = (bool(ev) and bool(mirrored)) if ev is not None else None
            out["replicas_mirrored"] = mirrored
            fb = list(getattr(engine, "exchange_fallback_from", []) or [])
            if os.environ.get("DAMD_BENCH_FALLBACK_FROM"):
                fb = [os.environ["DAMD_BENCH_FALLBACK_FROM"]] + fb
            out["fallback_from"] = fb
            transports = {k: round(v * 1e-3, 5) for k, v in (getattr(engine, "transport_us", None) or {}).items()}
            if transports:
                out["transport_ms_per_step"] = transports
            failed_selftest = [k for k in fb if not k.startswith("gang-exit")]
            if failed_selftest:
                out["transports_failed_selftest"] = failed_selftest
            out["rccl_ms_per_step"] = transports.get("rccl", round(dt * 1e3 / args.steps, 5)
                                                     if getattr(engine, "allreduce_kind", "") == "rccl" else None)
        if phases is not None:
            out["phases_ms"] = {k: (round(v, 5) if isinstance(v, float) else v) for k, v in phases.items()}
        print(json.dumps(out), flush=True)
    runtime.shutdown()


def _rccl_ranks(comm):
    nat = getattr(comm, "native", None)
    if nat is None:
        return None
    try:
        return int(nat.comm_count)
    except Exception:
        return None


if __name__ == "__main__":
    main()
