"""bench.py contract on CPU: ``python bench.py --gpus N`` without torchrun spawns the N
ranks itself and prints ONE JSON line for the whole job (reference README.md:363-392:
the same script runs on every worker)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=600):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TF_CONFIG", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["DAMD_DEVICE"] = "cpu"
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd="/tmp", env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, lines


@pytest.mark.dist
def test_bench_spawns_its_own_ranks():
    r, lines = _run(["--gpus", "2", "--engine", "generic", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["global_batch"] == 128 and out["config"]["parallelism"] == "dp2"
    assert out["steps"] == 3 and out["warmup"] == 1
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["allreduce"].startswith("torch")


@pytest.mark.dist
def test_bench_gang_fails_if_a_rank_fails():
    # rank 1 raises at its first step: the gang must exit non-zero, not hang
    r, lines = _run(["--gpus", "2", "--engine", "generic", "--steps", "3", "--warmup", "1"],
                    {"DAMD_FAIL_AT": "1:0"}, timeout=300)
    assert r.returncode != 0
    assert not lines


@pytest.mark.dist
def test_bench_retries_a_failed_gang_once():
    # rank 1 raises in the first attempt only (DAMD_FAIL_AT rank:step:attempt): the second
    # attempt (exchange pinned to RCCL on a GPU node; no effect on CPU) completes, and the
    # failed attempt prints no JSON line -- exactly one line for the job
    r, lines = _run(["--gpus", "2", "--engine", "generic", "--steps", "3", "--warmup", "1"],
                    {"DAMD_FAIL_AT": "1:0:0"}, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout
    assert "retrying with DAMD_ALLREDUCE=rccl" in r.stderr
    out = json.loads(lines[0])
    # the failed first attempt stays visible in the record
    assert out["fallback_from"] == ["gang-exit-1"], out


def test_bench_refuses_timing_probes():
    """A DAMD_PROBE_* variable (wrong-numerics timing probe) must never yield a bench line."""
    r, lines = _run(["--steps", "2", "--warmup", "1", "--engine", "generic"], {"DAMD_PROBE_HACC": "1"}, timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert not lines
    assert "refusing" in r.stderr


@pytest.mark.dist
@pytest.mark.timeout(600)
def test_bench_eight_ranks_dp8_window_has_no_host_collective():
    """BASELINE configs 3 / 5 are 8 ranks at global batch 512 (README.md:413: global batch =
    64 x workers).  bench.py --gpus 8 spawns 8 gloo ranks, prints ONE line for the job, and no
    control-plane collective (barrier / object all-gather) runs between t0 and the
    end-of-window device synchronize: the trailing barrier is outside the window and
    reported on its own as barrier_us."""
    r, lines = _run(["--gpus", "8", "--engine", "generic", "--steps", "3", "--warmup", "1"],
                    {"OMP_NUM_THREADS": "1"}, timeout=500)
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8
    assert out["config"]["parallelism"] == "dp8" and out["config"]["global_batch"] == 512
    assert out["control_collectives_in_window"] == 0
    assert out["barrier_us"] >= 0
    assert out["replicas_mirrored"] is True
    # value is the whole-job rate: global batch x steps / window
    assert abs(out["value"] - 512 * 1e3 / out["ms_per_step"]) / out["value"] < 1e-3


def test_bench_timed_window_has_no_collective_between_t0_and_sync():
    """Static check of bench.py's window: between t0 and t1 (the end-of-window device
    synchronize) the only calls are the steps and the synchronize -- the barrier and the
    all-gather of the per-rank times come after t1."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    body = src[src.index("    def timed(eng, k, final):"):src.index("    fail_at = runtime.fault_injection_step()")]
    win = body[body.index("t0 = time.perf_counter()"):body.index("t1 = time.perf_counter()")]
    for call in ("barrier()", "allgather_object", "broadcast_object", "all_reduce"):
        assert call not in win, call
    after = body[body.index("t1 = time.perf_counter()"):]
    assert "barrier()" in after and "allgather_object" in after
