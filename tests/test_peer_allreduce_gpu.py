"""The native xGMI peer-to-peer all-reduce (csrc/runtime/peer_comm.h) on one MI355X:
several ranks (processes) share the GPU and map each other's buffers over IPC, which
exercises the whole protocol (IPC export/map, per-block cross-rank flags, epochs across
calls, graph capture/replay) except the xGMI link itself.  On a multi-GPU node the same
code maps peers across xGMI and self-tests at engine start (make_peer_allreduce)."""
import json
import os

import numpy as np
import pytest

from distributed_amd import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = [pytest.mark.gpu, pytest.mark.dist]


def _env(out, **kw):
    e = {"DAMD_DEVICE": "cuda:0", "DAMD_COMM": "gloo", "DAMD_TEST_OUT": str(out), "PYTHONPATH": ROOT,
         "OMP_NUM_THREADS": "2", "DAMD_LOG_LEVEL": "WARNING",
         "DAMD_WATCHDOG_S": "20"}  # bounds every in-kernel cross-rank wait (a protocol bug fails fast)
    e.update({k: str(v) for k, v in kw.items()})
    return e


@pytest.mark.parametrize("world,blocks", [(2, 64), (4, 16)])
@pytest.mark.timeout(300)
def test_peer_allreduce_bitwise(tmp_path, world, blocks):
    # max_restarts=1: a new port range if the rendezvous port was taken (EADDRINUSE) in the
    # window between free_port_base's check and the bind; a protocol failure fails twice
    res = launch.launch_script([os.path.join(ROOT, "tests", "helpers", "peer_worker.py")], nproc=world,
                               env=_env(tmp_path, DAMD_PEER_BLOCKS=blocks), timeout=240, max_restarts=1)
    assert res.ok, res.returncodes
    rs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    for j in rs:
        assert j["ok"], "peer all-reduce could not be set up"
        assert j["errors"] == [], j["errors"]
        assert j["status"] == 0
    assert len({j["digest"] for j in rs}) == 1  # every rank holds the same result
    print(f"world {world}: {max(j['us_per_allreduce'] for j in rs):.1f} us per 1.39 MB all-reduce "
          "(ranks sharing one GPU)")


def _fused_run(tmp_path, name, world, init=None, **kw):
    worker = os.path.join(ROOT, "tests", "helpers", "dist_worker.py")
    d = tmp_path / name
    d.mkdir()
    env = dict(DAMD_TEST_PER_REPLICA=64 // world, DAMD_TEST_STEPS=8, DAMD_GRAPH_STEPS=5, **kw)
    if init is not None:
        env["DAMD_TEST_INIT_FROM"] = init
    res = launch.launch_script([worker], nproc=world, env=_env(d, **env), timeout=400)
    assert res.ok, (name, res.returncodes)
    runs = [([a for a in np.load(d / f"rank{r}.npz").values()], json.load(open(d / f"rank{r}.json")))
            for r in range(world)]
    w0, j0 = runs[0]
    assert j0["engine"] == "fused_convnet"
    for w, j in runs[1:]:  # mirrored replicas, identical History on every worker (README.md:229-231)
        assert all(np.array_equal(a, b) for a, b in zip(w0, w)), f"{name}: replicas diverged"
        assert j["history"] == j0["history"], name
    assert j0["iterations"] == 16
    return w0, j0, d


@pytest.mark.timeout(900)
def test_fused_exchanges_bitwise_equal_host_rank_order_reduction(tmp_path):
    """W = 2, 2 epochs x 8 momentum steps (graph replays, an epoch flush in between): the
    sharded exchange inside the step kernels, the standalone xGMI peer kernel, and the
    sharded exchange made to FAIL its start-up self-test (injected) -- which must fall back
    in process to the peer kernel before step 1 -- all end BITWISE equal (weights and
    History) to the host-gloo all-reduce: at W = 2 every transport computes a + b."""
    wh, jh, dh = _fused_run(tmp_path, "host", 2, DAMD_ALLREDUCE="off")
    assert jh["exchange"] == "host-gloo" and jh["exchange_verified"] is None, jh
    init = dh / "init0.npz"
    cases = {"sharded": dict(DAMD_ALLREDUCE="sharded"),
             "xgmi": dict(DAMD_ALLREDUCE="xgmi"),
             "injected": dict(DAMD_ALLREDUCE="auto", DAMD_XCHG_SELFTEST_INJECT="xgmi-sharded:1")}
    want = {"sharded": ("xgmi-sharded", []), "xgmi": ("xgmi-peer", []), "injected": ("xgmi-peer", ["xgmi-sharded"])}
    for name, kw in cases.items():
        w, j, _ = _fused_run(tmp_path, name, 2, init=init, **kw)
        kind, fb = want[name]
        assert j["exchange"] == kind and j["fallback_from"] == fb and j["exchange_verified"] is True, (name, j)
        for i, (a, b) in enumerate(zip(w, wh)):
            assert np.array_equal(a, b), (name, i, float(np.abs(a - b).max()))
        assert j["history"] == jh["history"], (name, j["history"], jh["history"])


@pytest.mark.timeout(900)
def test_fit_picks_the_measured_fastest_transport_and_bench_agrees(tmp_path):
    """README.md:398 "communication = CollectiveCommunication.AUTO": with the transport not
    pinned, fit() self-tests every candidate exchange and TIMES each passing one with the
    bench's window protocol (K steps + flush as one graph, engine/xchg_selftest.py), keeping
    the fastest; bench.py reports the same engine choice.  W = 2 sharing one GPU (no RCCL:
    the candidates are the sharded exchange and the peer kernel)."""
    w, j, _ = _fused_run(tmp_path, "auto", 2, DAMD_ALLREDUCE="auto")
    t = j["transport_us"]
    assert set(t) == {"xgmi-sharded", "xgmi-peer"}, t
    assert j["exchange"] == min(t, key=t.get), j
    assert j["exchange_verified"] is True
    import subprocess
    import sys

    port = launch.free_port_base(1)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--steps", "40", "--warmup", "10"], cwd=ROOT, capture_output=True, text=True, timeout=400,
                       env={**os.environ, **_env(tmp_path)})
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    print("fit:", t, "bench:", out.get("transport_ms_per_step"), out["allreduce"])
    assert out["allreduce"] == j["exchange"], (out, j)
    assert set(out["transport_ms_per_step"]) == set(t)
    assert out["control_collectives_in_window"] == 0 and out["exchange_verified"] is True


@pytest.mark.timeout(900)
def test_mid_run_exchange_fault_reruns_the_epoch_bitwise(tmp_path):
    """A bounded in-kernel exchange wait that expires AFTER a passing self-test (rank 1
    stalls 3 s before global step 5; the run's in-kernel deadline is 0.5 s): every rank
    votes at the epoch's end, fit() rebuilds the engine on the next transport from the
    epoch-start snapshot and re-runs the epoch -- no gang restart -- and the run ends
    BITWISE equal (weights, History) to the host-gloo all-reduce."""
    wh, jh, dh = _fused_run(tmp_path, "host", 2, DAMD_ALLREDUCE="off")
    w, j, _ = _fused_run(tmp_path, "fault", 2, init=dh / "init0.npz", DAMD_ALLREDUCE="auto",
                         DAMD_XCHG_FAULT_AT="1:5", DAMD_XCHG_TIMEOUT_S="0.5", DAMD_XCHG_FAULT_DELAY_S="3")
    assert any(f.endswith("(mid-run)") for f in j["fallback_from"]), j
    assert j["exchange"] in ("xgmi-sharded", "xgmi-peer") and j["exchange_verified"] is True, j
    for i, (a, b) in enumerate(zip(w, wh)):
        assert np.array_equal(a, b), (i, float(np.abs(a - b).max()))
    assert j["history"] == jh["history"], (j["history"], jh["history"])


@pytest.mark.timeout(600)
def test_fused_sharded_exchange_matches_single_rank(tmp_path):
    """world 2 x 32 rows == 1 rank x 64 rows (the same global batch), up to the grouping of
    the per-row gradient sums."""
    w0, j0, d2 = _fused_run(tmp_path, "wN", 2, DAMD_ALLREDUCE="sharded")
    w, j1, _ = _fused_run(tmp_path, "w1", 1, init=d2 / "init0.npz")
    # the 16-step weight UPDATES agree: the two runs differ only in how the per-row
    # gradients are grouped before the fp32 sums, and that 1-ulp fp32 noise flips some bf16
    # roundings of the activations, which the next steps carry on
    init = [a for a in np.load(d2 / "init0.npz").values()]
    for i, (a, b, w_0) in enumerate(zip(w0, w, init)):
        da, db = (a - w_0).ravel().astype(np.float64), (b - w_0).ravel().astype(np.float64)
        nb = np.linalg.norm(db)
        cos = float(da @ db / (np.linalg.norm(da) * nb + 1e-30))
        rel = float(np.linalg.norm(da - db) / nb)
        print(f"tensor {i}: update cos {cos:.5f} rel {rel:.4f}")
        assert cos > 0.995 and rel < 0.05, (i, cos, rel)
    for k in ("loss", "accuracy"):
        np.testing.assert_allclose(j0["history"][k], j1["history"][k], rtol=1e-3, atol=2e-3)


@pytest.mark.timeout(600)
def test_native_graph_peer_buckets_two_ranks_match_single_rank(tmp_path):
    """The native graph engine's bucketed, overlapped gradient all-reduce with two
    communicating ranks: a small ResNet, 4 buckets (DAMD_BUCKET_MB=0.05) each reduced by the
    xGMI peer kernel on the side stream as soon as backward has written it, inside the
    captured step.  Replicas bitwise mirrored, and the run is BITWISE equal (weights and
    History) to the same 2-rank run with the host-staged all-reduce: at W = 2 both compute
    a + b per element (fp32 addition commutes), with the same per-replica BN semantics, so a
    double-reduced, skipped or mis-tiled bucket cannot hide behind a tolerance."""
    worker = os.path.join(ROOT, "tests", "helpers", "dist_worker.py")
    common = dict(DAMD_TEST_MODEL="resnet_small", DAMD_TEST_STEPS=4, DAMD_TEST_ROWS=512, DAMD_FUSED=0,
                  DAMD_BUCKET_MB=0.05, DAMD_GRAPH_STEPS=2)
    d2 = tmp_path / "w2"
    d2.mkdir()
    res = launch.launch_script([worker], nproc=2, env=_env(d2, DAMD_ALLREDUCE="xgmi", DAMD_TEST_PER_REPLICA=32,
                                                          **common), timeout=400)
    assert res.ok, res.returncodes
    (w0, j0), (w1, j1) = [([a for a in np.load(d2 / f"rank{r}.npz").values()], json.load(open(d2 / f"rank{r}.json")))
                          for r in range(2)]
    assert j0["engine"] == "native_graph" and j0["exchange"] == "xgmi-peer-bucketed", j0
    assert all(np.array_equal(a, b) for a, b in zip(w0, w1)), "mirrored variables diverged"
    assert j0["history"] == j1["history"]
    dh = tmp_path / "wh"
    dh.mkdir()
    res = launch.launch_script([worker], nproc=2, env=_env(dh, DAMD_ALLREDUCE="off", DAMD_TEST_PER_REPLICA=32,
                                                          DAMD_TEST_INIT_FROM=d2 / "init0.npz", **common), timeout=400)
    assert res.ok, res.returncodes
    w = [a for a in np.load(dh / "rank0.npz").values()]
    jh = json.load(open(dh / "rank0.json"))
    assert jh["exchange"] == "host-gloo", jh
    for i, (a, b) in enumerate(zip(w0, w)):
        assert np.array_equal(a, b), (i, float(np.abs(a.astype(np.float64) - b).max()))
    assert j0["history"] == jh["history"], (j0["history"], jh["history"])
