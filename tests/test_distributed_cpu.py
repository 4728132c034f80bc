"""Multi-process data parallelism on CPU (gloo), launched like the reference's workers:
one process per worker, TF_CONFIG per rank (README.md:84-113, 319-357)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from distributed_amd import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "helpers", "dist_worker.py")
pytestmark = pytest.mark.dist


def _env(out, **kw):
    e = {"DAMD_DEVICE": "cpu", "DAMD_TEST_OUT": str(out), "PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2",
         "DAMD_LOG_LEVEL": "WARNING"}
    e.update({k: str(v) for k, v in kw.items()})
    return e


def _load(out, r):
    w = [a for a in np.load(os.path.join(out, f"rank{r}.npz")).values()]
    with open(os.path.join(out, f"rank{r}.json")) as f:
        return w, json.load(f)


@pytest.mark.timeout(300)
def test_two_workers_mirror_and_match_single_worker(tmp_path):
    d2 = tmp_path / "w2"
    d2.mkdir()
    # small buckets: 3 asynchronous all-reduces per step overlapped with backward
    res = launch.launch_script([WORKER], nproc=2, env=_env(d2, DAMD_TEST_PER_REPLICA=16, DAMD_CHECK_MIRRORS=1,
                                                           DAMD_TEST_DIVERGE=1, DAMD_BUCKET_MB=0.05), timeout=240)
    assert res.ok, res.returncodes
    (w0, j0), (w1, j1) = _load(d2, 0), _load(d2, 1)
    assert j0["world"] == j1["world"] == 2
    # mirrored variables: bitwise identical on every worker (init broadcast + same all-reduced grads)
    assert all(np.array_equal(a, b) for a, b in zip(w0, w1))
    # global metrics: identical History on every worker (README.md:229-231)
    assert j0["history"] == j1["history"]
    assert j0["iterations"] == 6
    # the mirror-divergence detector ran every epoch inside fit (no error) and catches a
    # 1e-6 perturbation of one replica's bias
    for r in (0, 1):
        assert open(d2 / f"diverge{r}.txt").read() == "detected"
    # N-worker DP at global batch B == 1 worker at batch B from the same initial weights
    d1 = tmp_path / "w1"
    d1.mkdir()
    res = launch.launch_script([WORKER], nproc=1, env=_env(d1, DAMD_TEST_PER_REPLICA=32,
                                                           DAMD_TEST_INIT_FROM=d2 / "init0.npz"), timeout=240)
    assert res.ok, res.returncodes
    ws, js = _load(d1, 0)
    for a, b in zip(w0, ws):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(j0["history"]["loss"], js["history"]["loss"], rtol=1e-5)


@pytest.mark.timeout(600)
def test_eight_workers_mirror_and_match_single_worker(tmp_path):
    """BASELINE configs 3 / 5 run 8 ranks: 8 workers x 8 rows per step == 1 worker x 64 rows
    from the same initial weights; replicas bitwise mirrored, History identical on all 8
    (README.md:229-231), rank-order sums over 8 ranks, ports base..base+7."""
    d8 = tmp_path / "w8"
    d8.mkdir()
    res = launch.launch_script([WORKER], nproc=8, env=_env(d8, DAMD_TEST_PER_REPLICA=8, DAMD_CHECK_MIRRORS=1,
                                                           DAMD_BUCKET_MB=0.05, OMP_NUM_THREADS=1), timeout=400)
    assert res.ok, res.returncodes
    outs = [_load(d8, r) for r in range(8)]
    w0, j0 = outs[0]
    assert j0["world"] == 8 and j0["iterations"] == 6
    for w, j in outs[1:]:
        assert all(np.array_equal(a, b) for a, b in zip(w0, w))
        assert j["history"] == j0["history"]
    d1 = tmp_path / "w1"
    d1.mkdir()
    res = launch.launch_script([WORKER], nproc=1, env=_env(d1, DAMD_TEST_PER_REPLICA=64,
                                                           DAMD_TEST_INIT_FROM=d8 / "init0.npz"), timeout=240)
    assert res.ok, res.returncodes
    ws, js = _load(d1, 0)
    for a, b in zip(w0, ws):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(j0["history"]["loss"], js["history"]["loss"], rtol=1e-5)


@pytest.mark.timeout(300)
def test_short_last_batch_with_many_buckets(tmp_path):
    """70 rows at global batch 64: the second step has 6 rows, all on rank 0, so rank 1
    has no rows but must issue the same per-bucket all-reduce sequence (tiny buckets:
    one per parameter).  Replicas stay mirrored and match one worker at batch 64."""
    d2 = tmp_path / "w2"
    d2.mkdir()
    res = launch.launch_script([WORKER], nproc=2, env=_env(d2, DAMD_TEST_PER_REPLICA=32, DAMD_TEST_ROWS=70,
                                                           DAMD_TEST_STEPS=0, DAMD_BUCKET_MB=0.001), timeout=240)
    assert res.ok, res.returncodes
    (w0, j0), (w1, j1) = _load(d2, 0), _load(d2, 1)
    assert all(np.array_equal(a, b) for a, b in zip(w0, w1))
    assert j0["history"] == j1["history"]
    assert j0["iterations"] == 4  # 2 epochs x ceil(70 / 64) steps
    d1 = tmp_path / "w1"
    d1.mkdir()
    res = launch.launch_script([WORKER], nproc=1, env=_env(d1, DAMD_TEST_PER_REPLICA=64, DAMD_TEST_ROWS=70,
                                                           DAMD_TEST_STEPS=0, DAMD_TEST_INIT_FROM=d2 / "init0.npz"),
                               timeout=240)
    assert res.ok, res.returncodes
    ws, js = _load(d1, 0)
    for a, b in zip(w0, ws):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(j0["history"]["loss"], js["history"]["loss"], rtol=1e-5)


def _reduce_fn(df, barrier):
    import json as _json
    import os as _os

    _os.environ["DAMD_DEVICE"] = "cpu"
    _os.environ["TF_CONFIG"] = _json.dumps({"cluster": {"worker": barrier["address"]},
                                            "task": {"type": "worker", "index": barrier["partition"]}})
    import distributed_amd as tf
    from distributed_amd.parallel import runtime

    s = tf.distribute.experimental.MultiWorkerMirroredStrategy()
    r = s.rank
    v = [[r + 1.0, 10.0 * r], [2.0, -r - 1.0]]
    out = {k: s.reduce(k, v).tolist() for k in ("sum", "mean", "max", "min")}
    out["mean_axis0"] = s.reduce(tf.distribute.ReduceOp.MEAN, v, axis=0).tolist()
    out["max_axis1"] = s.reduce("max", v, axis=1).tolist()
    runtime.shutdown()
    return out


def test_strategy_reduce_two_ranks():
    a, b = launch.barrier_apply(_reduce_fn, 2, on_error="raise")
    assert a == b
    assert a["sum"] == [[3.0, 10.0], [4.0, -3.0]]
    assert a["mean"] == [[1.5, 5.0], [2.0, -1.5]]
    assert a["max"] == [[2.0, 10.0], [2.0, -1.0]]
    assert a["min"] == [[1.0, 0.0], [2.0, -2.0]]
    # mean over both rows of both replicas: col0 (1+2+2+2)/4, col1 (0-1+10-2)/4
    assert a["mean_axis0"] == [1.75, 1.75]
    assert a["max_axis1"] == [10.0, 2.0]


def _ranked(df, barrier):
    import os as _os

    return f"{barrier['partition']}/{len(barrier['address'])}/{_os.environ['DAMD_LOCAL_RANK']}"


def _fails_on_1(df, barrier):
    if barrier["partition"] == 1:
        raise ValueError("boom")
    return "ok"


def _crash_first_attempt(df, barrier):
    import os as _os

    if barrier["partition"] == 0 and _os.environ.get("DAMD_RESTART_COUNT") == "0":
        _os._exit(3)  # hard crash of one task: the whole gang must be retried
    return int(_os.environ["DAMD_RESTART_COUNT"])


def test_barrier_apply_order_and_error_strings():
    out = launch.barrier_apply(_ranked, 3)
    assert out == ["0/3/0", "1/3/1", "2/3/2"]
    out = launch.barrier_apply(_fails_on_1, 3)  # tryCatch contract (README.md:176, 221)
    assert out[0] == "ok" and out[2] == "ok" and out[1] == "ValueError: boom"
    with pytest.raises(RuntimeError):
        launch.barrier_apply(_fails_on_1, 2, on_error="raise")


def test_barrier_apply_gang_restart():
    assert launch.barrier_apply(_crash_first_attempt, 2, max_restarts=1) == [1, 1]
    # at the deployment size (BASELINE config 5: 8 local ranks): one task's crash restarts
    # all 8, and every task of the second attempt reports it
    assert launch.barrier_apply(_crash_first_attempt, 8, max_restarts=1) == [1] * 8
    with pytest.raises(RuntimeError):
        launch.barrier_apply(_crash_first_attempt, 2, max_restarts=0)


def test_launcher_cli_gang_restart(tmp_path):
    script = tmp_path / "flaky.py"
    script.write_text(
        "import os, sys\n"
        "if os.environ['DAMD_LOCAL_RANK'] == '1' and os.environ['DAMD_RESTART_COUNT'] == '0': sys.exit(7)\n"
        "import json; c = json.loads(os.environ['TF_CONFIG'])\n"
        "open(os.path.join(%r, 'r%%s' %% c['task']['index']), 'w').write(os.environ['DAMD_RESTART_COUNT'])\n"
        % str(tmp_path))
    r = subprocess.run([sys.executable, "-m", "distributed_amd.launch", "--nproc", "2", "--max-restarts", "1",
                        str(script)], cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env={**os.environ, "PYTHONPATH": ROOT})
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "r0").read_text() == "1" and (tmp_path / "r1").read_text() == "1"
    r = subprocess.run([sys.executable, "-m", "distributed_amd.launch", "--nproc", "2", str(script)], cwd=ROOT,
                       capture_output=True, text=True, timeout=120, env={**os.environ, "PYTHONPATH": ROOT})
    assert r.returncode == 1 and "failed" in r.stderr


def _spark_closure(df, barrier):
    """The README's Spark closure (README.md:175-221), transliterated."""
    import os as _os

    _os.environ["DAMD_DEVICE"] = "cpu"
    _os.environ["OMP_NUM_THREADS"] = "2"
    try:
        from distributed_amd import r_api as k
        import distributed_amd as tf

        k.sys_setenv(TF_CONFIG=k.barrier_tf_config(barrier, base_port=int(_os.environ["SPARK_PORT_BASE"])))
        if k.tf_version() is None:
            k.install_tensorflow()
        strategy = tf.distribute.experimental.MultiWorkerMirroredStrategy()
        num_workers = 3
        batch_size = 64 * num_workers
        mnist = k.dataset_mnist()
        x_train = k.array_reshape(mnist["train"]["x"][:2048], k.c(2048, 28, 28, 1)) / 255
        y_train = mnist["train"]["y"][:2048]
        with strategy.scope():
            model = k.keras_model_sequential()
            k.layer_conv_2d(model, filters=32, kernel_size=3, activation="relu", input_shape=k.c(28, 28, 1))
            k.layer_max_pooling_2d(model)
            k.layer_flatten(model)
            k.layer_dense(model, units=64, activation="relu")
            k.layer_dense(model, units=10)
            k.compile(model, loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tf.keras.optimizers.SGD(learning_rate=0.001), metrics="accuracy")
        result = k.fit(model, x_train, y_train, batch_size=batch_size, epochs=3, steps_per_epoch=5, verbose=0)
        return str(max(result.metrics["accuracy"]))
    except Exception as e:  # error = function(e) e$message
        return str(e)


def _spark_closure_derived_world(df, barrier):
    """The README closure with the world size taken from the barrier (never
    hard-code num_workers), a smaller slice of rows, and the partition index returned."""
    import os as _os

    _os.environ["DAMD_DEVICE"] = "cpu"
    _os.environ["OMP_NUM_THREADS"] = "1"
    from distributed_amd import r_api as k
    import distributed_amd as tf

    k.sys_setenv(TF_CONFIG=k.barrier_tf_config(barrier, base_port=int(_os.environ["SPARK_PORT_BASE"])))
    strategy = tf.distribute.experimental.MultiWorkerMirroredStrategy()
    num_workers = len(barrier["address"])
    mnist = k.dataset_mnist()
    x_train = k.array_reshape(mnist["train"]["x"][:1024], k.c(1024, 28, 28, 1)) / 255
    y_train = mnist["train"]["y"][:1024]
    with strategy.scope():
        model = k.keras_model_sequential()
        k.layer_conv_2d(model, filters=32, kernel_size=3, activation="relu", input_shape=k.c(28, 28, 1))
        k.layer_max_pooling_2d(model)
        k.layer_flatten(model)
        k.layer_dense(model, units=64, activation="relu")
        k.layer_dense(model, units=10)
        k.compile(model, loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tf.keras.optimizers.SGD(learning_rate=0.001), metrics="accuracy")
    result = k.fit(model, x_train, y_train, batch_size=64 * num_workers, epochs=2, steps_per_epoch=2, verbose=0)
    return f"{barrier['partition']}/{strategy.num_replicas_in_sync}/{max(result.metrics['accuracy'])!r}"


@pytest.mark.timeout(600)
def test_spark_apply_eight_partitions_in_order(monkeypatch):
    """BASELINE config 5: spark_apply(barrier=TRUE) over sdf_len(8) -> 8 rows, in partition
    order, every rank training at world 8 and reporting the identical global accuracy."""
    monkeypatch.setenv("SPARK_PORT_BASE", str(launch.free_port_base(9)))
    sdf = launch.sdf_len(8, repartition=8)
    rows = launch.collect(launch.spark_apply(sdf, _spark_closure_derived_world, barrier=True,
                                             columns={"address": "character"}, timeout=500))
    assert len(rows) == 8
    vals = [r["address"] for r in rows]
    parts = [v.split("/") for v in vals]
    assert [int(p[0]) for p in parts] == list(range(8)), vals
    assert all(p[1] == "8" for p in parts), vals
    assert len({p[2] for p in parts}) == 1, vals


@pytest.mark.timeout(300)
def test_spark_apply_barrier_readme_closure(monkeypatch):
    monkeypatch.setenv("SPARK_PORT_BASE", str(launch.free_port_base(4)))
    sdf = launch.sdf_len(3, repartition=3)
    rows = launch.collect(launch.spark_apply(sdf, _spark_closure, barrier=True, columns={"address": "character"},
                                             timeout=240))
    assert len(rows) == 3
    vals = [r["address"] for r in rows]
    # every worker reports the identical (global) accuracy, like README.md:229-231
    assert len(set(vals)) == 1, vals
    assert 0.0 <= float(vals[0]) <= 1.0


def test_bench_two_ranks_cpu(tmp_path):
    """bench.py's multi-rank contract on CPU/gloo (torch.distributed.run, 127.0.0.1)."""
    port = launch.free_port_base(1)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--steps", "3", "--warmup", "1", "--engine", "generic"], cwd=ROOT, capture_output=True,
                       text=True, timeout=300,
                       env={**os.environ, "DAMD_DEVICE": "cpu", "OMP_NUM_THREADS": "2", "PYTHONPATH": ROOT})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 128 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and out["steps"] == 3 and out["scaling"] == "weak"


@pytest.mark.timeout(400)
def test_injected_failure_gang_restart_resumes_from_backup(tmp_path):
    """Rank 1 dies mid-epoch-3 on the first attempt (DAMD_FAIL_AT=1:7:0); the launcher
    restarts the gang, BackupAndRestore resumes after epoch 2, and the final weights equal
    an uninterrupted run's (README.md:400 "Workers will need to restart training")."""
    ft = os.path.join(ROOT, "tests", "helpers", "ft_worker.py")
    ref = tmp_path / "ref"
    ref.mkdir()
    res = launch.launch_script([ft], nproc=2, env=_env(ref), timeout=240)
    assert res.ok, res.returncodes
    run = tmp_path / "ft"
    run.mkdir()
    res = launch.launch_script([ft], nproc=2, env=_env(run, DAMD_FAIL_AT="1:7:0"), timeout=240, max_restarts=1)
    assert res.ok, res.returncodes
    w_ref, j_ref = _load(ref, 0)
    w_ft, j_ft = _load(run, 0)
    assert j_ft["attempt"] == 1 and j_ref["attempt"] == 0
    assert j_ft["iterations"] == j_ref["iterations"] == 12
    for a, b in zip(w_ft, w_ref):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)
    # the resumed attempt trained epochs 3-4 only
    assert len(j_ft["history"]["loss"]) == 2
    np.testing.assert_allclose(j_ft["history"]["loss"], j_ref["history"]["loss"][2:], rtol=1e-6)


@pytest.mark.timeout(120)
def test_rccl_communicator_bootstrap_two_ranks(tmp_path):
    """The RCCL world>1 path up to communicator construction: rank 0's ncclUniqueId is
    broadcast over the gloo control plane (TF_CONFIG rendezvous) to every rank, which then
    calls ncclCommInitRank on its own device (here: no device, so it stops at hipSetDevice)."""
    worker = os.path.join(ROOT, "tests", "helpers", "rccl_bootstrap_worker.py")
    res = launch.launch_script([worker], nproc=2, env=_env(tmp_path), timeout=100)
    assert res.ok, res.returncodes
    outs = [json.load(open(tmp_path / f"rccl{r}.json")) for r in (0, 1)]
    assert outs[0]["uid"] and outs[0]["uid"] == outs[1]["uid"] and len(outs[0]["uid"]) == 256
    for o in outs:
        if o["status"] == "constructed":
            assert o["comm_count"] == 2
        else:
            assert "hipSetDevice" in o["error"] or "device" in o["error"].lower(), o["error"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("epoch_sync", [True, False])
def test_batchnorm_moving_stats_are_replica_mean(tmp_path, epoch_sync):
    """BN moving statistics under MWMS (reference README.md:134-151: variables created in
    scope are mirrored; TF makes BN statistics SyncOnRead / MEAN).  Ranks see different
    data, so their local statistics differ; after fit every replica holds the replica
    mean, and the mirror check over ALL variables (statistics included) passes."""
    worker = os.path.join(ROOT, "tests", "helpers", "bn_worker.py")
    # without the epoch-end sync the in-fit mirror check would (rightly) raise: skip it there
    extra = {"DAMD_CHECK_MIRRORS": 1} if epoch_sync else {"DAMD_BN_SYNC": "0"}
    res = launch.launch_script([worker], nproc=2, env=_env(tmp_path, **extra), timeout=240)
    assert res.ok, res.returncodes
    outs = [json.load(open(tmp_path / f"bn{r}.json")) for r in (0, 1)]
    assert outs[0]["n_stats"] == 4
    assert outs[0]["fingerprint"] == outs[1]["fingerprint"]
    w0 = list(np.load(tmp_path / "bn0.npz").values())
    w1 = list(np.load(tmp_path / "bn1.npz").values())
    assert all(np.array_equal(a, b) for a, b in zip(w0, w1))
    if not epoch_sync:
        assert outs[0]["differed"], "per-rank statistics should differ before the sync"
        assert outs[0]["max_err"] < 1e-6


@pytest.mark.timeout(300)
def test_watchdog_turns_a_hung_rank_into_a_gang_restart(tmp_path):
    """Rank 1 stops responding in the middle of epoch 3 (first attempt only).  Rank 0 blocks
    in the gradient all-reduce; its collective watchdog fires after DAMD_WATCHDOG_S, exits
    with status 75, the launcher kills the gang and restarts it, and BackupAndRestore
    resumes from the epoch-2 backup: the result equals an uninterrupted run."""
    from distributed_amd.utils.watchdog import EXIT_CODE

    ft = os.path.join(ROOT, "tests", "helpers", "ft_worker.py")
    ref = tmp_path / "ref"
    ref.mkdir()
    res = launch.launch_script([ft], nproc=2, env=_env(ref), timeout=240)
    assert res.ok, res.returncodes
    run = tmp_path / "hang"
    run.mkdir()
    attempts = []
    res = launch.launch_script([ft], nproc=2, env=_env(run, DAMD_HANG_AT="1:7:0", DAMD_WATCHDOG_S=4), timeout=240,
                               max_restarts=1, on_failure=lambda rcs: attempts.append(list(rcs)))
    assert res.ok, res.returncodes
    assert res.attempts == 2
    assert EXIT_CODE in attempts[0], attempts  # the watchdog, not the launcher's timeout, ended attempt 1
    w_ref, j_ref = _load(ref, 0)
    w_h, j_h = _load(run, 0)
    assert j_h["attempt"] == 1 and j_h["iterations"] == j_ref["iterations"] == 12
    for a, b in zip(w_h, w_ref):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)
    assert len(j_h["history"]["loss"]) == 2  # resumed at epoch 3


def test_watchdog_unit():
    from distributed_amd.utils.watchdog import Watchdog

    fired, aborted = [], []
    wd = Watchdog(0.3, on_expire=fired.append)
    wd.add_abort(lambda: aborted.append(1))
    wd.arm("unit")
    for _ in range(6):  # beats keep it quiet
        import time as _t

        _t.sleep(0.1)
        wd.beat()
    assert not fired
    import time as _t

    _t.sleep(1.0)
    assert fired and aborted == [1] and "unit" in fired[0]
    wd.close()


def test_watchdog_beats_on_device_completion_not_enqueue():
    """A chunk whose device work never completes (a wedged collective: its event never
    signals) stops the beats even though the host enqueued it; the watchdog fires one
    deadline after the last COMPLETED chunk and names it."""
    import time as _t

    from distributed_amd.utils.watchdog import Watchdog

    class Ev:  # stand-in for torch.cuda.Event: query() is True once the work finished
        def __init__(self, done):
            self.done = done

        def query(self):
            return self.done

    fired = []
    wd = Watchdog(0.5, on_expire=fired.append, poll_s=0.05)
    wd.arm("start")
    late = Ev(False)
    wd.beat_when_done(Ev(True), "chunk 1")
    wd.beat_when_done(late, "chunk 2")
    _t.sleep(0.3)
    late.done = True  # chunk 2 completes late but within the deadline: a beat
    _t.sleep(0.3)
    assert not fired and wd._phase == "chunk 2"
    t0 = _t.monotonic()
    wd.beat_when_done(Ev(False), "chunk 3")  # enqueued, never completes
    while not fired and _t.monotonic() - t0 < 5:
        _t.sleep(0.02)
    assert fired and "'chunk 2'" in fired[0], fired
    assert _t.monotonic() - t0 < 0.5 + 0.3  # deadline (from chunk 2's completion) + a poll
    wd.close()


@pytest.mark.timeout(200)
def test_step_phases_include_the_allreduce_share(tmp_path):
    """bench.py --phases on 2 gloo ranks: forward / backward / all-reduce / optimizer times
    of the generic engine, reported next to the throughput."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TF_CONFIG", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["DAMD_DEVICE"] = "cpu"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--engine", "generic",
                        "--steps", "2", "--warmup", "1", "--phases", "3"], cwd=str(tmp_path), env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    ph = out["phases_ms"]
    for k in ("forward", "backward", "allreduce", "optimizer", "step"):
        assert ph[k] >= 0, ph
    assert ph["forward"] > 0 and ph["backward"] > 0
    assert abs(ph["step"] - (ph["forward"] + ph["backward"] + ph["allreduce"] + ph["optimizer"])) < 1e-3
