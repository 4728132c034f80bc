"""Data parallelism on the GPU with several ranks sharing ONE MI355X (the pool's boxes
have a single GPU; RCCL refuses two ranks on one device, so these runs use
``DAMD_COMM=gloo``: the gradient/metric buffer is all-reduced through host memory
between steps).  Everything else — the fused HIP step kernels' row offsets, the
1/global_batch loss scaling, the metric tail, the deferred SGD, the init broadcast — is
the same code the RCCL path runs, so N-rank == 1-rank equivalence here validates the
multi-GPU semantics (reference README.md:363-392, 229-231)."""
import json
import os

import numpy as np
import pytest

from distributed_amd import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "helpers", "dist_worker.py")
pytestmark = [pytest.mark.gpu, pytest.mark.dist]


def _env(out, **kw):
    # DAMD_ALLREDUCE=off: the host-staged gloo all-reduce (the xGMI peer kernel has its own
    # tests in test_peer_allreduce_gpu.py)
    e = {"DAMD_DEVICE": "cuda:0", "DAMD_COMM": "gloo", "DAMD_ALLREDUCE": "off", "DAMD_TEST_OUT": str(out), "PYTHONPATH": ROOT,
         "OMP_NUM_THREADS": "2", "DAMD_LOG_LEVEL": "WARNING"}
    e.update({k: str(v) for k, v in kw.items()})
    return e


def _load(out, r):
    w = [a for a in np.load(os.path.join(out, f"rank{r}.npz")).values()]
    with open(os.path.join(out, f"rank{r}.json")) as f:
        return w, json.load(f)


@pytest.mark.parametrize("engine", ["fused", "native_graph", "generic"])
@pytest.mark.timeout(600)
def test_two_ranks_one_gpu_match_single_rank(tmp_path, engine):
    fused = "1" if engine == "fused" else "0"
    ng = "1" if engine == "native_graph" else "0"
    d2 = tmp_path / "w2"
    d2.mkdir()
    res = launch.launch_script([WORKER], nproc=2, env=_env(d2, DAMD_TEST_PER_REPLICA=32, DAMD_FUSED=fused,
                                                           DAMD_NATIVE_GRAPH=ng),
                               timeout=420)
    assert res.ok, res.returncodes
    (w0, j0), (w1, j1) = _load(d2, 0), _load(d2, 1)
    assert j0["world"] == 2 and j0["engine"] == j1["engine"]
    assert j0["engine"] == {"fused": "fused_convnet", "native_graph": "native_graph", "generic": "generic"}[engine]
    assert all(np.array_equal(a, b) for a, b in zip(w0, w1)), "mirrored variables diverged"
    assert j0["history"] == j1["history"]
    d1 = tmp_path / "w1"
    d1.mkdir()
    res = launch.launch_script([WORKER], nproc=1, env=_env(d1, DAMD_TEST_PER_REPLICA=64, DAMD_FUSED=fused, DAMD_NATIVE_GRAPH=ng,
                                                           DAMD_TEST_INIT_FROM=d2 / "init0.npz"), timeout=420)
    assert res.ok, res.returncodes
    ws, js = _load(d1, 0)
    tol = {"generic": dict(rtol=1e-3, atol=1e-5), "fused": dict(rtol=2e-3, atol=2e-4),
           "native_graph": dict(rtol=5e-3, atol=5e-4)}[engine]
    for a, b in zip(w0, ws):
        np.testing.assert_allclose(a, b, **tol)
    np.testing.assert_allclose(j0["history"]["loss"], js["history"]["loss"], rtol=1e-3)
    np.testing.assert_allclose(j0["history"]["accuracy"], js["history"]["accuracy"], atol=1.5 / 64)


def test_strategy_reduce_world1_gpu():
    """World 1 on a GPU runs a size-1 RCCL communicator with no process group: host-value
    reduce must not reach torch.distributed."""
    import distributed_amd as tf
    from distributed_amd.parallel import runtime

    runtime.shutdown()
    s = tf.distribute.experimental.MultiWorkerMirroredStrategy()
    try:
        assert s.num_replicas_in_sync == 1 and s.device.type == "cuda"
        assert s.reduce("sum", [1.0, 2.0]).tolist() == [1.0, 2.0]
        assert s.reduce("mean", [[1.0, 3.0]], axis=1).tolist() == [2.0]
    finally:
        runtime.shutdown()
