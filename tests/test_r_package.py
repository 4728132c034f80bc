"""The R front-end (R/): structure checks that run without R, and the package's testthat
suite when Rscript + reticulate are present (they are not in this image, so that part
is skipped; the verbs themselves are covered through distributed_amd.r_api)."""
import json
import os
import re
import shutil
import subprocess

import pytest

from distributed_amd import r_api

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RPKG = os.path.join(ROOT, "R")


def _read(*p):
    with open(os.path.join(RPKG, *p)) as f:
        return f.read()


def test_description_and_namespace():
    desc = _read("DESCRIPTION")
    assert re.search(r"^Package: distributedamd$", desc, re.M)
    assert "reticulate" in desc
    exports = re.findall(r"^export\(\"?([^\")]+)\"?\)", _read("NAMESPACE"), re.M)
    # every verb used by the reference R snippets (README.md:46-75, 119-153, 171-247)
    for verb in ["tf", "tf_version", "install_tensorflow", "dataset_mnist", "array_reshape", "keras_model_sequential",
                 "layer_conv_2d", "layer_max_pooling_2d", "layer_flatten", "layer_dense", "compile", "fit",
                 "save_model_hdf5", "base64encode", "base64decode", "sdf_len", "spark_apply", "collect", "%>%"]:
        assert verb in exports, verb


def test_every_python_call_exists_in_r_api():
    src = "".join(_read("R", f) for f in os.listdir(os.path.join(RPKG, "R")) if f.endswith(".R"))
    called = set(re.findall(r"\.r\(\)\$([A-Za-z_0-9]+)\(", src))
    assert called, "no r_api calls found"
    missing = [c for c in sorted(called) if not hasattr(r_api, c)]
    assert not missing, missing


@pytest.mark.skipif(shutil.which("Rscript") is None, reason="R is not installed in this image")
def test_testthat_suite():  # pragma: no cover - needs R
    r = subprocess.run(["Rscript", "-e", f"testthat::test_dir('{RPKG}/tests/testthat', load_package='source')"],
                       capture_output=True, text=True, timeout=900, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stdout + r.stderr


# ---- the R spark_apply launch path, through its Python gang launcher ---------------------
def _shim_stage(tmp_path, behaviour, mode="return", max_restarts=0, n=3):
    import sys

    from distributed_amd import launch

    d = tmp_path / f"stage-{behaviour}-{mode}"
    d.mkdir()
    (d / "addresses.txt").write_text("\n".join(f"127.0.0.1:{8101 + i}" for i in range(n)))
    shim = os.path.join(os.path.dirname(__file__), "helpers", "r_runner_shim.py")
    fails = []
    gang = launch.launch_command([sys.executable, shim, str(d), mode], nproc=n, max_restarts=max_restarts,
                                 timeout=60, rank_arg=True, env={"DAMD_SHIM_BEHAVIOUR": behaviour},
                                 on_failure=lambda rcs: fails.append(rcs))
    res = [json.load(open(d / f"result-{i}.json")) for i in range(n)] if gang.ok else None
    return gang, res, fails


def test_r_barrier_stage_results_in_partition_order(tmp_path):
    gang, res, fails = _shim_stage(tmp_path, "ok")
    assert gang.ok and gang.attempts == 1 and not fails
    assert [r["value"] for r in res] == ["0/3/attempt0", "1/3/attempt0", "2/3/attempt0"]


def test_r_barrier_stage_kills_survivors_and_restarts(tmp_path):
    """Rank 1 crashes while rank 0 hangs: the crash is seen from its exit status (not a
    result-file timeout), rank 0 is killed, and the gang restarts as a whole."""
    import time

    t0 = time.time()
    gang, res, fails = _shim_stage(tmp_path, "crash1+hang0", max_restarts=1)
    assert gang.ok and gang.attempts == 2
    assert time.time() - t0 < 30  # far below the 60 s stage timeout
    assert len(fails) == 1 and fails[0][1] == 9 and fails[0][0] != 0  # survivor killed
    assert [r["value"] for r in res] == ["0/3/attempt1", "1/3/attempt1", "2/3/attempt1"]


def test_r_barrier_stage_error_contract(tmp_path):
    # on_error = "return": the error message is the partition's value (tryCatch contract)
    gang, res, _ = _shim_stage(tmp_path, "error1")
    assert gang.ok and res[1] == {"ok": False, "value": "boom in partition 1"} and res[0]["ok"]
    # on_error = "restart": an R error fails the gang like a crash
    gang, _, fails = _shim_stage(tmp_path, "error1", mode="restart", max_restarts=1)
    assert not gang.ok and gang.attempts == 2 and all(3 in f for f in fails)


def test_r_spark_apply_uses_the_gang_launcher():
    src = open(os.path.join(os.path.dirname(os.path.dirname(__file__)), "R", "R", "cluster.R")).read()
    assert "launch$launch_command(" in src and "rank_arg = TRUE" in src
    assert "tryCatch(list(ok = TRUE" in src and "status = 3" in src
