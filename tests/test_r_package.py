"""The R front-end (R/): structure checks that run without R, and the package's testthat
suite when Rscript + reticulate are present (they are not in this image, so that part
is skipped; the verbs themselves are covered through distributed_amd.r_api)."""
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
