"""The in-tree ``_C`` carries the hash of the sources it was built from, and the loader
refuses a module whose hash does not match the tree's ``csrc/`` (a stale
pushed binary must not run silently)."""
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

from distributed_amd import _build, native

ROOT = Path(__file__).resolve().parents[1]
SO = _build.PKG / f"_C{_build.EXT}"

pytestmark = pytest.mark.skipif(not SO.exists(), reason="_C not built")


def test_built_module_matches_tree():
    assert _build.embedded_hash(SO) == _build.source_hash()
    native.check_fresh()  # no raise


def test_touched_hip_source_is_refused(tmp_path):
    csrc = tmp_path / "csrc"
    shutil.copytree(_build.CSRC, csrc)
    native.check_fresh(SO, csrc)  # an identical copy: still fresh
    k = csrc / "kernels" / "gemm.hip"
    k.write_text(k.read_text() + "\n// touched\n")
    with pytest.raises(native.StaleExtensionError, match="other sources"):
        native.check_fresh(SO, csrc)
    # the loader itself refuses (no rebuild: build_if_missing=False), before importing
    code = ("import distributed_amd.native as n\n"
            "try:\n    n.load_C(build_if_missing=False)\nexcept n.StaleExtensionError as e:\n"
            "    print('REFUSED', e)\nelse:\n    print('LOADED')\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=str(ROOT), capture_output=True, text=True, timeout=120,
                       env={**os.environ, "DAMD_CSRC_ROOT": str(csrc), "PYTHONPATH": str(ROOT)})
    assert "REFUSED" in r.stdout, (r.stdout, r.stderr[-2000:])
    r = subprocess.run([sys.executable, "-c", code], cwd=str(ROOT), capture_output=True, text=True, timeout=120,
                       env={**os.environ, "DAMD_CSRC_ROOT": str(csrc), "DAMD_ALLOW_STALE": "1",
                            "PYTHONPATH": str(ROOT)})
    assert "LOADED" in r.stdout, (r.stdout, r.stderr[-2000:])
