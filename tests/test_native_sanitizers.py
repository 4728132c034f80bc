"""Host C++ under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 "race
detection / sanitizers"): the HDF5 tree writer/reader behind Keras checkpoints is built
as a standalone sanitized executable and run on a Keras-layout tree (write, read back,
byte-compare, failure paths).  Standalone, so no sanitizer runtime is injected into
the Python process."""
import os
import shutil
import subprocess

import pytest

from distributed_amd import _build


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
@pytest.mark.timeout(300)
def test_h5_tree_io_under_asan_ubsan(tmp_path):
    exe = _build.build_h5_selftest(tmp_path / "h5_selftest")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe), str(tmp_path / "t.h5")], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "h5 selftest OK" in r.stdout
    assert "runtime error" not in r.stderr  # UBSan reports
