import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the native extension")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "dist: spawns multiple processes (gloo)")


@pytest.fixture(autouse=True)
def _fresh_names():
    from distributed_amd.keras import backend

    backend.clear_session()
    yield
