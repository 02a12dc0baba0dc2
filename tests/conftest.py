import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libspe.so")
    config.addinivalue_line("markers", "slow: larger CPU-side cases")
    config.addinivalue_line("markers", "engine_fixed: GPU test that selects its path engine itself")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(params=["1", "2"], ids=["batch", "lds"], autouse=True)
def engine_env(request, monkeypatch):
    """Every GPU test runs on both path engines (SPE_ENGINE: 1 = 64-lane batch
    relaxation, 2 = LDS-resident per-source rows; the LDS engine falls back to
    batch when the graph does not fit).  CPU tests run once."""
    if request.node.get_closest_marker("gpu") is None or request.node.get_closest_marker("engine_fixed"):
        if request.param == "2":
            pytest.skip("engine-independent test (CPU, or picks its engine itself)")
        return
    monkeypatch.setenv("SPE_ENGINE", request.param)
