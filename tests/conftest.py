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
    config.addinivalue_line("markers", "shared_trees: runs the library default for pendant sources "
                                       "(shared anchor trees) instead of the bit-exact exact_sources mode")


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


@pytest.fixture(autouse=True)
def exact_sources_env(request, monkeypatch):
    """The bit-exact parity suite pins spe_table_opts.exact_sources (every pruned
    pendant source on its own lane, so latencies are the path-order sums bit for
    bit) through the Python mirror (SPE_EXACT_SOURCES) and the topology shim
    (SHADOW_SPE_EXACT_SOURCES).  Tests marked `shared_trees` run the library default
    instead -- hosts on one anchor share its relaxation; routes exact, latency /
    reliability within 1e-12 relative (tests/test_gpu_shared_trees.py, the C4
    full-size check in tests/test_gpu_bench_configs.py)."""
    if request.node.get_closest_marker("shared_trees"):
        monkeypatch.delenv("SPE_EXACT_SOURCES", raising=False)
        monkeypatch.delenv("SHADOW_SPE_EXACT_SOURCES", raising=False)
        return
    monkeypatch.setenv("SPE_EXACT_SOURCES", "1")
    monkeypatch.setenv("SHADOW_SPE_EXACT_SOURCES", "1")
