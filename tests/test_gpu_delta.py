"""GPU parity of the batch engine's experimental Delta-stepping schedule
(SPE_DELTA=<ms>, MEASUREMENTS.md): each lane group relaxes only offers below its
bucket bound, parks rows with larger offers and rescans them when its bound
advances.  The fixpoint is the same, so the rows must equal the oracle's bit for
bit at both relaxation widths (64 and 128 sources per row), on tie-free, pendant,
directed, vertex-loss and hub-heavy (in-degree > 64, relaxed by the same kernel
in this schedule) graphs."""
import numpy as np
import pytest

from oracle import Oracle
from shadow_amd import graphs

pytestmark = [pytest.mark.gpu, pytest.mark.engine_fixed]


@pytest.fixture(scope="module")
def spe():
    from shadow_amd import spe as m
    assert m.device_count() > 0, "no GPU visible"
    return m


def compare(gpu, ora, label):
    ok = ora["kind"] != 0
    np.testing.assert_array_equal(gpu["ok"], ok, err_msg=f"{label}: routability")
    for k in ("lat", "rel", "next", "hops"):
        a, b = gpu[k][ok], ora[k][ok]
        bad = np.flatnonzero(a != b)
        assert bad.size == 0, f"{label}: {k} differs at {bad.size} entries"


CASES = {
    "undirected_tiefree": lambda: graphs.gen_random_small(700, 2100, 31),
    "directed_tiefree": lambda: graphs.gen_random_small(500, 1500, 32, directed=True),
    "sparse_tree_like": lambda: graphs.gen_random_small(900, 60, 33),
    "vertex_loss": lambda: graphs.gen_random_small(400, 1200, 34, vloss_nonzero=True),
    "ba_hubs": lambda: graphs.gen_ba(3000, 3, seed=11),
}


@pytest.mark.parametrize("lanes", [64, 128])
@pytest.mark.parametrize("delta", [2.0, 25.0])
@pytest.mark.parametrize("name", sorted(CASES))
def test_delta_schedule_rows_match_oracle(spe, monkeypatch, name, delta, lanes):
    monkeypatch.setenv("SPE_DELTA", str(delta))
    top = CASES[name]()
    A = np.arange(top.n, dtype=np.int32)
    ora = Oracle(top).rows(A, A, tie_mode=1)
    g = spe.Graph(top)
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, lanes=lanes, groups=4)
    st = t.build()
    compare(t.download(), ora, f"{name} delta={delta} L={lanes}")
    assert st["iterations"] > 0


def test_delta_schedule_takes_more_rounds(spe, monkeypatch):
    """Buckets serialise the relaxation: a small Delta needs more rounds than
    the Gauss-Seidel default on the same table (the cost MEASUREMENTS.md measures)."""
    top = graphs.gen_ba(3000, 3, seed=11)
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    base = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, lanes=64, groups=4).build()["iterations"]
    monkeypatch.setenv("SPE_DELTA", "1.0")
    dl = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, lanes=64, groups=4).build()["iterations"]
    assert dl > base
