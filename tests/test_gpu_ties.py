"""Canonical ties on a graph with hubs (heavy vertices, in-degree > 64) and f64
path sums that tie: a Barabasi-Albert graph with latencies in tenths of a
millisecond.  Two in-neighbours u of a hub v often give the same fl(d[u] + w);
the route must then follow the canonical parent argmin (d[u], u),
which the oracle restates (tie_mode 1, shd-topology.c:1741's Dijkstra with a
documented tie-break).

Regression for a gfx950 code-generation fault (MEASUREMENTS.md): the short-circuit form
of the heavy-vertex partial's lexicographic compare kept the old parent entry on
lanes that won a tie on (d[u], u), so hubs recorded the losing parent on about
1 % of sources.  Every relaxation kernel shape, with and without the degree-3
contraction, and the LDS engine are checked entry for entry."""
import numpy as np
import pytest

from shadow_amd import graphs
from oracle import Oracle

pytestmark = [pytest.mark.gpu, pytest.mark.engine_fixed]


@pytest.fixture(scope="module")
def case():
    from shadow_amd import spe
    assert spe.device_count() > 0, "no GPU visible"
    top = graphs.gen_ba(3000, 3, 25)
    rng = np.random.default_rng(225)
    top.elat = rng.integers(1, 60, top.elat.shape[0]) * 0.1
    A = np.arange(top.n, dtype=np.int32)
    ref = Oracle(top).rows(A, A, tie_mode=1, nthreads=16)
    return spe, top, A, ref


SHAPES = {
    "ring128": dict(relax_kernel=2),
    "reg128": dict(relax_kernel=1),
    "k_relax64": dict(lanes=64),
    "ring128_groups2": dict(relax_kernel=2, groups=2),
}


@pytest.mark.parametrize("contract", [False, True], ids=["plain", "contracted"])
@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_decimal_ties_at_hubs_follow_the_canonical_parent(case, shape, contract):
    spe, top, A, ref = case
    if contract and not shape.startswith("ring"):
        pytest.skip("the degree-3 contraction runs on the LDS-ring relaxation only (spe_table_create)")
    g = spe.Graph(top)
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, exact_sources=True, no_contract=not contract,
                      **SHAPES[shape])
    t.build()
    assert (t.layout()["contracted_vertices"] > 0) == contract
    got = t.download()
    ok = ref["kind"] != 0
    for k in ("next", "hops"):
        bad = int(((got[k] != ref[k]) & ok).sum())
        assert bad == 0, f"{shape}: {k} differs at {bad} entries"
    for k in ("lat", "rel"):
        np.testing.assert_array_equal(got[k][ok], ref[k][ok], err_msg=f"{shape}: {k}")


def test_decimal_ties_lds_engine(case):
    spe, top, A, ref = case
    g = spe.Graph(top)
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_LDS)
    t.build()
    got = t.download()
    ok = ref["kind"] != 0
    for k in ("next", "hops", "lat", "rel"):
        np.testing.assert_array_equal(got[k][ok], ref[k][ok], err_msg=k)
