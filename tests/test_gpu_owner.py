"""GPU owner-replay mode (spe_table_opts.owner_rank) against the oracle's
simulation of the reference's path cache (first writer wins, either-direction
lookup: shd-topology.c:1292-1321, 1952-2034), for several source-run orders."""
import numpy as np
import pytest

from shadow_amd import graphs
from oracle import Oracle
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spe():
    from shadow_amd import spe as m
    assert m.device_count() > 0, "no GPU visible"
    return m


def orders(A, seed):
    rng = np.random.default_rng(seed)
    return {"identity": np.arange(A), "reverse": np.arange(A)[::-1].copy(), "random": rng.permutation(A)}


CASES = {
    "undirected": (lambda: graphs.gen_random_small(260, 700, 61, vloss_nonzero=True), None),
    "directed": (lambda: graphs.gen_random_small(200, 600, 62, directed=True), None),
    "prefer_direct": (lambda: graphs.gen_random_small(200, 500, 63), "prefer"),
    "partial_pendants": (lambda: graphs.gen_random_small(400, 120, 64), "partial"),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_owner_replay_matches_cache_simulation(spe, name):
    make, flavour = CASES[name]
    top = make()
    if flavour == "prefer":
        top.prefer_direct = True
    A = np.arange(top.n, dtype=np.int32)
    if flavour == "partial":
        A = np.sort(np.random.default_rng(3).choice(top.n, 150, replace=False)).astype(np.int32)
    o = Oracle(top)
    plain = o.rows(A, A)
    g = spe.Graph(top)
    for oname, order in orders(A.shape[0], 7).items():
        ora = o.rows_owner(A, order)
        # the replay is not a no-op: pairs answered by the reverse path fold their sums
        # and products in the other order (undirected: same route, different bits)
        assert (ora["lat"] != plain["lat"]).any() or (ora["rel"] != plain["rel"]).any()
        t = spe.PathTable(g, A, owner_order=order)
        t.build()
        compare(t.download(), ora, label=f"{name}/{oname}")
        t.close()


def test_owner_replay_needs_whole_table(spe):
    top = graphs.gen_random_small(200, 500, 65)
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    with pytest.raises(spe.SpeError):
        spe.PathTable(g, A, blocks=(0, 1), owner_order=np.arange(top.n))
