"""GPU parity of the shared anchor trees, the batch engine's default
for pruned pendant sources: the hosts on one anchor take the anchor's relaxation,
and a host's row is the anchor's row with its pendant edge folded in front.

The reference runs one Dijkstra per host (shd-topology.c:1741-1742) and folds each
path's latency and reliability in path order (:1413-1493).  Here routability, next
hops and hop counts must equal the oracle's exactly; latency and reliability agree
within 1e-12 relative (the north star allows 1e-9: a shared row adds the pendant
edge to the anchor's path sum instead of folding the path from the pendant), and
bit for bit where every latency is an integer (every sum exact).  Anchors whose
parent decisions lie within rounding of a tie are rebuilt one lane per source
(spe_build_stats.fallback_blocks).  The rest of the GPU suite pins
spe_table_opts.exact_sources (tests/conftest.py); this file runs the default.
"""
import numpy as np
import pytest

from shadow_amd import graphs
from oracle import Oracle

pytestmark = [pytest.mark.gpu, pytest.mark.engine_fixed, pytest.mark.shared_trees]

RTOL = 1e-12


@pytest.fixture(scope="module")
def spe():
    from shadow_amd import spe as m
    assert m.device_count() > 0, "no GPU visible"
    return m


def near(got, ref, label, exact_lat=False):
    ok = ref["kind"] != 0
    np.testing.assert_array_equal(got["ok"], ok, err_msg=f"{label}: routability")
    np.testing.assert_array_equal(got["next"][ok], ref["next"][ok], err_msg=f"{label}: next hop")
    np.testing.assert_array_equal(got["hops"][ok], ref["hops"][ok], err_msg=f"{label}: hops")
    if exact_lat:
        np.testing.assert_array_equal(got["lat"][ok], ref["lat"][ok], err_msg=f"{label}: latency")
    else:
        np.testing.assert_allclose(got["lat"][ok], ref["lat"][ok], rtol=RTOL, atol=0, err_msg=f"{label}: latency")
    np.testing.assert_allclose(got["rel"][ok], ref["rel"][ok], rtol=RTOL, atol=0, err_msg=f"{label}: reliability")
    assert (got["lat"][~ok] == -1).all() and (got["hops"][~ok] == 0).all(), f"{label}: unroutable entries"


def with_pendants(top, k, seed, integer=False):
    """top plus k pendant vertices on random anchors (several per anchor)."""
    rng = np.random.default_rng(seed)
    anc = rng.integers(0, top.n, k)
    n2 = top.n + k
    lat = rng.integers(1, 9, k).astype(np.float64) if integer else rng.uniform(0.5, 10.0, k)
    return graphs.Topology(n=n2, esrc=np.concatenate([top.esrc, np.arange(top.n, n2)]).astype(np.int32),
                           edst=np.concatenate([top.edst, anc]).astype(np.int32),
                           elat=np.concatenate([top.elat, lat]),
                           eloss=np.concatenate([top.eloss, rng.uniform(0, 0.01, k)]),
                           vloss=np.zeros(n2), directed=False, prefer_direct=False)


def tiered_case():
    top = graphs.gen_tiered(n_core=1500, n_stub=6000, n_attached=3000, seed=9)
    A = np.r_[graphs.tiered_attached(top, n_core=1500, n_attached=3000), np.arange(0, 1500, 7)]
    return top, A.astype(np.int32)


def all_of(top):
    return top, np.arange(top.n, dtype=np.int32)


# (graph + attached, oracle tie mode, latencies bit-exact)
CASES = {
    "ba_pendants": (lambda: all_of(with_pendants(graphs.gen_ba(2000, 3, 19), 1500, 4)), 0, False),
    "tiered": (tiered_case, 0, False),
    "tree_heavy": (lambda: all_of(graphs.gen_random_small(800, 150, 75)), 0, False),
    "integer": (lambda: all_of(with_pendants(graphs.gen_random_small(700, 300, 76, integer_weights=True), 600, 5,
                                             integer=True)), 1, True),
}


def build(spe, top, A, **kw):
    g = spe.Graph(top)
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, **kw)
    t.build()
    return g, t


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("groups", [1, 4])
def test_shared_rows_match_oracle_and_exact_build(spe, name, groups):
    mk, tie_mode, exact_lat = CASES[name]
    top, A = mk()
    g = spe.Graph(top)
    if groups > 1:   # the bench's slot order: hosts of one anchor adjacent
        A = g.order_sources(A)
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, groups=groups)
    st = t.build()
    assert t.layout()["shared_sources"] == 1, name
    core = g.info()["n_relax_vertices"]
    assert 0 < st["relaxed_lanes"] < len(A), f"{name}: {st}"
    got = t.download()
    ref = Oracle(top).rows(A, A, tie_mode=tie_mode)
    near(got, ref, f"{name} groups={groups}", exact_lat=exact_lat)
    if exact_lat:
        assert st["fallback_blocks"] == 0, f"{name}: integer sums need no fallback ({st})"
    te = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, groups=groups, exact_sources=True)
    se = te.build()
    assert te.layout()["shared_sources"] == 0 and se["relaxed_lanes"] == len(A)
    ex = te.download()
    for k in ("ok", "next", "hops"):
        np.testing.assert_array_equal(got[k], ex[k], err_msg=f"{name}: {k} vs exact build")
    # a core source is its own root: its row is the exact build's bit for bit (degree-3
    # and degree-4 core sources may be derived from their neighbours: not counted)
    deg = np.bincount(np.concatenate([top.esrc[top.esrc != top.edst], top.edst[top.esrc != top.edst]]),
                      minlength=top.n)
    rows_core = np.flatnonzero(deg[A] > 4)
    assert rows_core.size > 0 and core > 0
    for k in ("lat", "rel"):
        np.testing.assert_array_equal(got[k][rows_core], ex[k][rows_core], err_msg=f"{name}: core-source {k}")


def test_near_ties_fall_back_to_one_lane_per_source(spe):
    """Latencies in multiples of 0.1: equal real path lengths round differently
    from different offsets, so k_share_check flags their anchors and those blocks
    are rebuilt per source; every row still matches the oracle (canonical ties)."""
    top = with_pendants(graphs.gen_random_small(600, 400, 77), 700, 6)
    rng = np.random.default_rng(8)
    loop = top.esrc == top.edst
    top.elat = np.where(loop, top.elat, rng.integers(1, 6, top.elat.shape[0]) * 0.1)
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    A = g.order_sources(A)
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, groups=2)
    st = t.build()
    assert t.layout()["shared_sources"] == 1
    assert st["fallback_blocks"] > 0, st
    got = t.download()
    near(got, Oracle(top).rows(A, A, tie_mode=1), "decimal latencies")
    te = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, groups=2, exact_sources=True)
    te.build()
    ex = te.download()
    for k in ("ok", "next", "hops"):
        np.testing.assert_array_equal(got[k], ex[k], err_msg=f"decimal latencies: {k} vs exact build")


def test_shared_partial_blocks_source_trees_and_lookups(spe):
    """A block range of a shared table equals the same rows of the whole exact
    table; source trees of pendant hosts are their own (one lane per source);
    batched lookups on a whole shared table read its rows."""
    top, A = tiered_case()
    g = spe.Graph(top)
    A = g.order_sources(A)
    full = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, exact_sources=True)
    full.build()
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, blocks=(2, 7), groups=2)
    t.build()
    assert t.layout()["shared_sources"] == 1
    part = t.download(2 * 64, 7 * 64)
    ref = full.download(2 * 64, 7 * 64)
    for k in ("ok", "next", "hops"):
        np.testing.assert_array_equal(part[k], ref[k], err_msg=k)
    ok = ref["ok"]
    for k in ("lat", "rel"):
        np.testing.assert_allclose(part[k][ok], ref[k][ok], rtol=RTOL, atol=0, err_msg=k)
    for s in (2 * 64, 2 * 64 + 37, 7 * 64 - 1):
        np.testing.assert_array_equal(t.source_tree(s), full.source_tree(s), err_msg=f"source tree {s}")
    import torch
    ts = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH)
    ts.build()
    whole = ts.download()
    rng = np.random.default_rng(3)
    q = 1 << 16
    pairs = rng.integers(0, len(A), (q, 2)).astype(np.int32)
    dp = torch.from_numpy(pairs).cuda()
    lat = torch.empty(q, dtype=torch.float64, device="cuda")
    rel = torch.empty_like(lat)
    okq = torch.empty(q, dtype=torch.uint8, device="cuda")
    ts.lookup_batch(dp.data_ptr(), q, lat.data_ptr(), rel.data_ptr(), okq.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(okq.cpu().numpy(), whole["ok"][pairs[:, 0], pairs[:, 1]].astype(np.uint8))
    v = whole["ok"][pairs[:, 0], pairs[:, 1]]
    np.testing.assert_array_equal(lat.cpu().numpy()[v], whole["lat"][pairs[v, 0], pairs[v, 1]])
    np.testing.assert_array_equal(rel.cpu().numpy()[v], whole["rel"][pairs[v, 0], pairs[v, 1]])


def test_shared_multi_device_shares(spe):
    """Three shares of one GPU (peer gather): each part shares its own anchors."""
    top, A = tiered_case()
    g = spe.Graph(top)
    A = g.order_sources(A)
    t = spe.PathTable(g, A, devices=[0, 0, 0], engine=spe.SPE_ENGINE_BATCH)
    t.build()
    assert t.layout()["shared_sources"] == 1
    got = t.download()
    near(got, Oracle(top).rows(A, A), "three shares")
