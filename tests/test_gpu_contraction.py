"""GPU parity of the batch engine on its degree-3 contraction.

An independent set of relaxation vertices with exactly three neighbours is taken
out of the batch engine's relaxation graph and replaced by shortcut entries
between its neighbours (the two-add fold fl(fl(d[a] + w(a,x)) + w(x,b))); those
vertices' rows come from their three neighbours' rows.  The reference runs
igraph's Dijkstra on the whole graph (shd-topology.c:1741-1742), so every row
here must equal the oracle's and the uncontracted build's, bit for bit, including
removed vertices as sources and as targets, exact ties in canonical mode, pruned
pendants next to contracted vertices, ragged blocks and partial attachment.
"""
import numpy as np
import pytest

from shadow_amd import graphs
from oracle import Oracle

pytestmark = [pytest.mark.gpu, pytest.mark.engine_fixed]


@pytest.fixture(scope="module")
def spe():
    from shadow_amd import spe as m
    assert m.device_count() > 0, "no GPU visible"
    return m


def build(spe, top, A, **kw):
    g = spe.Graph(top)
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, lanes=128, **kw)
    t.build()
    return g, t


def same(a, b, label):
    for k in ("ok", "lat", "rel", "next", "hops"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=f"{label}: {k}")


def vs_oracle(got, ref, label):
    ok = ref["kind"] != 0
    np.testing.assert_array_equal(got["ok"], ok, err_msg=f"{label}: routability")
    for k in ("lat", "rel"):
        bad = np.flatnonzero(got[k][ok] != ref[k][ok])
        assert bad.size == 0, f"{label}: {k} differs at {bad.size} entries"
    np.testing.assert_array_equal(got["hops"][ok], ref["hops"][ok], err_msg=f"{label}: hops")
    np.testing.assert_array_equal(got["next"][ok], ref["next"][ok], err_msg=f"{label}: next hop")


def with_pendants(top, k, seed):
    """top plus k pendant vertices on random anchors (those anchors are never
    contracted; the pendants are pruned next to contracted neighbours)."""
    rng = np.random.default_rng(seed)
    anc = rng.integers(0, top.n, k)
    n2 = top.n + k
    return graphs.Topology(n=n2, esrc=np.concatenate([top.esrc, np.arange(top.n, n2)]).astype(np.int32),
                           edst=np.concatenate([top.edst, anc]).astype(np.int32),
                           elat=np.concatenate([top.elat, rng.uniform(1, 100, k)]),
                           eloss=np.concatenate([top.eloss, rng.uniform(0, 0.01, k)]),
                           vloss=np.zeros(n2), directed=False, prefer_direct=False)


# (graph, oracle tie mode); each has >= 10 % contractible relaxation vertices
CASES = {
    "ba_m3": (lambda: graphs.gen_ba(3000, 3, 17), 0),
    "random_sparse": (lambda: graphs.gen_random_small(700, 700, 71), 0),
    "ba_with_pendants": (lambda: with_pendants(graphs.gen_ba(2000, 3, 19), 300, 4), 0),
    "tie_heavy": (lambda: graphs.gen_random_small(500, 500, 72, integer_weights=True), 1),
}


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("groups", [1, 3])
def test_contracted_rows_equal_oracle_and_plain(spe, name, groups):
    mk, tie_mode = CASES[name]
    top = mk()
    A = np.arange(top.n, dtype=np.int32)
    g, t = build(spe, top, A, groups=groups)
    lay = t.layout()
    assert lay["contracted_vertices"] > 0, f"{name}: no contraction"
    assert lay["contracted_vertices"] < g.info()["n_relax_vertices"]
    got = t.download()
    ref = Oracle(top).rows(A, A, tie_mode=tie_mode)
    vs_oracle(got, ref, f"{name} groups={groups}")
    _, tp = build(spe, top, A, groups=groups, no_contract=True)
    assert tp.layout()["contracted_vertices"] == 0
    same(got, tp.download(), f"{name} groups={groups} vs plain")


def test_contracted_partial_attachment_and_source_trees(spe):
    """Removed vertices attached or not, sources among them, ragged blocks; the
    per-source parent trees of the contracted and the plain build agree."""
    top = graphs.gen_ba(2500, 3, 23)
    rng = np.random.default_rng(5)
    A = np.sort(rng.choice(top.n, size=5 * 64 + 29, replace=False)).astype(np.int32)
    g, t = build(spe, top, A, groups=2)
    assert t.layout()["contracted_vertices"] > 0
    got = t.download()
    vs_oracle(got, Oracle(top).rows(A, A), "partial")
    _, tp = build(spe, top, A, groups=2, no_contract=True)
    same(got, tp.download(), "partial vs plain")
    deg = np.bincount(np.concatenate([top.esrc, top.edst]), minlength=top.n)
    picks = [i for i in range(len(A)) if deg[A[i]] == 3][:3] + [0, len(A) - 1]
    for s in picks:
        pc, pp = t.source_tree(int(s)), tp.source_tree(int(s))
        np.testing.assert_array_equal(pc, pp, err_msg=f"source tree of slot {s}")


def test_contraction_skipped_where_it_does_not_apply(spe):
    """Vertex loss on some vertex (the rows' path-order re-fold walks plain edges
    only), 64-lane rows and graphs with few contractible vertices (C4's tiered core:
    its degree-3 vertices anchor pendants) keep the plain graph."""
    top = graphs.gen_random_small(400, 800, 73, vloss_nonzero=True)
    A = np.arange(top.n, dtype=np.int32)
    g, t = build(spe, top, A)
    assert t.layout()["contracted_vertices"] == 0
    vs_oracle(t.download(), Oracle(top).rows(A, A), "vertex loss")
    top = graphs.gen_ba(1500, 3, 29)
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    t64 = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, lanes=64)
    assert t64.layout()["contracted_vertices"] == 0
    top = graphs.gen_tiered(n_core=1500, n_stub=3000, n_attached=200, seed=7)
    A = graphs.tiered_attached(top, n_core=1500, n_attached=200)
    g, t = build(spe, top, A)
    assert t.layout()["contracted_vertices"] == 0
