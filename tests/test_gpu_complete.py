"""GPU parity of the offline completion tool (shadow_amd/complete.py): the
gfx950 SSSP rows + path-order jitter fold against the networkx restatement of
compute-topology-paths.py's worker() (oracle/topology_tools.py)."""
import os

import numpy as np
import pytest

import topology_tools as tt
from shadow_amd import complete, graphs, spe

pytestmark = [pytest.mark.gpu, pytest.mark.engine_fixed]


@pytest.mark.parametrize("n,extra,seed,step", [(200, 500, 1, 1), (600, 1500, 2, 5), (1500, 2500, 3, 7)])
def test_complete_paths_bit_exact_on_tie_free_graphs(n, extra, seed, step):
    top = graphs.gen_random_small(n, extra, seed)
    jit = np.random.default_rng(seed).uniform(0.0, 8.0, top.m)
    pois = np.arange(0, n, step, dtype=np.int32)
    got = complete.complete_paths(top, pois, jit)
    lat, jt, hops = tt.all_rows(top, jit, pois)
    assert np.array_equal(got["lat"], lat)
    assert np.array_equal(got["hops"], hops)
    assert np.array_equal(got["jitter"], jt)


def test_complete_paths_pendants_and_long_paths():
    """Pruned pendant sources / targets (their first / last edge is folded apart)
    and paths longer than the 64 edges the fold keeps in registers."""
    rng = np.random.default_rng(9)
    n_chain, n_pend = 150, 40
    src = list(range(n_chain - 1)) + list(rng.integers(0, n_chain, n_pend))
    dst = list(range(1, n_chain)) + list(range(n_chain, n_chain + n_pend))
    m = len(src)
    top = graphs.Topology(n=n_chain + n_pend, esrc=np.array(src, np.int32), edst=np.array(dst, np.int32),
                          elat=rng.uniform(0.5, 9.0, m), eloss=np.zeros(m), vloss=np.zeros(n_chain + n_pend))
    jit = rng.uniform(0, 3, m)
    pois = np.array([0, 1, 77, 149] + list(range(n_chain, n_chain + n_pend, 3)), np.int32)
    got = complete.complete_paths(top, pois, jit)
    lat, jt, hops = tt.all_rows(top, jit, pois)
    assert hops.max() > 64
    assert np.array_equal(got["lat"], lat)
    assert np.array_equal(got["hops"], hops)
    assert np.array_equal(got["jitter"], jt)


def test_complete_paths_shipped_topology(golden_dir):
    """The reference's shipped topology, every vertex a POI, against the committed
    networkx fixture: latency, mean jitter and hops bit-exact for all 183 x 183
    pairs.  (The graph has 1,392 igraph double ties; networkx's first-pushed
    choice happens to coincide with the canonical rule on every one of them.)"""
    z = np.load(os.path.join(golden_dir, "shipped_topology.npz"))
    c = np.load(os.path.join(golden_dir, "completion_shipped.npz"))
    top = graphs.Topology(n=int(z["n"]), esrc=z["esrc"], edst=z["edst"], elat=z["elat"], eloss=z["eloss"],
                          vloss=z["vloss"])
    got = complete.complete_paths(top, c["pois"], c["ejitter"])
    assert np.array_equal(got["lat"], c["lat"])
    assert np.array_equal(got["hops"], c["hops"])
    assert np.array_equal(got["jitter"], c["jitter"])


def test_complete_and_collapse_end_to_end(tmp_path):
    top = graphs.gen_random_small(300, 700, 4)
    rng = np.random.default_rng(4)
    top.eattrs["jitter"] = rng.uniform(0, 2, top.m)
    top.vattrs["geocode"] = [f"G{int(x)}" for x in rng.integers(0, 9, top.n)]
    pois = np.arange(0, top.n, 4, dtype=np.int32)
    comp = complete.complete_topology(top, pois)
    P = len(pois)
    assert comp.n == P and comp.m == P * (P + 1) // 2
    lat, jt, _ = tt.all_rows(top, top.eattrs["jitter"], pois)
    i, j = comp.esrc, comp.edst
    assert np.array_equal(comp.elat, lat[i, j]) and np.array_equal(comp.eattrs["jitter"], jt[i, j])
    col = complete.collapse_topology(comp)
    order, med, _ = tt.collapse(comp.esrc, comp.edst, {"latency": comp.elat, "jitter": comp.eattrs["jitter"]},
                                comp.vattrs["geocode"])
    assert col.n == len(order)
    for e in range(col.m):
        m = med[(int(col.esrc[e]), int(col.edst[e]))]
        assert col.elat[e] == m["latency"] and col.eattrs["jitter"][e] == m["jitter"]
    graphs.write_graphml_attrs(col, str(tmp_path / "collapsed.graphml"))
    back = graphs.load_graphml(str(tmp_path / "collapsed.graphml"))
    g = spe.Graph(back)   # the collapsed graph is a valid (complete) topology for the engine
    assert g.info()["complete"] == 1


def test_want_aux_argument_checks():
    top = graphs.gen_random_small(50, 80, 6)
    g = spe.Graph(top)
    with pytest.raises(spe.SpeError):
        spe.PathTable(g, np.arange(10, dtype=np.int32), want_aux=True)       # no aux attribute yet
    g.set_edge_aux(np.ones(top.m))
    with pytest.raises(spe.SpeError):
        spe.PathTable(g, np.arange(10, dtype=np.int32), want_aux=True, engine=2)
    t = spe.PathTable(g, np.arange(10, dtype=np.int32))
    t.build()
    with pytest.raises(spe.SpeError):
        t.download_aux()


def test_complete_paths_directed_graph():
    """Directed topologies: rows follow out-edges; the aux fold walks the same
    parent edges (the networkx oracle restates the tool on an undirected nx.Graph,
    so here the check is against the C oracle's directed rows plus a direct
    path-order jitter sum along its routes)."""
    from oracle import Oracle
    top = graphs.gen_random_small(150, 500, 8, directed=True)
    jit = np.random.default_rng(8).uniform(0.0, 3.0, top.m)
    pois = np.arange(0, top.n, 2, dtype=np.int32)
    got = complete.complete_paths(top, pois, jit)
    ref = Oracle(top).rows(pois, pois, force_sssp=True, tie_mode=1)
    off = ~np.eye(len(pois), dtype=bool)
    assert np.array_equal(got["lat"][off], ref["lat"][off])
    assert np.array_equal(got["hops"][off], ref["hops"][off])
    # jitter: path-order sum over the oracle's Dijkstra parent edges (no parallel edges here)
    o = Oracle(top)
    for i in range(0, len(pois), 7):
        s = int(pois[i])
        dist, peid, _ = o.dijkstra(s)
        for jx in range(0, len(pois), 5):
            t = int(pois[jx])
            if s == t:
                continue
            edges = []
            x = t
            while x != s:
                e = int(peid[x])
                edges.append(e)
                x = int(top.esrc[e])
            a = 0.0
            for e in reversed(edges):
                a += jit[e]
            assert got["jitter"][i, jx] == a / len(edges)
