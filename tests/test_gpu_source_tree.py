"""spe_table_source_tree / spe_graph_edge and the topology shim's per-path log
lines (shd-topology.c:1809-1829 with the path string of :1413-1493).

The tree of a row must BE the row: for every target, the parent walk from the
target back to the source has the row's hop count and first hop, and its
path-order latency fold is the row's latency bit for bit; the oracle's rows
then pin it.  Asking for a tree recomputes the source's block, so the table
must be unchanged afterwards (incl. the DIRECT overlay of preferdirectpaths)."""
import re

import numpy as np
import pytest

from oracle import Oracle
from shadow_amd import graphs
from shadow_amd import topology as T

pytestmark = [pytest.mark.gpu, pytest.mark.engine_fixed]


@pytest.fixture(scope="module")
def spe():
    from shadow_amd import spe as m
    assert m.device_count() > 0, "no GPU visible"
    return m


def walk(par, s, t):
    vs = [t]
    while vs[-1] != s:
        p = int(par[vs[-1]])
        assert p >= 0 and len(vs) <= par.shape[0], (s, t)
        vs.append(p)
    return vs[::-1]


CASES = {
    "tiefree": dict(n=400, extra_edges=1200, seed=71),
    "pendants": dict(n=600, extra_edges=40, seed=72),          # pruned sources and targets
    "directed": dict(n=300, extra_edges=900, seed=73, directed=True),
}


@pytest.mark.parametrize("engine", [1, 2, 3], ids=["batch", "lds", "fw"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_source_tree_is_the_row(spe, name, engine):
    top = graphs.gen_random_small(**CASES[name])
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    t = spe.PathTable(g, A, engine=engine, groups=2)
    t.build()
    before = t.download()
    ora = Oracle(top).rows(A[[0, 5, top.n - 1]], A)
    for i, s in enumerate((0, 5, top.n - 1)):
        par = t.source_tree(s)
        assert par[s] == -1
        row = {k: v[s] for k, v in before.items()}
        np.testing.assert_array_equal(row["lat"][row["ok"]], ora["lat"][i][row["ok"]])
        for tt in range(top.n):
            if tt == s or not row["ok"][tt]:
                continue
            vs = walk(par, s, tt)
            assert len(vs) - 1 == row["hops"][tt] and vs[1] == row["next"][tt], (s, tt)
            lat = 0.0
            for u, v in zip(vs[:-1], vs[1:]):
                lat += g.edge(u, v)[0]
            assert lat == row["lat"][tt], (s, tt, lat, row["lat"][tt])
    after = t.download()
    for k in ("lat", "rel", "next", "hops"):
        np.testing.assert_array_equal(after[k], before[k])


def test_source_tree_keeps_the_direct_overlay(spe):
    top = graphs.gen_random_small(300, 900, 44, self_loops=False)
    top.prefer_direct = True
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    for engine in (1, 2):
        t = spe.PathTable(g, A, engine=engine)
        t.build()
        before = t.download()
        t.source_tree(7)
        after = t.download()
        for k in ("lat", "rel", "next", "hops"):
            np.testing.assert_array_equal(after[k], before[k])


def test_graph_edge_lookup(spe):
    top = graphs.gen_random_small(100, 300, 74)
    g = spe.Graph(top)
    e = 17
    u, v = int(top.esrc[e]), int(top.edst[e])
    w, a = g.edge(u, v)
    assert w == top.elat[e] and a == 1.0 - top.eloss[e]
    assert g.edge(v, u) == (w, a)   # undirected
    adj = set(zip(top.esrc.tolist(), top.edst.tolist())) | set(zip(top.edst.tolist(), top.esrc.tolist()))
    x, y = next((x, y) for x in range(top.n) for y in range(top.n) if x != y and (x, y) not in adj)
    with pytest.raises(spe.SpeError):
        g.edge(x, y)
    with pytest.raises(spe.SpeError):
        g.edge(-1, 0)


def test_shim_per_path_log_lines_carry_the_path(tmp_path):
    """topology_* per-path info / debug lines print the reference's path string:
    the source id, then "<--[latency,loss]-->id" per edge; the vertices are the
    row's path (hops / first hop / latency fold as the oracle's row)."""
    t = graphs.gen_random_small(80, 200, 75)
    ips = [f"10.{v // 250}.{v % 250}.{1 + v % 7}" for v in range(t.n)]
    p = tmp_path / "g.graphml"
    graphs.write_graphml(t, str(p), ips=ips)
    top = T.Topology(str(p))
    verts = np.random.default_rng(75).choice(t.n, 20, replace=False).astype(np.int32)
    addrs = [T.ip(f"11.0.0.{i + 1}") for i in range(20)]
    for a, v in zip(addrs, verts):
        top.attach(a, ip_hint=ips[v])
    top.capture_logs(5)
    top.latency(addrs[0], addrs[3])
    logs = top.logs
    top.close()
    ora = Oracle(t).rows(verts[[0]], verts)
    pat = re.compile(r"shortest path v(\d+)<-->v(\d+) \((\d+)<-->(\d+)\) is ([0-9.]+) ms with ([0-9.]+) loss, "
                     r"path: (.*)")
    seen = 0
    for lvl, x in logs:
        m = pat.fullmatch(x)
        if not m:
            continue
        s, tt = int(m.group(1)), int(m.group(2))
        assert s == verts[0]
        j = int(np.flatnonzero(verts == tt)[0])
        hops = re.findall(r"<--\[([0-9.]+),([0-9.]+)\]-->v(\d+)", m.group(7))
        assert m.group(7).startswith(f"v{s}")
        vs = [s] + [int(h[2]) for h in hops]
        if tt == s:
            assert vs == [s, s]   # the row's [s] path: its self-loop
            continue
        assert vs[-1] == tt and len(vs) - 1 == ora["hops"][0, j] and vs[1] == ora["next"][0, j]
        lat = 0.0
        for u, v in zip(vs[:-1], vs[1:]):
            sel = ((t.esrc == u) & (t.edst == v)) | ((t.esrc == v) & (t.edst == u))
            lat += float(t.elat[np.flatnonzero(sel)[-1]])
        assert lat == ora["lat"][0, j]
        seen += 1
        assert (lvl == 4) == (tt == verts[3])
    assert seen >= 15


def test_source_tree_refuses_owner_replay_and_direct_tables(spe):
    top = graphs.gen_random_small(200, 600, 76)
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    t = spe.PathTable(g, A, owner_order=np.arange(top.n))
    t.build()
    with pytest.raises(spe.SpeError):
        t.source_tree(3)
    z = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "shipped_topology.npz"))
    shipped = graphs.Topology(n=int(z["n"]), esrc=z["esrc"], edst=z["edst"], elat=z["elat"], eloss=z["eloss"],
                              vloss=z["vloss"], directed=bool(z["directed"]), prefer_direct=bool(z["prefer_direct"]))
    gs = spe.Graph(shipped)
    td = spe.PathTable(gs, np.arange(shipped.n, dtype=np.int32))
    td.build()
    with pytest.raises(spe.SpeError):
        td.source_tree(0)
