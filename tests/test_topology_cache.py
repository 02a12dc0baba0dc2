"""The drop-in topology API's model of the reference's lazy path cache
(shd-topology.c:1269-1371 stores, :1952-2034 lookups, shd-path.c:53-56 packet
counters, :1914-1950 the dump at free), its answer modes, attach after seal and
the bounded host mirror.  GPU (the table is built on the device); values are
checked against the oracle, including its first-writer-wins cache replay
(Oracle.rows_owner)."""
import re

import numpy as np
import pytest

from shadow_amd import graphs
from shadow_amd import topology as T
from oracle import Oracle

pytestmark = [pytest.mark.gpu, pytest.mark.engine_fixed]


def setup(tmp_path, t, nverts, seed):
    ips = [f"10.{v // 250}.{v % 250}.{1 + v % 7}" for v in range(t.n)]
    p = tmp_path / "g.graphml"
    graphs.write_graphml(t, str(p), ips=ips)
    top = T.Topology(str(p))
    verts = np.random.default_rng(seed).choice(t.n, nverts, replace=False).astype(np.int32)
    addrs = []
    for i, v in enumerate(verts):
        a = T.ip(f"11.0.{i // 200}.{i % 200 + 1}")
        top.attach(a, ip_hint=ips[v])
        assert top.vertex_of(a) == v
        addrs.append(a)
    return top, verts, addrs


def test_packet_counts_exact_for_every_pair(tmp_path):
    """4,000 counted packets over ~1,600 distinct host pairs (the round-1 table
    dropped counts past ~1,024 pairs).  A packet counts on the cached Path its
    query hits: undirected (s, t) and (t, s) share one entry."""
    t = graphs.gen_random_small(90, 260, 21)
    top, verts, addrs = setup(tmp_path, t, 60, 21)
    rng = np.random.default_rng(4)
    inc = np.zeros((60, 60), np.int64)
    for i, j in rng.integers(0, 60, size=(4000, 2)):
        top.count_packet(addrs[i], addrs[j])
        inc[i, j] += 1
    assert np.count_nonzero(np.triu(inc + inc.T)) > 1024
    want = inc + inc.T - np.diag(np.diag(inc))
    got = np.array([[top.packets(addrs[i], addrs[j]) for j in range(60)] for i in range(60)])
    np.testing.assert_array_equal(got, want)
    top.close()


@pytest.mark.parametrize("directed", [False, True], ids=["undirected", "directed"])
def test_reference_answer_mode_replays_first_writer(tmp_path, directed):
    """TOPOLOGY_ANSWER_REFERENCE: sources run their Dijkstra rows in a chosen
    order (each one's first query misses); every later answer is then the one the
    reference's cache holds -- tree_t(t -> s) when t ran first, also for directed
    graphs -- against the oracle's cache replay in the same order."""
    t = graphs.gen_random_small(70, 200, 22, directed=directed)
    top, verts, addrs = setup(tmp_path, t, 30, 22)
    top.set_answer_mode(T.ANSWER_REFERENCE)
    perm = np.random.default_rng(5).permutation(30)
    last = perm[-1]
    for s in perm[:-1]:     # s's first query: (s, last) is cached in neither direction -> s's row runs
        top.latency(addrs[s], addrs[last])
    # (s, s): the row's [s] path for a source that ran, the SELF rule for the one
    # that has not (asked first: in a directed graph a (last, t) query runs last's row)
    o = Oracle(t)
    rows0 = o.rows(verts, verts, self_mode=0)
    rows1 = o.rows(verts, verts, self_mode=1)
    s0 = perm[0]
    assert top.latency(addrs[s0], addrs[s0]) == rows0["lat"][s0, s0]
    assert top.latency(addrs[last], addrs[last]) == rows1["lat"][last, last]
    assert top.reliability(addrs[last], addrs[last]) == rows1["rel"][last, last]
    ref = o.rows_owner(verts, list(perm))
    for i in range(30):
        for j in range(30):
            if i == j:
                continue
            ok, lat, rel = top.path_info(addrs[i], addrs[j])
            assert ok and lat == ref["lat"][i, j] and rel == ref["rel"][i, j], (i, j)
    # default mode: the source row whatever the order
    top.set_answer_mode(T.ANSWER_ROWS)
    for i in range(0, 30, 7):
        for j in range(30):
            assert top.latency(addrs[i], addrs[j]) == rows0["lat"][i, j]
    top.close()


def test_cached_path_dump_at_free(tmp_path):
    """topology_free logs one info line per cached Path (path_toString format,
    shd-path.c:58-71) with its packet count; the count of lines equals the
    cache size the model reports."""
    t = graphs.gen_random_small(50, 150, 23)
    top, verts, addrs = setup(tmp_path, t, 12, 23)
    top.capture_logs(4)
    top.count_packet(addrs[0], addrs[1])
    top.count_packet(addrs[1], addrs[0])
    top.latency(addrs[2], addrs[5])
    n_cached = top.cached_paths()
    assert n_cached >= 12   # rows of sources 0 and 2 (every target, minus pairs the other stored)
    logs = top.logs
    top.close()
    lines = [x for lvl, x in logs if x.startswith("Found path")]
    assert len(lines) == n_cached
    v0, v1 = int(verts[0]), int(verts[1])
    pat = re.compile(rf"Found path v{v0}<->v{v1} in cache: SourceIndex={v0} DestinationIndex={v1} "
                     r"Latency=[0-9.]+ Reliability=[0-9.]+ PacketCount=2 isDirect=False")
    assert any(pat.fullmatch(x) for x in lines), lines[:5]
    assert any(x.startswith("path cache cleared, spent") for _, x in logs)
    assert any(x.startswith("shortest path v") for lvl, x in logs if lvl == 4)


def test_attach_after_seal_rebuilds_and_keeps_counts(tmp_path):
    t = graphs.gen_random_small(120, 360, 24)
    ips = [f"10.{v // 250}.{v % 250}.{1 + v % 7}" for v in range(t.n)]
    p = tmp_path / "g.graphml"
    graphs.write_graphml(t, str(p), ips=ips)
    top = T.Topology(str(p))
    verts = np.random.default_rng(24).choice(t.n, 30, replace=False).astype(np.int32)
    addrs = [T.ip(f"11.0.0.{i + 1}") for i in range(30)]
    for i in range(20):
        top.attach(addrs[i], ip_hint=ips[verts[i]])
    assert top.seal() == 0
    for _ in range(3):
        top.count_packet(addrs[0], addrs[1])
    for i in range(20, 30):   # ten more vertices after the table is sealed
        top.attach(addrs[i], ip_hint=ips[verts[i]])
    ref = Oracle(t).rows(verts, verts)
    for i in range(30):
        for j in range(20, 30):
            assert top.latency(addrs[i], addrs[j]) == ref["lat"][i, j]
            assert top.reliability(addrs[j], addrs[i]) == ref["rel"][j, i]
    assert top.packets(addrs[0], addrs[1]) == 3
    top.close()


@pytest.mark.parametrize("budget", ["0", "2000"], ids=["device-reads", "one-row"])
def test_bounded_host_mirror(tmp_path, monkeypatch, budget):
    """Above SHADOW_SPE_MIRROR_BYTES the host mirrors only source rows read
    repeatedly, within the budget (a 70-host row is 1,120 B: one fits 2,000), and
    reads single {latency, reliability} records from HBM otherwise
    (spe_table_get_latrel / spe_table_get_row_latrel): same answers."""
    monkeypatch.setenv("SHADOW_SPE_MIRROR_BYTES", budget)
    t = graphs.gen_random_small(200, 600, 25)
    top, verts, addrs = setup(tmp_path, t, 70, 25)
    ref = Oracle(t).rows(verts, verts)
    for i in range(0, 70, 3):
        for j in range(0, 70, 2):
            assert top.path_info(addrs[i], addrs[j]) == (True, ref["lat"][i, j], ref["rel"][i, j])
    top.close()
