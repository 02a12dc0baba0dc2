"""CPU tests of the offline completion / collapse tool (shadow_amd/complete.py,
SURVEY.md §8f-3) and of its oracle (oracle/topology_tools.py, a networkx
restatement of src/tools/topology/compute-topology-paths.py / collapse-topology.py).
The GPU part (complete_paths) is in tests/test_gpu_complete.py."""
import os

import numpy as np
import pytest

import topology_tools as tt
from oracle import Oracle
from shadow_amd import complete, graphs


def _shipped(golden_dir):
    z = np.load(os.path.join(golden_dir, "shipped_topology.npz"))
    return graphs.Topology(n=int(z["n"]), esrc=z["esrc"], edst=z["edst"], elat=z["elat"], eloss=z["eloss"],
                           vloss=z["vloss"], directed=bool(z["directed"]), prefer_direct=bool(z["prefer_direct"])), z


def test_oracle_latencies_equal_igraph_restatement_on_shipped_topology(golden_dir):
    """Pin: the networkx restatement of the completion tool and the C restatement
    of igraph Dijkstra (tests/golden/shipped_topology.npz) give bit-identical
    path latencies -- both fold the path from the source, 0 + w1 + w2 + ...."""
    top, z = _shipped(golden_dir)
    c = np.load(os.path.join(golden_dir, "completion_shipped.npz"))
    off = ~np.eye(top.n, dtype=bool)
    assert np.array_equal(c["lat"][off], z["sssp_lat"][off])
    assert np.all(np.diag(c["lat"]) == 5.0) and np.all(np.diag(c["jitter"]) == 0.0)
    # 737 unordered pairs are shorter through other vertices than over their direct edge
    direct = z["direct_lat"]
    assert int(((c["lat"] < direct) & off).sum()) == 2 * 737


def test_oracle_matches_igraph_restatement_on_tie_free_graph():
    top = graphs.gen_random_small(120, 300, 11)
    jit = np.random.default_rng(3).uniform(0, 5, top.m)
    pois = np.arange(0, top.n, 3, dtype=np.int32)
    lat, jt, hops = tt.all_rows(top, jit, pois)
    r = Oracle(top).rows(pois, pois, force_sssp=True, tie_mode=1)
    off = ~np.eye(len(pois), dtype=bool)
    assert np.array_equal(lat[off], r["lat"][off])
    assert np.array_equal(hops[off], r["hops"][off])


def test_ensure_nonzero_latency_matches_oracle():
    rng = np.random.default_rng(5)
    src = rng.integers(0, 6, 200)
    dst = rng.integers(0, 6, 200)
    lat = rng.uniform(0.1, 9.0, 200)
    lat[rng.integers(0, 200, 30)] = 0.0
    lat[rng.integers(0, 200, 5)] = -1.0
    got = complete.ensure_nonzero_latency(src, dst, lat)
    ref = tt.ensure_nonzero_latency(src.tolist(), dst.tolist(), lat.tolist())
    assert got.tolist() == ref
    assert np.array_equal(complete.ensure_nonzero_latency(src, dst, np.abs(lat) + 1), np.abs(lat) + 1)


def _complete_graph(P, seed, ncodes=7):
    rng = np.random.default_rng(seed)
    ii, jj = np.triu_indices(P)
    geo = [f"G{int(x)}" for x in rng.integers(0, ncodes, P)]
    geo[3] = None   # a vertex without geocode: its edges are skipped
    return graphs.Topology(n=P, esrc=ii.astype(np.int32), edst=jj.astype(np.int32),
                           elat=rng.uniform(1, 300, ii.shape[0]).round(3), eloss=np.zeros(ii.shape[0]),
                           vloss=np.zeros(P), vertex_ids=[f"p{i}" for i in range(P)],
                           vattrs={"geocode": geo, "type": ["client"] * P, "countrycode": [f"C{i}" for i in range(P)]},
                           eattrs={"jitter": rng.uniform(0, 4, ii.shape[0])})


@pytest.mark.parametrize("seed", [1, 2])
def test_collapse_matches_oracle(seed):
    top = _complete_graph(40, seed)
    got = complete.collapse_topology(top)
    order, med, rep = tt.collapse(top.esrc, top.edst, {"latency": top.elat, "packetloss": top.eloss,
                                                        "jitter": top.eattrs["jitter"]}, top.vattrs["geocode"])
    assert got.n == len(order)
    assert [got.vattrs["geocode"][i] for i in range(got.n)] == order
    assert got.vattrs["countrycode"] == [top.vattrs["countrycode"][v] for v in rep]
    assert set(got.vattrs["type"]) == {"cluster"} and set(got.vattrs["asn"]) == {0}
    assert got.vertex_ids == [f"poi-{i + 1}" for i in range(got.n)]
    assert got.m == len(med)
    for e in range(got.m):
        m = med[(int(got.esrc[e]), int(got.edst[e]))]
        assert got.elat[e] == m["latency"] and got.eloss[e] == m["packetloss"]
        assert got.eattrs["jitter"][e] == m["jitter"]


def test_select_pois():
    n = 60
    types = ["client"] * 40 + ["server"] * 5 + ["relay"] * 5 + ["pop"] * 10
    geo = [f"g{i % 12}" for i in range(n)]
    top = graphs.Topology(n=n, esrc=np.zeros(0, np.int32), edst=np.zeros(0, np.int32), elat=np.zeros(0),
                          eloss=np.zeros(0), vloss=np.zeros(n), vattrs={"type": types, "geocode": geo})
    p = complete.select_pois(top, sample_size=10, seed=1)
    assert set(range(40, 50)) <= set(p.tolist())                  # every server and relay
    assert not set(range(50, 60)) & set(p.tolist())                # no pop
    clients = [v for v in p.tolist() if v < 40]
    assert {geo[v] for v in clients} == {geo[v] for v in range(40)}   # every client geocode covered
    assert np.array_equal(p, complete.select_pois(top, sample_size=10, seed=1))
    assert set(complete.select_pois(top, sample_size=100).tolist()) == set(range(50))


def test_graphml_roundtrip_keeps_attributes(tmp_path):
    top = _complete_graph(12, 4)
    top.vattrs["geocode"][3] = "X"
    path = str(tmp_path / "c.graphml")
    graphs.write_graphml_attrs(top, path)
    back = graphs.load_graphml(path)
    assert back.vertex_ids == top.vertex_ids
    assert np.array_equal(back.elat, top.elat) and np.array_equal(back.eattrs["jitter"], top.eattrs["jitter"])
    assert back.vattrs["type"] == top.vattrs["type"]
