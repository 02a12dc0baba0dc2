"""The drop-in topology API (include/shd_topology_spe.h) exercised like the
reference's own users do: topology_new on a GraphML file, attach hosts, then
per-packet queries.  CPU part: exports + validation failures (no GPU needed);
GPU part: values against the oracle."""
import json
import os
import subprocess

import numpy as np
import pytest

from shadow_amd import graphs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_libshdtopo_exports_declared_api():
    so = os.path.join(ROOT, "shadow_amd", "libshdtopo.so")
    assert os.path.exists(so)
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    have = {l.split()[-1] for l in out.splitlines() if " T " in l}
    from shadow_amd import topology
    import re
    hdr = open(os.path.join(ROOT, "include", "shd_topology_spe.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    declared = set(re.findall(r"SHD_TOPO\((topology_[A-Za-z_]+)\)\s*\(", hdr))
    assert declared == set(topology.EXPORTS)
    assert declared <= have


@pytest.mark.parametrize("mutate,why", [
    (lambda t: t.elat.__setitem__(0, 0.0), "latency must be > 0"),
    (lambda t: t.eloss.__setitem__(1, 1.5), "packetloss in [0,1]"),
])
def test_topology_new_rejects_invalid_graph(tmp_path, mutate, why):
    """shd-topology.c:1026-1109 / :2485-2490: validation failure -> NULL (before any GPU work)."""
    from shadow_amd import topology
    t = graphs.gen_random_small(20, 30, 1)
    mutate(t)
    p = tmp_path / "bad.graphml"
    graphs.write_graphml(t, str(p))
    assert not topology.lib().topology_new(str(p).encode()), why


def test_topology_new_rejects_disconnected(tmp_path):
    from shadow_amd import topology
    t = graphs.gen_random_small(20, 30, 2)
    t.n += 1   # an isolated vertex: not one strong component (shd-topology.c:785-791)
    t.vloss = np.append(t.vloss, 0.0)
    p = tmp_path / "disc.graphml"
    graphs.write_graphml(t, str(p))
    assert not topology.lib().topology_new(str(p).encode())


@pytest.mark.gpu
def test_examples_config_one_vertex(tmp_path, golden_dir):
    """resource/examples/shadow.config.xml: 150 hosts on the 1-vertex graph ->
    every pair 50.0 ms / 0.95, routable; packet counters per pair."""
    from shadow_amd import topology as T
    kat = json.load(open(os.path.join(golden_dir, "kat_1vertex.json")))["examples"]
    p = tmp_path / "ex.graphml"
    p.write_text(kat["graphml"])
    top = T.Topology(str(p))
    hosts = [T.ip(f"11.0.0.{i + 1}") for i in range(150)]
    for h in hosts:
        down, up = top.attach(h, rand=[0.37])
        assert (down, up) == (17038, 2251)
    assert top.latency(hosts[0], hosts[1]) == 50.0 and top.reliability(hosts[0], hosts[1]) == 0.95
    assert top.routable(hosts[3], hosts[3])
    top.count_packet(hosts[0], hosts[1])
    top.count_packet(hosts[0], hosts[1])
    # counters live on the vertex-pair path (shd-path.c:53-56): every host here is on vertex 0
    assert top.packets(hosts[0], hosts[1]) == 2 and top.packets(hosts[5], hosts[9]) == 2
    unknown = T.ip("12.0.0.1")
    assert top.latency(hosts[0], unknown) == -1.0 and not top.routable(unknown, hosts[0])
    assert top.path_info(hosts[0], unknown) == (False, -1.0, -1.0)
    assert top.path_info(hosts[0], hosts[1]) == (True, 50.0, 0.95)
    assert top.min_latency() == 50.0
    top.close()


@pytest.mark.gpu
def test_attach_by_ip_and_query_against_oracle(tmp_path):
    """Hosts attach by exact IP hint (shd-topology.c:2117-2137); queries return the
    per-source row values of the oracle."""
    from oracle import Oracle
    from shadow_amd import topology as T
    t = graphs.gen_random_small(120, 300, 9)
    ips = [f"10.{v // 250}.{v % 250}.{1 + v % 7}" for v in range(t.n)]
    p = tmp_path / "g.graphml"
    graphs.write_graphml(t, str(p), ips=ips)
    top = T.Topology(str(p))
    rng = np.random.default_rng(3)
    verts = rng.choice(t.n, 40, replace=False)
    addrs = []
    for i, v in enumerate(verts):
        a = T.ip(f"11.0.{i // 200}.{i % 200 + 1}")
        top.attach(a, ip_hint=ips[v])
        assert top.vertex_of(a) == v
        addrs.append(a)
    # slots follow first-attach order; oracle rows over the same attached set
    ref = Oracle(t).rows(verts, verts)
    for i in range(0, 40, 3):
        for j in range(40):
            assert top.latency(addrs[i], addrs[j]) == ref["lat"][i, j]
            assert top.reliability(addrs[i], addrs[j]) == ref["rel"][i, j]
            assert top.path_info(addrs[i], addrs[j]) == (True, ref["lat"][i, j], ref["rel"][i, j])
    top.close()


@pytest.mark.gpu
def test_examples_hosts_attach_like_the_reference(tmp_path, golden_dir):
    """C1: the shipped 183-vertex topology under the examples
    config's 150 un-hinted hosts (server, webclient, bulkclient x 50).  Shadow's
    seed chain master(1) -> slave -> host (shadow_amd/shadow_random.py, glibc
    rand_r) drives the shim's attach; every host lands on the vertex the
    reference's round((k-1) * nextDouble) rule picks over all 183 candidates."""
    from shadow_amd import shadow_random as sr
    from shadow_amd import topology as T
    z = np.load(os.path.join(golden_dir, "shipped_topology.npz"))
    top_g = graphs.Topology(n=int(z["n"]), esrc=z["esrc"], edst=z["edst"], elat=z["elat"], eloss=z["eloss"],
                            vloss=z["vloss"])
    p = tmp_path / "shipped.graphml"
    graphs.write_graphml(top_g, str(p))
    top = T.Topology(str(p))
    cfg = [("server", 50), ("webclient", 50), ("bulkclient", 50)]
    streams = sr.host_streams(cfg, seed=1)
    expect = [sr.unhinted_vertex(h, top_g.n) for _, h in sr.host_streams(cfg, seed=1)]
    assert [n for n, _ in streams][:2] == ["server1", "server2"] and len(streams) == 150
    for i, (name, h) in enumerate(streams):
        a = T.ip(f"11.0.0.{i + 1}")
        top.attach(a, rand=[h.next_double()])
        assert top.vertex_of(a) == expect[i], name
    assert len(set(expect)) > 90   # ~105 distinct vertices for 150 draws over 183
    # the shipped graph is complete: every attached pair answers its DIRECT edge (golden rows)
    for i in range(0, 150, 7):
        for j in range(0, 150, 11):
            a, b = T.ip(f"11.0.0.{i + 1}"), T.ip(f"11.0.0.{j + 1}")
            assert top.latency(a, b) == z["direct_lat"][expect[i], expect[j]]
            assert top.reliability(a, b) == z["direct_rel"][expect[i], expect[j]]
    top.close()


def test_shadow_random_streams():
    from shadow_amd import shadow_random as sr
    a, b = sr.Random(1), sr.Random(1)
    xs = [a.rand() for _ in range(5)]
    assert xs == [b.rand() for _ in range(5)] and all(0 <= x <= sr.RAND_MAX for x in xs)
    r = sr.Random(7)
    u = r.next_double()
    assert 0.0 <= u <= 1.0
    assert sr.unhinted_vertex(sr.Random(7), 183) == int(182 * u + 0.5)
