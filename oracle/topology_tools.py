"""CPU restatement of the reference's offline topology tools, used as the
parity oracle for shadow_amd/complete.py.

TEST INFRASTRUCTURE ONLY: imported by tests/ and tools/gen_golden.py -- never
by shadow_amd/.

The reference tools are Python 2 + networkx 1.x scripts
(src/tools/topology/compute-topology-paths.py, collapse-topology.py) that do not
run under Python 3.10; this module restates their per-source / per-edge logic
with the same dependency (networkx, here 3.4.2: `single_source_dijkstra_path`
keeps the 1.x semantics -- binary heap, strict `<` relaxation) and the same
float arithmetic (Python `sum` over the path's edge list, then `/ len`).
"""
from __future__ import annotations

import networkx as nx
import numpy as np


def nx_graph(top, jitter):
    """nx.Graph of the topology with weight = latency (compute-topology-paths.py:160-161).
    Self-loops are kept (they never shorten a path)."""
    G = nx.Graph()
    G.add_nodes_from(range(top.n))
    for e in range(top.m):
        a, b = int(top.esrc[e]), int(top.edst[e])
        G.add_edge(a, b, weight=float(top.elat[e]), latency=float(top.elat[e]), jitter=float(jitter[e]))
    return G


def source_rows(G, src, pois):
    """worker() of compute-topology-paths.py:15-38 for one source: per POI target
    the path latency float(sum(l)) and mean jitter sum(j)/len(j); a one-vertex
    path (target == source) gives (5.0, 0.0).  Unreachable targets are absent."""
    path = nx.single_source_dijkstra_path(G, src)
    out = {}
    poiset = set(pois)
    for dst, p in path.items():
        if dst not in poiset:
            continue
        lat, jit = [], []
        if len(p) <= 1:
            lat.append(5.0)
            jit.append(0.0)
        else:
            for i in range(len(p) - 1):
                e = G[p[i]][p[i + 1]]
                lat.append(float(e["latency"]))
                jit.append(float(e["jitter"]))
        out[dst] = (float(sum(lat)), float(sum(jit) / float(len(jit))), len(p) - 1)
    return out


def all_rows(top, jitter, pois):
    """Ordered-pair matrices (P x P): latency, mean jitter, hops; NaN / -1 unreachable."""
    G = nx_graph(top, jitter)
    P = len(pois)
    lat = np.full((P, P), np.nan)
    jit = np.full((P, P), np.nan)
    hops = np.full((P, P), -1, np.int64)
    col = {int(v): i for i, v in enumerate(pois)}
    for i, s in enumerate(pois):
        for dst, (l, j, h) in source_rows(G, int(s), pois).items():
            lat[i, col[dst]] = l
            jit[i, col[dst]] = j
            hops[i, col[dst]] = h
    return lat, jit, hops


def ensure_nonzero_latency(src, dst, lat):
    """compute-topology-paths.py:98-116: latencies <= 0 become the mean of the
    positive self-loop (s == d) or inter-vertex latencies, in edge order."""
    lat = [float(x) for x in lat]
    lintra = [l for s, d, l in zip(src, dst, lat) if l > 0.0 and s == d]
    linter = [l for s, d, l in zip(src, dst, lat) if l > 0.0 and s != d]
    zeros = [i for i, l in enumerate(lat) if l <= 0.0]
    if zeros:
        lintramean = float(sum(lintra)) / float(len(lintra)) if lintra else float("nan")
        lintermean = float(sum(linter)) / float(len(linter)) if linter else float("nan")
        for i in zeros:
            lat[i] = lintramean if src[i] == dst[i] else lintermean
    return lat


def collapse(src, dst, eattrs, geocode):
    """collapse-topology.py:20-49 over an edge list: cluster id per geocode in
    order of first appearance (source before target of each edge), every edge
    mapped onto its (unordered) cluster pair, each attribute the numpy median of
    the values landing there.  Edges with a missing geocode endpoint are skipped.
    Returns (cluster geocodes, {(a, b): {attr: median}}, representative vertex
    of each cluster)."""
    geoid, order, rep = {}, [], []
    acc = {}
    for e in range(len(src)):
        s, d = int(src[e]), int(dst[e])
        gs, gd = geocode[s], geocode[d]
        if gs is None or gd is None:
            continue
        for g, v in ((gs, s), (gd, d)):
            if g not in geoid:
                geoid[g] = len(order)
                order.append(g)
                rep.append(v)
        a, b = geoid[gs], geoid[gd]
        key = (min(a, b), max(a, b))
        slot = acc.setdefault(key, {})
        for name, vals in eattrs.items():
            slot.setdefault(name, []).append(float(vals[e]))
    med = {k: {name: float(np.median(v)) for name, v in attrs.items()} for k, attrs in acc.items()}
    return order, med, rep
