"""Offline topology completion and collapse on the GPU path engine (SURVEY.md
§8f-3): the MI355X equivalent of the reference's Python-2/networkx pipeline

  topology.pruned --compute-topology-paths.py--> topology.complete
                  --collapse-topology.py-->      topology (one vertex per geocode)

(src/tools/topology/readme:1-6).  The all-pairs part -- one Dijkstra per point
of interest, compute-topology-paths.py:15-38 -- runs as SSSP rows of the gfx950
batch engine (`spe.PathTable(force_sssp=True, want_aux=True)`): per ordered POI
pair the path latency, folded in path order from 0.0 exactly as Python's
``sum`` over the path's edge list, and the path-order sum of the edge jitters
(the ``aux`` fold), divided here by the hop count as the reference's
``sum(j) / len(j)``.  The rest is host-side bookkeeping over the P x P result,
as in the reference (which is Python too): POI selection (:128-151), the
undirected merge into a complete graph (:41-46), ``ensure_nonzero_latency``
(:98-116) and the per-geocode median collapse (collapse-topology.py:20-49).

Deliberate, documented differences (tests/test_complete.py):
  * client sampling uses a seeded numpy generator (the reference calls the
    unseeded ``random.sample``) and takes every client when there are fewer than
    the sample size (the reference raises);
  * for an unordered POI pair the reference keeps whichever worker's row was
    written last (process scheduling order); here the row of the POI that comes
    first in ``pois`` (rows differ only in the last bits of the fold);
  * route tie-breaks follow the engine's canonical rule; networkx keeps the
    first-pushed equal-distance path.  Identical on tie-free weights.
  * cluster ids ``poi-k`` follow this module's edge order.
There is no CPU fallback: without libspe.so / a GPU, SpeError is raised.
"""
from __future__ import annotations

import argparse
import math
import sys
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import graphs, spe

SELF_LATENCY = 5.0     # compute-topology-paths.py:26-28: a one-vertex path
SELF_JITTER = 0.0


def select_pois(top: graphs.Topology, sample_size: int = 10000, seed: int = 0) -> np.ndarray:
    """compute-topology-paths.py:128-151: clients (type 'client', sampled, plus
    one per geocode the sample misses), servers and relays; vertex ids sorted."""
    types = top.vattrs.get("type")
    if types is None:
        raise ValueError("select_pois: vertices need a 'type' attribute")
    geo = top.vattrs.get("geocode", [None] * top.n)
    clients = [v for v in range(top.n) if types[v] == "client"]
    others = [v for v in range(top.n) if types[v] in ("server", "relay")]
    codes: Dict[str, int] = {}
    for v in clients:
        codes[geo[v]] = v            # last client of each geocode (vertex order)
    if len(clients) > sample_size:
        rng = np.random.default_rng(seed)
        clients = sorted(int(x) for x in rng.choice(np.array(clients), sample_size, replace=False))
    for v in clients:
        codes.pop(geo[v], None)
    pois = set(clients) | set(codes.values()) | set(others)
    return np.array(sorted(pois), dtype=np.int32)


def complete_paths(top: graphs.Topology, pois: Sequence[int], jitter: Optional[np.ndarray] = None,
                   device: int = 0, max_table_bytes: float = 8e9) -> Dict[str, np.ndarray]:
    """Ordered-pair P x P matrices on the GPU: latency (path-order sum), jitter
    (mean over the path's edges), hops; (s, s) = (5.0, 0.0, 0); unreachable:
    latency = jitter = NaN, hops = -1."""
    pois = np.ascontiguousarray(pois, np.int32)
    P = int(pois.shape[0])
    if jitter is None:
        jitter = top.eattrs.get("jitter")
    if jitter is None:
        jitter = np.zeros(top.m)
    jitter = np.asarray(jitter, np.float64)
    g = spe.Graph(top, device=device)
    g.set_edge_aux(jitter)
    nblk = (P + 63) // 64
    per_block = 64.0 * P * 30.0             # latrel 16 + next 4 + hops 2 + aux 8 bytes per entry
    chunk = max(1, min(nblk, int(max_table_bytes // per_block)))
    lat = np.empty((P, P))
    jit = np.empty((P, P))
    hops = np.empty((P, P), np.int32)
    for b0 in range(0, nblk, chunk):
        b1 = min(nblk, b0 + chunk)
        t = spe.PathTable(g, pois, force_sssp=True, want_aux=True, blocks=(b0, b1))
        t.build()
        r0, r1 = b0 * 64, min(P, b1 * 64)
        d = t.download(r0, r1, fields=("lat", "hops"))
        aux = t.download_aux(r0, r1)
        t.close()
        bad = ~d["ok"]
        h = d["hops"]
        lat[r0:r1] = d["lat"]
        lat[r0:r1][bad] = np.nan
        np.divide(aux, h, out=jit[r0:r1], where=h > 0)
        jit[r0:r1][bad | (h <= 0)] = np.nan
        hops[r0:r1] = h
        hops[r0:r1][bad] = -1
    idx = np.arange(P)
    lat[idx, idx] = SELF_LATENCY
    jit[idx, idx] = SELF_JITTER
    hops[idx, idx] = 0
    g.close()
    return {"lat": lat, "jitter": jit, "hops": hops}


def ensure_nonzero_latency(src: np.ndarray, dst: np.ndarray, lat: np.ndarray) -> np.ndarray:
    """compute-topology-paths.py:98-116, vectorised: latencies <= 0 take the mean
    of the positive self-loop (s == d) or inter-vertex latencies, each mean the
    left-to-right float sum over edge order divided by the count."""
    lat = np.array(lat, np.float64)
    zero = lat <= 0.0
    if not zero.any():
        return lat
    intra = (~zero) & (src == dst)
    inter = (~zero) & (src != dst)

    def mean(x):   # Python's float(sum(list)) / len: sequential left fold
        s = 0.0
        for v in x.tolist():
            s += v
        return s / len(x) if len(x) else math.nan

    lat[zero & (src == dst)] = mean(lat[intra])
    lat[zero & (src != dst)] = mean(lat[inter])
    return lat


def complete_topology(top: graphs.Topology, pois: Sequence[int], jitter: Optional[np.ndarray] = None,
                      device: int = 0) -> graphs.Topology:
    """The complete undirected graph over the POIs (compute-topology-paths.py:
    41-46, 152-173): one edge per unordered pair incl. the self-loop, latency /
    jitter from complete_paths, packetloss 0.0; POI vertex attributes copied."""
    pois = np.ascontiguousarray(pois, np.int32)
    P = int(pois.shape[0])
    r = complete_paths(top, pois, jitter, device)
    if np.isnan(r["lat"]).any():
        raise ValueError("complete_topology: some POI pair is unroutable (the reference asserts connectivity)")
    ii, jj = np.triu_indices(P)                 # row of the POI listed first (module docstring)
    lat = ensure_nonzero_latency(ii, jj, r["lat"][ii, jj])
    out = graphs.Topology(n=P, esrc=ii.astype(np.int32), edst=jj.astype(np.int32), elat=lat,
                          eloss=np.zeros(ii.shape[0]), vloss=np.asarray(top.vloss)[pois].copy(),
                          directed=False, prefer_direct=False,
                          vertex_ids=[(top.vertex_ids[v] if top.vertex_ids else f"v{v}") for v in pois.tolist()],
                          vattrs={k: [vals[v] for v in pois.tolist()] for k, vals in top.vattrs.items()},
                          eattrs={"jitter": r["jitter"][ii, jj]}, name=top.name + ":complete")
    return out


def _grouped_median(key: np.ndarray, vals: np.ndarray, nkeys: int) -> np.ndarray:
    """numpy.median of `vals` per key (odd: the middle value; even: (lo + hi) / 2)."""
    o = np.lexsort((vals, key))
    k, v = key[o], vals[o]
    start = np.searchsorted(k, np.arange(nkeys), "left")
    cnt = np.searchsorted(k, np.arange(nkeys), "right") - start
    lo = start + (cnt - 1) // 2
    hi = start + cnt // 2
    lo = np.clip(lo, 0, max(0, len(v) - 1))
    hi = np.clip(hi, 0, max(0, len(v) - 1))
    med = np.where(cnt % 2 == 1, v[lo], (v[lo] + v[hi]) / 2.0) if len(v) else np.zeros(nkeys)
    return np.where(cnt > 0, med, np.nan)


def collapse_topology(top: graphs.Topology, key: str = "geocode") -> graphs.Topology:
    """collapse-topology.py:20-56: one 'cluster' vertex per geocode, named
    poi-1, poi-2, ... in order of first appearance over the edges (source before
    target); each complete-graph edge lands on its unordered cluster pair and
    every edge attribute becomes the median of the values landing there.  A
    cluster copies the attributes of its first vertex, with type 'cluster' and
    asn 0.  Edges with an endpoint lacking the geocode are skipped."""
    geo = top.vattrs.get(key)
    if geo is None:
        raise ValueError(f"collapse_topology: vertices need a '{key}' attribute")
    keep = np.array([geo[int(a)] is not None and geo[int(b)] is not None for a, b in zip(top.esrc, top.edst)], bool)
    src, dst = top.esrc[keep].astype(np.int64), top.edst[keep].astype(np.int64)
    # first appearance order over (src0, dst0, src1, dst1, ...)
    seq = np.empty(2 * src.shape[0], np.int64)
    seq[0::2], seq[1::2] = src, dst
    codes: Dict[str, int] = {}
    rep: List[int] = []
    vcode = np.full(top.n, -1, np.int64)
    for v in seq.tolist():
        if vcode[v] >= 0:
            continue
        c = codes.get(geo[v])
        if c is None:
            c = codes[geo[v]] = len(rep)
            rep.append(v)
        vcode[v] = c
    C = len(rep)
    a, b = vcode[src], vcode[dst]
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    pair = lo * C + hi
    # pairs in order of first appearance (the collapsed graph's edge order)
    uniq, first = np.unique(pair, return_index=True)
    order = uniq[np.argsort(first)]
    kid = np.searchsorted(uniq, pair)
    attrs = {"latency": top.elat[keep], "packetloss": top.eloss[keep]}
    for name, vals in top.eattrs.items():
        attrs[name] = np.asarray(vals)[keep]
    med = {name: _grouped_median(kid, vals, uniq.shape[0]) for name, vals in attrs.items()}
    sel = np.searchsorted(uniq, order)
    vattrs = {k: [vals[v] for v in rep] for k, vals in top.vattrs.items()}
    vattrs["type"] = ["cluster"] * C
    vattrs["asn"] = [0] * C
    return graphs.Topology(n=C, esrc=(order // C).astype(np.int32), edst=(order % C).astype(np.int32),
                           elat=med["latency"][sel], eloss=med["packetloss"][sel],
                           vloss=np.asarray(top.vloss)[rep].copy(), directed=False, prefer_direct=top.prefer_direct,
                           vertex_ids=[f"poi-{i + 1}" for i in range(C)], vattrs=vattrs,
                           eattrs={k: med[k][sel] for k in top.eattrs}, name=top.name + ":collapsed")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="GPU topology completion (compute-topology-paths.py) and collapse")
    ap.add_argument("input", help="pruned topology GraphML (.xml or .xz)")
    ap.add_argument("complete", help="output: complete graph over the POIs")
    ap.add_argument("--collapsed", default=None, help="also write the per-geocode collapse here")
    ap.add_argument("--sample", type=int, default=10000, help="client sample size (CLIENT_SAMPLE_SIZE)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--all-vertices", action="store_true", help="every vertex is a POI")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    top = graphs.load_graphml(a.input)
    pois = np.arange(top.n, dtype=np.int32) if a.all_vertices else select_pois(top, a.sample, a.seed)
    comp = complete_topology(top, pois, device=a.device)
    graphs.write_graphml_attrs(comp, a.complete)
    if a.collapsed:
        graphs.write_graphml_attrs(collapse_topology(comp), a.collapsed)
    print(f"{len(pois)} POIs -> {comp.m} edges", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
