"""Topology inputs: GraphML ingest with igraph's index semantics, and the
deterministic synthetic generators for the benchmark configs.

GraphML semantics restated from the reference's loader (igraph's GraphML reader,
called at src/main/routing/shd-topology.c:371):
  * vertex index = order of first reference (a <node>, or an <edge> endpoint
    naming an id not declared yet), edge id = order of <edge> elements;
  * numeric attributes parse with strtod semantics (Python float() is the same
    correctly-rounded conversion), a missing numeric value is NaN (the
    reference then treats the attribute as absent, shd-topology.c:315-332);
  * <graph edgedefault="directed|undirected">;
  * the graph attribute ``preferdirectpaths`` is read as a string and is true
    for a case-insensitive prefix "true"/"yes"/"1" (shd-topology.c:745-775);
  * values are looked up by their exact igraph attribute name ("latency",
    "packetloss", ...: igraph_cattribute_has_attr / EAN / VAN with the
    canonical names, shd-topology.c:272-354); the reference's case-insensitive
    prefix match (:178-267) drives its attribute TYPE checks, whose results
    overwrite one another (check_attribute_types, :550-707).
"""
from __future__ import annotations

import lzma
import math
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

GRAPHML_NS = "{http://graphml.graphdrawing.org/xmlns}"


@dataclass
class Topology:
    """Edge-list form of a topology graph (igraph ids) -- what spe_graph_desc carries."""

    n: int
    esrc: np.ndarray  # int32[m]
    edst: np.ndarray  # int32[m]
    elat: np.ndarray  # f64[m] latency, ms
    eloss: np.ndarray  # f64[m] packetloss
    vloss: np.ndarray  # f64[n] packetloss, NaN = absent
    directed: bool = False
    prefer_direct: bool = False
    vertex_ids: Optional[List[str]] = None
    vattrs: Dict[str, list] = field(default_factory=dict)
    eattrs: Dict[str, np.ndarray] = field(default_factory=dict)   # optional f64 edge attrs (jitter)
    name: str = ""

    @property
    def m(self) -> int:
        return int(self.esrc.shape[0])

    def validate(self) -> None:
        """The reference's per-edge checks (shd-topology.c:1026-1109): latency > 0,
        loss in [0,1]; raises ValueError like topology_new returning NULL."""
        if self.m and not np.all(self.elat > 0):
            raise ValueError("edge latency must be > 0")
        if self.m and not np.all((self.eloss >= 0) & (self.eloss <= 1)):
            raise ValueError("edge packetloss must be in [0,1]")
        if self.m and (self.esrc.min() < 0 or self.edst.min() < 0 or
                       max(self.esrc.max(), self.edst.max()) >= self.n):
            raise ValueError("edge endpoint out of range")


def _attr_match(name: str, canonical: str) -> bool:
    return name == canonical


def _attr_prefix(name: str, canonical: str) -> bool:
    """g_ascii_strncasecmp(name, canonical, len(canonical)) == 0 (shd-topology.c:178-267)."""
    return name is not None and name[:len(canonical)].lower() == canonical


_VCHECK = [("id", "string"), ("ip", "string"), ("citycode", "string"), ("countrycode", "string"),
           ("asn", "numeric"), ("type", "string"), ("bandwidthdown", "numeric"), ("bandwidthup", "numeric"),
           ("packetloss", "numeric"), ("geocode", "string")]
_ECHECK = [("latency", "numeric"), ("jitter", "numeric"), ("packetloss", "numeric")]


def _igraph_type(attr_type: str) -> str:
    t = (attr_type or "string").lower()
    return "numeric" if t in ("int", "long", "float", "double") else ("boolean" if t == "boolean" else "string")


def check_attribute_types(keys) -> bool:
    """_topology_checkGraphAttributes (shd-topology.c:550-707) over the <key>
    declarations in document order, `keys` = [(attr.name, attr.type, for)]:
    every attribute whose name prefix-matches a known one gets a type check that
    OVERWRITES the running result; the required-attribute checks (exact names)
    can only clear it.  Hence only the last prefix-matched edge attribute's type
    counts, plus the presence of "latency" and "packetloss"."""
    def dom(f, d):
        return f in (d, "all")
    ok = True
    for name, typ, f in keys:
        if dom(f, "graph") and _attr_prefix(name, "preferdirectpaths"):
            ok = _igraph_type(typ) == "string"
    for name, typ, f in keys:
        if not dom(f, "node"):
            continue
        for canon, want in _VCHECK:
            if _attr_prefix(name, canon):
                ok = _igraph_type(typ) == want
                break
    vnames = {n for n, _, f in keys if dom(f, "node")}
    if "bandwidthdown" not in vnames or "bandwidthup" not in vnames:
        ok = False
    for name, typ, f in keys:
        if not dom(f, "edge"):
            continue
        for canon, want in _ECHECK:
            if _attr_prefix(name, canon):
                ok = _igraph_type(typ) == want
                break
    enames = {n for n, _, f in keys if dom(f, "edge")}
    if "latency" not in enames or "packetloss" not in enames:
        ok = False
    return ok


def load_graphml(source: str, is_text: bool = False) -> Topology:
    """Parse a GraphML file (optionally .xz) or a GraphML string."""
    if is_text:
        root = ET.fromstring(source)
    elif source.endswith(".xz"):
        with lzma.open(source, "rb") as f:
            root = ET.fromstring(f.read())
    else:
        root = ET.parse(source).getroot()

    def tag(el):
        return el.tag.replace(GRAPHML_NS, "")

    keys = {}
    key_list = []
    for k in root:
        if tag(k) == "key":
            key_list.append((k.get("attr.name"), k.get("attr.type", "string"), k.get("for", "all")))
            default = None
            for d in k:
                if tag(d) == "default":
                    default = d.text
            keys[k.get("id")] = (k.get("attr.name"), k.get("attr.type", "string"),
                                 k.get("for", "all"), default)
    graph = None
    for g in root:
        if tag(g) == "graph":
            graph = g
            break
    if graph is None:
        raise ValueError("no <graph> element")
    directed = graph.get("edgedefault", "directed") == "directed"

    index: Dict[str, int] = {}
    vdata: List[Dict[str, str]] = []
    edges = []
    gdata: Dict[str, str] = {}

    def vid(name: str) -> int:
        if name not in index:
            index[name] = len(index)
            vdata.append({})
        return index[name]

    for el in graph:
        t = tag(el)
        if t == "node":
            v = vid(el.get("id"))
            for d in el:
                if tag(d) == "data":
                    vdata[v][d.get("key")] = d.text or ""
        elif t == "edge":
            a, b = vid(el.get("source")), vid(el.get("target"))
            dd = {}
            for d in el:
                if tag(d) == "data":
                    dd[d.get("key")] = d.text or ""
            edges.append((a, b, dd))
        elif t == "data":
            gdata[el.get("key")] = el.text or ""

    def numeric(text):
        if text is None or text.strip() == "":
            return math.nan
        return float(text)

    def find_key(kind: str, canonical: str):
        for kid, (name, typ, for_, default) in keys.items():
            if name is not None and for_ in (kind, "all") and _attr_match(name, canonical):
                return kid, default
        return None, None

    n = len(index)
    m = len(edges)
    if not check_attribute_types(key_list):
        raise ValueError("topology validation failed because of problem with graph, vertex, or edge attributes")
    lat_k, lat_def = find_key("edge", "latency")
    loss_k, loss_def = find_key("edge", "packetloss")
    esrc = np.array([e[0] for e in edges], dtype=np.int32)
    edst = np.array([e[1] for e in edges], dtype=np.int32)
    elat = np.array([numeric(e[2].get(lat_k, lat_def)) for e in edges], dtype=np.float64)
    eloss = np.array([numeric(e[2].get(loss_k, loss_def)) for e in edges], dtype=np.float64)
    vl_k, vl_def = find_key("node", "packetloss")
    vloss = np.full(n, math.nan)
    if vl_k is not None:
        vloss = np.array([numeric(vd.get(vl_k, vl_def)) for vd in vdata], dtype=np.float64)
    pref = False
    pk, pdef = find_key("graph", "preferdirectpaths")
    if pk is not None:
        val = gdata.get(pk, pdef) or ""
        low = val.lower()
        pref = low.startswith("true") or low.startswith("yes") or low.startswith("1")
    names = [None] * n
    for name, i in index.items():
        names[i] = name
    vattrs = {}
    for canon in ("ip", "citycode", "countrycode", "geocode", "type", "bandwidthdown", "bandwidthup"):
        kid, kdef = find_key("node", canon)
        if kid is not None:
            vattrs[canon] = [vd.get(kid, kdef) for vd in vdata]
    eattrs = {}
    jk, jdef = find_key("edge", "jitter")
    if jk is not None:
        eattrs["jitter"] = np.array([numeric(e[2].get(jk, jdef)) for e in edges], dtype=np.float64)
    top = Topology(n=n, esrc=esrc, edst=edst, elat=elat, eloss=eloss, vloss=vloss,
                   directed=directed, prefer_direct=pref, vertex_ids=names, vattrs=vattrs, eattrs=eattrs)
    return top


# --------------------------------------------------------------------------
# Synthetic generators.  All undirected, simple, one component,
# continuous PCG64 weights (tie-free), latency >= 0.5 ms, a self-loop on every
# attached vertex (latency U(0.5, 2.0), loss 0), vertex packetloss present = 0.0.
# --------------------------------------------------------------------------

def _finish(n, pairs, lat, loss, attached, rng, name, vloss=None) -> Topology:
    pairs = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
    loops = np.asarray(attached, dtype=np.int64)
    loop_lat = rng.uniform(0.5, 2.0, size=loops.shape[0])
    esrc = np.concatenate([pairs[:, 0], loops]).astype(np.int32)
    edst = np.concatenate([pairs[:, 1], loops]).astype(np.int32)
    elat = np.concatenate([lat, loop_lat]).astype(np.float64)
    eloss = np.concatenate([loss, np.zeros(loops.shape[0])]).astype(np.float64)
    if vloss is None:
        vloss = np.zeros(n)
    return Topology(n=n, esrc=esrc, edst=edst, elat=elat, eloss=eloss,
                    vloss=np.asarray(vloss, dtype=np.float64), directed=False, name=name)


def barabasi_albert_pairs(n: int, m: int, rng: np.random.Generator) -> np.ndarray:
    """Preferential attachment: vertex k>m joins with m distinct edges to earlier
    vertices chosen proportionally to degree (repeated-endpoint list)."""
    pairs = np.empty(((n - m) * m, 2), dtype=np.int64)
    repeated = np.empty(2 * m * n + m, dtype=np.int64)
    rl = 0
    targets = list(range(m))
    w = 0
    for src in range(m, n):
        for t in targets:
            pairs[w, 0] = src
            pairs[w, 1] = t
            w += 1
        repeated[rl:rl + m] = targets
        rl += m
        repeated[rl:rl + m] = src
        rl += m
        chosen = set()
        while len(chosen) < m:
            idx = rng.integers(0, rl, size=2 * m)
            for i in idx:
                chosen.add(int(repeated[i]))
                if len(chosen) == m:
                    break
        targets = sorted(chosen)
    return pairs[:w]


def gen_ba(n: int = 50000, m: int = 3, seed: int = 3, attached: Optional[np.ndarray] = None,
           lat_range=(1.0, 100.0)) -> Topology:
    """C3: power-law AS-like graph, latency U(1,100) ms, loss U(0,0.01); A = all."""
    rng = np.random.Generator(np.random.PCG64(seed))
    pairs = barabasi_albert_pairs(n, m, rng)
    lat = rng.uniform(lat_range[0], lat_range[1], size=pairs.shape[0])
    loss = rng.uniform(0.0, 0.01, size=pairs.shape[0])
    att = np.arange(n) if attached is None else attached
    return _finish(n, pairs, lat, loss, att, rng, f"ba{n}_m{m}_s{seed}")


def gen_rgg(n: int = 10000, seed: int = 2, mean_degree: float = 12.0) -> Topology:
    """C2: random geometric graph in [0,1)^2, r = sqrt(deg/(pi n)), largest
    component kept and relabelled; latency = 1 + 200 d ms, loss U(0,0.01)."""
    from scipy.spatial import cKDTree
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components

    rng = np.random.Generator(np.random.PCG64(seed))
    pts = rng.random((n, 2))
    r = math.sqrt(mean_degree / (math.pi * n))
    pairs = np.array(sorted(cKDTree(pts).query_pairs(r)), dtype=np.int64).reshape(-1, 2)
    adj = coo_matrix((np.ones(len(pairs)), (pairs[:, 0], pairs[:, 1])), shape=(n, n))
    _, lab = connected_components(adj, directed=False)
    big = np.bincount(lab).argmax()
    keep = np.flatnonzero(lab == big)
    remap = -np.ones(n, dtype=np.int64)
    remap[keep] = np.arange(keep.shape[0])
    sel = (lab[pairs[:, 0]] == big) & (lab[pairs[:, 1]] == big)
    pairs = remap[pairs[sel]]
    d = np.linalg.norm(pts[keep][pairs[:, 0]] - pts[keep][pairs[:, 1]], axis=1)
    lat = 1.0 + 200.0 * d
    loss = rng.uniform(0.0, 0.01, size=pairs.shape[0])
    nk = keep.shape[0]
    return _finish(nk, pairs, lat, loss, np.arange(nk), rng, f"rgg{n}_s{seed}")


def gen_tiered(n_core: int = 20000, n_stub: int = 180000, n_attached: int = 100000,
               seed: int = 4) -> Topology:
    """C4: BA core (m=3, latency U(5,150)) + stub vertices with one edge each to a
    uniform core vertex (latency U(0.5,10)); attached = the first n_attached stubs."""
    rng = np.random.Generator(np.random.PCG64(seed))
    core = barabasi_albert_pairs(n_core, 3, rng)
    core_lat = rng.uniform(5.0, 150.0, size=core.shape[0])
    stubs = np.arange(n_core, n_core + n_stub, dtype=np.int64)
    anchor = rng.integers(0, n_core, size=n_stub)
    stub_pairs = np.stack([stubs, anchor], axis=1)
    stub_lat = rng.uniform(0.5, 10.0, size=n_stub)
    pairs = np.concatenate([core, stub_pairs])
    lat = np.concatenate([core_lat, stub_lat])
    loss = rng.uniform(0.0, 0.01, size=pairs.shape[0])
    att = np.arange(n_core, n_core + n_attached)
    top = _finish(n_core + n_stub, pairs, lat, loss, att, rng, f"tiered{n_core}+{n_stub}_s{seed}")
    return top


def tiered_attached(top: Topology, n_core: int = 20000, n_attached: int = 100000) -> np.ndarray:
    return np.arange(n_core, n_core + n_attached, dtype=np.int32)


def gen_random_small(n: int, extra_edges: int, seed: int, integer_weights: bool = False,
                     directed: bool = False, self_loops: bool = True, vloss_nonzero: bool = False,
                     multi: int = 0) -> Topology:
    """Small test graphs: a random spanning tree plus random extra edges.
    integer_weights=True produces deliberate distance ties; multi>0 adds parallel
    edges; directed graphs get both directions of the spanning tree so they are
    strongly connected."""
    rng = np.random.Generator(np.random.PCG64(seed))
    perm = rng.permutation(n)
    tree = [(int(perm[i]), int(perm[rng.integers(0, i)])) for i in range(1, n)]
    pairs = list(tree)
    if directed:
        pairs += [(b, a) for (a, b) in tree]
    seen = set((a, b) for a, b in pairs)
    if not directed:
        seen |= set((b, a) for a, b in pairs)
    tries = 0
    while len(pairs) < len(tree) * (2 if directed else 1) + extra_edges and tries < 100 * extra_edges + 100:
        tries += 1
        a, b = int(rng.integers(0, n)), int(rng.integers(0, n))
        if a == b or (a, b) in seen:
            continue
        seen.add((a, b))
        if not directed:
            seen.add((b, a))
        pairs.append((a, b))
    for _ in range(multi):
        a, b = pairs[int(rng.integers(0, len(pairs)))]
        pairs.append((a, b))
    pairs = np.array(pairs, dtype=np.int64)
    if integer_weights:
        lat = rng.integers(1, 4, size=pairs.shape[0]).astype(np.float64)
        loss = rng.integers(0, 3, size=pairs.shape[0]) * 0.005
    else:
        lat = rng.uniform(0.5, 50.0, size=pairs.shape[0])
        loss = rng.uniform(0.0, 0.01, size=pairs.shape[0])
    vloss = rng.uniform(0.0, 0.02, size=n) if vloss_nonzero else np.zeros(n)
    att = np.arange(n) if self_loops else np.array([], dtype=np.int64)
    top = _finish(n, pairs, lat, loss, att, rng, f"small{n}_s{seed}", vloss=vloss)
    top.directed = directed
    if integer_weights and self_loops:
        top.elat[-n:] = rng.integers(1, 3, size=n).astype(np.float64)
    return top


def write_graphml(top: Topology, path: str, ips=None, bandwidth: int = 10240) -> None:
    """Write a topology as GraphML the reference (and topology_new) accepts:
    node attrs packetloss / bandwidthdown / bandwidthup (+ ip), edge latency /
    packetloss; vertex i gets id "v{i}"."""
    out = ['<?xml version="1.0" encoding="utf-8"?>',
           '<graphml xmlns="http://graphml.graphdrawing.org/xmlns">',
           '<key attr.name="packetloss" attr.type="double" for="edge" id="e1"/>',
           '<key attr.name="latency" attr.type="double" for="edge" id="e0"/>',
           '<key attr.name="ip" attr.type="string" for="node" id="n3"/>',
           '<key attr.name="bandwidthup" attr.type="int" for="node" id="n2"/>',
           '<key attr.name="bandwidthdown" attr.type="int" for="node" id="n1"/>',
           '<key attr.name="packetloss" attr.type="double" for="node" id="n0"/>']
    if top.prefer_direct:
        out.insert(2, '<key attr.name="preferdirectpaths" attr.type="string" for="graph" id="g0"/>')
    out.append(f'<graph edgedefault="{"directed" if top.directed else "undirected"}">')
    if top.prefer_direct:
        out.append('<data key="g0">true</data>')
    for v in range(top.n):
        d = [f'<data key="n1">{bandwidth}</data>', f'<data key="n2">{bandwidth}</data>']
        if not math.isnan(top.vloss[v]):
            d.append(f'<data key="n0">{repr(float(top.vloss[v]))}</data>')
        if ips is not None and ips[v]:
            d.append(f'<data key="n3">{ips[v]}</data>')
        out.append(f'<node id="v{v}">{"".join(d)}</node>')
    for e in range(top.m):
        out.append(f'<edge source="v{int(top.esrc[e])}" target="v{int(top.edst[e])}">'
                   f'<data key="e0">{repr(float(top.elat[e]))}</data>'
                   f'<data key="e1">{repr(float(top.eloss[e]))}</data></edge>')
    out.append("</graph></graphml>")
    with open(path, "w") as f:
        f.write("\n".join(out))


_VATTR_TYPES = {"bandwidthdown": "int", "bandwidthup": "int", "asn": "int"}


def write_graphml_attrs(top: Topology, path: str) -> None:
    """GraphML of a topology with all its attributes: vertex ids from
    ``vertex_ids`` (else "v{i}"), node packetloss + every ``vattrs`` entry, edge
    latency / packetloss + every ``eattrs`` entry (the completion and collapse
    tools' output, compute-topology-paths.py:173 / collapse-topology.py:55)."""
    from xml.sax.saxutils import escape, quoteattr
    keys = ['<key attr.name="packetloss" attr.type="double" for="node" id="n0"/>']
    vk = {}
    for i, name in enumerate(sorted(top.vattrs)):
        vk[name] = f"n{i + 1}"
        keys.append(f'<key attr.name="{name}" attr.type="{_VATTR_TYPES.get(name, "string")}" for="node" '
                    f'id="{vk[name]}"/>')
    keys += ['<key attr.name="latency" attr.type="double" for="edge" id="e0"/>',
             '<key attr.name="packetloss" attr.type="double" for="edge" id="e1"/>']
    ek = {}
    for i, name in enumerate(sorted(top.eattrs)):
        ek[name] = f"e{i + 2}"
        keys.append(f'<key attr.name="{name}" attr.type="double" for="edge" id="{ek[name]}"/>')
    if top.prefer_direct:
        keys.append('<key attr.name="preferdirectpaths" attr.type="string" for="graph" id="g0"/>')
    out = ['<?xml version="1.0" encoding="utf-8"?>', '<graphml xmlns="http://graphml.graphdrawing.org/xmlns">']
    out += keys
    out.append(f'<graph edgedefault="{"directed" if top.directed else "undirected"}">')
    if top.prefer_direct:
        out.append('<data key="g0">true</data>')
    ids = top.vertex_ids if top.vertex_ids is not None else [f"v{v}" for v in range(top.n)]
    for v in range(top.n):
        d = []
        if not math.isnan(top.vloss[v]):
            d.append(f'<data key="n0">{repr(float(top.vloss[v]))}</data>')
        for name, kid in vk.items():
            x = top.vattrs[name][v]
            if x is not None:
                d.append(f'<data key="{kid}">{escape(str(x))}</data>')
        out.append(f'<node id={quoteattr(str(ids[v]))}>{"".join(d)}</node>')
    for e in range(top.m):
        d = [f'<data key="e0">{repr(float(top.elat[e]))}</data>', f'<data key="e1">{repr(float(top.eloss[e]))}</data>']
        for name, kid in ek.items():
            d.append(f'<data key="{kid}">{repr(float(top.eattrs[name][e]))}</data>')
        out.append(f'<edge source={quoteattr(str(ids[int(top.esrc[e])]))} '
                   f'target={quoteattr(str(ids[int(top.edst[e])]))}>{"".join(d)}</edge>')
    out.append("</graph></graphml>")
    with open(path, "w") as f:
        f.write("\n".join(out))
