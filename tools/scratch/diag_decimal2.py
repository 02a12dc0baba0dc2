import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np, heapq
from shadow_amd import graphs, spe
top = graphs.gen_ba(3000, 3, 25)
rng = np.random.default_rng(225)
top.elat = rng.integers(1, 60, top.elat.shape[0]) * 0.1
A = np.arange(top.n, dtype=np.int32)
s = 1665
adj = [[] for _ in range(top.n)]
for a, b, w in zip(top.esrc, top.edst, top.elat):
    if a == b: continue
    adj[a].append((b, w)); adj[b].append((a, w))
d = [float('inf')] * top.n; d[s] = 0.0
pq = [(0.0, s)]; done = [False]*top.n
while pq:
    du, u = heapq.heappop(pq)
    if done[u]: continue
    done[u] = True
    for v, w in adj[u]:
        alt = du + w
        if alt < d[v]:
            d[v] = alt; heapq.heappush(pq, (alt, v))
def par(v):
    best = None
    for u, w in adj[v]:
        if d[u] + w == d[v] and d[u] + w > d[u]:
            if best is None or (d[u], u) < (d[best], best): best = u
    return best
g = spe.Graph(top)
for kw in (dict(exact_sources=True, no_contract=True), dict(exact_sources=True)):
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, **kw)
    t.build()
    pt = t.source_tree(s)
    row = t.download(s, s + 1)
    bad = [v for v in range(top.n) if v != s and pt[v] != par(v)]
    print(kw, "differing parents", len(bad))
    for v in bad[:6]:
        print(" v", v, "d", repr(d[v]), "engine", pt[v], "canon", par(v), "cands", [(u, repr(d[u]), repr(d[u]+w)) for u, w in adj[v] if d[u] + w == d[v]])
    lat = row["lat"][0]
    dd = np.array(d); ok = np.isfinite(dd)
    print(" lat mismatches", int((lat[ok] != np.where(dd[ok]==0,1,dd[ok])).sum()))
