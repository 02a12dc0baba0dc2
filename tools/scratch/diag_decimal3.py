import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np, heapq
from shadow_amd import graphs, spe
from oracle import Oracle
top = graphs.gen_ba(3000, 3, 25)
rng = np.random.default_rng(225)
top.elat = rng.integers(1, 60, top.elat.shape[0]) * 0.1
A = np.arange(top.n, dtype=np.int32)
adj = [[] for _ in range(top.n)]
for a, b, w in zip(top.esrc, top.edst, top.elat):
    if a == b: continue
    adj[a].append((int(b), w)); adj[b].append((int(a), w))
def dij(s):
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
    return d
def par(d, v):
    best = None
    for u, w in adj[v]:
        if d[u] + w == d[v] and d[u] + w > d[u]:
            if best is None or (d[u], u) < (d[best], best): best = u
    return best
g = spe.Graph(top)
ref = Oracle(top).rows(A, A, tie_mode=1)
ok = ref["kind"] != 0
for kw in (dict(exact_sources=True, no_contract=True), dict(exact_sources=True)):
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, **kw)
    t.build()
    dl = t.download()
    mis = ((dl["next"] != ref["next"]) & ok).any(axis=1)
    rows = np.flatnonzero(mis)
    print(kw, "rows", rows.size, rows[:10])
    for s in rows[:3]:
        d = dij(int(s))
        pt = t.source_tree(int(s))
        bad = [v for v in range(top.n) if v != s and pt[v] != par(d, v)]
        print(" src", s, "differing parents", len(bad))
        for v in bad[:3]:
            print("   v", v, "d", repr(d[v]), "engine", pt[v], "canon", par(d, v), "cands",
                  [(u, repr(d[u])) for u, w in adj[v] if d[u] + w == d[v]], "engine-par d", repr(d[pt[v]]) if pt[v] >= 0 else None,
                  "eng alt", repr(d[pt[v]] + dict(adj[v])[pt[v]]) if pt[v] >= 0 else None)
    t.close()
