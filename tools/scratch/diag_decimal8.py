import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np, heapq
from shadow_amd import graphs, spe
from oracle import Oracle
top = graphs.gen_ba(3000, 3, 25)
rng = np.random.default_rng(225)
top.elat = rng.integers(1, 60, top.elat.shape[0]) * 0.1
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
A = np.array([1, 39, 58, 184, 300, 436, 448, 552, 585, 593], np.int32)
for rep in range(2):
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, exact_sources=True, no_contract=True, lanes=64)
    t.build()
    for i, s in enumerate(A):
        d = dij(int(s))
        pt = t.source_tree(i)
        bad = [(v, int(pt[v]), par(d, v)) for v in range(top.n) if v != s and pt[v] != par(d, v)]
        if bad: print("rep", rep, "slot", i, "src", s, "bad", bad[:4], flush=True)
    t.close()
