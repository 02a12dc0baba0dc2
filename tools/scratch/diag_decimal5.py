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
nbs = [sorted(set(u for u, _ in adj[v])) for v in range(top.n)]
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
t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, exact_sources=True, no_contract=True)
t.build()
dl = t.download()
rows = np.flatnonzero(((dl["next"] != ref["next"]) & ok).any(axis=1))
stats = {"heavy": 0, "light": 0, "same_seg": 0, "diff_seg": 0, "eng_smaller_d": 0}
ex = []
for s in rows[:30]:
    d = dij(int(s))
    pt = t.source_tree(int(s))
    for v in range(top.n):
        if v == s or pt[v] == par(d, v): continue
        deg = len(nbs[v])
        stats["heavy" if deg > 64 else "light"] += 1
        c, e = par(d, v), pt[v]
        if deg > 64:
            sc, se = nbs[v].index(c) // 64, nbs[v].index(e) // 64
            stats["same_seg" if sc == se else "diff_seg"] += 1
        if d[e] < d[c]: stats["eng_smaller_d"] += 1
        if len(ex) < 8: ex.append((int(s), v, deg, c, e, repr(d[c]), repr(d[e]), len(nbs[c]), len(nbs[e])))
print(stats)
for x in ex: print(x)
