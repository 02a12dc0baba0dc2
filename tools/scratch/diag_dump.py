import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np, heapq
from shadow_amd import graphs, spe
top = graphs.gen_ba(3000, 3, 25)
rng = np.random.default_rng(225)
top.elat = rng.integers(1, 60, top.elat.shape[0]) * 0.1
n = top.n
adj = [dict() for _ in range(n)]
for a, b, w in zip(top.esrc, top.edst, top.elat):
    a, b = int(a), int(b)
    if a == b: continue
    if b not in adj[a] or w < adj[a][b]: adj[a][b] = w; adj[b][a] = w
iptr = [0]; icol = []; iw = []
for v in range(n):
    for u in sorted(adj[v]): icol.append(u); iw.append(adj[v][u])
    iptr.append(len(icol))
g = spe.Graph(top)
A = np.array([1, 39, 58, 184, 300, 436, 448, 552, 585, 593], np.int32)
os.environ["SPE_DUMP_STATE"] = "/tmp/state.bin"
t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, exact_sources=True, no_contract=True, lanes=64)
t.build()
raw = open("/tmp/state.bin", "rb").read()
L = 64
ne = len(raw) // 12
D = np.frombuffer(raw[:ne * 8], np.float64).reshape(-1, n, L)
P = np.frombuffer(raw[ne * 8:], np.int32).reshape(-1, n, L)
print("groups", D.shape[0])
bad = 0
for j, s in enumerate(A):
    d = D[0, :, j]
    for v in range(n):
        if v == s or not np.isfinite(d[v]): continue
        # fixpoint check
        best = None
        for k in range(iptr[v], iptr[v + 1]):
            u = icol[k]; alt = d[u] + iw[k]
            if not alt > d[u]: continue
            if best is None or (alt, d[u], u) < best[:3]: best = (alt, d[u], u, k)
        pk = P[0, v, j]
        if best[0] != d[v] or pk != best[3]:
            bad += 1
            if bad <= 10:
                print("src", s, "v", v, "deg", iptr[v+1]-iptr[v], "D", repr(d[v]), "P->u", icol[pk] if pk >= 0 else pk,
                      "alt via P", repr(d[icol[pk]] + iw[pk]) if pk >= 0 else None, "du(P)", repr(d[icol[pk]]) if pk >= 0 else None,
                      "canon u", best[2], "du", repr(best[1]), "alt", repr(best[0]))
print("bad", bad)
