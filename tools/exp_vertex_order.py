"""C3 build time under vertex renumberings of the same graph (the relaxation
order and the state rows' memory order follow vertex ids): identity (BA birth
order: hubs first), random, BFS from the largest hub, degree-descending."""
import time
from collections import deque

import numpy as np

from shadow_amd import graphs, spe

base = graphs.gen_ba(50000, 3, 3)
n = base.n


def relabel(perm):   # perm[old] = new
    t = graphs.gen_ba(50000, 3, 3)
    t.esrc = perm[t.esrc].astype(t.esrc.dtype)
    t.edst = perm[t.edst].astype(t.edst.dtype)
    return t


nl = base.esrc != base.edst
deg = np.bincount(np.concatenate([base.esrc[nl], base.edst[nl]]), minlength=n)
adj = [[] for _ in range(n)]
for a, b in zip(base.esrc[nl], base.edst[nl]):
    adj[a].append(b)
    adj[b].append(a)
root = int(np.argmax(deg))
seen = np.zeros(n, bool)
order = []
q = deque([root])
seen[root] = True
while q:
    x = q.popleft()
    order.append(x)
    for y in sorted(adj[x], key=lambda y: -deg[y]):
        if not seen[y]:
            seen[y] = True
            q.append(y)
order += [v for v in range(n) if not seen[v]]
bfs = np.empty(n, np.int64)
bfs[np.array(order)] = np.arange(n)
rng = np.random.default_rng(1)
orders = {"identity": np.arange(n), "random": rng.permutation(n), "bfs_hub": bfs,
          "degree_desc": np.argsort(np.argsort(-deg, kind="stable"), kind="stable")}
for name, perm in orders.items():
    top = relabel(perm)
    g = spe.Graph(top)
    A = g.order_sources(np.arange(n, dtype=np.int32))
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH)
    t.build()
    ts = []
    for _ in range(2):
        t0 = time.perf_counter()
        st = t.build()
        ts.append(time.perf_counter() - t0)
    print(f"{name:12s} table {min(ts):.4f} s  rounds {st['active_rounds']}  lanes {st['relaxed_lanes']}", flush=True)
    del t, g
