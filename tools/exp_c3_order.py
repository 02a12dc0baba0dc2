"""Experiment: does a source-locality slot order help C3 (no pendants)?
Times the batch engine over the first K source blocks for slot orders:
natural (id), voronoi (vertices grouped by their nearest of n/64 random centres,
multi-source Dijkstra, then by distance), hub (grouped by highest-degree
neighbour).  Prints relax ms / sources/s per order."""
import sys
import time

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import dijkstra

sys.path.insert(0, ".")
import bench  # noqa: E402
from shadow_amd import spe  # noqa: E402

top, att, desc = bench.workload("c3")
n = top.n
keep = top.esrc != top.edst
a = sp.coo_matrix((top.elat[keep], (top.esrc[keep], top.edst[keep])), shape=(n, n)).tocsr()
a = a.minimum(a.T) + (a - a.T).maximum(0) + (a.T - a).maximum(0) if False else (a + a.T).tocsr()
rng = np.random.default_rng(1)
orders = {"natural": att}
centres = rng.choice(n, n // 64, replace=False)
d, pred, src = dijkstra(a, indices=centres, min_only=True, return_predecessors=True)
orders["voronoi"] = np.lexsort((d, src)).astype(np.int32)
deg = np.diff(a.indptr)
hub = np.array([a.indices[a.indptr[v]:a.indptr[v + 1]][np.argmax(deg[a.indices[a.indptr[v]:a.indptr[v + 1]]])]
                for v in range(n)])
orders["hub"] = np.lexsort((np.arange(n), hub)).astype(np.int32)
g = spe.Graph(top)
K = int(sys.argv[1]) if len(sys.argv) > 1 else 128
for name, o in orders.items():
    t = spe.PathTable(g, o)
    t.build_blocks(0, 16)
    t.profile(True)
    t0 = time.perf_counter()
    rounds = 0
    for b in range(16, 16 + K, 16):
        rounds += t.build_blocks(b, b + 16)["iterations"]
    el = time.perf_counter() - t0
    kp = t.kernel_profile()
    print(f"{name:8s} {K * 64 / el:9.1f} sources/s  relax {kp['relax']['ms']:.1f} ms  rounds {rounds}", flush=True)
    t.close()
