"""Design experiment (not product code): does the relaxation-vertex numbering
change the batch engine's speed through L2 locality?  The C3 graph is relabelled
by several orderings; slot i is always the same original vertex, so every
ordering builds the same rows (up to tie-breaks), only the HBM layout differs."""
import sys, time, os
import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import reverse_cuthill_mckee, breadth_first_order
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shadow_amd import graphs, spe

top = graphs.gen_ba(50000, 3, 3)
n = top.n
M = sp.coo_matrix((np.ones(top.m), (top.esrc, top.edst)), shape=(n, n)).tocsr()
M = (M + M.T).tocsr()
deg = np.diff(M.indptr)
orders = {
    "identity": np.arange(n),
    "random": np.random.default_rng(0).permutation(n),
    "rcm": reverse_cuthill_mckee(M, symmetric_mode=True),
    "degree": np.argsort(-deg, kind="stable"),
    "bfs_hub": breadth_first_order(M, int(np.argmax(deg)), directed=False, return_predecessors=False),
}
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 64
for name, order in orders.items():
    newid = np.empty(n, np.int64)
    newid[order] = np.arange(n)   # order[k] = old vertex placed at position k
    t2 = graphs.Topology(n=n, esrc=newid[top.esrc].astype(np.int32), edst=newid[top.edst].astype(np.int32),
                         elat=top.elat, eloss=top.eloss, vloss=top.vloss[order])
    att = newid[np.arange(n)].astype(np.int32)
    g = spe.Graph(t2, device=0)
    t = spe.PathTable(g, att, blocks=(0, nb))
    t.build_blocks(0, 16)
    t.profile(True)
    t0 = time.perf_counter()
    t.build_blocks(0, nb)
    el = time.perf_counter() - t0
    kp = t.kernel_profile()
    st = t.stats()
    print(f"{name:10s} {nb*64/el:9.0f} sources/s  relax {kp['relax']['ms']:8.1f} ms / {kp['relax']['launches']} "
          f"heavy {kp['heavy']['ms']:6.1f} rows {kp['rows']['ms']:6.1f}  iters {st['iterations']}", flush=True)
    t.close(); g.close()
