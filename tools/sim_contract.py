"""Design model (not product code): does contracting an independent set of
degree-3 vertices out of C3's relaxation graph (each replaced by the three
shortcut entries between its neighbours, weight w1 + w2) cut the shipped
schedule's traffic?  Runs tools/sim_records.c's GS mode (mode 0) on both graphs
for the same 128-source groups and reports weighted lines per group.

    gcc -O2 -shared -fPIC -o tools/_sim_records.so tools/sim_records.c
    python tools/sim_contract.py [groups]
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import sim_records as sr  # noqa: E402
from shadow_amd import graphs  # noqa: E402


def csr(n, a, b, w):
    r = np.concatenate([a, b])
    c = np.concatenate([b, a])
    ww = np.concatenate([w, w])
    o = np.lexsort((c, r))
    r, c, ww = r[o], c[o], ww[o]
    ptr = np.zeros(n + 1, dtype=np.int32)
    np.add.at(ptr, r + 1, 1)
    return np.cumsum(ptr).astype(np.int32), c.astype(np.int32), ww.astype(np.float64)


def main():
    ng = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    kmax = int(sys.argv[2]) if len(sys.argv) > 2 else 3   # contract degrees 3..kmax
    c4 = len(sys.argv) > 3 and sys.argv[3] == "c4"
    if c4:   # C4: the BA core; sources = the attached stubs' anchors (duplicates kept)
        top = graphs.gen_tiered()
        n, ptr, col, w = sr.csr_of(top, True)
        nl = top.esrc != top.edst
        dfull = np.bincount(np.concatenate([top.esrc[nl], top.edst[nl]]), minlength=top.n)
        cid = -np.ones(top.n, np.int64)
        cid[dfull > 1] = np.arange(int((dfull > 1).sum()))
        att = graphs.tiered_attached(top)
        isatt = np.zeros(top.n, bool)
        isatt[att] = True
        e = nl & (isatt[top.esrc] | isatt[top.edst])
        anc_of = np.where(isatt[top.esrc[e]], top.edst[e], top.esrc[e])
        src_all = cid[anc_of]
    else:
        top = graphs.gen_ba()
        n, ptr, col, w = sr.csr_of(top, False)
    deg = np.diff(ptr)
    # greedy independent set of degree-3 vertices with three distinct neighbours
    X = np.zeros(n, bool)
    blocked = np.zeros(n, bool)
    cand = np.concatenate([np.flatnonzero(deg == k) for k in range(3, kmax + 1)])
    for v in cand:
        nb = col[ptr[v]:ptr[v + 1]]
        if blocked[v] or len(set(nb.tolist())) != len(nb):
            continue
        X[v] = True
        blocked[v] = True
        blocked[nb] = True
    keep = ~X
    ids = -np.ones(n, np.int64)
    ids[keep] = np.arange(keep.sum())
    nc = int(keep.sum())
    ea, eb, ew = [], [], []
    for v in range(n):   # original edges between kept vertices (each once)
        if not keep[v]:
            continue
        for k in range(ptr[v], ptr[v + 1]):
            u = col[k]
            if keep[u] and u > v:
                ea.append(ids[v]); eb.append(ids[u]); ew.append(w[k])
    for x in np.flatnonzero(X):   # shortcuts via x
        nb = col[ptr[x]:ptr[x + 1]]
        ws = w[ptr[x]:ptr[x + 1]]
        for i in range(len(nb)):
            for j in range(i + 1, len(nb)):
                ea.append(ids[nb[i]]); eb.append(ids[nb[j]]); ew.append(ws[i] + ws[j])
    cptr, ccol, cw = csr(nc, np.array(ea), np.array(eb), np.array(ew))
    print(f"C3: {n} vertices / {ptr[-1]} entries -> contracted {nc} vertices / {cptr[-1]} entries "
          f"({X.sum()} vertices of degree 3..{kmax} removed)")
    if c4:
        # a removed anchor seeds its three neighbours; modelled by its lightest neighbour
        src_k = src_all.copy()
        for i in np.flatnonzero(X[src_all]):
            a = src_all[i]
            src_k[i] = col[ptr[a] + int(np.argmin(w[ptr[a]:ptr[a + 1]]))]
        rngv = np.random.default_rng(7)
        cent = rngv.choice(np.unique(src_all), size=len(src_all) // 64, replace=False)
        from scipy.sparse import csr_matrix
        from scipy.sparse.csgraph import dijkstra
        dist, _, owner = dijkstra(csr_matrix((w, col, ptr), shape=(n, n)), indices=cent, min_only=True,
                                  return_predecessors=True)
        perm = np.lexsort((dist[src_all], owner[src_all]))
        order = src_all[perm]
        order_k = src_k[perm]
    else:
        sources = np.flatnonzero(keep)
        order = sr.voronoi_order(n, ptr, col, w, sources, 64)
        order_k = order
    lib = C.CDLL(os.path.join(os.path.dirname(__file__), "_sim_records.so"))
    P = C.c_void_p
    lib.sim_run.argtypes = [C.c_int32, P, P, P, P, C.c_int, C.POINTER(sr.Out)]
    rng = np.random.default_rng(11)
    picks = rng.choice(len(order) // 128, size=ng, replace=False)
    tot = {"full": 0.0, "contracted": 0.0}
    for gi in picks:
        src = np.ascontiguousarray(order[gi * 128:(gi + 1) * 128], dtype=np.int32)
        srck = np.ascontiguousarray(order_k[gi * 128:(gi + 1) * 128], dtype=np.int32)
        for name, (nn, pp, cc, ww, ss) in {"full": (n, ptr, col, w, src),
                                           "contracted": (nc, cptr, ccol, cw, ids[srck].astype(np.int32))}.items():
            o = sr.Out()
            ss = np.ascontiguousarray(ss, dtype=np.int32)
            lib.sim_run(nn, pp.ctypes.data, cc.ctypes.data, ww.ctypes.data, ss.ctypes.data, 0, C.byref(o))
            lines = o.rd_lines + 0.5 * o.wr_lines
            tot[name] += lines
            print(f"  group {gi} {name}: rounds {o.rounds} visits {o.visits} nbr lines {o.nbr_lines} "
                  f"weighted lines {lines:.3g}", flush=True)
    # rows of the removed targets read three anchors' rows (D + route: 24 lines) instead of one
    extra = sum((deg[x] - 1) * 24 for x in np.flatnonzero(X))
    print(f"weighted lines per group: full {tot['full'] / ng:.4g}, contracted {tot['contracted'] / ng:.4g} "
          f"+ rows of removed targets {extra:.3g} -> ratio {(tot['contracted'] / ng + extra) / (tot['full'] / ng):.3f}")


if __name__ == "__main__":
    main()
