"""Design tool: per-round histogram of k_relax_s's schedule on C3 (BA 50k) for
128-lane groups of clustered sources (Voronoi cells as spe_order_sources), and
how many own-row / neighbour lines the settle bound (tools/sim_final.c) would
skip.  VERDICT r05 Next #2 asked for this histogram before any change.

    gcc -O2 -shared -fPIC -o tools/_sim_final.so tools/sim_final.c
    python tools/sim_final.py [groups]
"""
import ctypes as C
import os
import sys

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import dijkstra

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from shadow_amd.graphs import gen_ba  # noqa: E402

FIELDS = ("visits", "lane_updates", "own_lines", "own_lines_final", "nbr_lines", "nbr_lines_final", "rows_all_final")


class RoundOut(C.Structure):
    _fields_ = [(k, C.c_int64) for k in FIELDS]


def main():
    ng = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    top = gen_ba(50000, 3, 3)
    n = top.n
    m = top.esrc != top.edst
    a, b, w = top.esrc[m], top.edst[m], top.elat[m]
    relabel = os.environ.get("RELABEL", "")
    if relabel:   # vertex processing order: new id = rank under the key
        deg = np.bincount(np.r_[a, b], minlength=n)
        rng0 = np.random.default_rng(9)
        key = {"degree": -deg, "random": rng0.permutation(n), "revid": -np.arange(n)}[relabel]
        perm = np.empty(n, np.int64)
        perm[np.argsort(key, kind="stable")] = np.arange(n)
        a, b = perm[a], perm[b]
    else:
        perm = np.arange(n)
    A = sp.coo_matrix((np.r_[w, w], (np.r_[a, b], np.r_[b, a])), shape=(n, n)).tocsr()
    A.sum_duplicates()
    A.sort_indices()
    ptr, col, ww = A.indptr.astype(np.int32), A.indices.astype(np.int32), A.data.astype(np.float64)
    lib = C.CDLL(os.path.join(HERE, "_sim_final.so"))
    rng = np.random.default_rng(1)
    K = (n + 63) // 64
    grouping = os.environ.get("GROUPING", "voronoi")
    Ag = A.copy()
    if grouping == "hops":   # Voronoi cells by hop count instead of latency
        Ag.data[:] = 1.0
    D, _, srcs = dijkstra(Ag, directed=False, indices=rng.permutation(n)[:K], min_only=True, return_predecessors=True)
    order = np.lexsort((D, srcs))
    if grouping == "cell128":   # cells of 128 sources (K/2 centres): one cell per group
        D, _, srcs = dijkstra(A, directed=False, indices=rng.permutation(n)[:K // 2], min_only=True,
                              return_predecessors=True)
        order = np.lexsort((D, srcs))
    pick = rng.choice(n // 128, ng, replace=False)
    tot = None
    MAXR = 64
    for gi in pick:
        src = np.ascontiguousarray(order[gi * 128:(gi + 1) * 128], dtype=np.int32)
        outs = (RoundOut * MAXR)()
        r = lib.sim_final(C.c_int32(n), ptr.ctypes.data_as(C.c_void_p), col.ctypes.data_as(C.c_void_p),
                          ww.ctypes.data_as(C.c_void_p), src.ctypes.data_as(C.c_void_p), C.c_double(float(ww.min())),
                          C.c_int32(MAXR), outs, C.c_int(int(os.environ.get('PER_ITEM', '0'))), C.c_int(int(os.environ.get('ORDER', '0'))))
        arr = np.array([[getattr(outs[i], f) for f in FIELDS] for i in range(r)], dtype=float)
        if tot is None or arr.shape[0] > tot.shape[0]:
            pad = np.zeros((arr.shape[0], len(FIELDS)))
            if tot is not None:
                pad[:tot.shape[0]] = tot
            tot = pad
        tot[:arr.shape[0]] += arr
    tot /= ng
    print(f"C3 BA 50k, {ng} groups of 128 clustered sources, per group and round (means):")
    print("round  visits  lane_upd  own_lines  own_after_bound  nbr_lines  nbr_after_bound  rows_all_final")
    for i, row in enumerate(tot):
        print(f"{i:5d} {row[0]:7.0f} {row[1]:9.0f} {row[2]:10.0f} {row[3]:16.0f} {row[4]:10.0f} {row[5]:16.0f} {row[6]:15.0f}")
    s = tot.sum(0)
    print(f"total  visits/vertex {s[0] / n:.2f}  lane updates/(vertex,lane) {s[1] / n / 128:.2f}  "
          f"own lines {s[2]:.0f} -> {s[3]:.0f} ({s[3] / s[2]:.2f})  nbr lines {s[4]:.0f} -> {s[5]:.0f} "
          f"({s[5] / s[4]:.2f})  all lines {s[2] + s[4]:.0f} -> {s[3] + s[5]:.0f} ({(s[3] + s[5]) / (s[2] + s[4]):.2f})")


if __name__ == "__main__":
    main()
