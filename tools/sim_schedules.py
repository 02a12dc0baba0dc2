"""Design tool: row visits / lane updates / neighbour-row reads per vertex for one
64-source group on C3 (BA 50k), under (a) the shipped Gauss-Seidel rounds,
(b) Delta-stepping gates (one bound per group, or per lane) and (c) source
groupings (random, Voronoi cells as spe_order_sources, 64 copies of one source
= perfect alignment).  Results are quoted in DESIGN.md section 8.

    gcc -O2 -shared -fPIC -o tools/_sim_delta.so tools/sim_delta.c
    python tools/sim_schedules.py
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


class Out(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("rounds", "visits", "lane_updates", "nbr_rows", "nbr_lines", "fires")]


def main():
    top = gen_ba()
    n = top.n
    m = top.esrc != top.edst
    a, b, w = top.esrc[m], top.edst[m], top.elat[m]
    A = sp.coo_matrix((np.r_[w, w], (np.r_[a, b], np.r_[b, a])), shape=(n, n)).tocsr()
    A.sort_indices()
    ptr, col, ww = A.indptr.astype(np.int32), A.indices.astype(np.int32), A.data.astype(np.float64)
    lib = C.CDLL(os.path.join(HERE, "_sim_delta.so"))

    def run(src, mode, delta):
        o = Out()
        s = np.ascontiguousarray(src, dtype=np.int32)
        lib.simd(C.c_int32(n), ptr.ctypes.data_as(C.c_void_p), col.ctypes.data_as(C.c_void_p),
                 ww.ctypes.data_as(C.c_void_p), s.ctypes.data_as(C.c_void_p), C.c_int(mode), C.c_double(delta),
                 C.byref(o))
        return [o.rounds, o.visits / n, o.lane_updates / (64 * n), o.nbr_rows / n, o.nbr_lines / n, o.fires / n]

    rng = np.random.default_rng(1)
    K = (n + 63) // 64
    D, _, srcs = dijkstra(A, directed=False, indices=rng.permutation(n)[:K], min_only=True, return_predecessors=True)
    order = np.lexsort((D, srcs))
    pick = rng.choice(n // 64, 4, replace=False)
    groups = {"voronoi": [order[i * 64:(i + 1) * 64] for i in pick],
              "random": [rng.choice(n, 64, replace=False) for _ in pick],
              "one source x64": [np.full(64, rng.integers(n)) for _ in pick]}
    print("grouping        schedule        rounds visits/v lane-upd nbr-rows/v nbr-lines/v fires/v")
    for gname, gs in groups.items():
        for mode, deltas in ((0, [0]), (1, [5, 20, 40]), (2, [5, 20])):
            if gname != "voronoi" and mode:
                continue
            for dl in deltas:
                r = np.array([run(g, mode, dl) for g in gs], dtype=float).mean(0)
                sched = ["gauss-seidel", f"delta/group {dl}", f"delta/lane {dl}"][mode]
                print(f"{gname:15s} {sched:15s} {r[0]:6.1f} {r[1]:8.2f} {r[2]:8.2f} {r[3]:10.2f} {r[4]:11.2f} {r[5]:7.2f}")


if __name__ == "__main__":
    main()
