"""Driver for tools/sim_records.c (design model, not product code): GS vs
stale-record relaxation on C3 (BA 50k) or the C4 core, a few 128-source groups
taken from a Voronoi-cell source order like spe_order_sources'.

    gcc -O2 -shared -fPIC -o tools/_sim_records.so tools/sim_records.c
    python tools/sim_records.py [c3|c4] [groups]

Result (C3, 3 groups, MEASUREMENTS.md): GS 605 weighted lines per vertex and group,
REC 795, DIST 771 -- neither alternative beats the shipped schedule.
"""
import ctypes as C
import os
import sys

import numpy as np
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import dijkstra

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from shadow_amd import graphs  # noqa: E402

FIELDS = ["rounds", "visits", "lane_updates", "rd_lines", "wr_lines", "nbr_lines", "own_lines", "route_lines",
          "par_rd", "par_wr", "tree_visits", "tree_rounds", "tree_rd", "tree_wr", "max_hops", "prune_row",
          "prune_line16", "prune_line32", "nbr_reads"]


class Out(C.Structure):
    _fields_ = [(f, C.c_int64) for f in FIELDS]


def csr_of(top, core_only):
    keep = top.esrc != top.edst
    a, b, w = top.esrc[keep], top.edst[keep], top.elat[keep]
    n = top.n
    if core_only:   # C4: the relaxation graph is the 20k BA core (stubs are pendants)
        deg = np.bincount(np.concatenate([a, b]), minlength=n)
        core = deg > 1
        sel = core[a] & core[b]
        a, b, w = a[sel], b[sel], w[sel]
        ids = -np.ones(n, dtype=np.int64)
        ids[core] = np.arange(core.sum())
        a, b, n = ids[a], ids[b], int(core.sum())
    r = np.concatenate([a, b])
    c = np.concatenate([b, a])
    ww = np.concatenate([w, w])
    o = np.lexsort((c, r))
    r, c, ww = r[o], c[o], ww[o]
    ptr = np.zeros(n + 1, dtype=np.int32)
    np.add.at(ptr, r + 1, 1)
    ptr = np.cumsum(ptr).astype(np.int32)
    return n, ptr, c.astype(np.int32), ww.astype(np.float64)


def voronoi_order(n, ptr, col, w, sources, cell, seed=7):
    rng = np.random.default_rng(seed)
    k = max(1, len(sources) // cell)
    centres = rng.choice(sources, size=k, replace=False)
    g = csr_matrix((w, col, ptr), shape=(n, n))
    dist, _, owner = dijkstra(g, indices=centres, min_only=True, return_predecessors=True)
    # owner = the centre index reaching each vertex
    cid = owner[sources]
    return sources[np.lexsort((dist[sources], cid))]


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    ng = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    if cfg == "c3":
        top = graphs.gen_ba()
        n, ptr, col, w = csr_of(top, False)
        sources = np.arange(n)
    else:
        top = graphs.gen_tiered()
        n, ptr, col, w = csr_of(top, True)
        sources = np.random.default_rng(1).integers(0, n, size=100000)   # stubs' anchors (approx.)
        sources = np.unique(sources)
    order = voronoi_order(n, ptr, col, w, sources, 64)
    lib = C.CDLL(os.path.join(os.path.dirname(__file__), "_sim_records.so"))
    P = C.c_void_p
    lib.sim_run.argtypes = [C.c_int32, P, P, P, P, C.c_int, C.POINTER(Out)]
    rng = np.random.default_rng(11)
    picks = rng.choice(len(order) // 128, size=ng, replace=False)
    tot = {m: np.zeros(len(FIELDS)) for m in (0, 1, 2)}
    for gi in picks:
        src = np.ascontiguousarray(order[gi * 128:(gi + 1) * 128], dtype=np.int32)
        for mode in (0, 1, 2):
            o = Out()
            lib.sim_run(n, ptr.ctypes.data, col.ctypes.data, w.ctypes.data, src.ctypes.data, mode, C.byref(o))
            tot[mode] += np.array([getattr(o, f) for f in FIELDS], dtype=float)
            print(mode, {f: getattr(o, f) for f in FIELDS}, flush=True)
    for mode in (0, 1, 2):
        t = dict(zip(FIELDS, tot[mode] / ng))
        relax = t["rd_lines"] + 0.5 * t["wr_lines"]
        extra = t["par_rd"] + 0.5 * t["par_wr"] + t["tree_rd"] + 0.5 * t["tree_wr"]
        print(f"mode {mode}: rounds {t['rounds']:.1f} visits/vertex {t['visits'] / n:.2f} "
              f"lane updates/(v,lane) {t['lane_updates'] / n / 128:.2f}  lines/vertex: relax rd {t['rd_lines'] / n:.1f} "
              f"wr {t['wr_lines'] / n:.1f} (nbr {t['nbr_lines'] / n:.1f} own {t['own_lines'] / n:.1f} "
              f"route {t['route_lines'] / n:.1f}); parent rd {t['par_rd'] / n:.1f}; tree visits/vertex "
              f"{t['tree_visits'] / n:.2f} rounds {t['tree_rounds']:.0f} rd {t['tree_rd'] / n:.1f} wr {t['tree_wr'] / n:.1f}; "
              f"weighted (wr = 0.5) total {(relax + extra) / n:.1f}")


if __name__ == "__main__":
    main()
