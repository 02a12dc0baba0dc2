"""CPU model for DESIGN §6: what a source-block share of C3
costs in relaxation lanes when derived rows must stay inside the share.

Approximates the library's derivation rule (spe_graph_prep.cpp contract_degree3:
an independent set of degree-3 vertices removed; derived = every removed vertex
plus an independent set, in the contracted graph, of kept vertices with <= 5
contracted entries and <= 1 removed neighbour (then <= 3 plain ones); legs end
at root lanes) and the slot order (Voronoi cells of ceil(A/64) seeded centres,
then distance to the centre).  For N shares of contiguous slot blocks it counts,
per share:
  own      roots whose slots are in the share
  current  own + the share's derived sources missing some leg root (what the
           library builds today: such sources take a lane)
  closed   own + every foreign root a derived source of the share needs
           (neighbourhood-closed shares: the roots are replicated)
  ideal    all roots / N
Prints the max over shares (the step waits for the slowest rank).

    python tools/model_share_closure.py [--n 50000]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import dijkstra

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shadow_amd import graphs  # noqa: E402


def model(n: int, seed: int = 3):
    top = graphs.gen_ba(n=n, m=3, seed=seed)
    keep = top.esrc != top.edst
    a, b, w = top.esrc[keep], top.edst[keep], top.elat[keep]
    g = sp.coo_matrix((np.concatenate([w, w]), (np.concatenate([a, b]), np.concatenate([b, a]))), shape=(n, n)).tocsr()
    g.sum_duplicates()
    nb = [g.indices[g.indptr[v]:g.indptr[v + 1]] for v in range(n)]
    deg = np.diff(g.indptr)
    removed = np.zeros(n, bool)
    for v in range(n):   # independent set of degree-3 vertices
        if deg[v] == 3 and not removed[nb[v]].any():
            removed[v] = True
    nrem = np.array([int(removed[nb[v]].sum()) for v in range(n)])
    cdeg = np.array([int((~removed[nb[v]]).sum()) + 2 * nrem[v] for v in range(n)])
    derived = removed.copy()
    cand = [v for v in range(n) if not removed[v] and cdeg[v] <= 5 and nrem[v] <= 1 and
            (nrem[v] == 0 or deg[v] - nrem[v] <= 3)]
    cand.sort(key=lambda v: (nrem[v], cdeg[v]))
    near = np.zeros(n, bool)
    for x in cand:
        if near[x]:
            continue
        derived[x] = True
        near[x] = True
        for u in nb[x]:
            if removed[u]:
                near[[c for c in nb[u] if c != x]] = True
            else:
                near[u] = True
    xnb = np.full(n, -1)
    for x in np.flatnonzero(derived & ~removed):
        for u in nb[x]:
            if removed[u]:
                xnb[u] = x
    legs = {}
    for v in np.flatnonzero(derived):
        r = set()
        if removed[v]:
            for u in nb[v]:
                if u != xnb[v]:
                    r.add(int(u))
                else:
                    r.update(int(k) for k in nb[u] if not removed[k])
        else:
            for u in nb[v]:
                if removed[u]:
                    r.update(int(c) for c in nb[u] if c != v)
                else:
                    r.add(int(u))
        legs[int(v)] = r
    assert all(not derived[u] for r in legs.values() for u in r), "a leg ends at a derived source"
    # slot order: Voronoi cells of ceil(n/64) seeded centres, then distance
    rng = np.random.default_rng(1)
    centres = rng.choice(n, size=(n + 63) // 64, replace=False)
    dist, _, src = dijkstra(g, indices=centres, min_only=True, return_predecessors=True)
    order = np.lexsort((dist, src))
    return order, derived, legs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50000)
    args = ap.parse_args()
    order, derived, legs = model(args.n)
    n = args.n
    roots_total = int((~derived).sum())
    print(f"n={n}: derived {int(derived.sum())} (removed + kept), roots {roots_total}")
    nblk = (n + 63) // 64
    for N in (1, 2, 4, 8):
        worst = {"own": 0, "current": 0, "closed": 0}
        for r in range(N):
            b0, b1 = r * nblk // N, (r + 1) * nblk // N
            share = order[b0 * 64:min(n, b1 * 64)]
            mine = set(int(v) for v in share)
            own = {v for v in mine if not derived[v]}
            der = [v for v in mine if derived[v]]
            missing = sum(1 for v in der if not legs[v] <= own)
            need = set(own)
            for v in der:
                need |= legs[v]
            worst["own"] = max(worst["own"], len(own))
            worst["current"] = max(worst["current"], len(own) + missing)
            worst["closed"] = max(worst["closed"], len(need))
        print(f"N={N}: lanes per share (max over shares) own {worst['own']}, current {worst['current']}, "
              f"closed {worst['closed']}, ideal {roots_total / N:.0f}, no derivation {n // N}")


if __name__ == "__main__":
    main()
