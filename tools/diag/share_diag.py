"""Diagnostic: where shared-anchor rows differ from the exact build (GPU)."""
import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle")); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
from shadow_amd import graphs, spe
from test_gpu_shared_trees import with_pendants

top = with_pendants(graphs.gen_ba(2000, 3, 19), 1500, 4)
A0 = np.arange(top.n, dtype=np.int32)
g = spe.Graph(top)
deg = np.bincount(np.concatenate([top.esrc[top.esrc != top.edst], top.edst[top.esrc != top.edst]]), minlength=top.n)
for label, order, kw in (("nat g4", False, dict(groups=4)), ("ord g4", True, dict(groups=4)),
                         ("ord g4 nc", True, dict(groups=4, no_contract=True)),
                         ("ord g4 L64", True, dict(groups=4, lanes=64)),
                         ("ord g1 L128", True, dict(groups=2, lanes=128)),
                         ("ord g40", True, dict(groups=40))):
    A = g.order_sources(A0) if order else A0
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, **kw)
    st = t.build()
    lay = t.layout()
    te = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, exact_sources=True, **kw)
    te.build()
    a, b = t.download(), te.download()
    bad = (a["next"] != b["next"]).any(axis=1)
    rows = np.flatnonzero(bad)
    print(label, "cx", lay["contracted_vertices"], "lanes", lay["lanes_per_group"], "stats", {k: st[k] for k in ("relaxed_lanes", "fallback_blocks", "iterations")},
          "bad rows", rows.size, "of", len(A), "core among bad", int((deg[A[rows]] > 1).sum()),
          "first", rows[:10].tolist(), "blocks", np.unique(rows // 64)[:20].tolist(), flush=True)
