import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np
from shadow_amd import graphs, spe
from oracle import Oracle
top = graphs.gen_ba(3000, 3, 25)
rng = np.random.default_rng(225)
top.elat = rng.integers(1, 60, top.elat.shape[0]) * 0.1
A = np.arange(top.n, dtype=np.int32)
g = spe.Graph(top)
A = g.order_sources(A)
ref = Oracle(top).rows(A, A, tie_mode=1)
ok = ref["kind"] != 0
print("double ties (oracle)", ref.get("double_ties"))
for name, kw in (("exact_cx", dict(exact_sources=True)), ("exact_nocx", dict(exact_sources=True, no_contract=True)),
                 ("default", {}), ("default_nocx", dict(no_contract=True))):
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, **kw)
    st = t.build()
    d = t.download()
    mis = (d["next"] != ref["next"]) & ok
    rows = np.flatnonzero(mis.any(axis=1))
    print(name, "next mismatches", int(mis.sum()), "rows", rows.size, "hops mism", int(((d["hops"] != ref["hops"]) & ok).sum()),
          "derived", st["derived_sources"], "fallback", st["fallback_blocks"], "lanes", st["relaxed_lanes"],
          "lay", t.layout()["contracted_vertices"], t.layout()["shared_sources"])
    if rows.size:
        r = rows[0]; c = np.flatnonzero(mis[r])[:5]
        print("  e.g. src", A[r], "targets", A[c], "got", d["next"][r, c], "ref", ref["next"][r, c], "lat", d["lat"][r,c], ref["lat"][r,c])
    t.close()
