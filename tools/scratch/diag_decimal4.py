import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np
from shadow_amd import graphs, spe
from oracle import Oracle
for gname, mk in (("ba_decimal", lambda: graphs.gen_ba(3000, 3, 25)), ("rand_decimal", lambda: graphs.gen_random_small(3000, 6000, 77))):
    top = mk()
    rng = np.random.default_rng(225)
    top.elat = rng.integers(1, 60, top.elat.shape[0]) * 0.1
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    ref = Oracle(top).rows(A, A, tie_mode=1)
    ok = ref["kind"] != 0
    for name, kw in (("ring128", dict(relax_kernel=2)), ("reg128", dict(relax_kernel=1)), ("k_relax64", dict(lanes=64)),
                     ("ring128_groups2", dict(relax_kernel=2, groups=2)), ("lds", dict(engine=spe.SPE_ENGINE_LDS))):
        kw2 = dict(engine=spe.SPE_ENGINE_BATCH, exact_sources=True, no_contract=True)
        kw2.update(kw)
        t = spe.PathTable(g, A, **kw2)
        st = t.build()
        dl = t.download()
        mis = ((dl["next"] != ref["next"]) & ok)
        print(gname, name, "rows", int(mis.any(axis=1).sum()), "pairs", int(mis.sum()), "layout", t.layout()["lanes_per_group"], t.layout()["relax_kernel"], "heavy_info", flush=True)
        t.close()
