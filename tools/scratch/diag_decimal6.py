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
ref = Oracle(top).rows(A, A, tie_mode=1)
ok = ref["kind"] != 0
for kw in (dict(no_contract=True), dict()):
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, exact_sources=True, **kw)
    t.build()
    dl = t.download()
    mis = (dl["next"] != ref["next"]) & ok
    print(os.environ.get("SPE_LIB"), kw, "rows", int(mis.any(axis=1).sum()), "pairs", int(mis.sum()), flush=True)
