import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np
from shadow_amd import graphs, spe
from oracle import Oracle
top = graphs.gen_ba(3000, 3, 25)
rng = np.random.default_rng(225)
top.elat = rng.integers(1, 60, top.elat.shape[0]) * 0.1
g = spe.Graph(top)
allA = np.arange(top.n, dtype=np.int32)
ref_all = Oracle(top).rows(allA, allA, tie_mode=1)
bad_rows = [1, 39, 58, 184, 300, 436, 448, 552, 585, 593]
for name, A in (("single", None), ("pairs10", np.array(bad_rows, np.int32)), ("first128", np.arange(128, dtype=np.int32)),
                ("bad+rest", np.r_[np.array(bad_rows, np.int32), np.setdiff1d(allA, bad_rows)].astype(np.int32))):
    tot = 0
    sets = [np.array([s] + [v for v in range(top.n) if v != s], np.int32) for s in bad_rows[:4]] if A is None else [A]
    for AA in sets:
        for lanes in (64, 128):
            t = spe.PathTable(g, AA, engine=spe.SPE_ENGINE_BATCH, exact_sources=True, no_contract=True, lanes=lanes)
            t.build()
            dl = t.download(0, min(len(AA), 64))
            ref = Oracle(top).rows(AA[:min(len(AA), 64)], AA, tie_mode=1)
            ok = ref["kind"] != 0
            mis = (dl["next"] != ref["next"]) & ok
            tot += int(mis.sum())
            print(name, "lanes", lanes, "A", len(AA), "rows with mismatch", int(mis.any(axis=1).sum()), "pairs", int(mis.sum()), flush=True)
            t.close()
