import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np
from shadow_amd import graphs, spe
top = graphs.gen_ba(3000, 3, 25)
rng = np.random.default_rng(225)
top.elat = rng.integers(1, 60, top.elat.shape[0]) * 0.1
g = spe.Graph(top)
A = np.array([1, 39, 58, 184, 300, 436, 448, 552, 585, 593], np.int32)
t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, exact_sources=True, no_contract=True, lanes=64)
t.build()
slot = int(sys.argv[1])
pt = t.source_tree(slot)
v = int(os.environ["SPE_DBG_V"])
print("tree parent of", v, "=", pt[v], flush=True)
