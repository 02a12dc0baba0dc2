"""Round-6 debug aid for the route pass (SPE_ROUTE_PASS=1 builds, run with SPE_LIB):
builds the directed tie-free parity graph REPS times with SPE_ROUTE_DEBUG=1, which
makes a pass that does not complete print its first stuck lanes and one parent chain."""
import os, sys
sys.path.insert(0, os.getcwd())
os.environ["SPE_ROUTE_DEBUG"] = "1"
import numpy as np
from shadow_amd import graphs, spe
top = graphs.gen_random_small(n=500, extra_edges=1500, seed=32, directed=True)
A = np.arange(top.n, dtype=np.int32)
g = spe.Graph(top)
t = spe.PathTable(g, A)
print("layout", t.layout(), flush=True)
for rep in range(int(os.environ.get("REPS", "20"))):
    try:
        t.build()
        print("built ok", rep, flush=True)
    except Exception as e:
        print("ERR", rep, e, flush=True)
        break
