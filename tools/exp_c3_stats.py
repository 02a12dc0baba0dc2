"""One C3 whole-table build (the bench's workload and slot order) with a
SPE_RELAX_STATS library (SPE_LIB=build_ab/stats*/libspe.so): the library prints
`spe-relax-stats ... round r items .. entries .. lines .. kept .. lanes_changed ..
items_changed ..` per relaxation round on stderr (VERDICT r05 Next #2's
histogram: rows visited, changed lanes per visited row, lines read)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shadow_amd import graphs, spe

top = graphs.gen_ba(50000, 3, 3)
g = spe.Graph(top)
A = g.order_sources(np.arange(top.n, dtype=np.int32))
t = spe.PathTable(g, A)
t.build()
st = t.stats()
print(f"c3 build: {st['seconds']:.3f} s, {st['iterations']} rounds, {st['relaxed_lanes']} lanes", file=sys.stderr)
