"""Per-launch times of one C3 whole-table build (SPE_TRACE=1: the library prints
`spe-trace <kind> <ms>` per timed launch; kinds as spe.h SPE_K_*)."""
import os
import sys

import numpy as np

os.environ["SPE_TRACE"] = "1"
from shadow_amd import graphs, spe

top = graphs.gen_ba(50000, 3, 3)
g = spe.Graph(top)
A = g.order_sources(np.arange(top.n, dtype=np.int32))
for rep in range(2):
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH)
    t.profile(True)
    print(f"--- build {rep}", file=sys.stderr, flush=True)
    t.build()
    del t
