"""Cost of building C3 block ranges of several sizes (the chunks of the multi-GPU
schedules): seconds per block against the whole table."""
import time

import numpy as np

from shadow_amd import graphs, spe

top = graphs.gen_ba(50000, 3, 3)
g = spe.Graph(top)
A = g.order_sources(np.arange(top.n, dtype=np.int32))
nblk = (len(A) + 63) // 64
for nb in (7, 26, 98, 196, 391, 782):
    b0 = (nblk - nb) // 2
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, blocks=(b0, b0 + nb))
    t.build()   # warm (code objects, allocations)
    t0 = time.perf_counter()
    st = t.build()
    el = time.perf_counter() - t0
    print(f"blocks {nb:4d}: {el * 1e3:8.1f} ms = {el * 1e3 / nb:.3f} ms/block; lanes {st['relaxed_lanes']}, "
          f"derived {st['derived_sources']}, rounds {st['active_rounds']}", flush=True)
    del t
