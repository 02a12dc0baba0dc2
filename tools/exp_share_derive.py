"""Derived rows under block-range shares (the multi-GPU split): how many sources
of a 1/N share of the C3 table are derived, and how many relaxation lanes the
share needs, against the whole table on one GPU."""
import sys
import time

import numpy as np

from shadow_amd import graphs, spe

top = graphs.gen_ba(50000, 3, 3)
g = spe.Graph(top)
A = g.order_sources(np.arange(top.n, dtype=np.int32))
nblk = (len(A) + 63) // 64
for N in (1, 2, 4, 8):
    b1 = (nblk + N - 1) // N
    t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, blocks=(0, b1))
    t0 = time.perf_counter()
    st = t.build()
    el = time.perf_counter() - t0
    print(f"N={N}: share blocks 0..{b1} ({b1 * 64} sources): derived {st['derived_sources']}, "
          f"relaxed lanes {st['relaxed_lanes']}, fallback blocks {st['fallback_blocks']}, build {el:.3f} s", flush=True)
    del t
