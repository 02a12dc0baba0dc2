"""Round-6 diagnostic: single-entry host reads (spe_table_get_latrel) from several
threads at once, straight on the library through a small C harness
(tools/mt_reads.c, built into build_ab/libmtreads.so), on the C3 and C4 tables.

Finding (profiles/r06_prefault.log): the first host load of each 64-KB window of the
large-BAR mapping takes a driver page fault, and the faults serialise; the library's
background pre-fault (spe_table_layout.host_prefault) fills the mapping from the first
host read on.  This prints the rates while it runs and after it is done, and its time
for 1 and 2 threads (SPE_HOST_PREFAULT)."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from shadow_amd import graphs, spe  # noqa: E402

mt = C.CDLL(os.path.join(ROOT, "build_ab", "libmtreads.so"))
mt.mt_reads.restype = C.c_double
mt.mt_reads.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int64]

for name in ("c3", "c4"):
    top = graphs.gen_ba(50000, 3, 3) if name == "c3" else graphs.gen_tiered()
    att = np.arange(top.n, dtype=np.int32) if name == "c3" else graphs.tiered_attached(top)
    g = spe.Graph(top)
    att = g.order_sources(att)
    for pf in (("1", "2") if name == "c4" else ("1", "0")):
        os.environ["SPE_HOST_PREFAULT"] = pf
        t = spe.PathTable(g, att)
        t.build()
        t.get_latrel(0, 1)   # decides host reads, starts the pre-fault
        t0 = time.perf_counter()
        r = mt.mt_reads(t.h, t.A, 1, 50000)
        lay = t.layout()
        print(f"{name} SPE_HOST_PREFAULT={pf}: while it runs ({time.perf_counter() - t0:.2f} s in): "
              f"1 thread {r:.0f} get_latrel/s; state {lay['host_prefault']} after {lay['host_prefault_s']:.2f} s",
              flush=True)
        while t.layout()["host_prefault"] == 1:
            time.sleep(0.05)
        lay = t.layout()
        print(f"{name} SPE_HOST_PREFAULT={pf}: state {lay['host_prefault']}, {lay['host_prefault_s']:.3f} s "
              f"over {lay['elems'] * 16 / 1e9:.1f} GB of records", flush=True)
        for nt in (1, 4, 16):
            r = mt.mt_reads(t.h, t.A, nt, 100000)
            print(f"{name} SPE_HOST_PREFAULT={pf} after: {nt:2d} threads (C): {r:.0f} get_latrel/s in all", flush=True)
        t.close()
    del g
