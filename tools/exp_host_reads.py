"""Round-6 diagnostic: does a C3 / C4-size table take host loads for single
entries (spe_table_layout.host_reads), how fast are get_latrel calls from
Python, and where does the table sit in /proc/self/maps."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shadow_amd import graphs, spe  # noqa: E402

for name in ("c3", "c4"):
    if name == "c3":
        top = graphs.gen_ba(50000, 3, 3)
        att = np.arange(top.n, dtype=np.int32)
    else:
        top = graphs.gen_tiered()
        att = graphs.tiered_attached(top)
    g = spe.Graph(top)
    att = g.order_sources(att)
    t = spe.PathTable(g, att)
    t.build()
    lay = t.layout()
    t.get_latrel(0, 1)
    lay = t.layout()
    p = lay["latrel"]
    span = lay["elems"] * 16
    maps = [l for l in open("/proc/self/maps") if True]
    hit = []
    for l in maps:
        a, b = (int(x, 16) for x in l.split()[0].split("-"))
        if b > p and a < p + span:
            hit.append(l.strip())
    print(f"{name}: host_reads {lay['host_reads']}, latrel {p:#x} span {span / 1e9:.1f} GB, "
          f"{len(hit)} mappings over it: {hit[:4]}{' ...' if len(hit) > 4 else ''}", flush=True)
    rng = np.random.default_rng(1)
    pr = rng.integers(0, t.A, (100000, 2))
    t0 = time.perf_counter()
    for s, u in pr:
        t.get_latrel(int(s), int(u))
    el = time.perf_counter() - t0
    print(f"{name}: {len(pr)} get_latrel calls from Python: {1e6 * el / len(pr):.2f} us/call", flush=True)
    t.close()
    del g
