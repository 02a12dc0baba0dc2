"""Design experiment (not product code): time the C3 batch build of `nb` blocks
under the current SPE_* environment knobs (one line per run)."""
import sys, time, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shadow_amd import graphs, spe

cfg = sys.argv[2] if len(sys.argv) > 2 else "c3"
top = graphs.gen_ba(50000, 3, 3) if cfg == "c3" else graphs.gen_tiered()
att = np.arange(top.n, dtype=np.int32) if cfg == "c3" else graphs.tiered_attached(top)
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 64
g = spe.Graph(top, device=0)
t = spe.PathTable(g, att, blocks=(0, nb), groups=int(os.environ.get("X_GROUPS", "0")))
t.build_blocks(0, 16)
t.profile(True)
t0 = time.perf_counter()
t.build_blocks(0, nb)
el = time.perf_counter() - t0
kp = t.kernel_profile()
st = t.stats()
knobs = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("SPE_"))
print(f"[{knobs}] {nb*64/el:9.0f} sources/s  relax {kp['relax']['ms']:8.1f} ms / {kp['relax']['launches']} "
      f"heavy {kp['heavy']['ms']:6.1f} rows {kp['rows']['ms']:6.1f} init {kp['init']['ms']:5.1f} iters {st['iterations']}",
      flush=True)
