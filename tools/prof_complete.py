"""Where the completion tool's wall time goes (diagnostic)."""
import sys, os, time, cProfile, pstats
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shadow_amd import complete, graphs
top = graphs.gen_tiered()
jit = np.random.default_rng(7).uniform(0, 5, top.m)
pois = np.arange(20000, 30000, dtype=np.int32)
complete.complete_paths(top, pois[:256], jit)
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
complete.complete_paths(top, pois, jit)
pr.disable()
print("total", time.perf_counter() - t0)
pstats.Stats(pr).sort_stats("cumulative").print_stats(12)
