import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
from shadow_amd import graphs, spe
top = graphs.gen_ba(3000, 3, 25)
rng = np.random.default_rng(225)
top.elat = rng.integers(1, 60, top.elat.shape[0]) * 0.1
n = top.n
adj = [dict() for _ in range(n)]
for a, b, w in zip(top.esrc, top.edst, top.elat):
    a, b = int(a), int(b)
    if a == b: continue
    if b not in adj[a] or w < adj[a][b]: adj[a][b] = w; adj[b][a] = w
iptr = [0]; icol = []
for v in range(n):
    for u in sorted(adj[v]): icol.append(u)
    iptr.append(len(icol))
g = spe.Graph(top)
A = np.array([1, 39, 58, 184, 300, 436, 448, 552, 585, 593], np.int32)
path = "/tmp/rounds.bin"
if os.path.exists(path): os.remove(path)
os.environ["SPE_DUMP_ROUNDS"] = path
t = spe.PathTable(g, A, engine=spe.SPE_ENGINE_BATCH, exact_sources=True, no_contract=True, lanes=64)
t.build()
raw = open(path, "rb").read()
L = 64; ne = n * L
# heavy plan: segments of 64 entries of vertices with in-degree > 64, in vertex order
segs = []
for x in range(n):
    if iptr[x+1] - iptr[x] > 64:
        for kb in range(iptr[x], iptr[x+1], 64): segs.append((x, kb))
nseg = len(segs)
np_ = L * nseg
per = ne * 12 + np_ * 24
R = len(raw) // per
print("rounds", R, "nseg", nseg, "bytes", len(raw), per)
j, v = 1, 20
s20 = [i for i, (x, kb) in enumerate(segs) if x == v]
for r in range(R):
    base = r * per
    D = np.frombuffer(raw[base:base + ne * 8], np.float64).reshape(n, L)
    P = np.frombuffer(raw[base + ne * 8:base + ne * 12], np.int32).reshape(n, L)
    o = base + ne * 12
    pa = np.frombuffer(raw[o:o + np_ * 8], np.float64).reshape(nseg, L)
    pd = np.frombuffer(raw[o + np_ * 8:o + np_ * 16], np.float64).reshape(nseg, L)
    pu = np.frombuffer(raw[o + np_ * 16:o + np_ * 24], np.int32).reshape(nseg, L, 2)
    pk = P[v, j]
    print("round", r + 1, "D20", repr(D[v, j]), "P20->", icol[pk] if pk >= 0 else pk, "D109", repr(D[109, j]),
          "| segs", [(int(pu[q, j, 0]), repr(pd[q, j]), repr(pa[q, j])) for q in s20])
