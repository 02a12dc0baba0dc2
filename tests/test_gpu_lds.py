"""LDS-resident engine (one workgroup per source row, SPE_ENGINE_LDS) at config C2
size: the 10k-vertex random geometric graph of BASELINE.json configs[1].

* a sample of full rows bit-exact against the oracle (igraph Dijkstra restatement
  + shd-topology.c row rules, `oracle/oracle.c`);
* the whole 10k x 10k table identical, field by field, to the 64-lane batch
  engine (two independent relaxation schemes converging to the same least
  fixpoint);
* the explicit LDS request on a graph that does not fit fails loudly.
"""
import numpy as np
import pytest

from shadow_amd import graphs
from oracle import Oracle

pytestmark = [pytest.mark.gpu, pytest.mark.engine_fixed]


@pytest.fixture(scope="module")
def spe():
    from shadow_amd import spe as m
    assert m.device_count() > 0, "no GPU visible"
    return m


@pytest.fixture(scope="module")
def c2():
    top = graphs.gen_rgg(10000, 2)
    return top, np.arange(top.n, dtype=np.int32)


def _build(spe, top, att, engine, **kw):
    g = spe.Graph(top)
    t = spe.PathTable(g, att, engine=engine, **kw)
    t.profile(True)
    t.build()
    kp = t.kernel_profile()
    used = "lds" if kp["lds"]["launches"] > 0 else "relax"
    assert kp[used]["launches"] > 0
    assert used == ("lds" if engine == spe.SPE_ENGINE_LDS else "relax"), f"engine {engine} ran {used}"
    return t, g


def test_c2_lds_rows_vs_oracle(spe, c2, monkeypatch):
    monkeypatch.delenv("SPE_ENGINE", raising=False)
    top, att = c2
    t, g = _build(spe, top, att, spe.SPE_ENGINE_LDS)
    rng = np.random.default_rng(11)
    rows = np.sort(rng.choice(top.n, size=96, replace=False))
    ref = Oracle(top).rows(att[rows], att)
    ok = ref["kind"] != 0
    for r_i, r in enumerate(rows):
        got = t.download(int(r), int(r) + 1)
        o = ok[r_i]
        assert (got["ok"][0] == o).all()
        for k in ("lat", "rel", "next", "hops"):
            a, b = got[k][0][o], ref[k][r_i][o]
            bad = np.flatnonzero(a != b)
            assert bad.size == 0, f"row {r}: {k} differs at {bad.size} targets"


def test_c2_lds_equals_batch_engine(spe, c2, monkeypatch):
    monkeypatch.delenv("SPE_ENGINE", raising=False)
    top, att = c2
    t1, _ = _build(spe, top, att, spe.SPE_ENGINE_LDS)
    a = t1.download()
    t1.close()
    t2, _ = _build(spe, top, att, spe.SPE_ENGINE_BATCH)
    b = t2.download()
    for k in ("lat", "rel", "next", "hops", "ok"):
        bad = np.count_nonzero(a[k] != b[k])
        assert bad == 0, f"{k}: {bad} entries differ between engines"
    assert a["ok"].all()   # one component


def test_lds_engine_refuses_large_graph(spe, monkeypatch):
    monkeypatch.delenv("SPE_ENGINE", raising=False)
    top = graphs.gen_ba(20000, 3, 9)
    g = spe.Graph(top)
    with pytest.raises(spe.SpeError):
        spe.PathTable(g, np.arange(64, dtype=np.int32), engine=spe.SPE_ENGINE_LDS)
