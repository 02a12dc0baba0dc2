"""Single-entry reads by host loads (spe_table_get / spe_table_get_latrel on a
large-BAR host): the per-packet read of the drop-in
(shd-worker.c:235-247 -> topology_getPathInfo -> spe_table_get_latrel) must
return exactly the table the device holds -- every field bit for bit against
spe_table_download -- whether the library reads the mapped device memory with a
host load (spe_table_layout.host_reads = 1) or copies each entry
(SPE_HOST_READS=0)."""
import time

import numpy as np
import pytest

from shadow_amd import graphs

pytestmark = [pytest.mark.gpu]


@pytest.fixture(scope="module")
def spe():
    from shadow_amd import spe as m
    assert m.device_count() > 0, "no GPU visible"
    return m


def _check_entries(t, ref, pairs):
    for s, u in pairs:
        e = t.get(int(s), int(u))
        for k, f in (("lat", "latency"), ("rel", "reliability"), ("next", "next_hop"), ("hops", "hops")):
            assert e[f] == ref[k][s, u] or (np.isnan(e[f]) and np.isnan(ref[k][s, u])), (s, u, k, e[f], ref[k][s, u])
        lat, rel = t.get_latrel(int(s), int(u))
        assert np.float64(lat).tobytes() == np.float64(ref["lat"][s, u]).tobytes(), (s, u)
        assert np.float64(rel).tobytes() == np.float64(ref["rel"][s, u]).tobytes(), (s, u)


@pytest.mark.parametrize("mode", ["auto", "copies"])
def test_single_entries_equal_the_download(spe, mode, monkeypatch):
    if mode == "copies":
        monkeypatch.setenv("SPE_HOST_READS", "0")
    top = graphs.gen_random_small(1500, 4500, 11)
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    t = spe.PathTable(g, A)
    t.build()
    assert t.layout()["host_reads"] == -1   # decided at the first read
    ref = t.download()
    rng = np.random.default_rng(3)
    pairs = np.concatenate([rng.integers(0, t.A, (3000, 2)), np.stack([np.arange(50)] * 2, 1)])   # + self entries
    t0 = time.perf_counter()
    _check_entries(t, ref, pairs)
    el = time.perf_counter() - t0
    hr = t.layout()["host_reads"]
    print(f"host_reads={hr}: {len(pairs)} get + get_latrel pairs in {el:.3f} s")
    assert hr == (0 if mode == "copies" else hr) and hr in (0, 1)
    # a second build of the same table (every block rewritten): reads see the new records
    t.build()
    _check_entries(t, ref, pairs[:500])
    t.close()


def test_host_reads_on_a_block_range_table(spe):
    """A table owning blocks [2, 5) of the sources: offsets are block-relative."""
    top = graphs.gen_random_small(800, 2400, 12)
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    full = spe.PathTable(g, A)
    full.build()
    ref = full.download()
    t = spe.PathTable(g, A, blocks=(2, 5))
    t.build()
    rng = np.random.default_rng(4)
    for s, u in zip(rng.integers(2 * 64, 5 * 64, 400), rng.integers(0, t.A, 400)):
        assert t.get_latrel(int(s), int(u)) == (ref["lat"][s, u], ref["rel"][s, u])
        assert t.get(int(s), int(u))["next_hop"] == ref["next"][s, u]


def test_download_by_dma_equals_staged(spe, monkeypatch):
    """spe_table_download of many blocks DMAs straight into the caller's arrays
    (hipHostRegister); SPE_DOWNLOAD_STAGED=1 forces the pinned staging path.  Both
    give the same table, every field."""
    top = graphs.gen_random_small(1200, 3600, 13)
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    t = spe.PathTable(g, A)
    t.build()
    direct = t.download()
    monkeypatch.setenv("SPE_DOWNLOAD_STAGED", "1")
    staged = t.download()
    for k in ("lat", "rel", "next", "hops"):
        assert direct[k].tobytes() == staged[k].tobytes(), k


@pytest.mark.parametrize("threads", ["0", "3"])
def test_host_prefault(spe, threads, monkeypatch):
    """The first host read starts the background pre-fault of the mapping
    (spe_table_layout.host_prefault: 1 running, 2 done; SPE_HOST_PREFAULT=0: -1 off);
    entries read while it runs and after it ends equal the download, and closing the
    table while it runs stops it."""
    monkeypatch.setenv("SPE_HOST_PREFAULT", threads)
    top = graphs.gen_random_small(1400, 4200, 14)
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    t = spe.PathTable(g, A)
    t.build()
    ref = t.download()
    assert t.layout()["host_prefault"] == 0
    rng = np.random.default_rng(5)
    pairs = rng.integers(0, t.A, (600, 2))
    _check_entries(t, ref, pairs[:300])
    lay = t.layout()
    if lay["host_reads"] != 1:
        assert lay["host_prefault"] == 0
        pytest.skip("no large-BAR host mapping: copies, nothing to pre-fault")
    if threads == "0":
        assert lay["host_prefault"] == -1
    else:
        assert lay["host_prefault"] in (1, 2)
        t0 = time.perf_counter()
        while t.layout()["host_prefault"] == 1 and time.perf_counter() - t0 < 30:
            time.sleep(0.01)
        lay = t.layout()
        assert lay["host_prefault"] == 2 and lay["host_prefault_s"] > 0
        print(f"pre-fault of {lay['elems'] * 16 / 1e6:.0f} MB on {threads} threads: {lay['host_prefault_s']:.4f} s")
    _check_entries(t, ref, pairs[300:])
    t2 = spe.PathTable(g, A)   # closed while (probably) still running
    t2.build()
    t2.get_latrel(0, 1)
    t2.close()
    t.close()
