"""On-disk path-table cache (spe_table_save / spe_table_load):
a saved table reloads bit-identically into a fresh table with the same key, and
a file for another graph, attached set or option set is refused."""
import numpy as np
import pytest

from shadow_amd import graphs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spe():
    from shadow_amd import spe as m
    assert m.device_count() > 0, "no GPU visible"
    return m


def test_save_load_roundtrip(spe, tmp_path):
    top = graphs.gen_random_small(400, 1200, 61)
    A = np.arange(0, top.n, 3, dtype=np.int32)   # 134 attached: a ragged last block
    g = spe.Graph(top)
    t = spe.PathTable(g, A)
    t.build()
    ref = t.download()
    path = str(tmp_path / "t.bin")
    t.save(path)
    t2 = spe.PathTable(g, A)
    assert t2.key() == t.key()
    t2.load(path)
    got = t2.download()
    for k in ("lat", "rel", "next", "hops"):
        np.testing.assert_array_equal(got[k], ref[k])
    assert t2.min_latency() == t.min_latency()


def test_key_covers_graph_attached_and_options(spe, tmp_path):
    top = graphs.gen_random_small(300, 900, 62)
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    t = spe.PathTable(g, A)
    t.build()
    path = str(tmp_path / "t.bin")
    t.save(path)
    other_top = graphs.gen_random_small(300, 900, 63)
    variants = [spe.PathTable(g, A[::-1].copy()),                 # attached order
                spe.PathTable(g, A, self_mode=spe.SPE_SELF_RULE),  # self mode
                spe.PathTable(g, A, force_sssp=True),              # forced regime
                spe.PathTable(g, A, blocks=(1, 3)),                # block range
                spe.PathTable(spe.Graph(other_top), A)]            # other graph
    keys = {t.key()} | {v.key() for v in variants}
    assert len(keys) == 1 + len(variants)
    for v in variants:
        with pytest.raises(spe.SpeError):
            v.load(path)


def test_truncated_file_is_refused(spe, tmp_path):
    top = graphs.gen_random_small(200, 600, 64)
    A = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    t = spe.PathTable(g, A)
    t.build()
    path = tmp_path / "t.bin"
    t.save(str(path))
    data = path.read_bytes()
    path.write_bytes(data[: len(data) // 2])
    t2 = spe.PathTable(g, A)
    with pytest.raises(spe.SpeError):
        t2.load(str(path))
    with pytest.raises(spe.SpeError):   # still unbuilt
        t2.download()
