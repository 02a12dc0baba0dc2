"""Multi-device tables in one process (spe_table_opts.devices, spe_multi.cpp):
Shadow is single-process (shd-master.c:390-394), so the library drives every
GPU itself -- contiguous source-block shares, one host thread and stream per
device, chunk-wise broadcasts of the {latency, reliability} records while the
next chunk builds (RCCL ncclBroadcast groups, or peer copies), and optionally a
local remainder every device builds itself (the compute-versus-gather split,
DESIGN §6).  CPU: the share / split / gather-offset arithmetic.
GPU: the single-device path through the API with RCCL, and a 3-way split on one
GPU (peer gather: RCCL refuses a repeated device) against the oracle."""
import numpy as np
import pytest

from shadow_amd import graphs
from oracle import Oracle


@pytest.mark.parametrize("A,N", [(1, 1), (64, 8), (100, 8), (50000, 8), (50000, 3), (100000, 8), (6400, 7)])
def test_device_shares_contiguous_and_padded(A, N):
    from shadow_amd import spe
    sh = spe.device_shares(A, N)
    nblk = -(-A // 64)
    cb = -(-nblk // N)
    assert sh[0][0] == 0 and sh[-1][1] == nblk
    for d, (b0, b1) in enumerate(sh):
        # share d starts at d * cb: its records sit at byte offset d * cb * A * 64 * 16 of
        # every replica, which is where an in-place all-gather puts rank d's send buffer
        assert b0 == min(nblk, d * cb) and b1 == min(nblk, (d + 1) * cb) and b1 - b0 <= cb
        if d:
            assert b0 == sh[d - 1][1]


@pytest.mark.parametrize("A,N,x", [(100000, 8, 0.39), (50000, 8, 0.88), (700, 3, 0.5), (64, 2, 0.3), (50000, 8, 0.0),
                                   (6400, 7, 1.0)])
def test_device_split_arithmetic(A, N, x):
    """spe_device_split: equal contiguous shares of [0, S), S = N floor(x nblk / N),
    the local remainder [S, nblk); x = 1 is spe_device_shares."""
    from shadow_amd import spe
    sh, S = spe.device_split(A, N, x)
    nblk = -(-A // 64)
    if x >= 1.0:
        assert sh == spe.device_shares(A, N) and S == nblk
        return
    cb = int(np.floor(x * nblk / N))
    assert S == N * cb <= nblk
    assert sh == [(d * cb, (d + 1) * cb) for d in range(N)]
    # the model's x* lands C4 at N = 8 near 40 % shared
    from shadow_amd import dist as sd
    assert abs(sd.shared_fraction(8, 0.28, 160e9, 300e9) - 0.393) < 0.01


def test_device_shares_rejects_bad_arguments():
    from shadow_amd import spe
    with pytest.raises(spe.SpeError):
        spe.device_shares(10, 0)
    with pytest.raises(spe.SpeError):
        spe.device_split(10, 2, 1.5)


def _check_table(t, top, att, label):
    out = t.download()
    ref = Oracle(top).rows(att, att)
    ok = ref["kind"] != 0
    np.testing.assert_array_equal(out["ok"], ok, err_msg=label)
    for k in ("lat", "rel", "next", "hops"):
        np.testing.assert_array_equal(out[k][ok], ref[k][ok], err_msg=f"{label}: {k}")
    return ref


@pytest.mark.gpu
@pytest.mark.engine_fixed
def test_single_device_through_the_multi_device_api_rccl():
    from shadow_amd import spe
    top = graphs.gen_random_small(600, 1800, 61)
    att = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    t = spe.PathTable(g, att, devices=[0], gather=spe.SPE_GATHER_RCCL)
    st = t.build()
    assert st["n_devices"] == 1 and st["gather"] == spe.SPE_GATHER_RCCL
    _check_table(t, top, att, "devices=[0] rccl")
    lay = t.layout()
    assert lay["n_devices"] == 1 and lay["block_end"] == t.nblocks and lay["next_hop"] is None


@pytest.mark.gpu
@pytest.mark.engine_fixed
@pytest.mark.parametrize("engine", [1, 2, 3], ids=["batch", "lds", "fw"])
def test_three_shares_peer_gather_on_one_gpu(engine):
    """Devices [0, 0, 0]: three part tables on one GPU, each building its share
    into its own replica; the peer gather completes every replica.  download
    (routed to the owners), get and the batched lookup (the home replica, i.e.
    the gathered records of all shares) all match the oracle."""
    import torch
    from shadow_amd import spe
    top = graphs.gen_random_small(700, 2100, 62)
    att = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    t = spe.PathTable(g, att, devices=[0, 0, 0], engine=engine)
    # FW: the closure's 11 row blocks are split 4 / 4 / 3 over the shares, pivot
    # row panels broadcast by peer copies, every share's rows then walk it
    st = t.build()
    assert st["n_devices"] == 3 and st["gather"] == spe.SPE_GATHER_PEER and st["gather_seconds"] > 0
    ref = _check_table(t, top, att, "3 shares")
    e = t.get(650, 3)
    assert e["latency"] == ref["lat"][650, 3] and e["next_hop"] == ref["next"][650, 3]
    q = 200_000
    pairs = torch.randint(0, t.A, (q, 2), dtype=torch.int32, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    lat = torch.empty(q, dtype=torch.float64, device="cuda")
    rel = torch.empty(q, dtype=torch.float64, device="cuda")
    ok = torch.empty(q, dtype=torch.uint8, device="cuda")
    t.lookup_batch(pairs.data_ptr(), q, lat.data_ptr(), rel.data_ptr(), ok.data_ptr())
    p = pairs.cpu().numpy()
    np.testing.assert_array_equal(lat.cpu().numpy(), ref["lat"][p[:, 0], p[:, 1]])
    np.testing.assert_array_equal(rel.cpu().numpy(), ref["rel"][p[:, 0], p[:, 1]])
    assert t.min_latency() == ref["lat"][ref["kind"] != 0].min()
    lay = t.layout()
    assert lay["n_devices"] == 3 and lay["elems"] == 3 * (-(-t.nblocks // 3)) * t.A * 64


@pytest.mark.gpu
@pytest.mark.engine_fixed
def test_topology_shim_on_two_shares(tmp_path, monkeypatch):
    """topology_new's SHADOW_SPE_DEVICES device list (here the one GPU twice)."""
    from shadow_amd import topology as T
    monkeypatch.setenv("SHADOW_SPE_DEVICES", "0,0")
    t = graphs.gen_random_small(300, 900, 63)
    ips = [f"10.{v // 250}.{v % 250}.{1 + v % 7}" for v in range(t.n)]
    p = tmp_path / "g.graphml"
    graphs.write_graphml(t, str(p), ips=ips)
    top = T.Topology(str(p))
    verts = np.random.default_rng(63).choice(t.n, 150, replace=False).astype(np.int32)
    addrs = [T.ip(f"11.0.0.{i + 1}") for i in range(150)]
    for a, v in zip(addrs, verts):
        top.attach(a, ip_hint=ips[v])
    ref = Oracle(t).rows(verts, verts)
    for i in range(0, 150, 5):
        for j in range(0, 150, 3):
            assert top.path_info(addrs[i], addrs[j]) == (True, ref["lat"][i, j], ref["rel"][i, j])
    top.close()


@pytest.mark.gpu
@pytest.mark.engine_fixed
def test_fw_engine_single_device_rccl_broadcasts():
    """FW engine through the multi-device API with RCCL (one rank: every pivot
    panel and the final row exchange go through ncclBroadcast)."""
    from shadow_amd import spe
    top = graphs.gen_random_small(500, 1500, 64)
    att = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    t = spe.PathTable(g, att, devices=[0], gather=spe.SPE_GATHER_RCCL, engine=spe.SPE_ENGINE_FW)
    st = t.build()
    assert st["gather"] == spe.SPE_GATHER_RCCL and t.layout()["engine"] == spe.SPE_ENGINE_FW
    _check_table(t, top, att, "fw devices=[0] rccl")


@pytest.mark.gpu
@pytest.mark.engine_fixed
def test_fw_engine_c2_four_shares_equals_lds_engine():
    """C2 at full size on the multi-device FW path (four shares on one GPU: 157
    closure row blocks over 4 devices, 157 pivot-panel broadcasts): the table
    equals the LDS engine's entry for entry."""
    from shadow_amd import spe
    top = graphs.gen_rgg(10000, 2)
    att = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    tf = spe.PathTable(g, att, devices=[0, 0, 0, 0], engine=spe.SPE_ENGINE_FW)
    tf.build()
    tl = spe.PathTable(g, att, engine=spe.SPE_ENGINE_LDS)
    tl.build()
    for r0 in range(0, top.n, 2500):
        r1 = min(top.n, r0 + 2500)
        a, b = tf.download(r0, r1), tl.download(r0, r1)
        for k in ("ok", "lat", "rel", "next", "hops"):
            bad = np.count_nonzero(a[k] != b[k])
            assert bad == 0, f"rows {r0}:{r1} {k}: {bad} entries differ"


@pytest.mark.gpu
@pytest.mark.engine_fixed
@pytest.mark.parametrize("frac", [0.5, 1e-6], ids=["half-shared", "all-local"])
def test_split_three_shares_overlap_on_one_gpu(frac):
    """The compute-versus-gather split on three shares of one GPU (peer copies):
    the first S blocks are built share by share in chunks whose records are copied
    to the other replicas while the next chunk builds, the rest built by every
    part itself.  Every replica then answers lookups from its own records
    (spe_lookup_batch_replica) equal to the oracle, and download / get / min
    latency route to the part that built each row."""
    import torch
    from shadow_amd import spe
    top = graphs.gen_random_small(1200, 3600, 64)
    att = np.arange(top.n, dtype=np.int32)
    g = spe.Graph(top)
    t = spe.PathTable(g, att, devices=[0, 0, 0], engine=spe.SPE_ENGINE_BATCH, groups=1, shared_fraction=frac)
    st = t.build()
    nblk = t.nblocks
    sh, S = spe.device_split(top.n, 3, frac)
    assert st["shared_blocks"] == min(S, nblk) and st["local_blocks"] == nblk - min(S, nblk)
    assert st["gather"] == spe.SPE_GATHER_PEER
    ref = _check_table(t, top, att, f"split {frac}")
    for s_slot, t_slot in ((5, 900), (700, 3), (1199, 1199)):
        e = t.get(s_slot, t_slot)
        assert e["latency"] == ref["lat"][s_slot, t_slot] and e["hops"] == ref["hops"][s_slot, t_slot]
    q = 100_000
    gen = torch.Generator(device="cuda").manual_seed(9)
    pairs = torch.randint(0, t.A, (q, 2), dtype=torch.int32, device="cuda", generator=gen)
    p = pairs.cpu().numpy()
    for rep in range(3):
        assert t.replica_device(rep) == 0
        lat = torch.empty(q, dtype=torch.float64, device="cuda")
        rel = torch.empty(q, dtype=torch.float64, device="cuda")
        ok = torch.empty(q, dtype=torch.uint8, device="cuda")
        t.lookup_batch_replica(rep, pairs.data_ptr(), q, lat.data_ptr(), rel.data_ptr(), ok.data_ptr())
        np.testing.assert_array_equal(lat.cpu().numpy(), ref["lat"][p[:, 0], p[:, 1]], err_msg=f"replica {rep}")
        np.testing.assert_array_equal(rel.cpu().numpy(), ref["rel"][p[:, 0], p[:, 1]], err_msg=f"replica {rep}")
    assert t.min_latency() == ref["lat"][ref["kind"] != 0].min()
    with pytest.raises(spe.SpeError):
        t.replica_device(3)
