"""N>1 path on CPU: source-block sharding and the table all-gather, world_size 2
over gloo (the GPU path uses the same code over RCCL)."""
import os

import numpy as np
import pytest

from shadow_amd import dist as sd
from shadow_amd import graphs


def test_shard_ranges_cover_every_block_once():
    for A in (1, 63, 64, 65, 150, 50000):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                b0, b1 = sd.rank_block_range(A, r, world)
                seen += list(range(b0, b1))
            assert seen == list(range(sd.nblocks(A)))


def test_sb64_roundtrip_matches_layout():
    sys_path_oracle()
    from oracle import Oracle
    top = graphs.gen_random_small(150, 400, 3)
    A = np.arange(top.n, dtype=np.int32)
    r = Oracle(top).rows(A, A)
    r["hops"] = r["hops"].astype(np.uint16)
    f = sd.rows_to_sb64(r, 0, top.n, sd.nblocks(top.n))
    back = sd.sb64_to_rows(f, top.n, 0, top.n)
    for k in ("lat", "rel", "next"):
        np.testing.assert_array_equal(back[k], r[k])
    # element (s, t) is where include/spe.h says it is
    s, t = 77, 12
    e = ((s // 64) * top.n + t) * 64 + s % 64
    assert f["lr"][e, 0] == r["lat"][s, t] and f["lr"][e, 1] == r["rel"][s, t] and f["next"][e] == r["next"][s, t]


def sys_path_oracle():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = os.path.join(root, "oracle")
    if p not in sys.path:
        sys.path.insert(0, p)


def _worker(rank, world, port, out_q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys_path_oracle()
    from oracle import Oracle
    top = graphs.gen_random_small(200, 600, 5)
    A = np.arange(top.n, dtype=np.int32)
    per = sd.shard_blocks(top.n, world)
    b0, b1 = sd.rank_block_range(top.n, rank, world)
    rows = Oracle(top).rows(A[b0 * 64:min(top.n, b1 * 64)], A)   # this rank's source rows only
    rows["hops"] = rows["hops"].astype(np.uint16)
    shard = sd.rows_to_sb64(rows, rank * per * 64, top.n, per)
    tshard = {k: torch.from_numpy(v) for k, v in shard.items()}
    full = sd.allgather_table(tshard, world, dist)
    got = sd.sb64_to_rows({k: v.numpy() for k, v in full.items()}, top.n, 0, top.n)
    ref = Oracle(top).rows(A, A)
    ok = all(np.array_equal(got[k], ref[k]) for k in ("lat", "rel", "next")) and \
        np.array_equal(got["hops"].astype(np.int32), ref["hops"])
    out_q.put((rank, ok))
    dist.destroy_process_group()


def test_gloo_world2_sharded_build_and_allgather():
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def test_chunk_plan_covers_every_block_once():
    for nblk in (1, 7, 157, 782, 1563):
        for world in (1, 2, 3, 8):
            for groups in (1, 16, 48, 64):
                rounds, G = sd.chunk_plan(nblk, world, groups)
                assert 1 <= G <= max(1, groups) and rounds * world * G >= nblk
                assert rounds * world * G - nblk < world * rounds   # balanced padding
                seen = []
                for r in range(world):
                    for k, c, b0, b1 in sd.rank_chunks(nblk, world, r, rounds, G):
                        assert c == k * world + r
                        seen += list(range(b0, b1))
                assert sorted(seen) == list(range(nblk))


def test_chunk_schedule_front_loaded_and_covering():
    """bench.py's N > 1 rounds: a short first round, then rounds of `groups`, the
    last trimmed; every block built exactly once, rounds contiguous."""
    for nblk in (1, 7, 157, 782, 1563):
        for world in (1, 2, 3, 8):
            for groups in (1, 16, 25, 98):
                sizes = sd.chunk_schedule(nblk, world, groups)
                assert all(1 <= g <= max(1, groups) for g in sizes)
                assert world * sum(sizes) >= nblk
                if world > 1 and len(sizes) > 1:
                    assert sizes[0] <= -(-groups // 4)
                seen, off = [], 0
                for r in range(world):
                    ch = sd.rank_chunks_sched(nblk, world, r, sizes)
                    assert [c[1] for c in ch] == list(np.cumsum([0] + [world * g for g in sizes[:-1]]))
                    for k, o, g, b0, b1 in ch:
                        assert b0 == min(nblk, o + r * g) and b1 == min(nblk, o + (r + 1) * g)
                        seen += list(range(b0, b1))
                assert sorted(seen) == list(range(nblk))


def _sched_worker(rank, world, port, out_q, mode="all_gather"):
    """The same with chunk_schedule + allgather_span (what bench.py runs); mode
    "p2p" gathers with allgather_span_p2p (world - 1 concurrent peer exchanges,
    asynchronous and waited at the end, as bench.py overlaps them)."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys_path_oracle()
    from oracle import Oracle
    top = graphs.gen_random_small(700, 2100, 8)
    A = np.arange(top.n, dtype=np.int32)
    nblk = sd.nblocks(top.n)
    sizes = sd.chunk_schedule(nblk, world, 2)
    blk = top.n * 64
    lr = torch.full((world * sum(sizes) * blk, 2), float("nan"), dtype=torch.float64)
    o = Oracle(top)
    works = []
    for k, off, g, b0, b1 in sd.rank_chunks_sched(nblk, world, rank, sizes):
        if b1 > b0:
            rows = o.rows(A[b0 * 64:min(top.n, b1 * 64)], A)
            rows["hops"] = rows["hops"].astype(np.uint16)
            f = sd.rows_to_sb64(rows, b0 * 64, top.n, b1 - b0)
            lr[b0 * blk:b1 * blk] = torch.from_numpy(f["lr"])
        if mode == "p2p":
            w = sd.allgather_span_p2p(lr, off, g, world, rank, blk, dist, async_op=True)
            if w is not None:
                works.append(w)
        else:
            sd.allgather_span(lr, off, g, world, rank, blk, dist)
    for w in works:
        w.wait()
    ref = o.rows(A, A)
    e = sd.sb64_index(np.repeat(A, top.n), np.tile(A, top.n), top.n)
    got = lr.numpy()[e]
    ok = np.array_equal(got[:, 0], ref["lat"].ravel()) and np.array_equal(got[:, 1], ref["rel"].ravel())
    out_q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "all_gather"), (3, "all_gather"), (2, "p2p"), (3, "p2p")])
def test_gloo_chunk_schedule_allgather(world, mode):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sched_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def _chunk_worker(rank, world, port, out_q):
    """bench.py's N > 1 step on CPU: round-robin chunks, each round's records
    all-gathered in place (sd.allgather_round) into the replicated SB64 table."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys_path_oracle()
    from oracle import Oracle
    top = graphs.gen_random_small(300, 900, 6)
    A = np.arange(top.n, dtype=np.int32)
    nblk = sd.nblocks(top.n)
    rounds, G = sd.chunk_plan(nblk, world, 2)
    chunk_elems = G * top.n * 64
    lr = torch.full((rounds * world * chunk_elems, 2), float("nan"), dtype=torch.float64)
    o = Oracle(top)
    for k, c, b0, b1 in sd.rank_chunks(nblk, world, rank, rounds, G):
        if b1 > b0:   # this rank's rows, written where the table keeps them
            rows = o.rows(A[b0 * 64:min(top.n, b1 * 64)], A)
            rows["hops"] = rows["hops"].astype(np.uint16)
            f = sd.rows_to_sb64(rows, b0 * 64, top.n, G)
            lr[c * chunk_elems:(c + 1) * chunk_elems] = torch.from_numpy(f["lr"])
        sd.allgather_round(lr, k, world, rank, chunk_elems, dist)
    ref = o.rows(A, A)
    e = sd.sb64_index(np.repeat(A, top.n), np.tile(A, top.n), top.n)
    got = lr.numpy()[e]
    ok = np.array_equal(got[:, 0], ref["lat"].ravel()) and np.array_equal(got[:, 1], ref["rel"].ravel())
    out_q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_round_robin_chunks_allgather(world):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_chunk_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def test_shared_fraction_model():
    """dist.shared_fraction: x* = T1 N / ((N - 1)(S / B + T1)), clipped."""
    assert sd.shared_fraction(1, 0.3, 160e9, 300e9) == 1.0
    x4 = sd.shared_fraction(8, 0.28, 160e9, 300e9)     # C4 at N = 8: share ~40 %, recompute the rest
    assert 0.35 < x4 < 0.45
    x3 = sd.shared_fraction(8, 0.45, 40e9, 300e9)      # C3: mostly shared
    assert x4 < x3 < 1.0
    assert sd.shared_fraction(8, 5.0, 1e6, 300e9) == 1.0   # gathers are free: shard everything
    # at x*, the build and the gather terms of the model meet
    N, t1, S, B = 8, 0.28, 160e9, 300e9
    x = sd.shared_fraction(N, t1, S, B)
    assert abs(t1 * (x / N + 1 - x) - x * (N - 1) / N * S / B) < 1e-9


def test_split_schedule_covers_every_block_once():
    """Sharded rounds (every gathered part inside [0, S)) plus the local remainder
    [S, nblk) every rank builds: each block is built by exactly one rank or by all
    ranks, and a rank's packed next-hop slots cover exactly what it built."""
    for nblk in (1, 9, 157, 782, 1563):
        for world in (2, 3, 8):
            for groups in (1, 26, 391):
                for frac in (0.0, 0.1, 0.39, 0.88, 1.0):
                    sizes, S = sd.split_schedule(nblk, world, groups, frac)
                    l0, l1 = sd.local_span(nblk, S)
                    if frac < 1.0:
                        assert S <= nblk and S == world * sum(sizes)
                    else:
                        assert S >= nblk and l1 == l0
                    shared = []
                    for r in range(world):
                        built = []
                        for k, off, g, b0, b1 in sd.rank_chunks_sched(nblk, world, r, sizes):
                            assert off + world * g <= max(S, nblk) or frac >= 1.0
                            built += list(range(b0, b1))
                        shared += built
                        slots, nslot = sd.rank_next_hop_slots(nblk, world, r, sizes, S)
                        packed = []
                        for b0, b1, s0 in slots:
                            assert s0 == len(packed)
                            packed += list(range(b0, b1))
                        assert packed == built + list(range(l0, l1)) and nslot == len(packed)
                    assert sorted(shared) == list(range(min(S, nblk)))
                    assert sorted(shared + list(range(l0, l1))) == list(range(nblk))


def _split_worker(rank, world, port, out_q):
    """bench.py's N > 1 step with the compute-versus-gather split on a reduced
    C4-shaped workload (tiered graph, stub hosts): sharded rounds all-gathered in
    place, the remainder built by every rank; every rank must end with the whole
    record span, and its packed next hops / hop counts equal the oracle's for the
    blocks it built."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys_path_oracle()
    from oracle import Oracle
    top = graphs.gen_tiered(n_core=300, n_stub=1200, n_attached=700, seed=9)
    A = graphs.tiered_attached(top, n_core=300, n_attached=700)
    nA = A.shape[0]
    nblk = sd.nblocks(nA)
    sizes, S = sd.split_schedule(nblk, world, 2, 0.45)
    l0, l1 = sd.local_span(nblk, S)
    blk = nA * 64
    lr = torch.full((max(S, nblk) * blk, 2), float("nan"), dtype=torch.float64)
    slots, nslot = sd.rank_next_hop_slots(nblk, world, rank, sizes, S)
    nx = np.full(nslot * blk, -7, dtype=np.int32)
    hp = np.zeros(nslot * blk, dtype=np.uint16)
    slot_of = {(b0, b1): s0 for b0, b1, s0 in slots}
    o = Oracle(top)

    def build(b0, b1):
        rows = o.rows(A[b0 * 64:min(nA, b1 * 64)], A)
        rows["hops"] = rows["hops"].astype(np.uint16)
        f = sd.rows_to_sb64(rows, b0 * 64, nA, b1 - b0)
        lr[b0 * blk:b1 * blk] = torch.from_numpy(f["lr"])
        s0 = slot_of[(b0, b1)]
        nx[s0 * blk:(s0 + b1 - b0) * blk] = f["next"]
        hp[s0 * blk:(s0 + b1 - b0) * blk] = f["hops"]

    for k, off, g, b0, b1 in sd.rank_chunks_sched(nblk, world, rank, sizes):
        if b1 > b0:
            build(b0, b1)
        sd.allgather_span(lr, off, g, world, rank, blk, dist)
    if l1 > l0:
        build(l0, l1)
    ref = o.rows(A, A)
    e = sd.sb64_index(np.repeat(np.arange(nA), nA), np.tile(np.arange(nA), nA), nA)
    got = lr.numpy()[e]
    ok = np.array_equal(got[:, 0], ref["lat"].ravel()) and np.array_equal(got[:, 1], ref["rel"].ravel())
    for b0, b1, s0 in slots:
        for s in range(b0 * 64, min(nA, b1 * 64)):
            idx = sd.sb64_index(s, np.arange(nA), nA, b0) + s0 * blk
            ok &= np.array_equal(nx[idx], ref["next"][s]) and np.array_equal(hp[idx].astype(np.int32), ref["hops"][s])
    out_q.put((rank, bool(ok), S, l1 - l0))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_split_schedule_c4_shaped(world):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] for r in res), res
    assert all(r[2] > 0 and r[3] > 0 for r in res)   # both parts of the split ran
