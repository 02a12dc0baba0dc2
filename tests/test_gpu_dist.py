"""The N>1 path on the GPU: two ranks (processes) on one MI355X each build their
own contiguous source-block share of the table into caller-owned device buffers
(spe_table_opts.ext_*, as bench.py --full-table does per GPU), the shares are
all-gathered (gloo here; RCCL all_gather_into_tensor across GPUs), and the
assembled table must equal the oracle's rows."""
import os

import numpy as np
import pytest

from shadow_amd import dist as sd
from shadow_amd import graphs

pytestmark = [pytest.mark.gpu, pytest.mark.engine_fixed]


def _worker(rank, world, port, engine, out_q):
    try:
        import sys
        import torch
        import torch.distributed as dist
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, os.path.join(root, "oracle"))
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import Oracle
        from shadow_amd import spe
        top = graphs.gen_random_small(900, 2500, 12)
        A = np.arange(top.n, dtype=np.int32)
        per = sd.shard_blocks(top.n, world)
        b0, b1 = sd.rank_block_range(top.n, rank, world)
        elems = per * top.n * 64
        lr = torch.full((elems, 2), -1.0, dtype=torch.float64, device="cuda")
        nx = torch.full((elems,), -1, dtype=torch.int32, device="cuda")
        hp = torch.zeros(elems, dtype=torch.int16, device="cuda")
        g = spe.Graph(top, device=0)
        t = spe.PathTable(g, A, blocks=(b0, b1), ext=[lr.data_ptr(), nx.data_ptr(), hp.data_ptr()], engine=engine)
        t.build()
        torch.cuda.synchronize()
        shard = {"lr": lr.cpu(), "next": nx.cpu(), "hops": hp.cpu().view(torch.uint8).view(torch.int16)}
        full = sd.allgather_table(shard, world, dist)
        got = sd.sb64_to_rows({"lr": full["lr"].numpy(), "next": full["next"].numpy(),
                               "hops": full["hops"].numpy().view(np.uint16)}, top.n, 0, top.n)
        ref = Oracle(top).rows(A, A)
        ok = (all(np.array_equal(got[k], ref[k]) for k in ("lat", "rel", "next")) and
              np.array_equal(got["hops"].astype(np.int32), ref["hops"]))
        out_q.put((rank, ok))
        dist.destroy_process_group()
    except Exception as e:   # report instead of hanging the parent
        out_q.put((rank, repr(e)))


@pytest.mark.parametrize("engine", [1, 2], ids=["batch", "lds"])
def test_two_ranks_share_one_gpu_build_and_allgather(engine):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, engine, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=150) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
