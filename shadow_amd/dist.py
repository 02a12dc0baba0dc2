"""Multi-GPU sharding of the path table, one process per GPU.

Source rows are independent, so ranks compute disjoint sets of 64-row source
blocks with no communication.  Two layouts:
  * contiguous shares (rank_block_range): one run of blocks per rank, one
    all_gather_into_tensor per field at the end (also what the in-library
    multi-device table does, spe_device_shares);
  * round-robin chunks (chunk_plan / rank_chunks, bench.py): the blocks are
    dealt in rounds of world x G, one build launch per rank per round, and each
    round's records are all-gathered IN PLACE (they are contiguous in the SB64
    table) while the next round builds -- the gather hides behind the build.
Equal shard sizes: the block count is padded (padding blocks are never read).
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import numpy as np

WAVE = 64
# table fields as stored on the device (include/spe.h spe_table_layout):
# "lr" = {latency, reliability} f64 pairs, then next hop and hop count
FIELDS = (("lr", np.float64, 2), ("next", np.int32, 1), ("hops", np.uint16, 1))


def nblocks(n_attached: int) -> int:
    return (n_attached + WAVE - 1) // WAVE


def shard_blocks(n_attached: int, world: int) -> int:
    """Blocks per rank (padded so every rank holds the same number)."""
    return max(1, math.ceil(nblocks(n_attached) / world))


def rank_block_range(n_attached: int, rank: int, world: int) -> Tuple[int, int]:
    """[b0, b1) of real blocks owned by `rank` (may be empty for trailing ranks)."""
    per = shard_blocks(n_attached, world)
    nb = nblocks(n_attached)
    return min(nb, rank * per), min(nb, (rank + 1) * per)


def sb64_index(s_slot, t_slot, n_attached: int, block_begin: int = 0):
    """Element offset of (s, t) in an SB64 field (include/spe.h spe_table_layout)."""
    s_slot = np.asarray(s_slot, np.int64)
    t_slot = np.asarray(t_slot, np.int64)
    return ((s_slot // WAVE - block_begin) * n_attached + t_slot) * WAVE + s_slot % WAVE


def rows_to_sb64(rows: Dict[str, np.ndarray], row_begin: int, n_attached: int, nblk: int) -> Dict[str, np.ndarray]:
    """Host rows (row-major [rows][A]: lat, rel, next, hops) -> SB64 fields covering
    `nblk` blocks starting at block row_begin // 64; missing rows are unroutable
    (-1 / -1 / -1 / 0)."""
    assert row_begin % WAVE == 0
    b0 = row_begin // WAVE
    elems = nblk * n_attached * WAVE
    lr = np.full((elems, 2), -1.0, dtype=np.float64)
    nxt = np.full(elems, -1, dtype=np.int32)
    hops = np.zeros(elems, dtype=np.uint16)
    for r in range(rows["lat"].shape[0]):
        idx = sb64_index(row_begin + r, np.arange(n_attached), n_attached, b0)
        lr[idx, 0] = rows["lat"][r]
        lr[idx, 1] = rows["rel"][r]
        nxt[idx] = rows["next"][r]
        hops[idx] = rows["hops"][r].astype(np.uint16)
    return {"lr": lr, "next": nxt, "hops": hops}


def sb64_to_rows(fields: Dict[str, np.ndarray], n_attached: int, row_begin: int, row_end: int) -> Dict[str, np.ndarray]:
    t = np.arange(n_attached)
    idx = [sb64_index(s, t, n_attached) for s in range(row_begin, row_end)]
    lr = np.asarray(fields["lr"]).reshape(-1, 2)
    return {"lat": np.stack([lr[i, 0] for i in idx]), "rel": np.stack([lr[i, 1] for i in idx]),
            "next": np.stack([fields["next"][i] for i in idx]), "hops": np.stack([fields["hops"][i] for i in idx])}


def allgather_table(shard: Dict, world: int, dist):
    """all_gather_into_tensor each SB64 field.  `shard[name]` is a torch tensor
    holding this rank's padded block run; returns the full (padded) fields."""
    import torch
    full = {}
    gloo = dist.get_backend() == "gloo"
    for name, _, _ in FIELDS:
        x = shard[name]
        xb = x.contiguous().view(-1).view(torch.uint8)   # raw bytes: not every backend takes uint16
        out = torch.empty(xb.numel() * world, dtype=torch.uint8, device=x.device)
        if gloo:
            parts = list(out.chunk(world))
            dist.all_gather(parts, xb)
            out = torch.cat(parts)
        else:
            dist.all_gather_into_tensor(out, xb)
        full[name] = out.view(x.dtype).reshape((-1,) + tuple(x.shape[1:]))
    return full


def chunk_plan(nblk: int, world: int, groups: int) -> Tuple[int, int]:
    """(rounds, G): rounds of world x G blocks, G <= groups (one build launch),
    balanced so the padding is at most world x rounds - 1 blocks."""
    rounds = max(1, math.ceil(nblk / (world * max(1, groups))))
    return rounds, math.ceil(nblk / (world * rounds))


def rank_chunks(nblk: int, world: int, rank: int, rounds: int, G: int):
    """[(round, chunk, b0, b1)] of `rank`: chunk c = round * world + rank covers
    blocks [c * G, (c + 1) * G) clipped to nblk (may be empty)."""
    out = []
    for k in range(rounds):
        c = k * world + rank
        out.append((k, c, min(nblk, c * G), min(nblk, (c + 1) * G)))
    return out


def chunk_schedule(nblk: int, world: int, groups: int, lead: int = 4):
    """Per-round chunk sizes (blocks per rank) for the overlapped build + gather:
    round k covers the contiguous blocks [off_k, off_k + world * sizes[k]).  At
    N > 1 the first round is short (groups / lead) so the first all-gather starts
    early -- the step is then about the first build plus the gathers, which xGMI
    bounds -- then rounds of `groups`; the last one is trimmed to what
    is left.  N = 1: uniform rounds (chunk_plan's)."""
    groups = max(1, groups)
    if world <= 1:
        rounds, G = chunk_plan(nblk, 1, groups)
        return [G] * rounds
    sizes, left = [], nblk
    first = max(1, -(-groups // lead))
    while left > 0:
        g = first if not sizes else groups
        g = min(g, -(-left // world))
        sizes.append(g)
        left -= world * g
    return sizes


def rank_chunks_sched(nblk: int, world: int, rank: int, sizes):
    """[(round, first block of the round, size, b0, b1)] of `rank` under chunk_schedule."""
    out, off = [], 0
    for k, g in enumerate(sizes):
        out.append((k, off, g, min(nblk, off + rank * g), min(nblk, off + (rank + 1) * g)))
        off += world * g
    return out


def allgather_span(lr, off: int, g: int, world: int, rank: int, blk_elems: int, dist, async_op: bool = False):
    """All-gather one chunk_schedule round in place: blocks [off, off + world * g)
    of the SB64 records, rank r's part being [off + r g, off + (r + 1) g)."""
    grp = lr[off * blk_elems:(off + world * g) * blk_elems]
    own = lr[(off + rank * g) * blk_elems:(off + (rank + 1) * g) * blk_elems]
    if dist.get_backend() == "gloo":
        parts = [p.clone() for p in grp.chunk(world)]
        dist.all_gather(parts, own.clone())
        for p, dst in zip(parts, grp.chunk(world)):
            dst.copy_(p)
        return None
    return dist.all_gather_into_tensor(grp, own, async_op=async_op)


class _Requests:
    """The P2P requests of one gather, waited on together (the async handle)."""

    def __init__(self, reqs):
        self.reqs = list(reqs)

    def wait(self):
        for r in self.reqs:
            r.wait()
        return True


def allgather_span_p2p(lr, off: int, g: int, world: int, rank: int, blk_elems: int, dist, async_op: bool = False):
    """The same in-place gather as allgather_span, as world - 1 concurrent
    point-to-point exchanges per rank (one batch_isend_irecv group: every peer's part
    arrives over its own xGMI link at once, SURVEY §5's 7 concurrent peer copies per
    GPU) instead of the collective's own algorithm.  bench.py measures both and
    gathers with the faster (split.calibration)."""
    grp = lr[off * blk_elems:(off + world * g) * blk_elems]
    parts = list(grp.chunk(world))
    own = parts[rank]
    ops = []
    for p in range(world):
        if p == rank:
            continue
        ops.append(dist.P2POp(dist.isend, own, p))
        ops.append(dist.P2POp(dist.irecv, parts[p], p))
    if not ops:
        return None
    reqs = _Requests(dist.batch_isend_irecv(ops))
    if async_op:
        return reqs
    reqs.wait()
    return None


def allgather_round(lr, k: int, world: int, rank: int, chunk_elems: int, dist, async_op: bool = False):
    """All-gather round k's records in place: rank r's chunk (k * world + r) sits
    at element (k * world + r) * chunk_elems of `lr` on every rank, so the round
    is one contiguous span (RCCL all_gather_into_tensor; gloo on CPU gathers a
    list and copies back)."""
    grp = lr[k * world * chunk_elems:(k + 1) * world * chunk_elems]
    own = lr[(k * world + rank) * chunk_elems:(k * world + rank + 1) * chunk_elems]
    if dist.get_backend() == "gloo":
        parts = [p.clone() for p in grp.chunk(world)]
        dist.all_gather(parts, own.clone())
        for p, dst in zip(parts, grp.chunk(world)):
            dst.copy_(p)
        return None
    return dist.all_gather_into_tensor(grp, own, async_op=async_op)


# ---- compute-versus-gather split.  Gathering a share costs xGMI time,
# recomputing it costs build time: with T1 the one-GPU whole-table build time and
# S / B the time to receive the whole record span, sharding a fraction x of the
# blocks (built once, all-gathered) and building the rest [S, nblk) on every rank
# (no exchange) takes about max(T1 (x / N + 1 - x), x (N - 1) / N S / B) when the
# gathers overlap the local builds.  The two terms meet at
#   x* = T1 N / ((N - 1) (S / B + T1)),
# clipped to [0, 1] (x = 1: pure sharding, the C3 regime; C4 at N = 8 with
# S = 160 GB: x* ~ 0.4).

def shared_fraction(world: int, t1_s: float, span_bytes: float, gather_bps: float) -> float:
    """x*: the fraction of the source blocks to shard and all-gather (the rest is
    built by every rank), from the one-GPU build time and the gather bandwidth."""
    if world <= 1:
        return 1.0
    if gather_bps <= 0 or t1_s <= 0:
        return 1.0
    x = t1_s * world / ((world - 1) * (span_bytes / gather_bps + t1_s))
    return float(min(1.0, max(0.0, x)))


def split_schedule(nblk: int, world: int, groups: int, shared_frac: float, lead: int = 4):
    """(sizes, S): chunk_schedule rounds over the first S blocks (every round holds
    world equal parts, so S = world * sum(sizes) and no gathered part reaches past
    S), and the local remainder [S, nblk) that every rank builds itself.
    shared_frac >= 1 (or a world of 1): every block sharded, S may exceed nblk
    (padding blocks, never read)."""
    if world <= 1 or shared_frac >= 1.0:
        sizes = chunk_schedule(nblk, world, groups, lead)
        return sizes, world * sum(sizes)
    want = int(math.floor(max(0.0, shared_frac) * nblk / world))   # blocks per rank
    if want <= 0:
        return [], 0
    sizes = chunk_schedule(want * world, world, groups, lead)
    return sizes, world * sum(sizes)


def local_span(nblk: int, S: int) -> Tuple[int, int]:
    """The blocks every rank builds itself under split_schedule."""
    return min(nblk, S), nblk


def rank_next_hop_slots(nblk: int, world: int, rank: int, sizes, S: int):
    """Where a rank keeps next hop / hop count: its own sharded chunks, then the
    local remainder, packed contiguously -> [(b0, b1, slot0)] with slot0 the first
    packed block of [b0, b1), and the packed block count."""
    out, slot = [], 0
    for _, _, _, b0, b1 in rank_chunks_sched(nblk, world, rank, sizes):
        if b1 > b0:
            out.append((b0, b1, slot))
            slot += b1 - b0
    l0, l1 = local_span(nblk, S)
    if l1 > l0:
        out.append((l0, l1, slot))
        slot += l1 - l0
    return out, slot
