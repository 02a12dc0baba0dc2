"""Multi-GPU sharding of the path table.

Source rows are independent, so ranks own disjoint, contiguous runs of 64-row
source blocks and compute them with no communication.  When a replicated table
is wanted, every rank's SB64 block run is one contiguous span of each field, so
one all_gather_into_tensor per field (RCCL over xGMI; gloo on CPU in tests)
assembles the full table in place.  Equal shard sizes: the block count is
padded to a multiple of the world size (padding blocks hold unroutable rows).
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import numpy as np

WAVE = 64
FIELDS = (("lat", np.float64), ("rel", np.float64), ("next", np.int32), ("hops", np.uint16))


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
    """Host rows (row-major [rows][A]) -> SB64 fields covering `nblk` blocks starting at
    block row_begin // 64; missing rows are unroutable (-1 / -1 / -1 / 0)."""
    assert row_begin % WAVE == 0
    b0 = row_begin // WAVE
    out = {}
    fill = {"lat": -1.0, "rel": -1.0, "next": -1, "hops": 0}
    for name, dt in FIELDS:
        f = np.full(nblk * n_attached * WAVE, fill[name], dtype=dt)
        src = rows[name]
        for r in range(src.shape[0]):
            s = row_begin + r
            idx = sb64_index(s, np.arange(n_attached), n_attached, b0)
            f[idx] = src[r].astype(dt)
        out[name] = f
    return out


def sb64_to_rows(fields: Dict[str, np.ndarray], n_attached: int, row_begin: int, row_end: int) -> Dict[str, np.ndarray]:
    out = {}
    t = np.arange(n_attached)
    for name, _ in FIELDS:
        f = fields[name]
        out[name] = np.stack([f[sb64_index(s, t, n_attached)] for s in range(row_begin, row_end)])
    return out


def allgather_table(shard: Dict, world: int, dist):
    """all_gather_into_tensor each SB64 field.  `shard[name]` is a torch tensor
    holding this rank's padded block run; returns the full (padded) fields."""
    import torch
    full = {}
    gloo = dist.get_backend() == "gloo"
    for name, _ in FIELDS:
        x = shard[name]
        xb = x.view(torch.uint8)   # move raw bytes: not every backend takes uint16
        out = torch.empty(xb.numel() * world, dtype=torch.uint8, device=x.device)
        if gloo:
            parts = list(out.chunk(world))
            dist.all_gather(parts, xb)
            out = torch.cat(parts)
        else:
            dist.all_gather_into_tensor(out, xb)
        full[name] = out.view(x.dtype)
    return full
