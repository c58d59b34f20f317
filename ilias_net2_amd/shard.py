"""Sharding a packet batch over ranks (one process per GPU).

Packets are independent, so a global batch is split into
contiguous slices with no data-path collective; each rank hashes its slice on
its own device.  The byte-balanced split for variable-length batches is the
same rule the C ABI's multi-device ``net2_sha2_batch`` uses
(csrc/sha2_shim.cpp): device d starts at the first packet whose running byte
count reaches d/N of the total.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np


def shard_range(n: int, world: int, rank: int):
    """Contiguous [lo, hi) slice of n equal-cost packets for `rank`."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return n * rank // world, n * (rank + 1) // world


def shard_cuts_by_bytes(lens: Sequence[int], world: int) -> List[int]:
    """world+1 cut points over packets so each slice carries ~equal bytes."""
    lens = np.asarray(lens, dtype=np.uint64)
    n = len(lens)
    nd = max(1, min(world, n)) if n else 1
    cuts = [0] * (world + 1)
    cuts[world] = n
    if n == 0:
        return cuts
    total = int(lens.sum())
    csum = np.cumsum(lens)
    d = 1
    for i in range(n):
        while d < nd and int(csum[i]) * nd >= total * d:
            cuts[d] = i + 1
            d += 1
        if d >= nd:
            break
    for k in range(d, world):
        cuts[k] = n
    return cuts


def gather_digests(local: np.ndarray, group=None) -> Optional[np.ndarray]:
    """All-gather per-rank digest slices (rank order) into the full array.

    Used for verification only; the hot path never moves digests between
    ranks."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(local))
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(dist.get_world_size(group))]
    dist.all_gather(sizes, torch.tensor([t.shape[0]], dtype=torch.int64), group=group)
    mx = int(max(s.item() for s in sizes))
    pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype)
    pad[: t.shape[0]] = t
    bufs = [torch.zeros_like(pad) for _ in sizes]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[: int(s.item())] for b, s in zip(bufs, sizes)]).numpy()
