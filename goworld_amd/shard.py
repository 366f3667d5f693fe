"""Space sharding across GPUs: one process per GPU, every
rank owns a contiguous block of spaces balanced by entity count.  GoWorld
spaces are independent AOI managers (Space.go:33), so the hot path has no
data exchange between ranks: each rank runs its own world and only the
benchmark's counters are reduced (MAX of the timed region, SUM of work).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def assign_spaces(counts: Sequence[int], world_size: int) -> List[Tuple[int, int]]:
    """Contiguous [begin, end) space ranges per rank, balanced by entity count.

    Rank r takes the spaces whose cumulative-count midpoint falls in
    [r*T/W, (r+1)*T/W) -- contiguous, deterministic, and within one space's
    count of the ideal share.  Empty ranks get an empty range.
    """
    c = np.asarray(counts, np.float64)
    if world_size < 1:
        raise ValueError("world_size must be >= 1")
    if c.size == 0:
        return [(0, 0)] * world_size
    T = c.sum()
    if T <= 0:
        cuts = np.linspace(0, c.size, world_size + 1).round().astype(int)
        return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world_size)]
    mid = np.cumsum(c) - c / 2.0
    owner = np.minimum((mid * world_size / T).astype(np.int64), world_size - 1)
    out = []
    for r in range(world_size):
        idx = np.nonzero(owner == r)[0]
        out.append((int(idx[0]), int(idx[-1]) + 1) if idx.size else (int(np.searchsorted(owner, r)),) * 2)
    return out


def reduce_over_ranks(dist, elapsed: float, work: Sequence[float], device) -> Tuple[float, List[float]]:
    """MAX of the timed region and SUM of the work counters over all ranks
    (the bench contract).  `dist` None = single process."""
    if dist is None:
        return float(elapsed), [float(w) for w in work]
    import torch
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([float(w) for w in work], dtype=torch.float64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return float(t.item()), [float(v) for v in s.tolist()]
