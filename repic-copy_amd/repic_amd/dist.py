"""Micrograph sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

SURVEY.md §8(e): micrographs are independent, so each rank takes a contiguous shard of the
reference-order micrograph list.  The only data-dependent exchange is the global box-id
offset of each shard (ids are a process-wide counter in the reference, common.py:23,108-112):
an ``all_gather`` of one int64 per rank.  After the run one ``all_reduce`` combines the
node-level counters, and one ``all_reduce(MIN)`` agrees on the first micrograph at which the
reference would have crashed so that no rank writes outputs beyond it.
"""
from __future__ import annotations

import numpy as np


def shard_bounds(weights, world: int):
    """Contiguous shard boundaries balancing the sum of ``weights`` (e.g. n_a*n_b pair work).

    Returns ``world + 1`` indices; shard r is ``[b[r], b[r+1])``.
    """
    w = np.asarray(weights, dtype=np.float64)
    n = len(w)
    if world <= 1 or n == 0:
        return [0] + [n] * max(world, 1)
    c = np.concatenate([[0.0], np.cumsum(w)])
    tot = c[-1]
    b = [0]
    for r in range(1, world):
        b.append(int(np.searchsorted(c, tot * r / world, side="left")))
    b.append(n)
    for r in range(1, world + 1):
        b[r] = max(b[r], b[r - 1])
    return b


def exclusive_offsets(values, group=None, device=None):
    """All-gather one int64 per rank and return (this rank's exclusive prefix, total)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(values)], dtype=torch.int64, device=device)
    world = dist.get_world_size(group)
    allv = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(allv, t, group=group)
    vals = [int(v.item()) for v in allv]
    r = dist.get_rank(group)
    return sum(vals[:r]), sum(vals)


def reduce_counts(counts, group=None, device=None):
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=device)
    dist.all_reduce(t, group=group)
    return [int(v) for v in t.tolist()]


def first_failure(local_index, group=None, device=None):
    """Global index of the first failing micrograph (``None`` where a rank has none)."""
    import torch
    import torch.distributed as dist
    big = np.iinfo(np.int64).max
    t = torch.tensor([big if local_index is None else int(local_index)], dtype=torch.int64,
                     device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    v = int(t.item())
    return None if v == big else v
