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


def gather_rows(values, group=None, device=None):
    """All-gather one int64 vector per rank -> list (by rank) of lists."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    world = dist.get_world_size(group)
    allv = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(allv, t, group=group)
    return [[int(v) for v in a.tolist()] for a in allv]


class PeerFailure(RuntimeError):
    """Another rank failed (its own exception is raised there)."""


def agree(local_exc, values=(), group=None, device=None):
    """One exchange after fallible per-rank work: every rank learns whether any rank failed
    (so no rank is left blocked in a later collective) and gets the gathered ``values``.
    Re-raises this rank's exception, or raises PeerFailure naming the failed ranks."""
    rows = gather_rows([0 if local_exc is None else 1] + list(values), group, device)
    bad = [r for r, row in enumerate(rows) if row[0]]
    if local_exc is not None:
        raise local_exc
    if bad:
        raise PeerFailure(f"get_cliques failed on rank(s) {bad}")
    return [row[1:] for row in rows]


def pair_work(sizes):
    """Pair-loop work estimate of one micrograph from its k per-picker box counts (or file
    sizes): sum over picker pairs j < l of n_j * n_l (get_cliques.py:135-138)."""
    s = np.asarray(sizes, dtype=np.float64)
    return float((s.sum() ** 2 - (s * s).sum()) / 2.0)


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
