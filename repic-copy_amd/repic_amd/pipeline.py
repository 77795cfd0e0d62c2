"""Batch packing and device execution of the get_cliques hot path.

Packs many micrographs into one SoA/CSR batch (``box_off`` per (micrograph, picker), x / y /
score f64 arrays, per-micrograph global id base) and runs ``rgc_run`` on it.  Results are
split back into per-micrograph records for the writers.
"""
from __future__ import annotations

import numpy as np

from . import _lib


class Batch:
    """Host-side packed batch."""

    def __init__(self, k, box_size, box_off, id_base, x, y, score):
        self.k, self.box_size = k, int(box_size)
        self.box_off = np.ascontiguousarray(box_off, np.int64)
        self.id_base = np.ascontiguousarray(id_base, np.int64)
        self.x = np.ascontiguousarray(x, np.float64)
        self.y = np.ascontiguousarray(y, np.float64)
        self.score = np.ascontiguousarray(score, np.float64)

    @property
    def n_mg(self):
        return len(self.id_base)

    @property
    def n_boxes(self):
        return int(self.box_off[-1])

    @classmethod
    def pack(cls, k, box_size, micrographs, id_bases=None):
        """``micrographs``: list of k (x, y, score) triples per micrograph."""
        counts = np.array([[len(t[0]) for t in mg] for mg in micrographs], np.int64).reshape(-1)
        box_off = np.zeros(len(counts) + 1, np.int64)
        np.cumsum(counts, out=box_off[1:])
        if id_bases is None:
            per_mg = counts.reshape(-1, k).sum(axis=1) if len(counts) else np.zeros(0, np.int64)
            id_bases = np.concatenate([[0], np.cumsum(per_mg)[:-1]]) if len(per_mg) else per_mg
        cat = lambda j: (np.concatenate([t[j] for mg in micrographs for t in mg])  # noqa: E731
                         if len(counts) else np.zeros(0))
        return cls(k, box_size, box_off, id_bases, cat(0), cat(1), cat(2))

    @classmethod
    def from_counts(cls, k, box_size, counts, x, y, score):
        """From per-(micrograph, picker) box counts and the concatenated arrays (synth.packed);
        id bases as in ``pack``."""
        counts = np.asarray(counts, np.int64)
        box_off = np.zeros(len(counts) + 1, np.int64)
        np.cumsum(counts, out=box_off[1:])
        per_mg = counts.reshape(-1, k).sum(axis=1)
        id_bases = np.concatenate([[0], np.cumsum(per_mg)[:-1]]) if len(per_mg) else per_mg
        return cls(k, box_size, box_off, id_bases, x, y, score)

    def slice(self, m0, m1):
        k = self.k
        b0, b1 = int(self.box_off[m0 * k]), int(self.box_off[m1 * k])
        return Batch(k, self.box_size, self.box_off[m0 * k:m1 * k + 1] - b0,
                     self.id_base[m0:m1], self.x[b0:b1], self.y[b0:b1], self.score[b0:b1])


class MgResult:
    __slots__ = ("status", "cc_max", "cc_cnt", "n_vert", "n_edges", "rows", "w", "conf",
                 "consensus", "members", "order")


def run_batch(ctx: _lib.Context, batch: Batch, get_cc=False, multi_out=False, timing=False,
              members=False, no_fused=False):
    """Run one packed batch on the device; returns list[MgResult] (batch-local box indices)."""
    flags = _lib.F_HOST_OUTPUTS
    if members:
        flags |= _lib.F_MEMBERS
    if no_fused:
        flags |= _lib.F_NO_FUSED
    if get_cc:
        flags |= _lib.F_GET_CC
    if multi_out:
        flags |= _lib.F_MULTI_OUT
    if timing:
        flags |= _lib.F_TIMING
    r = ctx.run(batch.n_mg, batch.k, batch.box_size, batch.box_off, batch.id_base, batch.x,
                batch.y, batch.score, flags)
    out = []
    for m in range(batch.n_mg):
        q = MgResult()
        q.status = int(r.status[m])
        q.cc_max, q.cc_cnt = int(r.cc_max[m]), int(r.cc_cnt[m])
        q.n_vert, q.n_edges = int(r.n_vert[m]), int(r.n_edges_mg[m])
        c0 = int(r.clique_base[m])
        c1 = c0 + int(r.clique_cnt[m])
        q.rows = r.rows[c0:c1].copy()
        q.w = r.w[c0:c1].copy()
        q.conf = r.conf[c0:c1].copy()
        q.consensus = r.consensus[c0:c1].copy()
        q.members = r.members[c0:c1].copy() if r.members is not None else None
        q.order = r.order[c0:c1].copy() if r.order is not None else None
        out.append(q)
    return out


def split_batches(counts_per_mg, max_boxes):
    """Contiguous micrograph ranges with at most ``max_boxes`` boxes each (>= 1 mg)."""
    out, start, acc = [], 0, 0
    for i, c in enumerate(counts_per_mg):
        if i > start and acc + c > max_boxes:
            out.append((start, i))
            start, acc = i, 0
        acc += c
    if start < len(counts_per_mg):
        out.append((start, len(counts_per_mg)))
    return out
