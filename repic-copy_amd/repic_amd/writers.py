"""Per-micrograph output files, exactly the set the reference writes.

reference get_cliques.py:125-129 (skip -> empty ``<base>.box``) and :204-229:
``<base>_weight_vector.pickle`` (float32[C]), ``<base>_consensus_coords.pickle`` (list of
``(x, y, id)`` tuples, or the ``--multi_out`` table), ``<base>_consensus_confidences.pickle``
(float32[C]), ``<base>_constraint_matrix.pickle`` (scipy ``coo_matrix``, int64 data, int32
indices, shape (V, C)) and ``<base>_runtime.tsv`` ("seconds\\tlargest CC\\tnumber of CCs").
All pickles use ``pickle.HIGHEST_PROTOCOL`` so the unchanged ``run_ilp`` reads them.
"""
from __future__ import annotations

import os
import pickle
from concurrent.futures import ThreadPoolExecutor

import numpy as np
from scipy.sparse import coo_matrix

LABELS = ("weight_vector", "consensus_coords", "consensus_confidences", "constraint_matrix")


def write_skip(out_dir: str, base: str):
    with open(os.path.join(out_dir, base + ".box"), "wt"):
        pass


def constraint_matrix(rows: np.ndarray, n_vert: int):
    """coo_matrix(([1]*nnz, (rows, cols)), shape=(V, C)) with cols = [j]*k (:192-202)."""
    C, k = rows.shape
    cols = np.repeat(np.arange(C, dtype=np.int32), k)
    data = np.ones(C * k, dtype=np.int64)
    return coo_matrix((data, (rows.reshape(-1).astype(np.int32), cols)), shape=(n_vert, C))


def consensus_coords(x, y, ids):
    return list(zip(x.tolist(), y.tolist(), ids.tolist()))


def multi_out_coords(methods, member_tuples, order, k, get_cc, picker_coords):
    """--multi_out table (get_cliques.py:175-178, 206-213).

    Members are sorted by the node attribute "name" that add_nodes_to_graph (:30-37)
    assigns: every node is (re)named ``node_names[0]`` when added as the first box of a
    pair and ``node_names[1]`` as the second, so clique members of pickers 0..k-2 end up
    ``methods[0]`` and the picker k-1 member ``methods[1]``; sorted() is stable, so the
    former keep networkx's node iteration order (``order``).
    """
    rows = [list(methods)]
    for j in range(len(member_tuples)):
        mt = member_tuples[j]
        first = [mt[p] for p in order[j] if p != k - 1]
        rows.append(first + [mt[k - 1]])
    if not get_cc:
        clique_set = set([val for clique in rows for val in clique])
        for p in range(k):
            for val in set(picker_coords[p]).difference(clique_set):
                e = [None] * k
                e[p] = val
                rows.append(e)
    return rows


def write_micrograph(out_dir, base, w, coords, conf, A, seconds, cc_max, cc_cnt):
    for label, val in zip(LABELS, (w, coords, conf, A)):
        with open(os.path.join(out_dir, f"{base}_{label}.pickle"), "wb") as o:
            pickle.dump(val, o, protocol=pickle.HIGHEST_PROTOCOL)
    with open(os.path.join(out_dir, f"{base}_runtime.tsv"), "wt") as o:
        o.write("\t".join([str(seconds), str(cc_max), str(cc_cnt)]) + "\n")


def write_micrograph_raw(out_dir, base, w, conf, rows, n_vert, cx, cy, cid, coords, seconds,
                         cc_max, cc_cnt):
    """write_micrograph from the device results: the consensus tuples and the COO matrix are
    built here (in the writer thread or process), not on the submitting thread."""
    if coords is None:
        coords = consensus_coords(cx, cy, cid)
    write_micrograph(out_dir, base, w, coords, conf, constraint_matrix(rows, n_vert), seconds,
                     cc_max, cc_cnt)


def _write_chunk(items):
    """Writer-process task: a chunk of (kind, args) writes, in order."""
    for kind, args in items:
        if kind == 0:
            write_skip(*args)
        elif kind == 1:
            write_micrograph_raw(*args)
        else:
            write_group(*args)
    return len(items)


def write_group(out_dir, items, w, conf, rows, cx, cy, cid):
    """Writer task for a group of micrographs in reference order, from flat arrays over the
    group's cliques (micrograph by micrograph): ``items`` = (base, n_cliques, n_vert, cc_max,
    cc_cnt, seconds, coords) per micrograph, or (base, -1, ...) for a skipped one (empty
    ``<base>.box``); ``coords`` is the prebuilt --multi_out table, else None and the
    consensus tuples come from cx / cy / cid."""
    c0 = 0
    for base, n, n_vert, cc_max, cc_cnt, seconds, coords in items:
        if n < 0:
            write_skip(out_dir, base)
            continue
        c1 = c0 + n
        write_micrograph_raw(out_dir, base, w[c0:c1], conf[c0:c1], rows[c0:c1], n_vert,
                             cx[c0:c1] if coords is None else None,
                             cy[c0:c1] if coords is None else None,
                             cid[c0:c1] if coords is None else None, coords, seconds, cc_max,
                             cc_cnt)
        c0 = c1


class Writer:
    """Pooled writer.  Pickling the per-micrograph objects holds the GIL, so large runs write
    from a pool of spawned processes (started early, chunks of ``chunk`` micrographs per
    task, raw arrays shipped, objects built in the worker); small runs use threads (file
    creation releases the GIL).  ``close()`` waits for every pending write and re-raises the
    first I/O error, so the files of every micrograph before a crash exist, as in the
    reference."""

    def __init__(self, threads=None, processes=False, chunk=32):
        self.threads = threads or min(16, (os.cpu_count() or 1))
        self.procs = bool(processes) and self.threads > 1
        self.chunk = chunk
        if self.procs:
            import multiprocessing as mp
            from concurrent.futures import ProcessPoolExecutor
            self._pool = ProcessPoolExecutor(self.threads, mp_context=mp.get_context("spawn"))
            for _ in range(self.threads):   # start the workers now: they import while the
                self._pool.submit(_write_chunk, [])   # device runs
        else:
            self._pool = ThreadPoolExecutor(max_workers=self.threads) if self.threads > 1 else None
        self._futs = []
        self._bases = set()
        self._items = []

    def _submit(self, kind, args):
        base = args[1]
        if base in self._bases:      # same output name twice: keep the reference's order
            self._flush()
            self._drain()
        self._bases.add(base)
        if self._pool is None:
            _write_chunk([(kind, args)])
        elif self.procs:
            self._items.append((kind, args))
            if len(self._items) >= self.chunk:
                self._flush()
        else:
            self._futs.append(self._pool.submit(_write_chunk, [(kind, args)]))
        if len(self._futs) > 4 * self.threads:
            self._drain(len(self._futs) // 2)

    def _flush(self):
        if self._items:
            self._futs.append(self._pool.submit(_write_chunk, self._items))
            self._items = []

    def _drain(self, n=None):
        n = len(self._futs) if n is None else n
        done, self._futs = self._futs[:n], self._futs[n:]
        for f in done:
            f.result()

    def skip(self, out_dir, base):
        self._submit(0, (out_dir, base))

    def micrograph(self, out_dir, base, w, conf, rows, n_vert, cx, cy, cid, coords, seconds,
                   cc_max, cc_cnt):
        self._submit(1, (out_dir, base, w, conf, rows, n_vert, cx, cy, cid, coords, seconds,
                         cc_max, cc_cnt))

    def group(self, out_dir, items, w, conf, rows, cx, cy, cid):
        """A group of micrographs (write_group) as one task; a base name already written
        earlier in the run waits for every pending write first (the reference's order)."""
        names = [it[0] for it in items]
        if any(b in self._bases for b in names):
            self._flush()
            self._drain()
        self._bases.update(names)
        args = (out_dir, items, w, conf, rows, cx, cy, cid)
        if self._pool is None:
            write_group(*args)
            return
        self._flush()
        self._futs.append(self._pool.submit(_write_chunk, [(2, args)]))
        if len(self._futs) > 4 * self.threads:
            self._drain(len(self._futs) // 2)

    def close(self):
        try:
            if self._pool is not None:
                self._flush()
            self._drain()
        finally:
            if self._pool is not None:
                self._pool.shutdown(wait=True)
